#!/bin/bash
# steady-state A/B (300-tick burn-in) of the round-2 final kernel vs now; rocprofv3 passes of c2 and c5
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3x
mkdir -p $O
export ASTRO_AB_ANY_ABI=1
for wl in c3 c2 c5; do
  timeout -k 10 300 python tools/ab.py --libs libastro_hip_r2,libastro_hip_dpp --workload $wl --rounds 4 > $O/ab_r2_$wl.log 2>&1 || exit $?
  grep '^{' $O/ab_r2_$wl.log | cut -c1-200
done
unset ASTRO_AB_ANY_ABI
WLS="c2 c5" bash tools/gpu_r3r.sh
