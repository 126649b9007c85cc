#!/bin/bash
# quad instance: planet update on the helpers (qpl) vs on the step waves (dpp); round-2 kernel vs now; rocprofv3 passes of c3
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3v
mkdir -p $O
export ASTRO_AB_ANY_ABI=1
timeout -k 10 300 python tools/ab.py --libs libastro_hip_dpp,libastro_hip_qpl --workload c2 --rounds 5 > $O/ab_c2.log 2>&1 || exit $?
grep '^{' $O/ab_c2.log | cut -c1-200
for wl in c3 c2 c5; do   # the round-2 final kernel (a2820fe, ABI 12) vs the current one
  timeout -k 10 300 python tools/ab.py --libs libastro_hip_r2,libastro_hip_dpp --workload $wl --rounds 5 > $O/ab_r2_$wl.log 2>&1 || exit $?
  grep '^{' $O/ab_r2_$wl.log | cut -c1-200
done
unset ASTRO_AB_ANY_ABI
WLS=c3 bash tools/gpu_r3r.sh
