#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp ASTRO_AB_ANY_ABI=1
mkdir -p gpurun_out/r3i
timeout -k 10 300 python tools/ab.py --libs libastro_hip_q4,libastro_hip_nodraw,libastro_hip_nopend,libastro_hip_nopd --workload c3 --rounds 5 > gpurun_out/r3i/ab_ablate_reset.log 2>&1
rc=$?; grep "^{" gpurun_out/r3i/ab_ablate_reset.log; exit $rc
