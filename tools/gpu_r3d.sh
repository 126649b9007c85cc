#!/bin/bash
# Regression hunt vs the round-2 build + the driver-style bench lines and
# their rocprofv3 kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3d
mkdir -p $O
step() {
  local name=$1 limit=$2; shift 2
  local t0=$SECONDS
  timeout -k 10 "$limit" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc $((SECONDS - t0))s"
  tail -2 $O/$name.log | cut -c1-300
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return $rc
}
export ASTRO_AB_ANY_ABI=1
step ab_c3 300 python tools/ab.py --libs libastro_hip_r2,libastro_hip_cur,libastro_hip_noseen --workload c3 --rounds 5
step ab_c2 300 python tools/ab.py --libs libastro_hip_r2,libastro_hip_cur,libastro_hip_noseen --workload c2 --rounds 4
step stamps_cur 200 python tools/stamps_r3.py --workload c3 --lib libastro_hip_stamps
step stamps_r2 200 python tools/stamps_r3.py --workload c3 --lib libastro_hip_r2stamps
unset ASTRO_AB_ANY_ABI
step bench20 300 python bench.py --steps 20 --warmup 5
step bench1000 300 python bench.py --no-cpu --no-single
step prof20 300 rocprofv3 --kernel-trace --stats -d $O/prof20 -o run -f csv -- python bench.py --steps 20 --warmup 5 --no-cpu --no-single
step prof1000 300 rocprofv3 --kernel-trace --stats -d $O/prof1000 -o run -f csv -- python bench.py --no-cpu --no-single
exit 0
