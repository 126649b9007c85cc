#!/bin/bash
# Round-3 GPU session on the committed library: GPU tests, smoke, the
# driver-style short bench and the long one, c5/c2 lines, the helper
# fault-injection check, and rocprofv3 kernel stats of the driver-style run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3c
mkdir -p $O
step() {
  local name=$1 limit=$2; shift 2
  local t0=$SECONDS
  timeout -k 10 "$limit" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc $((SECONDS - t0))s"
  tail -2 $O/$name.log | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return $rc
}
step pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step bench20 300 python bench.py --steps 20 --warmup 5
step bench1000 300 python bench.py --no-cpu --no-single
step bench_c5 300 python bench.py --workload c5 --no-cpu --no-single
step bench_c2 300 python bench.py --workload c2 --no-cpu --no-single
ASTRO_LIB=astro_amd/libastro_hip_droppost.so step fault 120 python tools/fault_check.py
step fault_ok 120 python tools/fault_check.py
step prof20 300 rocprofv3 --kernel-trace --stats -d $O/prof20 -o run -f csv -- python bench.py --steps 20 --warmup 5 --no-cpu --no-single
step prof1000 300 rocprofv3 --kernel-trace --stats -d $O/prof1000 -o run -f csv -- python bench.py --no-cpu --no-single
ASTRO_AB_ANY_ABI=1 step ab_r2 300 python tools/ab.py --libs libastro_hip_r2,libastro_hip_sym8,libastro_hip_lref --workload c3 --rounds 4
ASTRO_AB_ANY_ABI=1 step ab_r2_c2 300 python tools/ab.py --libs libastro_hip_r2,libastro_hip_sym8,libastro_hip_lref --workload c2 --rounds 4
exit 0
