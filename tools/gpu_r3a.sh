#!/bin/bash
# Round-3 first GPU session: GPU tests, smoke, short (driver-style) and long
# bench lines for c3, the partial-line read microbenchmark with request-size
# counters.  Every GPU step has its own limit; a crash/timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3a
mkdir -p $O
step() {
  local name=$1 limit=$2; shift 2
  local t0=$SECONDS
  timeout -k 10 "$limit" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc $((SECONDS - t0))s"
  tail -2 $O/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return $rc
}
step pytest 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step bench20 300 python bench.py --steps 20 --warmup 5
step bench1000 300 python bench.py --no-cpu --no-single
step ab_c3 300 python tools/ab.py --libs libastro_hip_sym8,libastro_hip_hbul --workload c3 --rounds 5
step ab_c5 300 python tools/ab.py --libs libastro_hip_sym8,libastro_hip_hbul --workload c5 --rounds 3
step bench_c5 300 python bench.py --workload c5 --no-cpu --no-single
step bench_c2 300 python bench.py --workload c2 --no-cpu --no-single
exit 0
