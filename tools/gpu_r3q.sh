#!/bin/bash
# round-3 measurement pass A: GPU suite, smoke, the bench lines (driver-style c3 first)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3q2
mkdir -p $O
step() {
  local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  grep -E "^\{|passed|failed|Error|error|SMOKE" $O/$name.log | tail -3 | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
  return $rc
}
step pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step bench_c3_20a 200 python bench.py --steps 20 --warmup 5
step bench_c3 300 python bench.py
step bench_c3_20b 200 python bench.py --steps 20 --warmup 5
step bench_c2 200 python bench.py --workload c2 --cpu-seconds 3
step bench_c5 300 python bench.py --workload c5 --cpu-seconds 3
step bench_c3any 200 python bench.py --workload c3any --cpu-seconds 3 --no-single
step bench_c3_1m 300 python bench.py --n-env 1048576 --steps 300 --cpu-seconds 3 --no-single --no-features
exit 0
