#!/bin/bash
# header-first A/B, then measurement pass A (GPU suite, smoke, bench lines)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3u
mkdir -p $O
step() {
  local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  grep -E "^\{|passed|failed|Error|error" $O/$name.log | tail -6 | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
  return $rc
}
export ASTRO_AB_ANY_ABI=1
L=libastro_hip_dpp,libastro_hip_hdrfirst
step ab_c3 300 python tools/ab.py --libs $L --workload c3 --rounds 5
step ab_c2 300 python tools/ab.py --libs $L --workload c2 --rounds 3
unset ASTRO_AB_ANY_ABI
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
