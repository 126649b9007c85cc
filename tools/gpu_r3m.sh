#!/bin/bash
# write-through end stores of the non-helper one-tick instance (WT_FINAL 8) vs plain; full GPU tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3m
mkdir -p $O
step() {
  local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  grep -E "^\{|passed|failed|Error|error" $O/$name.log | tail -6 | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
  return $rc
}
L=libastro_hip_wtd0,libastro_hip_wtd8
step ab_1m 400 python tools/ab.py --libs $L --workload c3 --n-env 1048576 --rounds 3
step ab_256k 300 python tools/ab.py --libs $L --workload c3 --n-env 262144 --rounds 3
step ab_c5 300 python tools/ab.py --libs $L --workload c5 --rounds 3
step pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
exit 0
