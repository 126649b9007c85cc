#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3k
mkdir -p $O
step() {
  local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  grep -E "^\{|passed|failed|Error|error" $O/$name.log | tail -5 | cut -c1-1500
  if [ $rc -ne 0 ]; then exit $rc; fi
  return $rc
}
step pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
export ASTRO_AB_ANY_ABI=1
step ab_c3 300 python tools/ab.py --libs libastro_hip_q4,libastro_hip_nodraw,libastro_hip_undr,libastro_hip_undr2 --workload c3 --rounds 5
step ab_c2 300 python tools/ab.py --libs libastro_hip_q4,libastro_hip_undr,libastro_hip_undr2 --workload c2 --rounds 4
unset ASTRO_AB_ANY_ABI
step bench20 300 python bench.py --steps 20 --warmup 5
exit 0
