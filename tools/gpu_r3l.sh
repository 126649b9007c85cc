#!/bin/bash
# write-through final stores (ASTRO_WT_FINAL masks 1, 3, 7) vs base, c3 / c2 / c5
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3l
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
L=libastro_hip_undr,libastro_hip_wt1,libastro_hip_wt3,libastro_hip_wt7
step ab_c3 300 python tools/ab.py --libs $L --workload c3 --rounds 5
step ab_c2 300 python tools/ab.py --libs $L --workload c2 --rounds 4
step ab_c5 300 python tools/ab.py --libs $L --workload c5 --rounds 3
exit 0
