#!/bin/bash
# reset pass: row broadcasts by DPP (row_newbcast / row_ror) vs ds_bpermute shuffles; GPU suite on the DPP build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3s
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
L=libastro_hip_nodpp,libastro_hip_dpp
step ab_c3 300 python tools/ab.py --libs $L --workload c3 --rounds 5
step ab_c2 300 python tools/ab.py --libs $L --workload c2 --rounds 3
step ab_1m 300 python tools/ab.py --libs $L --workload c3 --n-env 1048576 --rounds 3
unset ASTRO_AB_ANY_ABI
step pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
exit 0
