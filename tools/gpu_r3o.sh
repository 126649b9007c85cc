#!/bin/bash
# pair helpers pre-create every env's next game (ASTRO_PRECREATE 1) vs reset passes after the post (0); GPU suite; stamps
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3o
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
step pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
export ASTRO_AB_ANY_ABI=1
L=libastro_hip_pc0,libastro_hip_pc1
step ab_c3 300 python tools/ab.py --libs $L --workload c3 --rounds 5
step ab_c3any 300 python tools/ab.py --libs $L --workload c3any --rounds 3
step ab_c2 300 python tools/ab.py --libs $L --workload c2 --rounds 3
exit 0
