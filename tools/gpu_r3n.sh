#!/bin/bash
# nontemporal state loads (ASTRO_NT_LOADS 1 bullets, 3 + ships/planets) vs base; stamps; GPU suite
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3n
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
L=libastro_hip_base,libastro_hip_nt1,libastro_hip_nt3
step ab_c3 300 python tools/ab.py --libs $L --workload c3 --rounds 5
step ab_c2 300 python tools/ab.py --libs $L --workload c2 --rounds 4
step ab_c5 300 python tools/ab.py --libs $L --workload c5 --rounds 3
step stamps_c3 200 python tools/stamps_r3.py --workload c3 --lib libastro_hip_stamps --ticks 40
step stamps_c2 200 python tools/stamps_r3.py --workload c2 --lib libastro_hip_stamps --ticks 40
exit 0
