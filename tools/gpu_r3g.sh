#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3g
mkdir -p $O
step() {
  local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  grep "^{" $O/$name.log | tail -3 | cut -c1-2000
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return $rc
}
step stamps_c3 200 python tools/stamps_r3.py --workload c3 --lib libastro_hip_stamps --ticks 40
step test_core 300 python -u -m pytest tests/test_long_games.py tests/test_bots_logs.py -m gpu -x -q --timeout 120 -p no:cacheprovider
exit 0
