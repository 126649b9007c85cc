#!/bin/bash
# Quick GPU check: parity tests, default bench, optional extra steps ($EXTRA).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/q
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/q/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/q/pytest.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/q/bench.log 2>&1 || exit $?
tail -1 gpurun_out/q/bench.log
for x in ${EXTRA:-}; do
  timeout -k 10 300 $x > gpurun_out/q/$(basename ${x%% *}).log 2>&1 || exit $?
  cat gpurun_out/q/$(basename ${x%% *}).log
done
exit 0
