#!/bin/bash
# GPU tests: named test files first (TESTS), then optionally the whole -m gpu
# suite (FULL=1) and the default bench (BENCH=1).  Each step time-limited;
# anything but a clean pass/fail stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/t
step() {
  local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > gpurun_out/t/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -4 gpurun_out/t/$name.log
  if [ $rc -ne 0 ]; then exit $rc; fi
}
if [ -n "${TESTS:-}" ]; then
  step new 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider
fi
if [ "${FULL:-0}" = 1 ]; then
  step full 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
fi
if [ "${BENCH:-0}" = 1 ]; then
  step bench 600 python bench.py ${BENCH_ARGS:-}
fi
exit 0
