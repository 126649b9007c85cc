#!/bin/bash
# A targeted GPU-box session: selected parity tests (PYTEST_K), then the
# same-process A/B runs (AB_1.., tools/gpu_ab.sh).  Each step time-limited;
# a crash, abort or timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "${PYTEST_K:-}" ]; then
  timeout -k 10 "${PYTEST_LIMIT:-600}" python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
      --timeout-method thread -k "$PYTEST_K" > gpurun_out/pytest_sel.log 2>&1
  rc=$?
  tail -15 gpurun_out/pytest_sel.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
if [ -n "${AB_1:-}" ]; then
  bash tools/gpu_ab.sh || exit $?
fi
if [ -n "${BENCH_ARGS:-}" ]; then
  timeout -k 10 300 python bench.py $BENCH_ARGS > gpurun_out/bench_q.log 2>&1
  rc=$?
  tail -c 3000 gpurun_out/bench_q.log
  exit $rc
fi
exit 0
