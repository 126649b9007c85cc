#!/bin/bash
# Session-2 round-3 check of the committed build: full GPU suite, smoke,
# the bench as the driver runs it (20 steps) and the default bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/s2a
step() {
  local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > gpurun_out/s2a/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -3 gpurun_out/s2a/$name.log
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step full 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step b20 300 python bench.py --steps 20 --warmup 5
step bdef 300 python bench.py
exit 0
