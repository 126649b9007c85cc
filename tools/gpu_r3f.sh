#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3f
mkdir -p $O
step() {
  local name=$1 limit=$2; shift 2
  local t0=$SECONDS
  timeout -k 10 "$limit" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc $((SECONDS - t0))s"
  tail -2 $O/$name.log | cut -c1-300
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return $rc
}
step pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step bench20 300 python bench.py --steps 20 --warmup 5
step bench20b 300 python bench.py --steps 20 --warmup 5 --no-cpu --no-single
step bench20c 300 python bench.py --steps 20 --warmup 5 --no-cpu --no-single
step bench1000 300 python bench.py --no-cpu --no-single
exit 0
