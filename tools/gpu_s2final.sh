#!/bin/bash
# Round-3 second-session final check of the committed tree: full GPU suite,
# smoke, the bench as the driver runs it and the default bench, and a
# rocprofv3 kernel-stats pass of the 20-step command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/s2f; mkdir -p $OUT
step() {
  local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -3 $OUT/$name.log
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step full 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step b20 300 python bench.py --steps 20 --warmup 5
step bdef 300 python bench.py
step prof20 300 rocprofv3 --kernel-trace --stats -d $OUT/prof20 -o run -f csv -- python bench.py --steps 20 --warmup 5 --no-cpu --no-single --no-features --rollout 0 --calib 10
find $OUT/prof20 -type f ! -name 'run_kernel_stats.csv' ! -name 'run_kernel_trace.csv' -delete
exit 0
