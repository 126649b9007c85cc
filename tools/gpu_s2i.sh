#!/bin/bash
# last check of the committed tree: smoke, the driver-style line, the default line, rocprof stats of the 20-step command
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/s2i; mkdir -p $OUT
step() {
  local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -2 $OUT/$name.log | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step b20 300 python bench.py --steps 20 --warmup 5
step bdef 300 python bench.py
step prof20 300 rocprofv3 --kernel-trace --stats -d $OUT/prof20 -o run -f csv -- python bench.py --steps 20 --warmup 5 --no-cpu --no-single --no-features --rollout 0 --calib 10
find $OUT/prof20 -type f ! -name 'run_kernel_stats.csv' -delete
exit 0
