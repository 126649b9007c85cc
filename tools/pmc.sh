#!/bin/bash
# PMC passes (each its own rocprofv3 run: --pmc with --kernel-trace only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
ARGS="${PMC_BENCH_ARGS:---steps 200 --warmup 20 --no-cpu}"
i=0
for ctrs in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctrs -d gpurun_out/pmc/p$i -o run -f csv -- python bench.py $ARGS > gpurun_out/pmc/p$i.log 2>&1
  rc=$?; echo "pass $i ($ctrs) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc/p$i.log; exit $rc; fi
done
