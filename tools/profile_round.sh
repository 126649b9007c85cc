#!/bin/bash
# Round profile: rocprofv3 kernel-trace stats of the default bench, then
# FETCH_SIZE / WRITE_SIZE passes for the HBM traffic per launch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=${ROUND:-round1}
OUT=gpurun_out/$R
mkdir -p $OUT
WL=${WL:-c3}
ARGS="--workload $WL --no-cpu --rollout 0 --no-features${NENV:+ --n-env $NENV}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run -f csv -- python bench.py $ARGS > $OUT/stats_$WL.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/fetch -o run -f csv -- python bench.py $ARGS --steps 300 --calib 10 > $OUT/fetch_$WL.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/write -o run -f csv -- python bench.py $ARGS --steps 300 --calib 10 > $OUT/write_$WL.log 2>&1 || exit $?
python3 tools/traffic.py $OUT/fetch/run_counter_collection.csv $OUT/write/run_counter_collection.csv $OUT/traffic_${WL}_f32.json ${NENV:-65536} auto
