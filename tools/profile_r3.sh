#!/bin/bash
# Round-3 profiles of one workload, all from the SAME bench command the line
# is quoted on (burn-in included), so the numbers describe the same state:
#   1. rocprofv3 --kernel-trace --stats          -> kernel durations
#   2. --pmc FETCH_SIZE, 3. --pmc WRITE_SIZE      -> HBM bytes per launch
#   4. --pmc SQ_WAVES SQ_INSTS_VALU/SALU/F64      -> VALU issue per wave
#   5. --pmc TCC_EA0_RDREQ{,_32B,_64B,_128B}, 6. TCC_EA0_WRREQ{,_64B} -> request-sized bytes
# then tools/prof_summary.py writes traffic_<wl>_f32.json / pmc_<wl>_f32.json
# (with the bench run's own live-bullet and reset counts) under $OUT.
#   WL=c3 bash tools/profile_r3.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
WL=${WL:-c3}
OUT=${OUT:-gpurun_out/prof/$WL}
mkdir -p $OUT
ARGS="--workload $WL --no-cpu --no-single --no-features --steps ${PSTEPS:-300} ${EXTRA_ARGS:-}"
run() {
  local tag=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace "$@" -d $OUT/$tag -o run -f csv -- python bench.py $ARGS > $OUT/$tag.log 2>&1
  local rc=$?
  echo "$WL $tag rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/$tag.log; exit $rc; fi
}
run stats --stats
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
run insts --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_FMA_F64
if [ "${REQ:-1}" = 1 ]; then   # request sizes: the bytes behind FETCH_SIZE / WRITE_SIZE without the 2x guess
  run rdreq --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum
  run wrreq --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum
fi
PROFILE_ARGS="$ARGS" PROFILE_SCRIPT=tools/profile_r3.sh python3 tools/prof_summary.py $OUT $WL
rc=$?
du -sh $OUT/* | sort -h | tail -4
# keep the summaries, drop rocprofv3's raw per-dispatch files (gpurun returns at most 64 MiB)
for d in stats fetch write insts rdreq wrreq; do
  [ -d $OUT/$d ] && find $OUT/$d -type f ! -name 'run_kernel_stats.csv' -delete
done
exit $rc
