#!/bin/bash
# Round-end measurements on one GPU box: bench lines of every workload (the
# driver's own c3 command three times, the default 1,000-step c3 run) and,
# with PROF=1, the rocprofv3 stats + PMC traffic profiles (tools/profile_r3.sh).
# Every GPU step is time-limited; a failing step ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
b() {   # name limit args...
  local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" python bench.py "$@" > $O/$name.json 2> $O/$name.err
  local rc=$?
  echo "$name rc=$rc"; cat $O/$name.json | cut -c1-400
  if [ $rc -ne 0 ]; then tail -5 $O/$name.err; exit $rc; fi
}
if [ "${BENCH:-1}" = 1 ]; then
  b bench_c3_20a 300 --steps 20 --warmup 5
  b bench_c3_20b 300 --steps 20 --warmup 5
  b bench_c3_20c 300 --steps 20 --warmup 5
  b bench_c3 400
  b bench_c2 300 --workload c2 --no-single --no-features
  b bench_c5 300 --workload c5 --no-single --no-features
  b bench_c3any 300 --workload c3any --no-single --no-features --no-cpu
  b bench_c3_1m 300 --n-env 1048576 --no-single --no-features --no-cpu
fi
if [ "${PROF:-0}" = 1 ]; then
  for wl in ${PROF_WL:-c3 c2 c5}; do
    WL=$wl OUT=$O/prof/$wl bash tools/profile_r3.sh || exit $?
  done
fi
exit 0
