#!/bin/bash
# first-process-on-the-box check of the warm replays: the driver-style line first, then repeats
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/s2h; mkdir -p $OUT
for r in 1 2 3; do
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 --no-cpu --no-single --no-features --rollout 0 > $OUT/run.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { tail -5 $OUT/run.log; exit $rc; }
  grep '^{' $OUT/run.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(dict(rep=$r, wall_us=d['ms_per_step']*1e3, gpu_us=d['gpu_ms_per_step']*1e3, stream_us=d['gpu_ms_per_step_stream_events']*1e3, value=d['value'], warm_ms=d['warm_ms'])))" >> $OUT/b20.jsonl
  tail -1 $OUT/b20.jsonl
done
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/full.log 2>&1
rc=$?; echo "full rc=$rc"; tail -2 $OUT/full.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/b20_full.log 2>&1
rc=$?; echo "b20_full rc=$rc"; grep '^{' $OUT/b20_full.log | cut -c1-200
exit $rc
