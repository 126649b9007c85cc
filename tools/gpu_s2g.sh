#!/bin/bash
# the bench as the driver runs it, with the round's last bench changes (raw hipGraphLaunch, ev0 before the clock)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/s2g; mkdir -p $OUT
for r in 1 2 3 4; do
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 --no-cpu --no-single --no-features --rollout 0 > $OUT/run.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { tail -5 $OUT/run.log; exit $rc; }
  grep '^{' $OUT/run.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(dict(rep=$r, wall_us=d['ms_per_step']*1e3, gpu_us=d['gpu_ms_per_step']*1e3, stream_us=d['gpu_ms_per_step_stream_events']*1e3, value=d['value'], region=d['timed_region'])))" >> $OUT/b20.jsonl
  tail -1 $OUT/b20.jsonl
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/b20_full.log 2>&1
rc=$?; echo "b20_full rc=$rc"; grep '^{' $OUT/b20_full.log | cut -c1-200
timeout -k 10 300 python bench.py > $OUT/bdef.log 2>&1
rc=$?; echo "bdef rc=$rc"; grep '^{' $OUT/bdef.log | cut -c1-200
exit $rc
