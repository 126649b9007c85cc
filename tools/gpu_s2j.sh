#!/bin/bash
# raw hipGraphLaunch replays with and without DEBUG_CLR_GRAPH_PACKET_CAPTURE=0, 20-step c3 region
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/s2j; mkdir -p $OUT
for r in 1 2 3 4 5; do
  for s in base DEBUG_CLR_GRAPH_PACKET_CAPTURE=0; do
    E=""; [ "$s" != base ] && E="$s"
    timeout -k 10 150 env $E python bench.py --steps 20 --warmup 5 --no-cpu --no-single --no-features --rollout 0 --calib 10 > $OUT/run.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -5 $OUT/run.log; exit $rc; }
    grep '^{' $OUT/run.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(dict(setting='$s', rep=$r, wall_us=d['ms_per_step']*1e3, gpu_us=d['gpu_ms_per_step']*1e3, stream_us=d['gpu_ms_per_step_stream_events']*1e3, value=d['value'])))" >> $OUT/pc.jsonl
    tail -1 $OUT/pc.jsonl
  done
done
