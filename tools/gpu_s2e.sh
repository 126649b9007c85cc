#!/bin/bash
# torch CUDAGraph.replay() vs hipGraphLaunch directly in the 20-step timed region (c3)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/s2e; mkdir -p $OUT
for r in $(seq 1 ${REPS:-5}); do
  for m in torch raw; do
    timeout -k 10 150 python bench.py --steps 20 --warmup 5 --rollout 0 --no-cpu --no-single --no-features --calib 10 --replay $m > $OUT/run.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "$m rc=$rc"; tail -5 $OUT/run.log; exit $rc; }
    python3 - "$m" "$r" $OUT/run.log >> $OUT/replay.jsonl <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[3]) if l.startswith('{')][-1])
print(json.dumps(dict(replay=sys.argv[1], rep=int(sys.argv[2]), wall_us=d['ms_per_step'] * 1e3,
                      gpu_us=d['gpu_ms_per_step'] * 1e3, stream_us=(d.get('gpu_ms_per_step_stream_events') or 0) * 1e3,
                      value=d['value'], errors=d['device_errors'])))
PY
    tail -1 $OUT/replay.jsonl
  done
done
