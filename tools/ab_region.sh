#!/bin/bash
# Interleaved runs of the driver's c3 command (--steps 20 --warmup 5) under
# two bench settings, one bench process each (the region is what differs):
#   A="--warm-ms 20" B="--warm-ms 100" [C=... VARS="A B C"] N=4 bash tools/ab_region.sh
# -> gpurun_out/ab_region.jsonl, one line per run with its setting in "ab".
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/ab_region.jsonl
for k in $(seq 1 ${N:-4}); do
  for v in ${VARS:-A B}; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --no-single --no-features --rollout 0 ${!v} \
      > /tmp/abr.json 2> /tmp/abr.err
    rc=$?
    if [ $rc -ne 0 ]; then tail -5 /tmp/abr.err; exit $rc; fi
    python3 -c "
import json, sys
d = json.loads(open('/tmp/abr.json').read().strip().splitlines()[-1])
print(json.dumps(dict(ab=sys.argv[1], run=int(sys.argv[2]), value=d['value'], ms_per_step=d['ms_per_step'],
                      gpu_ms_per_step=d['gpu_ms_per_step'], graph_replay=d.get('gpu_ms_per_step_graph_replay'),
                      region_events=d.get('gpu_ms_per_step_stream_events'))))" "${!v}" $k | tee -a $OUT
  done
done
