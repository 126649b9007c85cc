#!/bin/bash
# HIP runtime knobs vs the driver-style 20-step c3 timed region (wall per
# step): each setting a fresh process, interleaved over rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/knobs; mkdir -p $OUT
ARGS="--steps ${KSTEPS:-20} --warmup 5 --no-cpu --no-single --no-features --rollout 0 --calib 10"
# a setting: ENV=VAL (an environment variable) or ARG=--flag=value (a bench argument)
# (DEBUG_HIP_FORCE_GRAPH_QUEUES=0 crashes the runtime: SIGFPE)
SETTINGS=${SETTINGS:-"base DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 DEBUG_HIP_GRAPH_BATCH_SIZE=1 AMD_DIRECT_DISPATCH=0 ARG=--graph=0"}
for r in $(seq 1 ${REPS:-4}); do
  for s in $SETTINGS; do
    E=""; A=""
    case $s in base) ;; ARG=*) A="${s#ARG=}"; A="${A/=/ }" ;; *) E="$s" ;; esac
    timeout -k 10 120 env $E python bench.py $ARGS $A > $OUT/run.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "$s rc=$rc"; tail -5 $OUT/run.log; exit $rc; fi
    python3 - "$s" "$r" $OUT/run.log >> $OUT/knobs.jsonl <<'PY'
import json, sys
line = [l for l in open(sys.argv[3]) if l.startswith('{')][-1]
d = json.loads(line)
print(json.dumps(dict(setting=sys.argv[1], rep=int(sys.argv[2]), wall_us=d['ms_per_step'] * 1e3,
                      gpu_us=d.get('gpu_ms_per_step', 0) * 1e3, value=d['value'],
                      stream_us=(d.get('gpu_ms_per_step_stream_events') or 0) * 1e3)))
PY
    tail -1 $OUT/knobs.jsonl
  done
done
# one kernel trace of the default setting: per-launch durations and gaps in the region
mkdir -p $OUT/trace
timeout -k 10 180 rocprofv3 --kernel-trace -d $OUT/trace -o run -f csv -- python bench.py $ARGS > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"
find $OUT/trace -name '*kernel_trace.csv' -exec cp {} $OUT/kernel_trace.csv \;
exit $rc
