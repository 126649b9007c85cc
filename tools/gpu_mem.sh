#!/bin/bash
# State-array memory kind A/B (BatchedEnv mem / ASTRO_MEM: default = hipMalloc,
# uncached, finegrained): parity tests under the uncached kind, then c3 bench
# lines (20 and 300 steps) per kind, interleaved; then one runtime-API trace
# of the 20-step region (hip-trace + kernel-trace) for the host-side costs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/mem; mkdir -p $OUT
if [ "${PARITY:-1}" = 1 ]; then
  ASTRO_MEM=uncached timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
      --timeout-method thread -p no:cacheprovider > $OUT/parity_uncached.log 2>&1
  rc=$?; echo "parity_uncached rc=$rc"; tail -3 $OUT/parity_uncached.log
  [ $rc -ne 0 ] && exit $rc
fi
BASE="--no-cpu --no-single --no-features --calib 10"
for r in $(seq 1 ${REPS:-3}); do
  for m in ${KINDS:-default uncached finegrained}; do
    for st in ${STEPSET:-20 300}; do
      W=5; [ $st -gt 20 ] && W=50
      RO=0; [ $st -gt 20 ] && RO=100
      ASTRO_MEM=$m timeout -k 10 150 python bench.py --steps $st --warmup $W --rollout $RO $BASE > $OUT/run.log 2>&1
      rc=$?
      if [ $rc -ne 0 ]; then echo "$m $st rc=$rc"; tail -5 $OUT/run.log; exit $rc; fi
      python3 - "$m" "$r" "$st" $OUT/run.log >> $OUT/mem.jsonl <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[4]) if l.startswith('{')][-1])
print(json.dumps(dict(mem=sys.argv[1], rep=int(sys.argv[2]), steps=int(sys.argv[3]), wall_us=d['ms_per_step'] * 1e3,
                      gpu_us=d['gpu_ms_per_step'] * 1e3, stream_us=(d.get('gpu_ms_per_step_stream_events') or 0) * 1e3,
                      value=d['value'], rollout_us=(d.get('rollout') or {}).get('gpu_ms_per_tick', 0) * 1e3)))
PY
      tail -1 $OUT/mem.jsonl
    done
  done
done
for r in $(seq 1 ${EREPS:-4}); do   # end detection: event vs stream busy-poll (20 steps, default memory)
  for e in event stream; do
    timeout -k 10 150 python bench.py --steps 20 --warmup 5 --rollout 0 --end-poll $e $BASE > $OUT/run.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "end $e rc=$rc"; tail -5 $OUT/run.log; exit $rc; fi
    python3 - "$e" "$r" $OUT/run.log >> $OUT/endpoll.jsonl <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[3]) if l.startswith('{')][-1])
print(json.dumps(dict(end_poll=sys.argv[1], rep=int(sys.argv[2]), wall_us=d['ms_per_step'] * 1e3,
                      gpu_us=d['gpu_ms_per_step'] * 1e3, value=d['value'])))
PY
    tail -1 $OUT/endpoll.jsonl
  done
done
if [ "${TRACE:-1}" = 1 ]; then
  timeout -k 10 180 rocprofv3 --kernel-trace --hip-trace -d $OUT/trace -o run -f csv -- \
      python bench.py --steps 20 --warmup 5 --rollout 0 $BASE > $OUT/trace.log 2>&1
  rc=$?; echo "trace rc=$rc"
  find $OUT/trace -name '*.csv' -size +2M -delete
fi
exit 0
