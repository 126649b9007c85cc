#!/bin/bash
# driver-style c3 runs (--steps 20 --warmup 5): wall per step with 0, 1 or 2 eager launches at the head of the timed region
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3z
mkdir -p $O
for rep in 1 2 3; do
  for h in 0 1 2; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --no-single --no-features --eager-head $h > $O/h${h}_$rep.log 2>&1 || exit $?
    python3 -c "
import json,sys
d=[json.loads(l) for l in open('$O/h${h}_$rep.log') if l.startswith('{\"metric')][-1]
print('head $h rep $rep wall %.2f gpu %.2f stream %.2f value %.3e' % (d['ms_per_step']*1e3, d['gpu_ms_per_step']*1e3, d['gpu_ms_per_step_stream_events']*1e3, d['value']))"
  done
done
