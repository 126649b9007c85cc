#!/bin/bash
# astro_step_many test; timed region from C (astro_step_many) vs graphs at 20 and 1000 steps; SQ wait/active counters
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3cc
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "step_many or rollout_equals" > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
show() { python3 -c "
import json
d=[json.loads(l) for l in open('$1') if l.startswith('{\"metric')][-1]
print('$1', 'wall %.2f gpu %.2f stream %.2f value %.3e' % (d['ms_per_step']*1e3, d['gpu_ms_per_step']*1e3, d['gpu_ms_per_step_stream_events']*1e3, d['value']))"; }
for rep in 1 2 3; do
  for l in graph c; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --no-single --no-features --launcher $l > $O/k20_${l}_$rep.log 2>&1 || exit $?
    show $O/k20_${l}_$rep.log
  done
done
for l in graph c; do
  timeout -k 10 300 python bench.py --no-cpu --no-single --no-features --launcher $l > $O/k1000_$l.log 2>&1 || exit $?
  show $O/k1000_$l.log
done
for wl in c3 c2; do
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT -d $O/w_$wl -o run -f csv -- python bench.py --workload $wl --no-cpu --no-single --no-features --steps 300 > $O/w_$wl.log 2>&1 || exit $?
  python3 tools/waits_summary.py $O/w_$wl $wl || exit $?
  find $O/w_$wl -type f ! -name 'waits_*.json' -delete
done
