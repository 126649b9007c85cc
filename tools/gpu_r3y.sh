#!/bin/bash
# bench GPU-time from back-to-back eager launches behind a spin; shim tests in both arena modes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3y
mkdir -p $O
step() {
  local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  grep -E "^\{|passed|failed|Error|error" $O/$name.log | tail -3 | cut -c1-200
  if [ $rc -ne 0 ]; then exit $rc; fi
  return $rc
}
step shim_tests 400 python -u -m pytest tests/test_long_games.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "shim"
step bench_c3_20a 200 python bench.py --steps 20 --warmup 5
step bench_c3_20b 200 python bench.py --steps 20 --warmup 5
step bench_c3 300 python bench.py --no-features
python3 - <<'PY'
import json
for f in ['bench_c3_20a', 'bench_c3_20b', 'bench_c3']:
    d = [json.loads(l) for l in open('gpurun_out/r3y/%s.log' % f) if l.startswith('{')][-1]
    print(f, 'value %.3e wall %.2f gpu %.2f graph %.2f stream %.2f frac %.3f single %s' % (
        d['value'], d['ms_per_step'] * 1e3, d['gpu_ms_per_step'] * 1e3, (d['gpu_ms_per_step_graph_replay'] or 0) * 1e3,
        d['gpu_ms_per_step_stream_events'] * 1e3, d['roofline']['frac'], d.get('single_game', {}).get('mode')))
PY
