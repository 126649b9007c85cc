#!/bin/bash
# Round-6 GPU session: selected tests (PYTEST_K, over the -m gpu suite), then
# A/B commands (AB: one shell command per line, output appended to
# gpurun_out/r6/ab.jsonl), then bench variants (BENCH_VARS: one argument
# string per line, each line run once into gpurun_out/r6/bench.jsonl).  Every
# GPU step time-limited; any failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6
mkdir -p $O
if [ -n "${PYTEST_K:-}" ]; then
  timeout -k 10 "${PYTEST_LIMIT:-600}" python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 \
      --timeout-method thread -k "$PYTEST_K" > $O/pytest.log 2>&1
  rc=$?
  tail -5 $O/pytest.log
  if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $O/pytest.log | head -20; exit $rc; fi
fi
if [ -n "${AB:-}" ]; then
  while IFS= read -r cmd; do
    [ -z "$cmd" ] && continue
    echo "ab: $cmd"
    timeout -k 10 "${AB_LIMIT:-400}" bash -c "$cmd" >> $O/ab.jsonl 2> $O/ab.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "ab rc=$rc"; tail -5 $O/ab.err; exit $rc; fi
  done <<< "$AB"
  tail -20 $O/ab.jsonl
fi
if [ -n "${BENCH_VARS:-}" ]; then
  while IFS= read -r args; do
    [ -z "$args" ] && continue
    timeout -k 10 300 python bench.py $args > $O/bench_one.json 2> $O/bench.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "bench rc=$rc: $args"; tail -5 $O/bench.err; exit $rc; fi
    python - "$args" <<'PY' >> $O/bench.jsonl
import json, sys
j = json.loads([l for l in open('gpurun_out/r6/bench_one.json') if l.startswith('{')][-1])
j['args'] = sys.argv[1]
print(json.dumps(j))
PY
    python - "$args" <<'PY'
import json, sys
j = json.loads([l for l in open('gpurun_out/r6/bench_one.json') if l.startswith('{')][-1])
r = j.get('region_host_us', {})
print(sys.argv[1], '| value %.3e wall %.2f gpu %.2f us/step' % (j['value'], j['ms_per_step'] * 1e3, j['gpu_ms_per_step'] * 1e3),
      {k: round(v, 1) for k, v in r.items()})
for k in ('rollout', 'rollout_script'):
    if k in j: print('  %s %.3f us/tick' % (k, j[k]['gpu_ms_per_tick'] * 1e3))
PY
  done <<< "$BENCH_VARS"
fi
exit 0
