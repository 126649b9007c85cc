#!/bin/bash
# Where a resident-rollout wave-tick's instructions go, by difference (no
# ablation builds): tools/pmc_rollout.sh over the c3 rollouts with and
# without auto-reset, and over config 2's bullet-less games at c3's size.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
B=${OUT_BASE:-gpurun_out/pmcr6}
for v in "full|--workload c3" "noreset|--workload c3 --no-reset" "nobullets|--workload c2 --n-env 65536" \
         "nobullets_noreset|--workload c2 --n-env 65536 --no-reset"; do
  name=${v%%|*}; args=${v#*|}
  OUT=$B/$name RD_ARGS="$args" bash tools/pmc_rollout.sh > $B.$name.log 2>&1 || { echo "$name failed"; tail -5 $B.$name.log; exit 1; }
  echo "$name ok"
done
python3 - "$B" <<'PY'
import json, sys
b = sys.argv[1]
rows = {}
for n in ('full', 'noreset', 'nobullets', 'nobullets_noreset'):
    rows[n] = json.load(open('%s/%s/summary.json' % (b, n)))['per_wave_tick']
keys = ('SQ_INSTS_VALU', 'SQ_INSTS_SALU', 'SQ_INSTS_LDS', 'SQ_ACTIVE_INST_VALU', 'SQ_WAVE_CYCLES', 'SQ_BUSY_CYCLES')
print(json.dumps({n: {k: round(r.get(k, 0.0), 1) for k in keys} for n, r in rows.items()}, indent=1))
json.dump(rows, open(b + '/breakdown.json', 'w'), indent=1)
PY
