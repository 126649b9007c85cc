#!/bin/bash
# c5 per-env cost vs env count: does 131,072 envs (4,096 pair waves at 3 per SIMD) pay a tail round?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/s2c; mkdir -p $OUT
for n in 98304 131072 163840 196608; do
  timeout -k 10 150 python bench.py --workload c5 --n-env $n --steps 200 --warmup 20 --no-cpu --no-single --no-features --rollout 0 --calib 10 > $OUT/run.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { tail -5 $OUT/run.log; exit $rc; }
  python3 - $n $OUT/run.log >> $OUT/c5_sizes.jsonl <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith('{')][-1])
n = int(sys.argv[1])
print(json.dumps(dict(n=n, gpu_us=d['gpu_ms_per_step'] * 1e3, ns_per_env=d['gpu_ms_per_step'] * 1e6 / n, value=d['value'])))
PY
  tail -1 $OUT/c5_sizes.jsonl
done
