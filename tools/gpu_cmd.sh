set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/s26
L=libastro_hip_w4,libastro_hip
for wl in c3 c2; do
  timeout -k 10 250 python tools/ab.py --libs $L --workload $wl > gpurun_out/s26/ab_$wl.jsonl 2>&1 || { tail -5 gpurun_out/s26/ab_$wl.jsonl; exit 1; }
done
cat gpurun_out/s26/ab_*.jsonl | grep -v amdgpu.ids | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['workload'], d['n'], d['lib'][12:] or 'main', round(d['us_per_launch_median'], 3), round(d['rollout_us_per_tick'], 3))
"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/s26/full.log 2>&1 || { tail -40 gpurun_out/s26/full.log; exit 1; }
tail -2 gpurun_out/s26/full.log
