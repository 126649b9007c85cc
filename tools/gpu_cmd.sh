set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/s29
L=libastro_hip_d0,libastro_hip_d1,libastro_hip_d2,libastro_hip_d4
for wl in c3 c2; do
  timeout -k 10 250 python tools/ab.py --libs $L --workload $wl > gpurun_out/s29/ab_$wl.jsonl 2>&1 || { tail -5 gpurun_out/s29/ab_$wl.jsonl; exit 1; }
done
cat gpurun_out/s29/ab_*.jsonl | grep -v amdgpu.ids | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['workload'], d['n'], d['lib'][12:] or 'main', round(d['us_per_launch_median'], 3), round(d['rollout_us_per_tick'], 3))
"
