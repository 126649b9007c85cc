set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/s17
L=libastro_hip_nohelp,libastro_hip_early_qw2,libastro_hip
for wl in c2 c3; do
  timeout -k 10 200 python tools/ab.py --libs $L --workload $wl > gpurun_out/s17/ab_$wl.jsonl 2>&1 || { tail -5 gpurun_out/s17/ab_$wl.jsonl; exit 1; }
done
cat gpurun_out/s17/ab_*.jsonl | grep -v amdgpu.ids | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['workload'], d['n'], d['lib'][12:] or 'main', round(d['us_per_launch_median'], 3), round(d['rollout_us_per_tick'], 3))
"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/s17/full.log 2>&1 || { tail -40 gpurun_out/s17/full.log; exit 1; }
tail -2 gpurun_out/s17/full.log
timeout -k 10 300 python bench.py > gpurun_out/s17/bench_c3.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload c2 --cpu-seconds 5 > gpurun_out/s17/bench_c2.log 2>&1 || exit 1
for f in gpurun_out/s17/bench_*.log; do grep metric $f | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step']*1e3, d['roofline']['frac'])"; done
