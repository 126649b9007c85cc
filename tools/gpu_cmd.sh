set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/s32
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/s32/full.log 2>&1 || { tail -40 gpurun_out/s32/full.log; exit 1; }
tail -2 gpurun_out/s32/full.log
timeout -k 10 300 python bench.py --workload c2 --cpu-seconds 5 > gpurun_out/s32/bench_c2.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/s32/bench_c3.log 2>&1 || exit 1
WL=c2 bash tools/profile_r2.sh || exit 1
python tools/trace_outliers.py gpurun_out/r2prof/c2/stats/run_kernel_trace.csv > gpurun_out/r2prof/c2/outliers_c2.json
for f in gpurun_out/s32/bench_*.log; do grep metric $f | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step']*1e3, d['roofline']['frac'], d.get('rollout',{}).get('ms_per_tick',0)*1e3)"; done
