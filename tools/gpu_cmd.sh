set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/s11
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/s11/full.log 2>&1 || { tail -40 gpurun_out/s11/full.log; exit 1; }
tail -2 gpurun_out/s11/full.log
timeout -k 10 300 python bench.py > gpurun_out/s11/bench_c3.log 2>&1 || exit 1
for wl in c2 c5 c3any; do timeout -k 10 300 python bench.py --workload $wl --cpu-seconds 5 > gpurun_out/s11/bench_$wl.log 2>&1 || exit 1; done
timeout -k 10 300 python bench.py --n-env 1048576 --no-cpu --steps 200 > gpurun_out/s11/bench_c3_1m.log 2>&1 || exit 1
WL=c5 bash tools/profile_r2.sh || exit 1
python tools/trace_outliers.py gpurun_out/r2prof/c5/stats/run_kernel_trace.csv > gpurun_out/r2prof/c5/outliers_c5.json
for f in gpurun_out/s11/bench_*.log; do echo $f; grep metric $f | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step']*1e3, d['roofline']['frac'], d['stats']['mean_live_bullets'], d['stats']['resets_per_step'], d.get('rollout',{}).get('ms_per_tick',0)*1e3, d.get('cpu_baseline',{}).get('value'))"; done
