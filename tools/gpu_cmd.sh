set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/s28
timeout -k 10 300 python bench.py > gpurun_out/s28/bench_c3.log 2>&1 || exit 1
for wl in c2 c5 c3any; do timeout -k 10 300 python bench.py --workload $wl --cpu-seconds 5 > gpurun_out/s28/bench_$wl.log 2>&1 || exit 1; done
timeout -k 10 300 python bench.py --n-env 1048576 --no-cpu --steps 200 > gpurun_out/s28/bench_c3_1m.log 2>&1 || exit 1
for wl in c3 c2; do WL=$wl bash tools/profile_r2.sh || exit 1; done
for wl in c3 c2; do python tools/trace_outliers.py gpurun_out/r2prof/$wl/stats/run_kernel_trace.csv > gpurun_out/r2prof/$wl/outliers_$wl.json; done
timeout -k 10 300 python tools/sweep.py --set c2 > gpurun_out/s28/stamps.jsonl 2>gpurun_out/s28/stamps.err || { tail gpurun_out/s28/stamps.err; exit 1; }
for f in gpurun_out/s28/bench_*.log; do grep metric $f | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step']*1e3, d['roofline']['frac'], d.get('rollout',{}).get('ms_per_tick',0)*1e3, d.get('observation',{}).get('ms',0)*1e3)"; done
