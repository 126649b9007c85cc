set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/s7
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/s7/full.log 2>&1 || { tail -30 gpurun_out/s7/full.log; exit 1; }
tail -2 gpurun_out/s7/full.log
timeout -k 10 300 python bench.py > gpurun_out/s7/bench_default.log 2>&1 || { tail gpurun_out/s7/bench_default.log; exit 1; }
for wl in c3 c2 c5; do WL=$wl bash tools/profile_r2.sh || exit 1; done
timeout -k 10 300 python tools/sweep.py --set c2 > gpurun_out/s7/stamps.jsonl 2>gpurun_out/s7/stamps.err || { tail gpurun_out/s7/stamps.err; exit 1; }
for wl in c3 c5; do python tools/trace_outliers.py gpurun_out/r2prof/$wl/stats/run_kernel_trace.csv > gpurun_out/r2prof/$wl/outliers_$wl.json; done
echo ok
