set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/s30
ASTRO_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 200 --warmup 20 --no-cpu > gpurun_out/s30/bench_2rank.log 2>&1 || { tail -20 gpurun_out/s30/bench_2rank.log; exit 1; }
grep metric gpurun_out/s30/bench_2rank.log | cut -c1-400
