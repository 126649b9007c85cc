set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r2
timeout -k 10 300 python bench.py --workload c2 --cpu-seconds 10 > gpurun_out/r2/bench_c2.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload c5 --cpu-seconds 10 > gpurun_out/r2/bench_c5.log 2>&1 || exit $?
ROUND=r2 WL=c5 NENV=131072 bash tools/profile_round.sh || exit $?
ROUND=r2 WL=c2 NENV=4096 bash tools/profile_round.sh || exit $?
