#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; a crash/abort/timeout (anything but
# exit 0 or an ordinary test failure, 1) ends the script there.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS="${ASTRO_STEPS:-pytest smoke bench prof}"
run() {
    local name=$1 limit=$2; shift 2
    local t0=$SECONDS
    timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc $((SECONDS - t0))s" | tee -a gpurun_out/rc.log
    tail -3 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
for s in $STEPS; do
  case $s in
    pytest) run pytest_gpu 1200 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    smoke)  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)  run bench 600 python bench.py ;;
    driver) run driver 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    prof)   run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -f csv -- \
                python bench.py --steps 300 --no-cpu ;;
  esac
done
