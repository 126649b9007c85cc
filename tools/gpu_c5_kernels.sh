#!/bin/bash
# Lane vs quad step kernel over env counts (bench.py timed region, no CPU leg).
#   CASES="c5:131072 c3:262144" bash tools/gpu_c5_kernels.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/kern
for c in ${CASES:-c5:131072 c3:131072}; do
  wl=${c%%:*}; n=${c##*:}
  for k in ${KERNELS:-lane quad}; do
    timeout -k 10 200 python bench.py --workload $wl --kernel $k --n-env $n --steps 300 --no-cpu --rollout 0 --no-features \
      > gpurun_out/kern/${k}_${wl}_$n.log 2>&1 || exit $?
    tail -1 gpurun_out/kern/${k}_${wl}_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$k $wl $n', '%.3g'%d['value'], round(d['roofline']['kernel_ms']*1e3, 2), 'us')"
  done
done
exit 0
