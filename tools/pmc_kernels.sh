#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmck
for k in lane quad; do
  i=0
  for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE GRBM_COUNT"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctrs -d gpurun_out/pmck/${k}$i -o run -f csv -- python bench.py --steps 200 --warmup 20 --no-cpu --kernel $k > gpurun_out/pmck/${k}$i.log 2>&1
    rc=$?; echo "$k pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/pmck/${k}$i.log; exit $rc; }
  done
done
