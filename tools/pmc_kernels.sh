#!/bin/bash
# PMC comparison of the step kernels: per kernel/workload, two counter passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmck
mkdir -p $OUT
for k in ${KERNELS:-lane quad}; do
 for wl in ${WLS:-c3}; do
  i=0
  for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_FMA_F64 GRBM_GUI_ACTIVE GRBM_COUNT"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctrs -d $OUT/${k}_${wl}_$i -o run -f csv -- python bench.py --steps 200 --warmup 20 --no-cpu --graph 0 --calib 10 --kernel $k --workload $wl --n-env 65536 > $OUT/${k}_${wl}_$i.log 2>&1
    rc=$?; echo "$k $wl pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/${k}_${wl}_$i.log; exit $rc; }
  done
 done
done
