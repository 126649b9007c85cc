#!/bin/bash
# PMC passes over tools/rollout_driver.py (each its own rocprofv3 run:
# --pmc with --kernel-trace only), then the per-wave-tick summary.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmcr}
mkdir -p $OUT
ARGS="${RD_ARGS:---workload c3}"
i=0
for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
            "SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_FMA_F64 SQ_ACTIVE_INST_LDS"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctrs -d $OUT/p$i -o run -f csv -- python tools/rollout_driver.py $ARGS > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; tail -2 $OUT/p$i.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
python3 tools/pmc_rollout_summary.py $OUT
