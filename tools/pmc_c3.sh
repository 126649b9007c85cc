#!/bin/bash
# PMC passes of the one-tick step kernel for library variants (LIBS), each
# pass its own rocprofv3 run (--pmc with --kernel-trace only), then the
# per-wave summary (tools/pmc_c3_summary.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
export ASTRO_AB_ANY_ABI=1
OUT=${OUT:-gpurun_out/pmc3}
mkdir -p $OUT
WL=${WL:-c3}
for lib in ${LIBS:-libastro_hip}; do
  i=0
  for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
              "SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_FMA_F64 SQ_ACTIVE_INST_LDS"; do
    i=$((i+1))
    ASTRO_LIB=$PWD/astro_amd/$lib.so timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctrs -d $OUT/${lib}_$i -o run -f csv -- \
        python bench.py --workload $WL --steps 200 --warmup 20 --no-cpu --no-single --no-features --rollout 0 --graph 0 --calib 10 \
        > $OUT/${lib}_$i.log 2>&1
    rc=$?; echo "$lib pass $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $OUT/${lib}_$i.log; exit $rc; fi
  done
done
python3 tools/pmc_c3_summary.py $OUT
