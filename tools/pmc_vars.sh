#!/bin/bash
# Dynamic instruction counts per library build (ablations): one rocprofv3
# --pmc pass per build, counters of the step kernel only.
#   LIBS="libastro_hip libastro_hip_abl_x" bash tools/pmc_vars.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmcv
mkdir -p $OUT
CTRS="${CTRS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_FMA_F64 SQ_WAVE_CYCLES SQ_BUSY_CYCLES}"
for lib in $LIBS; do
  for mode in "" "--noreset"; do
    tag=$lib${mode:+_noreset}
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $CTRS -d $OUT/$tag -o run -f csv -- \
        python tools/pmc_var.py --lib $lib $mode > $OUT/$tag.log 2>&1
    rc=$?; echo "$tag rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $OUT/$tag.log; exit $rc; fi
  done
done
exit 0
