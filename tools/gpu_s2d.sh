#!/bin/bash
# timing ablations (wrong results, timing only) of c5, c3, c2; then a hip-trace of the 20-step region
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/s2d; mkdir -p $OUT
LIBS=libastro_hip_abl_base,libastro_hip_abl_shipf,libastro_hip_abl_planf,libastro_hip_abl_sinc,libastro_hip_abl_bull
for wl in c5 c3 c2; do
  timeout -k 10 300 python tools/ab.py --libs $LIBS --workload $wl --rounds 3 >> $OUT/ablate.jsonl 2> $OUT/ablate_$wl.err
  rc=$?; echo "$wl rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/ablate_$wl.err; exit $rc; }
done
cat $OUT/ablate.jsonl
timeout -k 10 180 rocprofv3 --kernel-trace --hip-trace -d $OUT/trace -o run -f csv -- \
    python bench.py --steps 20 --warmup 5 --rollout 0 --no-cpu --no-single --no-features --calib 10 > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"
find $OUT/trace -name '*.csv' -size +1M -exec gzip {} \;
exit 0
