#!/bin/bash
# Variant check: workload state + timing of A/B libraries, then targeted
# float32 parity tests on the variant ($VAR).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3b
mkdir -p $O
VAR=${VAR:-libastro_hip_hbul2}
LIBS=${LIBS:-libastro_hip_sym8,libastro_hip_hrefac,$VAR}
step() {
  local name=$1 limit=$2; shift 2
  local t0=$SECONDS
  timeout -k 10 "$limit" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc $((SECONDS - t0))s"
  tail -4 $O/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return $rc
}
step vs_c3 200 python tools/varstats.py --libs $LIBS --workload c3
step vs_c5 200 python tools/varstats.py --libs $LIBS --workload c5
step vs_c2 200 python tools/varstats.py --libs $LIBS --workload c2
ASTRO_LIB=astro_amd/$VAR.so step pytest_var 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "config5 or full_size or config4 or config2 or planets_only_streams or (batched_auto_reset and float) or ragged"
step ab_c3 300 python tools/ab.py --libs $LIBS --workload c3 --rounds 4
exit 0
