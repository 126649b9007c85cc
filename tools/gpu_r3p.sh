#!/bin/bash
# 4-slot instances at 3 waves/SIMD (no spills) vs 4 (7 VGPRs spilled), 256k / 1M envs; then the c3 bench lines and profiles
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3p
mkdir -p $O
step() {
  local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  grep -E "^\{|passed|failed|Error|error" $O/$name.log | tail -6 | cut -c1-600
  if [ $rc -ne 0 ]; then exit $rc; fi
  return $rc
}
export ASTRO_AB_ANY_ABI=1
L=libastro_hip_p4w4,libastro_hip_p4w3
step ab_1m 400 python tools/ab.py --libs $L --workload c3 --n-env 1048576 --rounds 3
step ab_256k 300 python tools/ab.py --libs $L --workload c3 --n-env 262144 --rounds 3
unset ASTRO_AB_ANY_ABI
step bench_c3_20 300 python bench.py --steps 20 --warmup 5
step bench_c3 400 python bench.py
WL=c3 timeout -k 10 1000 bash tools/profile_r3.sh > $O/profile_c3.log 2>&1; echo "profile rc=$?"; tail -3 $O/profile_c3.log
exit 0
