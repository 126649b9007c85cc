#!/bin/bash
# 8-slot instances at 2 waves/SIMD (no spills) vs 3 (2 VGPRs spilled), c5; helper priority after the post; SQ wait/active counters of c3 and c2
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3aa
mkdir -p $O
export ASTRO_AB_ANY_ABI=1
timeout -k 10 300 python tools/ab.py --libs libastro_hip_base,libastro_hip_p8w2 --workload c5 --rounds 4 > $O/ab_c5.log 2>&1 || exit $?
grep '^{' $O/ab_c5.log | cut -c1-200
for wl in c3 c2; do   # helper waves at s_setprio 1 / 3 after the post vs 0
  timeout -k 10 300 python tools/ab.py --libs libastro_hip_base,libastro_hip_hp1,libastro_hip_hp3 --workload $wl --rounds 4 > $O/ab_hp_$wl.log 2>&1 || exit $?
  grep '^{' $O/ab_hp_$wl.log | cut -c1-200
done
unset ASTRO_AB_ANY_ABI
for wl in c3 c2; do
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT -d $O/w_$wl -o run -f csv -- python bench.py --workload $wl --no-cpu --no-single --no-features --steps 300 > $O/w_$wl.log 2>&1 || exit $?
  python3 tools/waits_summary.py $O/w_$wl $wl || exit $?
  find $O/w_$wl -type f ! -name 'waits_*.json' -delete
done
