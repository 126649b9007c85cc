#!/bin/bash
# Round profiles: rocprofv3 kernel stats + HBM traffic for c3, c5, c2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for c in ${CASES:-c3:65536 c5:131072 c2:4096}; do
  wl=${c%%:*}; n=${c##*:}
  ROUND=prof_$wl WL=$wl NENV=$n bash tools/profile_round.sh || exit $?
  cp gpurun_out/prof_$wl/stats/run_kernel_stats.csv gpurun_out/prof_$wl/rocprof_kernel_stats_$wl.csv
done
exit 0
