#!/bin/bash
# round-3 measurement pass B: rocprofv3 stats + PMC passes of the bench workloads named in $WLS
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for wl in ${WLS:-c3 c2}; do
  WL=$wl timeout -k 10 500 bash tools/profile_r3.sh > gpurun_out/profile_$wl.log 2>&1
  rc=$?
  echo "profile $wl rc=$rc"; tail -6 gpurun_out/profile_$wl.log | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
done
exit 0
