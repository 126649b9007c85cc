#!/bin/bash
# Same-process A/B runs of library builds (tools/ab.py) on the GPU box, one
# time-limited step per AB_<k> variable, results appended to gpurun_out/ab/:
#   AB_1="--libs libastro_hip,libastro_hip_x --workload c3" AB_2="..." bash tools/gpu_ab.sh
# A step that fails ends the script (nothing more runs on the GPU).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
export ASTRO_AB_ANY_ABI=1
mkdir -p gpurun_out/ab
for k in 1 2 3 4 5 6 7 8; do
  v="AB_$k"
  [ -z "${!v:-}" ] && continue
  echo "== $k: ${!v}"
  timeout -k 10 "${AB_LIMIT:-500}" python -u tools/ab.py ${!v} > gpurun_out/ab/ab_$k.jsonl 2> gpurun_out/ab/ab_$k.err
  rc=$?
  cat gpurun_out/ab/ab_$k.jsonl
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/ab/ab_$k.err; exit $rc; fi
done
exit 0
