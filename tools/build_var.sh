#!/bin/bash
# A/B library variant (float32 state, two ships: the bench workloads only):
#   tools/build_var.sh NAME [SRC] [extra hipcc flags...]
#   -> astro_amd/libastro_hip_NAME.so, for tools/ab.py --libs libastro_hip_NAME
set -eu
cd "$(dirname "$0")/.."
NAME=$1; shift
SRC=${1:-astro_amd/csrc/astro_kernels.hip}; [ $# -gt 0 ] && shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
  -fhip-fp32-correctly-rounded-divide-sqrt -fPIC -shared -Iinclude -DASTRO_ONLY_F32_S2 "$@" \
  "$SRC" -o astro_amd/libastro_hip_$NAME.so
