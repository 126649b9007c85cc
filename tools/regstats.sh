#!/bin/bash
# Static register/spill/instruction summary of the step kernels (CPU only):
#   tools/regstats.sh [extra hipcc flags]
set -u
cd "$(dirname "$0")/.."
OUT=${OUT:-/tmp/astro_isa.s}
export FILTER=${FILTER:-step}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
  -fhip-fp32-correctly-rounded-divide-sqrt -Iinclude --cuda-device-only -S "$@" \
  ${SRC:-astro_amd/csrc/astro_kernels.hip} -o $OUT 2>/dev/null || exit 1
python3 - "$OUT" <<'PY'
import os, re, sys
FILTER = os.environ.get('FILTER', 'step')
s = open(sys.argv[1]).read()
for m in re.finditer(r'\.name:\s+(\S+)\n(.*?)\.wavefront_size', s, re.S):
    name, body = m.group(1), m.group(2)
    if FILTER not in name: continue
    f = lambda k: (re.search(r'\.%s:\s+(\d+)' % k, body) or [None, '?'])[1]
    short = re.sub(r'_ZN12_GLOBAL__N_1\d+', '', name).split('EEv')[0]
    print('%-40s vgpr %4s spill %4s sgpr_spill %4s scratch %5s' % (short, f('vgpr_count'), f('vgpr_spill_count'), f('sgpr_spill_count'), f('private_segment_fixed_size')))
PY
