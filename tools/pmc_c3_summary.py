#!/usr/bin/env python3
"""Per-wave counters of the one-tick step kernel per library variant
(tools/pmc_c3.sh): instructions, and wave-cycles split into issuing,
issue-stalled and parked (quad-cycles x 4 = shader cycles)."""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/pmc3'
res = {}
for d in sorted(glob.glob(os.path.join(root, '*_[0-9]'))):
    lib = os.path.basename(d).rsplit('_', 1)[0]
    acc = collections.defaultdict(list)
    durs = []
    for path in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(path)):
            if 'astro_step_quad_kernel' not in r['Kernel_Name'] or ', false, true,' not in r['Kernel_Name']:
                continue   # the one-tick helper instance only
            acc[r['Counter_Name']].append(float(r['Counter_Value']))
    m = res.setdefault(lib, {})
    for c, v in acc.items():
        v = v[20:] or v
        m[c] = sum(v) / len(v)
out = {}
for lib, m in res.items():
    w = m.get('SQ_WAVES', 0) or 1
    per = {c: v / w for c, v in m.items() if c != 'SQ_WAVES'}
    for c in ('SQ_WAVE_CYCLES', 'SQ_WAIT_ANY', 'SQ_WAIT_INST_ANY', 'SQ_ACTIVE_INST_ANY', 'SQ_ACTIVE_INST_VALU',
              'SQ_ACTIVE_INST_LDS', 'SQ_BUSY_CYCLES'):
        if c in per:
            per[c] *= 4
    out[lib] = dict(waves=w, per_wave=per, valu_per_launch=m.get('SQ_INSTS_VALU'))
print(json.dumps(out, indent=1))
json.dump(out, open(os.path.join(root, 'summary.json'), 'w'), indent=1)
