#!/usr/bin/env python3
"""Per-wave and per-tick counters of the rollout launches (tools/pmc_rollout.sh)."""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/pmcr'
acc = collections.defaultdict(list)
names = set()
for path in glob.glob(os.path.join(root, 'p*', '**', '*counter_collection.csv'), recursive=True):
    for r in csv.DictReader(open(path)):
        k = r['Kernel_Name']
        if 'rollout' not in k and 'astro_step_quad_kernel<float, 2, 4, true' not in k:
            continue
        names.add(k.split('(')[0])
        acc[r['Counter_Name']].append(float(r['Counter_Value']))
m = {c: sum(v[1:]) / max(1, len(v) - 1) for c, v in acc.items()}   # (the burn-in launch first: dropped)
w = m.get('SQ_WAVES', 1.0)
ticks = int(os.environ.get('TICKS', '100'))
out = dict(kernels=sorted(names), waves=w, ticks_per_launch=ticks,
           per_wave_tick={c: v / w / ticks for c, v in m.items() if c != 'SQ_WAVES'},
           note='SQ_*_CYCLES / WAIT / ACTIVE count quad-cycles (x4 = shader cycles)')
print(json.dumps(out, indent=1))
json.dump(out, open(os.path.join(root, 'summary.json'), 'w'), indent=1)
