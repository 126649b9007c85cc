#!/usr/bin/env python3
"""Summarise tools/pmc_kernels.sh output: per-wave and per-SIMD counters of astro_step."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/pmck'
groups = collections.defaultdict(lambda: collections.defaultdict(list))
durs = collections.defaultdict(list)
for path in glob.glob(os.path.join(root, '*_*_*/run_counter_collection.csv')):
    tag = '_'.join(os.path.basename(os.path.dirname(path)).split('_')[:2])
    for r in csv.DictReader(open(path)):
        if 'astro_step' not in r['Kernel_Name']:
            continue
        groups[tag][r['Counter_Name']].append(float(r['Counter_Value']))
        durs[tag].append(int(r['End_Timestamp']) - int(r['Start_Timestamp']))
for tag, acc in sorted(groups.items()):
    m = {c: sum(v[20:]) / max(1, len(v[20:])) for c, v in acc.items()}
    w = m['SQ_WAVES']
    d = sorted(durs[tag])[len(durs[tag]) // 2] / 1e3
    print('%-10s waves %5d  VALU/wave %6.0f  SALU/wave %5.0f  f64(add+mul+fma)/wave %5.0f  '
          'wave_cyc %6.0f  wait_any %6.0f  wait_inst %6.0f  active %6.0f  VALU-busy/SIMD %6.0f  dur %.1f us'
          % (tag, w, m['SQ_INSTS_VALU'] / w, m['SQ_INSTS_SALU'] / w,
             (m['SQ_INSTS_VALU_ADD_F64'] + m['SQ_INSTS_VALU_MUL_F64'] + m['SQ_INSTS_VALU_FMA_F64']) / w,
             4 * m['SQ_WAVE_CYCLES'] / w, 4 * m['SQ_WAIT_ANY'] / w, 4 * m['SQ_WAIT_INST_ANY'] / w,
             4 * m['SQ_ACTIVE_INST_ANY'] / w, 4 * m['SQ_ACTIVE_INST_VALU'] / 1024, d))
