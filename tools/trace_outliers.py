#!/usr/bin/env python3
"""Per-launch durations of the one-tick step kernel from a rocprofv3
--kernel-trace CSV, in dispatch order: where in the bench run (reset,
burn-in, warm-up, timed region) the slow launches sit.

    python tools/trace_outliers.py gpurun_out/c5trace/run_kernel_trace.csv
"""
import csv
import json
import sys

import numpy as np


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    step = [r for r in rows if 'astro_step_quad_kernel<' in r['Kernel_Name']
            and r['Kernel_Name'].split('<', 1)[1].split(',')[3].strip() == 'false'
            or 'astro_step_kernel<' in r['Kernel_Name']]
    d = np.array([(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3 for r in step])
    order = np.argsort(-d)
    out = dict(launches=len(d), mean_us=float(d.mean()), median_us=float(np.median(d)), max_us=float(d.max()),
               top=[dict(index=int(k), us=round(float(d[k]), 2)) for k in order[:8]],
               first10_us=[round(float(x), 2) for x in d[:10]],
               mean_after_first_us=float(d[1:].mean()) if len(d) > 1 else None,
               max_after_first_us=float(d[1:].max()) if len(d) > 1 else None)
    # what ran just before the slowest launch
    k = int(order[0])
    t0 = int(step[k]['Start_Timestamp'])
    prev = [r['Kernel_Name'].split('(')[0][-60:] for r in rows if int(r['Start_Timestamp']) < t0][-3:]
    out['before_slowest'] = prev
    print(json.dumps(out))


if __name__ == '__main__':
    main()
