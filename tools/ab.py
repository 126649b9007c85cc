#!/usr/bin/env python3
"""A/B timing of library builds on the bench's own timed region (hipGraph
replays of 100 astro_step launches, c3 by default, after the bench's
300-tick burn-in; before round 3's last A/Bs there was none, so games were
young), interleaved over rounds so clock drift hits every build alike.

    python tools/ab.py --libs libastro_hip,libastro_hip_var[:kernel] [--workload c3] [--rounds 5]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from astro_amd import BatchedEnv, DEFAULT_CONFIG, _lib  # noqa: E402


def make(spec, wl, n, ticks, rollout, stamp_rows=False, stats=False):
    lib, _, kernel = spec.partition(':')
    _lib._lib = None
    _lib.load(os.path.join(ROOT, 'astro_amd', lib + '.so'))
    w = bench.WORKLOADS[wl]
    env = BatchedEnv(DEFAULT_CONFIG._replace(**w['cfg']), n, device='cuda:0', b_cap=w['b_cap'],
                     p_pad=w['p_pad'], auto_reset=True, kernel=kernel or 'auto', planets_only=w['planets_only'])
    env.reset()
    if stamp_rows:   # room for a -DASTRO_STAMPS build's per-wave rows (32 int64 per wave)
        lpe = dict(lane=1, quad=4, pair=2)[env.step_kernel]
        env.stats = torch.zeros((n * lpe + 63) // 64, 32, dtype=torch.int64, device='cuda:0')
    if rollout > 0:   # age the batch as bench.py does (games of every age, bullets in flight)
        env.rollout(rollout, 'random', tick0=1 << 40, stats=False)
    ctl = torch.from_numpy(bench.controls(0, n, env.S, ticks)).cuda()
    for t in range(50):
        env.launch(ctl[t].data_ptr(), stats=stats)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for t in range(50, 150):
                env.launch(ctl[t].data_ptr(), stats=stats)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    return env, g


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--libs', required=True)
    ap.add_argument('--workload', default='c3')
    ap.add_argument('--n-env', type=int, default=0)
    ap.add_argument('--rounds', type=int, default=5)
    ap.add_argument('--reps', type=int, default=5)
    ap.add_argument('--stats', action='store_true', help='time the counting launches (default: the counter-free '
                                                         'ones bench.py times)')
    ap.add_argument('--stamp-rows', action='store_true', help='per-wave stats rows (for -DASTRO_STAMPS builds)')
    ap.add_argument('--burn-in', type=int, default=300, help='random-policy rollout ticks after reset (bench.py: 300)')
    ap.add_argument('--rollout-policy', default='random', help="the rollout column's policy ('random', 'script', ...)")
    a = ap.parse_args()
    libs = a.libs.split(',')
    n = a.n_env or bench.WORKLOADS[a.workload]['n']
    res = {l: [] for l in libs}
    rolls = {l: [] for l in libs}
    for r in range(a.rounds):
        for lib in libs:
            env, g = make(lib, a.workload, n, 150, a.burn_in, a.stamp_rows, a.stats or a.stamp_rows)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            res[lib].append(e0.elapsed_time(e1) * 1e3 / (100 * a.reps))
            e0.record()
            env.rollout(100, a.rollout_policy, tick0=1000, stats=False)
            e1.record()
            torch.cuda.synchronize()
            rolls[lib].append(e0.elapsed_time(e1) * 1e3 / 100)
            del g, env
    for lib in libs:
        v = np.array(res[lib])
        print(json.dumps(dict(lib=lib, workload=a.workload, n=n, us_per_launch_median=float(np.median(v)),
                              us_all=[round(x, 3) for x in v],
                              rollout_us_per_tick=float(np.median(rolls[lib])), rollout_policy=a.rollout_policy)),
              flush=True)


if __name__ == '__main__':
    main()
