#!/usr/bin/env python3
"""Workload state of a library variant after the bench's burn-in and N
launches: mean live bullets, resets per launch, planets, device errors --
to see that an A/B variant steps the same games (tools/ab.py times them).
    python tools/varstats.py --libs libastro_hip,libastro_hip_x --workload c5"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from astro_amd import BatchedEnv, DEFAULT_CONFIG, _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--libs', required=True)
    ap.add_argument('--workload', default='c3')
    ap.add_argument('--launches', type=int, default=200)
    a = ap.parse_args()
    w = bench.WORKLOADS[a.workload]
    n = w['n']
    ctl = torch.from_numpy(bench.controls(0, n, 2, a.launches)).cuda()
    ref = None
    for lib in a.libs.split(','):
        _lib._lib = None
        _lib.load(os.path.join(ROOT, 'astro_amd', lib + '.so'))
        env = BatchedEnv(DEFAULT_CONFIG._replace(**w['cfg']), n, device='cuda:0', b_cap=w['b_cap'], p_pad=w['p_pad'],
                         auto_reset=True, planets_only=w['planets_only'])
        env.reset()
        s0 = env.stat_dict()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for t in range(a.launches):
            env.launch(ctl[t].data_ptr())
        e1.record()
        torch.cuda.synchronize()
        s1 = env.stat_dict()
        d = {k: s1[k] - s0[k] for k in s0}
        st = (env.hdr.clone(), env.ships.clone(), env.planets.clone(), env.bullets.clone())
        same = None if ref is None else all(torch.equal(x, y) for x, y in zip(st, ref))
        ref = ref or st
        print(json.dumps(dict(lib=lib, workload=a.workload, us_per_launch=e0.elapsed_time(e1) * 1e3 / a.launches,
                              mean_live_bullets=d['bullets_in'] / (n * a.launches), resets_per_launch=d['resets'] / a.launches,
                              mean_planets=d['planets'] / (n * a.launches), errors=env.device_errors(),
                              same_state_as_first=same)), flush=True)
        del env


if __name__ == '__main__':
    main()
