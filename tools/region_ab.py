#!/usr/bin/env python3
"""Same-process A/B of the bench's 20-step timed region: how the K launches
are handed to the GPU (hipGraph replays of various graph sizes, or the K
launches issued from C), alternated over many regions of one process so
box-level noise hits every variant alike.  Each region is what bench.py
times: synchronize, clock, submit, synchronize, clock (games continue from
region to region; controls cycle).

    python tools/region_ab.py [--steps 20] [--reps 40] [--variants 20 1+19 1+2+4+8+5 c]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from astro_amd import BatchedEnv, DEFAULT_CONFIG  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--reps', type=int, default=40)
    ap.add_argument('--variants', nargs='+', default=['20', '1+19', '1+2+4+8+5', 'c'])
    a = ap.parse_args()
    w = bench.WORKLOADS['c3']
    dev = torch.device('cuda', 0)
    env = BatchedEnv(DEFAULT_CONFIG, w['n'], device=dev, b_cap=w['b_cap'], p_pad=w['p_pad'], auto_reset=True,
                     planets_only=w['planets_only'])
    env.reset()
    env.rollout(300, 'random', tick0=1 << 40, stats=False)
    K = a.steps
    ctl = torch.from_numpy(bench.controls(0, w['n'], env.S, K)).to(dev)
    ptrs = [ctl[t].data_ptr() for t in range(K)]
    stream = torch.cuda.current_stream(dev)
    hgl = env.lib.hipGraphLaunch
    hgl.restype, hgl.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]
    sp = ctypes.c_void_p(stream.cuda_stream)
    rew = torch.empty(K, w['n'], env.S, dtype=torch.float32, device=dev)
    done = torch.empty(K, w['n'], dtype=torch.uint8, device=dev)
    subs = {}
    keep = []
    for v in a.variants:
        if v == 'c':
            subs[v] = lambda: env.launch_many(ptrs[0], K, rew.data_ptr(), done.data_ptr(), stats=False)
            continue
        sizes = [int(x) for x in v.split('+')]
        assert sum(sizes) == K, v
        cap = torch.cuda.Stream(dev)
        cap.wait_stream(stream)
        execs, k0 = [], 0
        with torch.cuda.stream(cap):
            for sz in sizes:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=cap):
                    for k in range(k0, k0 + sz):
                        env.launch(ptrs[k], stats=False)
                keep.append(g)
                execs.append(ctypes.c_void_p(g.raw_cuda_graph_exec()))
                k0 += sz
        stream.wait_stream(cap)

        def run(execs=execs):
            for e in execs:
                if hgl(e, sp) != 0:
                    raise RuntimeError('hipGraphLaunch failed')
        subs[v] = run
    for v in a.variants:   # every path once, untimed (first replays upload the graphs)
        subs[v]()
    torch.cuda.synchronize(dev)
    walls = {v: [] for v in a.variants}
    submit = {v: [] for v in a.variants}
    for r in range(a.reps):
        for v in a.variants:
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            subs[v]()
            t1 = time.perf_counter()
            torch.cuda.synchronize(dev)
            t2 = time.perf_counter()
            walls[v].append((t2 - t0) / K * 1e6)
            submit[v].append((t1 - t0) * 1e6)
    env.check_errors()
    for v in a.variants:
        x = np.array(walls[v])
        print(json.dumps(dict(variant=v, steps=K, reps=a.reps, wall_us_per_step_median=float(np.median(x)),
                              wall_us_per_step_p10=float(np.percentile(x, 10)),
                              wall_us_per_step_p90=float(np.percentile(x, 90)),
                              submit_us_median=float(np.median(submit[v])),
                              env_steps_per_s_median=w['n'] / (float(np.median(x)) * 1e-6))), flush=True)


if __name__ == '__main__':
    main()
