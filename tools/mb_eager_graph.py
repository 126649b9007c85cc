#!/usr/bin/env python3
"""Per-launch GPU time of a workload's one-tick launch, eager back-to-back
launches against the same launches replayed from a hipGraph, after the
bench's burn-in (event pairs on the launch stream).
    python tools/mb_eager_graph.py --workload c5 [--lib libastro_hip]"""
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
    ap.add_argument('--workload', default='c5')
    ap.add_argument('--lib', default='libastro_hip')
    ap.add_argument('--burn-in', type=int, default=300)
    ap.add_argument('--k', type=int, default=20)
    ap.add_argument('--reps', type=int, default=5)
    a = ap.parse_args()
    _lib._lib = None
    _lib.load(os.path.join(ROOT, 'astro_amd', a.lib + '.so'))
    w = bench.WORKLOADS[a.workload]
    n = w['n']
    env = BatchedEnv(DEFAULT_CONFIG._replace(**w['cfg']), n, device='cuda:0', b_cap=w['b_cap'], p_pad=w['p_pad'],
                     auto_reset=True, planets_only=w['planets_only'])
    env.reset()
    env.rollout(a.burn_in, 'random', tick0=1 << 40, stats=False)
    K = a.k
    ctl = torch.from_numpy(bench.controls(0, n, env.S, K * (2 * a.reps + 2))).cuda()
    ptr = lambda t: ctl[t % ctl.shape[0]].data_ptr()  # noqa: E731
    for t in range(5):
        env.launch(ptr(t))
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for t in range(K):
                env.launch(ptr(t))
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    out = dict(workload=a.workload, lib=a.lib, n=n, k=K, eager=[], graph=[], eager_stats_off=[])
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t = K
    for r in range(a.reps):
        e0.record()
        for _ in range(K):
            env.launch(ptr(t))
            t += 1
        e1.record()
        torch.cuda.synchronize()
        out['eager'].append(round(e0.elapsed_time(e1) * 1e3 / K, 3))
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        out['graph'].append(round(e0.elapsed_time(e1) * 1e3 / K, 3))
        e0.record()
        for _ in range(K):
            env.launch(ptr(t), stats=False)
            t += 1
        e1.record()
        torch.cuda.synchronize()
        out['eager_stats_off'].append(round(e0.elapsed_time(e1) * 1e3 / K, 3))
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
