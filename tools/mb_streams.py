#!/usr/bin/env python3
"""Config 3's 65,536 envs as S concurrent shards on S HIP streams of one GPU.

A one-tick launch reads its state in a burst at the start (every wave loads
its header, ships and planets at once), computes, and leaves its stores to
the end-of-launch write-back: the phases of one launch do not overlap.  Two
independent shards on two streams (HW queues) desynchronise: one shard's
load burst runs under the other's compute.  Measures GPU time per step of
the whole batch (all shards one tick) for shard counts 1, 2, 4, each shard
an env_offset slice of the same global batch (same games as one launch),
timed over graph replays of `--steps` launches per shard, after the bench's
300-tick burn-in.

    python tools/mb_streams.py [--steps 100] [--reps 5] [--shards 1,2,4] [--kernel auto]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from astro_amd import BatchedEnv, DEFAULT_CONFIG  # noqa: E402


def setup(n_total, shards, steps, kernel):
    w = bench.WORKLOADS['c3']
    n = n_total // shards
    envs, graphs, streams = [], [], []
    for k in range(shards):
        env = BatchedEnv(DEFAULT_CONFIG, n, device='cuda:0', b_cap=w['b_cap'], p_pad=w['p_pad'],
                         env_offset=k * n, auto_reset=True, kernel=kernel, planets_only=w['planets_only'])
        env.reset()
        env.rollout(300, 'random', tick0=1 << 40, stats=False)
        ctl = torch.from_numpy(bench.controls(k * n, n, env.S, steps + 10)).cuda()
        for t in range(10):
            env.launch(ctl[t].data_ptr())
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                for t in range(10, 10 + steps):
                    env.launch(ctl[t].data_ptr())
        torch.cuda.current_stream().wait_stream(s)
        envs.append((env, ctl))
        graphs.append(g)
        streams.append(s)
    torch.cuda.synchronize()
    for g in graphs:   # first replay uploads
        g.replay()
    torch.cuda.synchronize()
    return envs, graphs, streams


def timed(graphs, streams, steps):
    main = torch.cuda.current_stream()
    torch.cuda._sleep(2000000)   # the host submits every replay before the first one starts
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(main)
    for g, s in zip(graphs, streams):
        s.wait_stream(main)
        with torch.cuda.stream(s):
            g.replay()
    for s in streams:
        main.wait_stream(s)
    e1.record(main)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=100)
    ap.add_argument('--reps', type=int, default=5)
    ap.add_argument('--shards', default='1,2,4')
    ap.add_argument('--kernel', default='auto')
    ap.add_argument('--n', type=int, default=65536)
    a = ap.parse_args()
    for shards in [int(x) for x in a.shards.split(',')]:
        envs, graphs, streams = setup(a.n, shards, a.steps, a.kernel)
        us = [timed(graphs, streams, a.steps) for _ in range(a.reps)]
        for env, _ in envs:
            env.check_errors()
        print(json.dumps(dict(n_total=a.n, shards=shards, n_per_shard=a.n // shards, kernel=envs[0][0].step_kernel,
                              us_per_step=sorted(us)[len(us) // 2], us_all=[round(u, 3) for u in us],
                              env_steps_per_s=a.n / (sorted(us)[len(us) // 2] * 1e-6))), flush=True)
        del envs, graphs, streams
        torch.cuda.synchronize()


if __name__ == '__main__':
    main()
