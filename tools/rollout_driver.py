#!/usr/bin/env python3
"""A fixed rollout workload for rocprofv3 passes: the bench's c3 (or
--workload) batch, burned in, then --launches astro_rollout launches of
--ticks ticks with the on-device random policy (the bench's rollout line)."""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from astro_amd import BatchedEnv, DEFAULT_CONFIG  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--workload', default='c3')
    ap.add_argument('--n-env', type=int, default=0)
    ap.add_argument('--ticks', type=int, default=100)
    ap.add_argument('--launches', type=int, default=10)
    ap.add_argument('--burn-in', type=int, default=300)
    ap.add_argument('--b-cap', type=int, default=0, help='override the workload\'s bullet capacity')
    ap.add_argument('--lib', default='', help='a library variant under astro_amd/ (A/B builds)')
    ap.add_argument('--no-reset', action='store_true', help='timed rollouts without auto-reset (finished games '
                                                            're-stepped): the reset passes\' share by difference')
    ap.add_argument('--policy', default='random', help="the timed rollouts' policy ('random', 'script', ...)")
    a = ap.parse_args()
    if a.lib:
        from astro_amd import _lib
        _lib._lib = None
        _lib.load(os.path.join(ROOT, 'astro_amd', a.lib + '.so'))
    w = bench.WORKLOADS[a.workload]
    n = a.n_env or w['n']
    env = BatchedEnv(DEFAULT_CONFIG._replace(**w['cfg']), n, device='cuda:0', b_cap=a.b_cap or w['b_cap'], p_pad=w['p_pad'],
                     auto_reset=True, planets_only=w['planets_only'])
    env.reset()
    env.rollout(a.burn_in, 'random', tick0=1 << 40, stats=False)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for r in range(a.launches):
        env.rollout(a.ticks, a.policy, tick0=1000 + r * a.ticks, stats=False, auto_reset=not a.no_reset)
    e1.record()
    torch.cuda.synchronize()
    env.check_errors()
    print('us_per_tick %.3f' % (e0.elapsed_time(e1) * 1e3 / (a.ticks * a.launches)))


if __name__ == '__main__':
    main()
