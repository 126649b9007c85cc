#!/usr/bin/env python3
"""Launch driver for per-build PMC passes (tools/pmc_vars.sh): 200 eager
astro_step launches of a workload with the given library build.
    python tools/pmc_var.py --lib libastro_hip_abl_x [--workload c3] [--noreset]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from astro_amd import BatchedEnv, DEFAULT_CONFIG, _lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--lib', default='libastro_hip')
ap.add_argument('--workload', default='c3')
ap.add_argument('--noreset', action='store_true')
ap.add_argument('--ticks', type=int, default=200)
a = ap.parse_args()
_lib.load(os.path.join(ROOT, 'astro_amd', a.lib + '.so'))
w = bench.WORKLOADS[a.workload]
env = BatchedEnv(DEFAULT_CONFIG._replace(**w['cfg']), w['n'], device='cuda:0', b_cap=w['b_cap'],
                 p_pad=w['p_pad'], auto_reset=not a.noreset, planets_only=w['planets_only'])
env.reset()
ctl = torch.from_numpy(bench.controls(0, w['n'], env.S, a.ticks)).cuda()
for t in range(a.ticks):
    env.launch(ctl[t].data_ptr())
torch.cuda.synchronize()
print('ok', a.lib, env.stat_dict())
