#!/usr/bin/env python3
"""GPU time of ONE env's one-tick launch (the single-game drop-in's kernel):
the game's state in device memory against the shim's host-mapped arena,
200 launches back to back behind a spin kernel, event pair around them."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from astro_amd import BatchedEnv, DEFAULT_CONFIG, core  # noqa: E402


def timed(env, ctl, k=200):
    torch.cuda.synchronize()
    torch.cuda._sleep(3000000)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(k):
        env.launch(ctl.data_ptr(), stats=False)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / k


def main():
    cfg = DEFAULT_CONFIG
    out = {}
    ctl = torch.tensor([[3, 2]], dtype=torch.int8, device='cuda:0')
    for name, kw in (('device', dict()), ('device_quad', dict(kernel='quad')), ('device_lane', dict(kernel='lane'))):
        env = BatchedEnv(cfg, 1, device='cuda:0', dtype=torch.float64, b_cap=64, auto_reset=True, **kw)
        env.reset()
        out[name] = [round(timed(env, ctl), 3) for _ in range(3)]
        out[name + '_kernel'] = env.step_kernel
    st = core.create(cfg)
    rng = np.random.RandomState(0)
    for _ in range(30):
        st, _ = core.step(st, rng.randint(0, 6, size=2), cfg)
        if st is None:
            st = core.create(cfg)
    sh = core._shim(cfg, 0)
    out['mapped'] = [round(timed(sh.env, ctl), 3) for _ in range(3)]
    out['mapped_kernel'] = sh.env.step_kernel
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
