#!/usr/bin/env python3
"""Where a single-game tick's time goes (astro_amd.core, mapped arena):
the whole core.step call, astro_game_step alone (pack, launch, wait,
unpack in C) on a fixed state, and the Python around it."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from astro_amd import DEFAULT_CONFIG, core  # noqa: E402


def main():
    cfg = DEFAULT_CONFIG
    rng = np.random.RandomState(0)
    st = core.create(cfg)
    for _ in range(30):
        st, _ = core.step(st, rng.randint(0, 6, size=2), cfg)
        if st is None:
            st = core.create(cfg)
    sh = core._shim(cfg, 0)
    n = 3000
    # whole call, fixed state (the same input every time: no create)
    ctl = np.array([3, 2])
    t0 = time.perf_counter()
    for _ in range(n):
        core.step(st, ctl, cfg)
    whole = (time.perf_counter() - t0) / n * 1e6
    # C alone: the record as the last call left it
    f, ptr = sh.game_step, sh.tick_ptr
    t0 = time.perf_counter()
    for _ in range(n):
        f(ptr)
    c_only = (time.perf_counter() - t0) / n * 1e6
    print(json.dumps(dict(kernel=core.SHIM_KERNEL, step_env_kernel=sh.env.step_kernel, us_core_step=whole,
                          us_astro_game_step=c_only, us_python=whole - c_only)), flush=True)


if __name__ == '__main__':
    main()
