#!/usr/bin/env python3
"""Fault-injection check of the helper-wave wait (one-off, GPU box): with a
library built -DASTRO_DEBUG_DROP_POST the step waves never post their
finished envs, every helper's bounded wait must expire and the launch must
report ASTRO_ERR_HELPER_WAIT through AstroState.errors -- BatchedEnv.
check_errors() raises -- instead of running reset passes from a stale mask.
    ASTRO_LIB=astro_amd/libastro_hip_droppost.so python tools/fault_check.py"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from astro_amd import BatchedEnv, DEFAULT_CONFIG, _lib  # noqa: E402


def main():
    env = BatchedEnv(DEFAULT_CONFIG, 65536, device='cuda:0', b_cap=32, p_pad=4, planets_only=3)
    env.reset()
    ctl = torch.randint(0, 6, (65536, 2), dtype=torch.int8, device='cuda')
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    env.launch(ctl.data_ptr())
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    bits = int(env.errors.item())
    raised = None
    try:
        env.check_errors()
    except _lib.AstroError as e:
        raised = str(e)
    print(json.dumps(dict(lib=os.path.basename(_lib.LIB_PATH), launch_s=dt, error_bits=bits, raised=raised,
                          helper_waves=env.launch_waves()[1])), flush=True)


if __name__ == '__main__':
    main()
