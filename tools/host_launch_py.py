#!/usr/bin/env python3
"""Host cost per astro_step launch from Python (ctypes, env.launch) and from
C (env.launch_many), on a small batch so the GPU keeps up; one JSON line."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from astro_amd import BatchedEnv, DEFAULT_CONFIG  # noqa: E402


def main():
    n, k = 256, 2000
    env = BatchedEnv(DEFAULT_CONFIG, n, device='cuda:0', b_cap=32, auto_reset=True, use_key_table=False)
    env.reset()
    ctl = torch.randint(0, 6, (k, n, 2), dtype=torch.int8, device='cuda:0')
    rew = torch.empty(k, n, 2, device='cuda:0')
    done = torch.empty(k, n, dtype=torch.uint8, device='cuda:0')
    ptrs = [ctl[t].data_ptr() for t in range(k)]
    out = {}
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for t in range(k):
            env.launch(ptrs[t])
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        env.launch_many(ptrs[0], k, rew.data_ptr(), done.data_ptr())
        t3 = time.perf_counter()
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        out = dict(n_env=n, launches=k, py_host_us_per_launch=(t1 - t0) / k * 1e6,
                   py_until_done_us_per_launch=(t2 - t0) / k * 1e6, c_host_us_per_launch=(t3 - t2) / k * 1e6,
                   c_until_done_us_per_launch=(t4 - t2) / k * 1e6)
    print(json.dumps(out))


if __name__ == '__main__':
    main()
