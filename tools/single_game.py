#!/usr/bin/env python3
"""bench.py's single_game line alone: the drop-in astro_amd.core.step /
play latency (mapped and copy arenas) beside oracle/port.py on one core."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from astro_amd import DEFAULT_CONFIG  # noqa: E402

if __name__ == '__main__':
    for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 1):
        r = bench.single_game_latency(DEFAULT_CONFIG)
        r.pop('path', None)
        print(json.dumps(r), flush=True)
