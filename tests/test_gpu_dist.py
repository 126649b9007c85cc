"""The multi-GPU code path of bench.py on one GPU, over RCCL.

bench.py's multi-rank run initialises ``torch.distributed`` with the
``nccl`` backend (RCCL on ROCm), brackets its timed region with barriers and
reduces its timing and counters with device-tensor ``all_reduce``
(astro_amd/shard.py).  An 8-GPU node is not available to the build, so this
runs that same path at world size 1 (``ASTRO_DIST_INIT=1``: the process group
is initialised although there is one rank) as a real rank would, and checks
the line it prints.  Games are independent (astro/core.py:215-303): the
collective is timing and counters only, never on the hot path.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.gpu
def test_bench_rank_over_rccl_at_world_size_one():
    env = dict(os.environ, ASTRO_DIST_INIT='1', ASTRO_DIST_BACKEND='nccl', RANK='0', LOCAL_RANK='0',
               WORLD_SIZE='1', LOCAL_WORLD_SIZE='1', MASTER_ADDR='127.0.0.1', MASTER_PORT=str(_free_port()),
               PYTHONDONTWRITEBYTECODE='1')
    cmd = [sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', '1', '--steps', '6', '--warmup', '2',
           '--burn-in', '20', '--rollout', '4', '--no-features', '--no-single', '--calib', '4',
           '--cpu-seconds', '0.5', '--cpu-procs', '1', '--n-env', '4096', '--warm-ms', '2']
    p = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.strip().startswith('{')]
    assert len(lines) == 1, p.stdout
    j = json.loads(lines[0])
    assert j['dist'] == dict(initialized=True, backend='nccl', world=1, barrier='host-side gloo group',
                             reductions='device tensors (RCCL all_reduce)')
    assert j['ranks'] == 1 and j['n_gpus'] == 1 and j['value'] > 0
    agg = j['roofline']['aggregate']
    assert agg['n_gpus'] == 1 and agg['achieved'] > 0
    assert j['cpu_baseline']['kind'] == 'port' and j['cpu_baseline']['value'] > 0
    assert j['rollout']['launches'] >= 10
    assert j['device_errors'] == 0
