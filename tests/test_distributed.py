"""Multi-rank host logic on CPU with the gloo backend (world_size 2 and 4).

The GPU path shards envs by global id with no collective on the hot path;
what CAN be wrong without a GPU is the host side: shard ranges, per-rank seed
streams (must equal the matching slice of a 1-rank run) and the
max/sum-over-ranks reductions bench.py uses around the timed region."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as tmp

from astro_amd import shard
from astro_amd.config import DEFAULT_CONFIG


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, n_total, out_dir):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        off, cnt = shard.shard(n_total, rank, world)
        seeds = shard.stream_seeds(DEFAULT_CONFIG, off, cnt)
        wall = 1.0 + rank             # fake per-rank wall times
        mx = shard.max_over_ranks(wall)
        sm = shard.sum_over_ranks([cnt, rank])
        np.savez(os.path.join(out_dir, 'r%d.npz' % rank), off=off, cnt=cnt, seeds=seeds,
                 mx=mx, sm=np.array(sm))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('world,n_total', [(2, 1000), (4, 4099)])
def test_gloo_sharding_matches_single_rank(tmp_path, world, n_total):
    port = _free_port()
    tmp.spawn(_worker, args=(world, port, n_total, str(tmp_path)), nprocs=world, join=True)
    full = shard.stream_seeds(DEFAULT_CONFIG, 0, n_total)
    got = []
    for r in range(world):
        z = np.load(tmp_path / ('r%d.npz' % r))
        got.append(z['seeds'])
        assert float(z['mx']) == float(world)                 # max over ranks of 1 + rank
        assert z['sm'].tolist() == [float(n_total), float(sum(range(world)))]
    assert np.array_equal(np.concatenate(got), full)


def test_single_process_reductions_are_identity():
    assert shard.max_over_ranks(3.5) == 3.5
    assert shard.sum_over_ranks([1, 2]) == [1.0, 2.0]
