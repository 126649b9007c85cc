"""Env-batch sharding over the GPUs of a node (one process per GPU).

Games are independent (core.step touches one game, core.py:215-303), so a
run of n_total envs is split into contiguous ranges of global env ids; each
env's seed stream is keyed by its global id (BatchedEnv env_offset), which
makes per-env results identical for any GPU count.  No collective is needed
on the hot path; ``max_over_ranks`` is the only reduction (timing).
"""


def shard(n_total, rank, world):
    """(offset, count) of rank's contiguous share of n_total envs."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError('bad rank/world')
    base, rem = divmod(int(n_total), int(world))
    offset = rank * base + min(rank, rem)
    return offset, base + (1 if rank < rem else 0)


def max_over_ranks(value, device=None):
    """Max of a float over all ranks of the default process group (or the
    value itself when no group is initialised; a one-rank group still runs
    the all_reduce, so the collective path is the same at every size)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(values, device=None):
    """Element-wise sum of a list of numbers over all ranks."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return [float(v) for v in values]
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.tolist()


def stream_seeds(config, offset, count):
    """Seed-stream seeds of global envs offset .. offset+count-1: the first
    configs of generate_configs(config) (core.py:77-83), i.e.
    RandomState(config.seed).randint(1 << 30) drawn in sequence.  Host numpy,
    O(offset + count)."""
    import numpy as np
    seeds = np.random.RandomState(config.seed).randint(1 << 30, size=int(offset) + int(count))
    return seeds[int(offset):].astype(np.uint32)
