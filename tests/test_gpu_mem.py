"""The state arrays in each memory kind astro_dev_alloc offers (BatchedEnv
mem: hipMalloc, fine-grained, uncached) give the same games bit for bit.

The kind only changes how the L2 treats the arrays (include/astro_step.h
ASTRO_MEM_*), never the arithmetic: c3-shaped batches (3-planet games,
bullets, auto-reset) on the helper instance, the helper-less pair instance
and the K-tick rollout must match the default-memory run on every array.
"""
import numpy as np
import pytest
import torch

from astro_amd import BatchedEnv, DEFAULT_CONFIG

pytestmark = pytest.mark.gpu

ARRAYS = ('ships', 'ships_b', 'planets', 'bullets', 'hdr', 'stream')


def _run(mem, n, ticks, rollout):
    env = BatchedEnv(DEFAULT_CONFIG, n, device='cuda:0', b_cap=32, planets_only=3, mem=mem)
    env.reset()
    env.rollout(40, 'random', tick0=1 << 40, stats=False)   # games of several ages, bullets in flight
    g = torch.Generator().manual_seed(7)
    rew, done = [], []
    if rollout:
        env.rollout(ticks, 'random', tick0=5, stats=False)
    else:
        for t in range(ticks):
            c = torch.randint(0, 6, (n, env.S), generator=g, dtype=torch.int8).cuda()
            _, r, d = env.step(c)
            rew.append(r.clone())
            done.append(d.clone())
    torch.cuda.synchronize()
    env.check_errors()
    out = {k: getattr(env, k).cpu().numpy() for k in ARRAYS}
    if rew:
        out['reward'] = torch.stack(rew).cpu().numpy()
        out['done'] = torch.stack(done).cpu().numpy()
    return out


@pytest.mark.parametrize('mem', ['uncached', 'finegrained'])
@pytest.mark.parametrize('n, rollout', [(65536, False), (200000, False), (16384, True)])
def test_memory_kinds_bit_exact(mem, n, rollout):
    """n = 65,536: the pair instance with helper waves (config 3's); 200,000:
    the helper-less pair instance; a rollout: the K-tick kernel."""
    want = _run('default', n, 30, rollout)
    got = _run(mem, n, 30, rollout)
    for k in want:
        assert np.array_equal(got[k], want[k]), (mem, n, k)


def test_mem_argument_checked():
    with pytest.raises(ValueError):
        BatchedEnv(DEFAULT_CONFIG, 4, device='cuda:0', mem='pinned')
