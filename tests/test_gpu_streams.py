"""generate_configs streams far past MT19937's first 624 words, on the GPU.

Each env plays the games of ONE RandomState (core.py:77-83: generate_configs
draws ``randint(1 << 30)`` from the same generator for as long as the env
plays), so an RL-length run walks thousands of MT19937 outputs per env.  The
kernel's MTStream (cursor + per-env 624-word ring) must reproduce every one
of them: these tests run games that end at their first tick (or after a few)
so that each env draws 800-2,000 words -- past output 227 (where the lazy
init-key form stops being valid) and past 624 and 1,248 (whole twists) --
and compare every game seed and every created game with the oracle
(oracle/mt19937.py: numpy's legacy MT19937, pinned by tests/golden/).
"""
import numpy as np
import pytest
import torch

from oracle import batched
from tests import golden_io as gio

pytestmark = pytest.mark.gpu

CFG = gio.configs()
KERNELS = ['lane', 'quad', 'pair']


def _host_batch(env):
    h = env.to_host()
    return batched.Batch(h['tick'].astype(np.int32), h['nplanets'].astype(np.int32),
                         h['nbullets'].astype(np.int32), h['ships'].astype(np.float64),
                         h['ships_b'].astype(np.float64), h['planets'].astype(np.float64),
                         h['bullets'].astype(np.float64), (h['flags'] & 1).astype(bool))


# (planets_only, game length in ticks via max_time, steps)
#   fast: every game times out at its first tick, so with planets_only the
#         reset itself walks the stream (next_game's synchronous walk);
#   slow: 6-tick games, the running steps check one candidate each
#         (check_pending) before the game ends
VARIANTS = {
    'unfiltered_fast': (0, 1, 900),
    'filtered_fast': (3, 1, 420),
    'filtered_slow': (3, 6, 1500),
}


@pytest.mark.parametrize('kernel', KERNELS)
@pytest.mark.parametrize('variant', sorted(VARIANTS))
def test_streams_exact_past_624_draws(variant, kernel):
    planets_only, life, steps = VARIANTS[variant]
    cfg = CFG['default']
    cfg = cfg._replace(max_time=cfg.dt * life)
    n = 200
    from astro_amd import BatchedEnv
    env = BatchedEnv(cfg, n, device='cuda:0', b_cap=32, planets_only=planets_only, kernel=kernel)
    env.reset()
    draws = 2600
    if planets_only:
        seeds, idx = batched.filtered_game_draws(env.stream_seeds, draws // 5, planets_only,
                                                 cfg.max_planets, draws)
    else:
        seeds = batched.game_seeds(env.stream_seeds, draws)
        idx = np.broadcast_to(np.arange(draws), seeds.shape)
    games = np.ones(n, np.int64)
    rows = np.arange(n)
    ctl = torch.full((n, 2), 2, dtype=torch.int8, device='cuda')
    for t in range(steps):
        _, _, done = env.step(ctl)
        games += done.cpu().numpy() != 0
        got = env.game_seed.cpu().numpy().view(np.uint32)
        assert np.array_equal(got, seeds[rows, games - 1]), (variant, t)
    h = env.to_host()
    assert not (h['flags'] & 2).any()
    if planets_only:
        assert (h['nplanets'] == planets_only).all()
    # how far the streams went: the deepest game seed's draw index
    deepest = int(idx[rows, games - 1].max())
    assert deepest > 700, deepest
    # the games themselves: the last games created equal the oracle's
    # create() of the same seeds (every env at tick 0 in the fast variants)
    fresh = h['tick'] == 0
    if fresh.any():
        P = batched.make_params(cfg)
        want = batched.create(seeds[rows, games - 1][fresh], P, p_pad=env.p_pad, b_cap=32, store='f32')
        got = _host_batch(env).take(np.nonzero(fresh)[0])
        assert np.array_equal(got.nplanets, want.nplanets)
        assert np.array_equal(got.ships, want.ships.astype(np.float32).astype(np.float64))
        assert np.array_equal(got.ships_b, want.ships_b.astype(np.float32).astype(np.float64))
        pv = np.arange(env.p_pad)[None, :] < got.nplanets[:, None]
        assert np.array_equal(got.planets[pv], want.planets[pv].astype(np.float32).astype(np.float64))


def test_stream_reset_path_past_624_draws():
    """astro_reset without seeds (the stream's next game, astro_reset_kernel)
    keeps walking the same exact stream: 700 resets per env."""
    cfg = CFG['default']
    n = 100
    from astro_amd import BatchedEnv
    env = BatchedEnv(cfg, n, device='cuda:0', b_cap=8, planets_only=0)
    want = batched.game_seeds(env.stream_seeds, 700)
    for k in range(700):
        env.reset()
        assert np.array_equal(env.game_seed.cpu().numpy().view(np.uint32), want[:, k]), k
