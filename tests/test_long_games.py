"""BASELINE.json config 1 and whole games to their end, vs the reference.

Fixtures (tools/gen_golden.py, written by running the reference itself):
  * config1.npz    -- config 1: DEFAULT_CONFIG (seed 42), 1000 ticks of
                      RandomState(0).randint(0, 6, (1000, 2)) controls,
                      re-created with the same config whenever a game ends
                      (the input state of every tick, rewards, done codes);
  * long_games.npz -- core.play (core.py:377-410) under the reference's own
                      bots: test_script's games (test/test_core.py:88-98:
                      ScriptBot solo at max_time=20 wins, NothingBot vs
                      ScriptBot is won by ScriptBot) and a SOLO game that
                      reaches the 3000-tick timeout (core.py:257-260).

The CPU tests replay them through the oracle (oracle/port.py, the single-game
restatement) and the host ScriptBot; the GPU tests through the HIP kernel:
the reference-shaped shim (astro_amd.core) and BatchedEnv with float64
state, bit for bit.
"""
import json
import os

import numpy as np
import pytest
import torch

from astro_amd import bots as hbots
from astro_amd.config import Config, DEFAULT_CONFIG
from oracle import port
from tests import golden_io as gio

KERNELS = ['lane', 'quad', 'pair']


def _long():
    z = gio.load('long_games.npz')
    with open(os.path.join(gio.GOLDEN, 'long_games.json')) as f:
        index = json.load(f)
    for r in index:
        r['cfg'] = Config(**r['config'])
        for k in ('controls', 'ships', 'nbullets', 'reward'):
            r[k] = z[r['key'] + '__' + k]
    return index


def _bots(names, config, lib):
    return [lib.ScriptBot.create(config) if n == 'script' else lib.NothingBot() for n in names]


def _check_config1_state(st, z, t):
    n = int(z['nplanets'][t])
    assert np.array_equal(st.ships.x, z['ships'][t, :, 0:2]), t
    assert np.array_equal(st.ships.dx, z['ships'][t, :, 2:4]), t
    assert np.array_equal(st.ships.b, z['ships'][t, :, 4]), t
    assert np.array_equal(st.planets.x, z['planets'][t, :n, 0:2]), t
    assert np.array_equal(st.planets.dx, z['planets'][t, :n, 2:4]), t
    off = z['bullets_off']
    bl = z['bullets'][off[t]:off[t + 1]]
    assert np.array_equal(st.bullets.x, bl[:, 0:2]), t
    assert np.array_equal(st.bullets.dx, bl[:, 2:4]), t


def _run_config1(create, step):
    z = gio.load('config1.npz')
    ctl = z['control'].astype(np.int64)
    assert np.array_equal(ctl, np.random.RandomState(0).randint(0, 6, (1000, 2)))
    st = create()
    ended = 0
    for t in range(1000):
        _check_config1_state(st, z, t)
        st, rew = step(st, ctl[t])
        assert np.array_equal(rew, z['reward'][t]), t
        if st is None:
            assert z['done'][t] == (1 if rew.dtype.kind == 'i' else 2), t
            st = create()
            ended += 1
        else:
            assert z['done'][t] == 0, t
    assert ended == int((z['done'] > 0).sum()) > 0


# ------------------------------------------------------------------ CPU

def test_config1_trace_oracle():
    g = port.Game(DEFAULT_CONFIG)
    _run_config1(g.create, g.step)


@pytest.mark.parametrize('key', ['script_solo0', 'nothing_script2', 'solo_timeout'])
def test_long_games_oracle_closed_loop(key):
    """The oracle step driven by the host bots (astro_amd.bots) replays the
    reference's core.play exactly: every decision, every ship state, the
    length (1001, 335, 3000 ticks) and the winner."""
    r = next(r for r in _long() if r['key'] == key)
    cfg = r['cfg']
    S = 1 if cfg.solo else 2
    g = port.Game(cfg)
    bots = _bots(r['bots'], cfg, hbots)
    st = g.create()
    for t in range(r['ticks']):
        assert np.array_equal(st.ships.x, r['ships'][t, :S, 0:2]), t
        assert np.array_equal(st.ships.b, r['ships'][t, :S, 4]), t
        ctl = np.array([b(_roll(st, i)) for i, b in enumerate(bots)])
        assert np.array_equal(ctl, r['controls'][t]), t
        st, rew = g.step(st, ctl)
        assert (st is None) == (t == r['ticks'] - 1), t
    winner = None if np.max(rew) < 1 else int(np.argmax(rew))
    assert winner == r['winner']
    assert np.array_equal(np.pad(rew.astype(np.float64), (0, 2 - S)), r['reward'])


def test_long_games_fixture_invariants():
    """The reference's own test_script invariants hold in the fixture, and
    the SOLO game really runs to the 3000-tick timeout."""
    idx = {r['key']: r for r in _long()}
    for k in range(3):
        assert idx['script_solo%d' % k]['winner'] == 0
        assert idx['nothing_script%d' % k]['winner'] == 1
    t = idx['solo_timeout']
    assert t['ticks'] == 3000 and t['done'] == 2 and t['winner'] == 0


def _roll(state, i):
    from astro_amd.core import roll_ships
    return roll_ships(state, i)


# ------------------------------------------------------------------ GPU

@pytest.mark.gpu
@pytest.mark.parametrize('mode', ['mapped', 'mapped_py', 'copy'])
def test_config1_trace_through_hip_shim(mode, monkeypatch):
    """BASELINE config 1 through the drop-in surface: astro_amd.core.create /
    step (one float64 env on the HIP kernel) reproduce the reference's
    1000-tick trace bit for bit, re-creates included -- with the game's arena
    in host-mapped memory (the default; its packing in C, and in Python) and
    in device memory with copies."""
    from astro_amd import core
    if mode == 'mapped_py':
        monkeypatch.setattr(core, '_gamestep', None)
    else:
        assert mode != 'mapped' or core._gamestep is not None, 'astro_amd/_gamestep not built'
    mode = 'mapped' if mode == 'mapped_py' else mode
    monkeypatch.setattr(core, 'SHIM_MODE', mode)
    monkeypatch.setattr(core, '_ENVS', {})
    _run_config1(lambda: core.create(DEFAULT_CONFIG), lambda s, c: core.step(s, c, DEFAULT_CONFIG))
    sh = next(iter(core._ENVS.values()))
    assert sh.arena.mode == mode


@pytest.mark.gpu
def test_shim_c_packing_equals_python(monkeypatch):
    """The C packing of a mapped-arena tick (astro_amd/_gamestep) returns what
    the Python packing returns: the same values, dtypes and shapes of every
    State array (float32 at a game's first tick and for a lone planet), the
    same types of reload and t, and the same end-of-game reward (int64 on a
    collision), over whole games of every planet count."""
    from astro_amd import core
    assert core._gamestep is not None, 'astro_amd/_gamestep not built'
    monkeypatch.setattr(core, 'SHIM_MODE', 'mapped')
    monkeypatch.setattr(core, '_ENVS', {})
    gs = core._gamestep
    rng = np.random.RandomState(7)
    ends = set()
    for seed in range(12):
        cfg = DEFAULT_CONFIG._replace(seed=seed, max_planets=4)
        s = core.create(cfg)
        for _ in range(400):
            c = rng.randint(0, 6, size=2)
            monkeypatch.setattr(core, '_gamestep', gs)
            a, ra = core.step(s, c, cfg)
            monkeypatch.setattr(core, '_gamestep', None)
            b, rb = core.step(s, c, cfg)
            assert ra.dtype == rb.dtype and np.array_equal(ra, rb)
            if a is None or b is None:
                assert a is None and b is None
                ends.add(str(ra.dtype))
                break
            assert type(a.reload) is type(b.reload) and a.reload == b.reload
            assert type(a.t) is type(b.t) and a.t == b.t
            for f in ('ships', 'planets', 'bullets'):
                for g in ('x', 'dx', 'b'):
                    x, y = getattr(getattr(a, f), g), getattr(getattr(b, f), g)
                    if y is None:
                        assert x is None
                    else:
                        assert x.dtype == y.dtype and x.shape == y.shape and np.array_equal(x, y), (f, g)
            s = a
    assert ends   # games ended on the way


@pytest.mark.gpu
def test_shim_two_threads_interleaved(monkeypatch):
    """astro/server.py calls core.step from request threads: two games ticked
    concurrently through the same shim arena (same config, the host-mapped
    default) each stay their own game -- one thread replays config 1's
    reference trace, the other plays seed 7 against the oracle port."""
    import threading
    from astro_amd import core
    monkeypatch.setattr(core, '_ENVS', {})
    errors = []

    def trace():
        try:
            _run_config1(lambda: core.create(DEFAULT_CONFIG), lambda s, c: core.step(s, c, DEFAULT_CONFIG))
        except Exception as e:   # (reported by the main thread)
            errors.append(e)

    def other():
        try:
            cfg = DEFAULT_CONFIG._replace(seed=7)
            g = port.Game(cfg)
            rng = np.random.RandomState(1)
            st, want = core.create(cfg), g.create()
            for t in range(1500):
                ctl = rng.randint(0, 6, 2)
                st, rew = core.step(st, ctl, cfg)
                want, wrew = g.step(want, ctl)
                assert np.array_equal(rew, wrew) and rew.dtype == wrew.dtype, t
                if st is None:
                    assert want is None, t
                    st, want = core.create(cfg), g.create()
                else:
                    assert np.array_equal(st.ships.x, want.ships.x), t
                    assert np.array_equal(st.bullets.x, want.bullets.x), t
        except Exception as e:
            errors.append(e)
    th = [threading.Thread(target=f) for f in (trace, other)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors
    assert len(core._ENVS) == 1


@pytest.mark.gpu
def test_test_script_invariants_through_hip_shim():
    """test/test_core.py:88-98 on the HIP kernel: astro_amd.core.play with
    ScriptBot solo (max_time=20) -> winner 0; NothingBot vs ScriptBot ->
    winner 1; and the 3000-tick SOLO game to its timeout.  Every tick's
    controls equal the reference's."""
    from astro_amd import core
    for r in _long():
        cfg = r['cfg']
        game = core.play(cfg, _bots(r['bots'], cfg, hbots))
        assert len(game.ticks) == r['ticks'], r['key']
        assert game.winner == r['winner'], r['key']
        ctl = np.stack([t.control for t in game.ticks])
        assert np.array_equal(ctl, r['controls']), r['key']


@pytest.mark.gpu
@pytest.mark.parametrize('kernel', KERNELS)
def test_long_games_batched_float64_open_loop(kernel):
    """All the long games at once in one BatchedEnv (float64 state), their
    recorded controls replayed: every tick's ship state, bullet counts, the
    length (up to 3000 ticks: the timeout) and the outcome, bit for bit."""
    from astro_amd import BatchedEnv
    games = _long()
    by_cfg = {}
    for r in games:
        by_cfg.setdefault(r['cfg']._replace(seed=0), []).append(r)
    for cfg, gs in by_cfg.items():
        S = 1 if cfg.solo else 2
        env = BatchedEnv(cfg, len(gs), device='cuda:0', b_cap=64, dtype=torch.float64,
                         auto_reset=False, kernel=kernel)
        env.reset(seeds=np.array([r['cfg'].seed for r in gs], dtype=np.uint32))
        T = max(r['ticks'] for r in gs)
        alive = np.ones(len(gs), bool)
        for t in range(T):
            h = env.to_host()
            ctl = np.full((len(gs), S), 2, np.int8)
            for k, r in enumerate(gs):
                if alive[k]:
                    assert np.array_equal(h['ships'][k], r['ships'][t, :S, 0:4]), (r['key'], t)
                    assert np.array_equal(h['ships_b'][k], r['ships'][t, :S, 4]), (r['key'], t)
                    assert h['nbullets'][k] == r['nbullets'][t], (r['key'], t)
                    ctl[k] = r['controls'][t]
            _, rew, done = env.step(torch.from_numpy(ctl).cuda(), auto_reset=False)
            done = done.cpu().numpy()
            rew = rew.cpu().numpy()
            for k, r in enumerate(gs):
                if alive[k]:
                    last = t == r['ticks'] - 1
                    assert bool(done[k]) == last, (r['key'], t)
                    if last:
                        assert done[k] == r['done'] and np.array_equal(rew[k], r['reward'][:S])
                        alive[k] = False
        assert not alive.any()
