"""On-device bots (script.py:6-91) and batched core.play (core.py:377-410).

* astro_controls (core.Bots.control on the device) == the reference
  ScriptBot's decision on every golden input state of steps.npz, every
  ship's ego view (tests/golden/script_controls.npz, written by running the
  reference);
* the ScriptBot instance of the rollout kernel makes the same decisions
  (one scripted tick == one step with the fixture's controls);
* BatchedEnv.play with device ScriptBots reproduces the reference's games
  closed-loop: test/test_core.py:88-98's winners, the fixtures' game
  lengths (long_games.npz: up to the 3000-tick timeout), and 32
  NothingBot-vs-ScriptBot games against the CPU oracle + host ScriptBot.
"""
import numpy as np
import pytest
import torch

from astro_amd import bots as hbots
from astro_amd.core import roll_ships
from oracle import port
from tests import golden_io as gio
from tests.test_long_games import _long

pytestmark = pytest.mark.gpu

CFG = gio.configs()


def _loaded(tr, idx, cfg, dtype):
    from astro_amd import BatchedEnv
    S = 1 if cfg.solo else 2
    bcap = tr.max_bullets(idx) + 2
    B = tr.batch_in(idx, S, b_cap=bcap)
    env = BatchedEnv(cfg, idx.size, device='cuda:0', b_cap=bcap, p_pad=8, dtype=dtype, auto_reset=False)
    env.load_host(B.ships, B.ships_b, B.planets, B.bullets, B.tick, B.nplanets, B.nbullets)
    return env


def _dtype_rule_holds(tr, i):
    """The kernel infers the reference's dtypes from (tick, planets): ships
    float32 iff tick 0, planet x float32 iff tick 0 or one planet, planet dx
    float32 iff one planet.  True when golden state i has those dtypes."""
    fl = int(tr.z['dtype_flags'][i])
    t0 = int(tr.z['tick'][i]) == 0
    one = int(tr.z['nplanets'][i]) == 1
    return (bool(fl & 1) == t0 and bool(fl & 2) == (t0 or one) and bool(fl & 4) == one)


@pytest.mark.parametrize('dtype', [torch.float64, torch.float32])
def test_device_scriptbot_decisions_match_reference(dtype):
    tr = gio.Transitions('steps.npz')
    want = gio.load('script_controls.npz')['control']
    checked = 0
    for name, idx in tr.groups():
        cfg = CFG[name]
        S = 1 if cfg.solo else 2
        assert all(_dtype_rule_holds(tr, i) for i in idx), name
        env = _loaded(tr, idx, cfg, dtype)
        got = env.controls('script').cpu().numpy()
        bad = np.nonzero((got != want[idx, :S]).any(1))[0]
        assert bad.size == 0, (name, idx[bad[:5]], got[bad[:5]], want[idx[bad[:5]], :S])
        checked += idx.size * S
    assert checked > 15000


def test_rollout_scriptbot_tick_equals_step_with_reference_decisions():
    """One tick of the ScriptBot rollout kernel (pair instance) from every
    golden state == astro_step driven by the reference's decisions."""
    tr = gio.Transitions('steps.npz')
    want = gio.load('script_controls.npz')['control']
    for name, idx in tr.groups():
        cfg = CFG[name]
        S = 1 if cfg.solo else 2
        a = _loaded(tr, idx, cfg, torch.float64)
        b = _loaded(tr, idx, cfg, torch.float64)
        ra, da = a.rollout(1, 'script', auto_reset=False)
        _, rb, db = b.step(torch.from_numpy(want[idx, :S].astype(np.int8)).cuda(), auto_reset=False)
        assert torch.equal(da[0], db) and torch.equal(ra[0], rb), name
        run = db == 0
        for f in ('ships', 'ships_b'):
            assert torch.equal(getattr(a, f)[:, run], getattr(b, f)[:, run]), (name, f)
        assert torch.equal(a.hdr[run], b.hdr[run]), name


def test_device_play_reproduces_reference_games():
    """BatchedEnv.play with device bots, float64 state, closed loop: the
    games of test/test_core.py:88-98 (ScriptBot solo at max_time=20 wins;
    NothingBot vs ScriptBot is won by ScriptBot) and the 3000-tick SOLO
    game, each the reference's own length and winner (long_games.npz)."""
    from astro_amd import BatchedEnv
    groups = {}
    for r in _long():
        groups.setdefault((r['cfg']._replace(seed=0), tuple(r['bots'])), []).append(r)
    for (cfg, names), rs in groups.items():
        env = BatchedEnv(cfg, len(rs), device='cuda:0', b_cap=64, dtype=torch.float64, auto_reset=True)
        env.reset(seeds=np.array([r['cfg'].seed for r in rs], dtype=np.uint32))
        winner, length = env.play(names, games=1)
        for k, r in enumerate(rs):
            assert int(length[k, 0]) == r['ticks'], r['key']
            assert int(winner[k, 0]) == (-1 if r['winner'] is None else r['winner']), r['key']


def test_device_play_nothing_vs_script_matches_oracle():
    """32 NothingBot-vs-ScriptBot games (DEFAULT_CONFIG, max_time=20) played
    on the device == the CPU oracle driven by the host ScriptBot, closed
    loop: same winners and lengths."""
    from astro_amd import BatchedEnv
    from astro_amd.config import DEFAULT_CONFIG
    cfg = DEFAULT_CONFIG._replace(max_time=20)
    n = 32
    env = BatchedEnv(cfg, n, device='cuda:0', b_cap=64, dtype=torch.float64, auto_reset=True)
    seeds = env.stream_seeds[:n].copy()
    env.reset(seeds=seeds)
    winner, length = env.play(('nothing', 'script'), games=1)
    g = port.Game(cfg)
    bots = [hbots.NothingBot(), hbots.ScriptBot.create(cfg)]
    wins = 0
    for k in range(n):
        st = g.create(int(seeds[k]))
        t = 0
        while st is not None:
            ctl = np.array([b(roll_ships(st, i)) for i, b in enumerate(bots)])
            st, rew = g.step(st, ctl)
            t += 1
        w = -1 if np.max(rew) < 1 else int(np.argmax(rew))
        assert (int(winner[k, 0]), int(length[k, 0])) == (w, t), k
        wins += w == 1
    assert wins > n // 2


@pytest.mark.parametrize('bots', ['script', ('nothing', 'script'), ('script', 'random')])
def test_resident_scripted_rollout_equals_controls_then_step(bots):
    """The ScriptBot instance of the resident rollout (float32 state, b_cap
    <= 32: the state on chip for the K ticks) == K ticks of astro_controls
    (core.Bots.control on the device, pinned above to the reference's
    decisions) followed by astro_step with those controls, bit for bit on
    every state array, reward and done, auto-reset included; and the random
    ship's draws are the RANDOM policy's (global env id, tick)."""
    from astro_amd import BatchedEnv
    cfg = CFG['default']
    n, K, t0 = 1200, 70, 9
    envs = [BatchedEnv(cfg, n, device='cuda:0', b_cap=32, p_pad=4, dtype=torch.float32, auto_reset=True,
                       kernel='pair', env_offset=40) for _ in range(2)]
    for e in envs:
        e.reset()
        e.rollout(30, 'random', tick0=1 << 20)   # games of several ages first
    a, b = envs
    rew, done = a.rollout(K, bots, tick0=t0)
    for k in range(K):
        c = b.controls(bots, tick0=t0 + k)
        _, r, d = b.step(c)
        assert torch.equal(rew[k], r) and torch.equal(done[k], d), k
    for f in ('ships', 'ships_b', 'planets', 'bullets', 'hdr', 'stream', 'stream_ring'):
        assert torch.equal(getattr(a, f), getattr(b, f)), f
    assert a.stat_dict() == b.stat_dict()
    assert int(done.ne(0).sum()) > 0


def test_play_bookkeeping_independent_of_chunk():
    """play's per-env game accounting (several games per env and chunk,
    games straddling chunks) does not depend on the rollout chunk length."""
    from astro_amd import BatchedEnv
    cfg = CFG['short']
    res = []
    for chunk in (7, 256):
        env = BatchedEnv(cfg, 500, device='cuda:0', b_cap=32)
        env.reset()
        res.append(env.play('random', games=3, chunk=chunk))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    assert int(res[0][1].min()) >= 1 and (res[0][0] >= -1).all()
