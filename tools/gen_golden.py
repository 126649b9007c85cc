#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ by running the REFERENCE.

Test infrastructure only.  This script imports DouglasOrr/Astro's own
``astro/core.py`` / ``astro/util.py`` / ``astro/script.py`` from
``/root/reference`` (read-only, via a synthetic package so that
``astro/__init__.py``'s imports of ``rl``/``server`` -- which need the absent
``tensorboardX``/``lru`` -- are skipped) and records inputs and outputs of
``core.create`` (core.py:86-135), ``core.generate_configs`` (core.py:77-83) and
``core.step`` (core.py:215-303), and ``rl.ValueNetwork.get_features`` /
``to_batch`` (rl.py:36-112), as small ``.npz``/``.json`` fixtures.

It refuses to run when ``/root/reference`` is absent, so it never runs on the
GPU box; the fixtures it writes are plain data (inputs + expected outputs) and
are committed.  Nothing here is imported by the product package.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tools/gen_golden.py
"""
import itertools as it
import json
import os
import sys
import types

import numpy as np

REF = '/root/reference/astro'
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'tests', 'golden')
P_PAD = 8          # planet padding used by every fixture
S_PAD = 2          # ship padding


def _import_reference():
    if not os.path.isdir(REF):
        sys.exit('gen_golden: /root/reference is absent -- this script only '
                 'runs in the build container')
    sys.dont_write_bytecode = True
    pkg = types.ModuleType('astro')
    pkg.__path__ = [REF]
    sys.modules['astro'] = pkg
    from astro import core, util, script  # noqa: E402
    return core, util, script


core, util, script = _import_reference()

# Named configurations exercised by the fixtures (all derived from the
# reference presets, core.py:52-74).
CONFIGS = {
    'default': core.DEFAULT_CONFIG,
    'solo': core.SOLO_CONFIG,
    'solo_easy': core.SOLO_EASY_CONFIG,
    'mp8': core.DEFAULT_CONFIG._replace(max_planets=8),
    'mp3': core.DEFAULT_CONFIG._replace(max_planets=3),    # masked rejection
    'mp6_solo': core.SOLO_CONFIG._replace(max_planets=6),  # rejection + solo
    'rapid': core.DEFAULT_CONFIG._replace(reload_time=0.01),  # fires at tick 0
    'short': core.DEFAULT_CONFIG._replace(max_time=3.0, reload_time=0.05),
    'solo20': core.SOLO_CONFIG._replace(max_time=20),
}


def cfg_json():
    return {k: dict(v._asdict()) for k, v in CONFIGS.items()}


# ---------------------------------------------------------------------------
# State <-> padded arrays

def pack_state(state, nships):
    """Reference State -> padded float64 arrays + counts + dtype flags."""
    ships = np.zeros((S_PAD, 5))
    ships[:nships, 0:2] = state.ships.x
    ships[:nships, 2:4] = state.ships.dx
    ships[:nships, 4] = state.ships.b
    npl = state.planets.x.shape[0]
    planets = np.zeros((P_PAD, 4))
    planets[:npl, 0:2] = state.planets.x
    planets[:npl, 2:4] = state.planets.dx
    bullets = np.concatenate([state.bullets.x, state.bullets.dx], axis=1).astype(np.float64)
    flags = (int(state.ships.x.dtype == np.float32) |
             int(state.planets.x.dtype == np.float32) << 1 |
             int(state.planets.dx.dtype == np.float32) << 2 |
             int(state.bullets.x.dtype == np.float32) << 3)
    return ships, planets, npl, bullets, flags


def round_state(state):
    """Round every array of a State to float32 VALUES, keeping its dtype.

    This is the state a float32-storing implementation hands to step(): the
    reference's own promotion path (core.py:234-303) is kept because each
    array keeps its numpy dtype."""
    def r(a):
        return None if a is None else a.astype(np.float32).astype(a.dtype)
    B = core.Bodies
    return core.State(
        ships=B(x=r(state.ships.x), dx=r(state.ships.dx), b=r(state.ships.b)),
        planets=B(x=r(state.planets.x), dx=r(state.planets.dx), b=None),
        bullets=B(x=r(state.bullets.x), dx=r(state.bullets.dx), b=None),
        reload=state.reload, t=state.t)


class TransitionWriter:
    """Ragged store of teacher-forced (state_in, control) -> ref outputs."""

    def __init__(self):
        self.rows = []

    def add(self, cfg_name, tick, state_in, control, config):
        nships = state_in.ships.x.shape[0]
        out_state, reward = core.step(state_in, np.asarray(control), config)
        ships, planets, npl, bullets, flags = pack_state(state_in, nships)
        if out_state is None:
            done = 1 if reward.dtype.kind == 'i' else 2
            o_ships = np.zeros((S_PAD, 5))
            o_planets = np.zeros((P_PAD, 4))
            o_bullets = np.zeros((0, 4))
        else:
            done = 0
            o_ships, o_planets, _, o_bullets, _ = pack_state(out_state, nships)
        rew = np.zeros(S_PAD)
        rew[:nships] = reward
        ctl = np.full(S_PAD, 2, dtype=np.int64)
        ctl[:nships] = control
        self.rows.append(dict(
            cfg=list(CONFIGS).index(cfg_name), tick=tick, nships=nships,
            nplanets=npl, flags=flags, ships=ships, planets=planets,
            bullets=bullets, control=ctl, done=done, reward=rew,
            reward_int=int(reward.dtype.kind == 'i'),
            o_ships=o_ships, o_planets=o_planets, o_bullets=o_bullets))
        return out_state, reward

    def save(self, path):
        R = self.rows

        def ragged(key):
            arrs = [r[key] for r in R]
            off = np.zeros(len(arrs) + 1, dtype=np.int64)
            off[1:] = np.cumsum([a.shape[0] for a in arrs])
            flat = np.concatenate(arrs, axis=0) if arrs else np.zeros((0, 4))
            return flat, off
        bi, bio = ragged('bullets')
        bo, boo = ragged('o_bullets')
        np.savez_compressed(
            path,
            cfg=np.array([r['cfg'] for r in R], dtype=np.int32),
            tick=np.array([r['tick'] for r in R], dtype=np.int32),
            nships=np.array([r['nships'] for r in R], dtype=np.int32),
            nplanets=np.array([r['nplanets'] for r in R], dtype=np.int32),
            dtype_flags=np.array([r['flags'] for r in R], dtype=np.int32),
            in_ships=np.stack([r['ships'] for r in R]),
            in_planets=np.stack([r['planets'] for r in R]),
            in_bullets=bi, in_bullets_off=bio,
            control=np.stack([r['control'] for r in R]),
            out_done=np.array([r['done'] for r in R], dtype=np.int8),
            out_reward=np.stack([r['reward'] for r in R]),
            out_reward_int=np.array([r['reward_int'] for r in R], dtype=np.int8),
            out_ships=np.stack([r['o_ships'] for r in R]),
            out_planets=np.stack([r['o_planets'] for r in R]),
            out_bullets=bo, out_bullets_off=boo,
            cfg_names=np.array(list(CONFIGS)),
        )
        print('wrote', path, len(R), 'transitions')


# ---------------------------------------------------------------------------
# 1. create() + generate_configs()

def gen_create(k=256):
    out = {}
    for name, base in CONFIGS.items():
        configs = list(it.islice(core.generate_configs(base), k))
        seeds = np.array([c.seed for c in configs], dtype=np.uint32)
        npl = np.zeros(k, dtype=np.int32)
        sx = np.zeros((k, S_PAD, 2), np.float32)
        sdx = np.zeros((k, S_PAD, 2), np.float32)
        sb = np.zeros((k, S_PAD), np.float32)
        px = np.zeros((k, P_PAD, 2), np.float32)
        pdx = np.zeros((k, P_PAD, 2), np.float64)
        for i, c in enumerate(configs):
            s = core.create(c)
            n = s.ships.x.shape[0]
            assert s.ships.x.dtype == np.float32 and s.ships.b.dtype == np.float32
            npl[i] = s.planets.x.shape[0]
            sx[i, :n] = s.ships.x
            sdx[i, :n] = s.ships.dx
            sb[i, :n] = s.ships.b
            px[i, :npl[i]] = s.planets.x
            pdx[i, :npl[i]] = s.planets.dx
        for key, val in dict(seed=seeds, nplanets=npl, ships_x=sx, ships_dx=sdx,
                             ships_b=sb, planets_x=px, planets_dx=pdx).items():
            out['%s__%s' % (name, key)] = val
    np.savez_compressed(os.path.join(OUT, 'create.npz'), **out)
    print('wrote create.npz')

    gc = {}
    for seed in [42, 0, 1, 7, 123456789, (1 << 30) - 1, (1 << 32) - 1]:
        c = core.DEFAULT_CONFIG._replace(seed=seed)
        gc['seed_%d' % seed] = np.array(
            [x.seed for x in it.islice(core.generate_configs(c), 300)], dtype=np.uint32)
    np.savez_compressed(os.path.join(OUT, 'generate_configs.npz'), **gc)
    print('wrote generate_configs.npz')


# ---------------------------------------------------------------------------
# 2. Teacher-forced step transitions along reference games

def _controls(policy, rng, nships, state, bots):
    if policy == 'random':
        return rng.randint(0, 6, size=nships)
    if policy == 'nothing':
        return np.full(nships, 2)
    if policy == 'spin_fwd':
        return np.full(nships, 5)
    if policy == 'left_fwd':
        return np.full(nships, 1)
    if policy == 'script':
        return core.Bots.control(bots, state)
    raise ValueError(policy)


def gen_steps():
    w = TransitionWriter()
    plan = [
        # (config, policy, games, keep_every)
        ('default', 'random', 24, 1),
        ('default', 'nothing', 6, 2),
        ('default', 'script', 4, 3),
        ('solo', 'random', 6, 1),
        ('solo_easy', 'nothing', 2, 4),
        ('mp8', 'random', 16, 1),
        ('mp3', 'random', 6, 1),
        ('mp6_solo', 'spin_fwd', 4, 2),
        ('rapid', 'random', 6, 1),
        ('rapid', 'left_fwd', 3, 1),
        ('short', 'random', 8, 1),
        ('solo20', 'script', 2, 25),
    ]
    for cfg_name, policy, games, keep in plan:
        base = CONFIGS[cfg_name]
        for g, config in enumerate(it.islice(core.generate_configs(base), games)):
            rng = np.random.RandomState(1000 + g)
            nships = 1 if config.solo else 2
            bots = [script.ScriptBot.create(config) for _ in range(nships)]
            state = core.create(config)
            tick = 0
            while state is not None:
                ctl = _controls(policy, rng, nships, state, bots)
                nb_before = state.bullets.x.shape[0]
                # free-running reference step decides the trajectory
                nxt, reward = core.step(state, ctl, config)
                interesting = (tick == 0 or nxt is None or
                               (nxt is not None and nxt.bullets.x.shape[0] != nb_before))
                if interesting or tick % keep == 0:
                    w.add(cfg_name, tick, round_state(state), ctl, config)
                state = nxt
                tick += 1
    w.save(os.path.join(OUT, 'steps.npz'))


# ---------------------------------------------------------------------------
# 3. Hand-built edge cases through the reference step

def _mk(ships_x, ships_dx, ships_b, planets_x, planets_dx, bullets_x=(), bullets_dx=(),
        reload=0.0, t=0.0):
    f = lambda a, n: np.asarray(a, dtype=np.float64).reshape(n)  # noqa: E731
    B = core.Bodies
    nb = len(bullets_x)
    return core.State(
        ships=B(x=f(ships_x, (-1, 2)), dx=f(ships_dx, (-1, 2)), b=f(ships_b, (-1,))),
        planets=B(x=f(planets_x, (-1, 2)), dx=f(planets_dx, (-1, 2)), b=None),
        bullets=B(x=f(bullets_x, (nb, 2)), dx=f(bullets_dx, (nb, 2)), b=None),
        reload=reload, t=t)


def gen_edges():
    w = TransitionWriter()
    c = CONFIGS['default']
    solo = CONFIGS['solo']
    far = [[0.6, 0.6], [-0.6, -0.6]]
    still = [[0, 0], [0, 0]]
    cases = [
        # (name, config, state, control, tick)
        ('cull_quirk_kept', c, _mk(far, still, [0, 1], [[0, 0]], [[0, 0]],
                                   [[0.999, 0.0], [0.999, 0.999], [1.5, 0.0], [1.5, 1.5]],
                                   [[1, 0], [1, 1], [1, 0], [1, 1]]), [2, 2], 5),
        ('bullet_in_planet', c, _mk(far, still, [0, 1], [[0, 0]], [[0, 0]],
                                    [[0.19, 0.0], [0.0, -0.2], [0.3, 0.3]],
                                    [[0, 0], [0, 0], [0, 0]]), [2, 2], 5),
        ('coincident_bullets', c, _mk(far, still, [0, 1], [[0, 0]], [[0, 0]],
                                      [[0.4, 0.4], [0.4, 0.4]], [[0, 0.1], [0, 0.1]]), [2, 2], 5),
        ('planet_overlap_not_terminal', c, _mk(far, still, [0, 1],
                                               [[0.1, 0], [-0.1, 0]], [[0, 0.1], [0, -0.1]]),
         [2, 2], 5),
        ('ship_ship', c, _mk([[0.6, 0.6], [0.62, 0.6]], still, [0, 1], [[0, 0]], [[0, 0]]),
         [2, 2], 5),
        ('bullet_hits_ship1', c, _mk([[0.6, 0.6], [-0.6, -0.6]], still, [0, 1], [[0, 0]], [[0, 0]],
                                     [[-0.6, -0.61]], [[0, 1.5]]), [2, 2], 5),
        ('bullet_hits_ship0', c, _mk([[0.6, 0.6], [-0.6, -0.6]], still, [0, 1], [[0, 0]], [[0, 0]],
                                     [[0.6, 0.6249]], [[0, 1.5]]), [2, 2], 5),
        ('wrap_x', c, _mk([[0.999, 0.2], [-0.999, -0.2]], [[1, 0], [-1, 0]], [0, 1],
                          [[0, 0]], [[0, 0]]), [2, 2], 5),
        ('wrap_corner', c, _mk([[0.9999, -0.9999], [-0.5, 0.5]], [[1, -1], [0, 0]], [1, 2],
                               [[0, 0]], [[0, 0]]), [3, 0], 5),
        ('gravity_1_over_r', c, _mk([[0.1, 0.0], [0.0, 0.3]], still, [0, 0], [[0, 0]], [[0, 0]]),
         [2, 2], 5),
        ('thrust_rotate_all_controls_a', c, _mk(far, [[0.1, -0.2], [0.3, 0.05]], [0.3, 2.0],
                                                [[0, 0]], [[0, 0]]), [0, 1], 5),
        ('thrust_rotate_all_controls_b', c, _mk(far, [[0.1, -0.2], [0.3, 0.05]], [-40.0, 123.0],
                                                [[0, 0]], [[0, 0]]), [4, 5], 5),
        ('negative_and_large_controls', c, _mk(far, still, [0.5, 1.0], [[0, 0]], [[0, 0]]),
         [-1, 7], 5),
        ('fire_geometry', c, _mk([[0.6, 0.6], [-0.6, -0.6]], [[0.1, 0], [0, -0.1]], [0.7, 4.0],
                                 [[0, 0]], [[0, 0]], reload=0.29), [3, 3], 14),
        ('timeout_plain', c, _mk(far, still, [0, 1], [[0, 0]], [[0, 0]], t=59.98000000000378),
         [2, 2], 2999),
        ('timeout_solo_win', solo, _mk([[0.6, 0.6]], [[0, 0]], [0], [[0, 0]], [[0, 0]],
                                       t=59.98000000000378), [2], 2999),
        ('collision_beats_timeout', c, _mk([[0.6, 0.6], [-0.6, -0.6]], still, [0, 1],
                                           [[0, 0]], [[0, 0]], [[-0.6, -0.6]], [[0, 0]],
                                           t=59.98000000000378), [2, 2], 2999),
        ('planets_8', CONFIGS['mp8'], _mk(far, [[0.05, 0], [0, 0.05]], [0, 1],
                                          [[0.5 * np.sin(a), 0.5 * np.cos(a)] for a in
                                           np.linspace(0, 2 * np.pi, 8, endpoint=False) + 0.1],
                                          [[0.3 * np.cos(a), -0.3 * np.sin(a)] for a in
                                           np.linspace(0, 2 * np.pi, 8, endpoint=False) + 0.1]),
         [1, 5], 5),
        ('ship_in_planet_1e12_floor', c, _mk([[0.0, 0.0], [-0.6, -0.6]], still, [0, 1],
                                             [[0, 0], [0.5, 0]], [[0, 0], [0, 0]]), [2, 2], 5),
    ]
    names = []
    for name, cfg, state, ctl, tick in cases:
        cfg_name = [k for k, v in CONFIGS.items() if v == cfg][0]
        w.add(cfg_name, tick, round_state(state), ctl, cfg)
        names.append(name)
    w.save(os.path.join(OUT, 'edge_steps.npz'))
    with open(os.path.join(OUT, 'edge_steps_names.json'), 'w') as f:
        json.dump(names, f, indent=1)


# ---------------------------------------------------------------------------
# 4. Free-running open-loop games (exact float64 trajectories)

def gen_games():
    """Whole games under open-loop controls: the full float64 ship trajectory,
    bullet counts, outcome.  A float64-storing implementation must reproduce
    these bit for bit; a float32-storing one statistically."""
    out = {}
    index = []
    plan = [('default', 'random', 24), ('default', 'nothing', 8), ('solo', 'random', 8),
            ('mp8', 'random', 12), ('rapid', 'random', 4), ('short', 'random', 6),
            ('solo_easy', 'nothing', 2)]
    gid = 0
    for cfg_name, policy, games in plan:
        base = CONFIGS[cfg_name]
        for g, config in enumerate(it.islice(core.generate_configs(base), 100, 100 + games)):
            nships = 1 if config.solo else 2
            rng = np.random.RandomState(5000 + gid)
            tmax = int(round(config.max_time / config.dt)) + 2
            if policy == 'random':
                ctl = rng.randint(0, 6, size=(tmax, nships))
            else:
                ctl = np.full((tmax, nships), 2)
            state = core.create(config)
            ships, nbul, planets = [], [], []
            tick = 0
            while True:
                sp, pp, _, _, _ = pack_state(state, nships)
                ships.append(sp)
                planets.append(pp)
                nbul.append(state.bullets.x.shape[0])
                state, reward = core.step(state, ctl[tick], config)
                tick += 1
                if state is None:
                    break
            rew = np.zeros(2)
            rew[:nships] = reward
            key = 'g%03d' % gid
            out[key + '__seed'] = np.uint32(config.seed)
            out[key + '__controls'] = ctl[:tick].astype(np.int8)
            out[key + '__ships'] = np.stack(ships)
            out[key + '__planets'] = np.stack(planets)
            out[key + '__nbullets'] = np.array(nbul, dtype=np.int32)
            out[key + '__reward'] = rew
            winner = None if np.max(reward) < 1 else int(np.argmax(reward))
            index.append(dict(gid=gid, cfg=cfg_name, policy=policy, seed=int(config.seed),
                              ticks=tick, winner=winner,
                              done=1 if reward.dtype.kind == 'i' else 2))
            gid += 1
    np.savez_compressed(os.path.join(OUT, 'games.npz'), **out)
    with open(os.path.join(OUT, 'games.json'), 'w') as f:
        json.dump(index, f, indent=0)
    print('wrote games.npz', gid, 'games')


# ---------------------------------------------------------------------------
# 5. Fire / timeout schedule, measured through the reference step

def gen_schedule():
    """Fire ticks and the timeout tick of several configs, observed from the
    reference step itself (a solo ship parked far from a massless planet, so
    nothing ever collides): fire <=> the bullet count grows."""
    sched = {}
    variants = {
        'default': {}, 'rapid': dict(reload_time=0.01), 'r005': dict(reload_time=0.05),
        'r007': dict(reload_time=0.07), 'r02': dict(reload_time=0.2),
        'short': dict(max_time=3.0, reload_time=0.05), 'mt1': dict(max_time=1.0),
        'dt003': dict(dt=0.03, max_time=7.0, reload_time=0.1),
        'never': dict(reload_time=1000.0, max_time=5.0),
    }
    for name, kw in variants.items():
        cfg = core.DEFAULT_CONFIG._replace(solo=True, planet_mass=0.0, **kw)
        B = core.Bodies
        state = core.State(
            ships=B(x=np.array([[0.9, 0.9]]), dx=np.zeros((1, 2)), b=np.array([0.785])),
            planets=B(x=np.zeros((1, 2)), dx=np.zeros((1, 2)), b=None),
            bullets=B(x=np.zeros((0, 2)), dx=np.zeros((0, 2)), b=None), reload=0.0, t=0.0)
        fires, tick = [], 0
        reloads, ts = [], []
        while True:
            nb = state.bullets.x.shape[0]
            reloads.append(state.reload)
            ts.append(state.t)
            nxt, reward = core.step(state, np.array([2]), cfg)
            if nxt is None:
                break
            # fire <=> reload was decremented by reload_time (core.py:263,280)
            new = nxt.reload != state.reload + cfg.dt
            if new:
                fires.append(tick)
            state = nxt
            tick += 1
        sched[name] = dict(config=dict(cfg._asdict()), fire_ticks=fires, timeout_tick=tick,
                           reload=reloads[:50], t=ts[:50], t_last=ts[-1])
    with open(os.path.join(OUT, 'schedule.json'), 'w') as f:
        json.dump(sched, f)
    print('wrote schedule.json')


# ---------------------------------------------------------------------------
# 6. Known-answer tests from the reference's own tests, as data

def gen_kats():
    kat = {}
    x = np.array([[0, 0], [1.9, 1.9], [3.8, 1.9], [3.8, 0.0]])
    r = np.array([1, 1, 2, 0])
    kat['collisions'] = dict(x=x.tolist(), r=r.tolist(),
                             out=core._collisions(x, r).tolist())  # test_core.py:6-17
    b = np.arange(0, 2 * np.pi + 1e-3, np.pi / 2)
    kat['direction'] = dict(b=b.tolist(), out=util.direction(b).tolist())  # test_util.py:59-64
    w = np.array([[1.01, -0.95], [0.95, -1.01]])
    kat['wrap_unit_square'] = dict(x=w.tolist(), out=util.wrap_unit_square(w).tolist())
    rng = np.random.RandomState(3)
    wx = np.concatenate([rng.uniform(-3, 3, 200), [-1, 1, -3, 3, 0, -1e-17, 1 - 1e-16, -1 + 1e-17]])
    kat['wrap_random'] = dict(x=wx.tolist(), out=util.wrap_unit_square(wx).tolist())
    bb = np.concatenate([rng.uniform(-300, 300, 2000), np.arange(-20, 20, 0.125)]).astype(np.float32)
    dd = util.direction(bb)
    kat['direction_f32'] = dict(b=bb.astype(np.float64).tolist(),
                                out_bits=dd.view(np.uint32).tolist())
    with open(os.path.join(OUT, 'kat.json'), 'w') as f:
        json.dump(kat, f)
    print('wrote kat.json')


# ---------------------------------------------------------------------------
# 6. Observation features: rl.ValueNetwork.get_features / to_batch
#    (rl.py:36-112) of every input state of steps.npz

def _import_rl():
    """astro/rl.py imports tensorboardX at module level for its training
    logger; it is absent here and unused by get_features/to_batch, so an empty
    placeholder module is registered before the import (nothing of rl.py's
    feature code is touched)."""
    sys.modules.setdefault('tensorboardX', types.ModuleType('tensorboardX'))
    from astro import rl  # noqa: E402
    return rl


def gen_features():
    rl = _import_rl()
    z = np.load(os.path.join(OUT, 'steps.npz'))
    names = list(z['cfg_names'])
    feats, rows, dims = [], [], []
    for i in range(z['tick'].shape[0]):
        S = int(z['nships'][i])
        npl = int(z['nplanets'][i])
        fl = int(z['dtype_flags'][i])
        sh = z['in_ships'][i, :S]
        pl = z['in_planets'][i, :npl]
        off = z['in_bullets_off']
        bl = z['in_bullets'][off[i]:off[i + 1]]
        f32 = np.float32
        sdt = f32 if fl & 1 else np.float64
        B = core.Bodies
        state = core.State(
            ships=B(x=sh[:, 0:2].astype(sdt), dx=sh[:, 2:4].astype(sdt), b=sh[:, 4].astype(sdt)),
            planets=B(x=pl[:, 0:2].astype(f32 if fl & 2 else np.float64),
                      dx=pl[:, 2:4].astype(f32 if fl & 4 else np.float64), b=None),
            bullets=B(x=bl[:, 0:2].astype(f32 if fl & 8 else np.float64),
                      dx=bl[:, 2:4].astype(f32 if fl & 8 else np.float64), b=None),
            reload=0.0, t=0.0)
        f = rl.ValueNetwork.get_features(state)
        assert f.dtype == np.float32
        feats.append(f)
        rows.append(f.shape[0])
        dims.append(f.shape[1])
    off = np.zeros(len(rows) + 1, dtype=np.int64)
    off[1:] = np.cumsum(rows)
    flat = np.zeros((int(off[-1]), 15), dtype=np.float32)
    for i, f in enumerate(feats):
        flat[off[i]:off[i + 1], :f.shape[1]] = f
    # to_batch of a few groups of same-ship-count states (ragged rows -> -1 padding)
    groups, batches = [], []
    for name in ('default', 'solo', 'rapid'):
        idx = [i for i in range(len(rows)) if names[z['cfg'][i]] == name][:40:5]
        b = rl.ValueNetwork.to_batch([feats[i] for i in idx])
        groups.append(np.array(idx, dtype=np.int64))
        batches.append(b)
    np.savez_compressed(os.path.join(OUT, 'features.npz'), features=flat, features_off=off,
                        dims=np.array(dims, dtype=np.int32),
                        **{'batch_idx_%d' % k: g for k, g in enumerate(groups)},
                        **{'batch_%d' % k: b for k, b in enumerate(batches)})
    print('wrote features.npz', len(rows), 'states', int(off[-1]), 'rows')


# ---------------------------------------------------------------------------
# 7. A game log written by the reference (core.save_log, core.py:413-426)

def gen_log():
    config = CONFIGS['short']
    game = core.play(config, [script.NothingBot(), script.NothingBot()])
    import gzip
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, 'log.jsonl')
        core.save_log(path, game)
        data = open(path, 'rb').read()
    with gzip.GzipFile(os.path.join(OUT, 'log_short_nothing.jsonl.gz'), 'wb', mtime=0) as f:
        f.write(data)
    print('wrote log_short_nothing.jsonl.gz', len(game.ticks), 'ticks, winner', game.winner)


# ---------------------------------------------------------------------------
# 8. ScriptBot decisions (script.py:13-83) on every input state of steps.npz,
#    for each ship's ego view (core.roll_ships, core.py:306-327)

def gen_script_controls():
    z = np.load(os.path.join(OUT, 'steps.npz'))
    names = list(z['cfg_names'])
    out = np.full((z['tick'].shape[0], S_PAD), -1, dtype=np.int8)
    bots = {}
    for i in range(z['tick'].shape[0]):
        name = names[z['cfg'][i]]
        config = CONFIGS[name]
        if name not in bots:
            bots[name] = script.ScriptBot.create(config)
        S = int(z['nships'][i])
        npl = int(z['nplanets'][i])
        fl = int(z['dtype_flags'][i])
        sh = z['in_ships'][i, :S]
        pl = z['in_planets'][i, :npl]
        off = z['in_bullets_off']
        bl = z['in_bullets'][off[i]:off[i + 1]]
        f32 = np.float32
        sdt = f32 if fl & 1 else np.float64
        B = core.Bodies
        state = core.State(
            ships=B(x=sh[:, 0:2].astype(sdt), dx=sh[:, 2:4].astype(sdt), b=sh[:, 4].astype(sdt)),
            planets=B(x=pl[:, 0:2].astype(f32 if fl & 2 else np.float64),
                      dx=pl[:, 2:4].astype(f32 if fl & 4 else np.float64), b=None),
            bullets=B(x=bl[:, 0:2].astype(f32 if fl & 8 else np.float64),
                      dx=bl[:, 2:4].astype(f32 if fl & 8 else np.float64), b=None),
            reload=0.0, t=0.0)
        for k in range(S):
            out[i, k] = bots[name](core.roll_ships(state, k))
    np.savez_compressed(os.path.join(OUT, 'script_controls.npz'), control=out)
    print('wrote script_controls.npz', out.shape[0], 'states')


# ---------------------------------------------------------------------------
# 9. BASELINE.json config 1: DEFAULT_CONFIG (seed 42), 1000 ticks of
#    RandomState(0).randint(0, 6, (1000, 2)) controls, re-created on done

def gen_config1():
    config = core.DEFAULT_CONFIG
    ctl = np.random.RandomState(0).randint(0, 6, (1000, 2))
    state = core.create(config)
    ships, planets, npl, bl, boff, rew, done, gtick = [], [], [], [], [0], [], [], []
    g = 0
    for t in range(1000):
        sp, pp, n, b, _ = pack_state(state, 2)
        ships.append(sp)
        planets.append(pp)
        npl.append(n)
        bl.append(b)
        boff.append(boff[-1] + b.shape[0])
        gtick.append(g)
        state, reward = core.step(state, ctl[t], config)
        rew.append(np.asarray(reward, np.float64))
        if state is None:
            done.append(1 if reward.dtype.kind == 'i' else 2)
            state = core.create(config)
            g = 0
        else:
            done.append(0)
            g += 1
    np.savez_compressed(os.path.join(OUT, 'config1.npz'), control=ctl.astype(np.int8),
                        ships=np.stack(ships), planets=np.stack(planets), nplanets=np.array(npl, np.int32),
                        bullets=np.concatenate(bl).reshape(-1, 4), bullets_off=np.array(boff, np.int64),
                        reward=np.stack(rew), done=np.array(done, np.int8), game_tick=np.array(gtick, np.int32))
    print('wrote config1.npz', int(np.sum(np.array(done) > 0)), 'games ended')


# ---------------------------------------------------------------------------
# 10. Whole games to the end under the reference's own bots (core.play):
#     test_script's invariants (test/test_core.py:88-98, max_time=20) and
#     games that reach the full 3000-tick timeout (core.py:257-260)

def _record_play(key, config, bots, out, index, extra):
    game = core.play(config, bots)
    nships = 1 if config.solo else 2
    ctl = np.stack([t.control for t in game.ticks]).astype(np.int8)
    ships = np.stack([pack_state(t.state, nships)[0] for t in game.ticks])
    nbul = np.array([t.state.bullets.x.shape[0] for t in game.ticks], np.int32)
    reward = game.ticks[-1].reward
    rew = np.zeros(2)
    rew[:nships] = reward
    out[key + '__controls'] = ctl
    out[key + '__ships'] = ships
    out[key + '__nbullets'] = nbul
    out[key + '__reward'] = rew
    index.append(dict(key=key, config=dict(config._asdict()), ticks=len(game.ticks), winner=game.winner,
                      done=1 if reward.dtype.kind == 'i' else 2, **extra))
    return game


def gen_long_games():
    out, index = {}, {}
    rows = []
    # test_script (test_core.py:88-98)
    for k, config in enumerate(it.islice(core.generate_configs(core.SOLO_CONFIG._replace(max_time=20)), 3)):
        _record_play('script_solo%d' % k, config, [script.ScriptBot.create(config)], out, rows,
                     dict(bots=['script']))
    for k, config in enumerate(it.islice(core.generate_configs(core.DEFAULT_CONFIG._replace(max_time=20)), 3)):
        _record_play('nothing_script%d' % k, config, [script.NothingBot(), script.ScriptBot.create(config)],
                     out, rows, dict(bots=['nothing', 'script']))
    # a full-length game: the first SOLO game ScriptBot survives to the
    # 3000-tick timeout (no 1v1 ScriptBot game of the first 40 DEFAULT_CONFIG
    # configs lasts that long)
    for name, base, mk in [('solo_timeout', core.SOLO_CONFIG, lambda c: [script.ScriptBot.create(c)])]:
        for config in it.islice(core.generate_configs(base), 40):
            game = core.play(config, mk(config))
            if len(game.ticks) == 3000:
                _record_play(name, config, mk(config), out, rows,
                             dict(bots=['script'] * (1 if config.solo else 2)))
                break
        else:
            print('no', name, 'game found')
    index = rows
    np.savez_compressed(os.path.join(OUT, 'long_games.npz'), **out)
    with open(os.path.join(OUT, 'long_games.json'), 'w') as f:
        json.dump(index, f, indent=0)
    print('wrote long_games.npz', [(r['key'], r['ticks'], r['winner']) for r in index])


def main():
    if sys.argv[1:] == ['config1']:
        gen_config1()
        return
    if sys.argv[1:] == ['long']:
        gen_long_games()
        return
    if sys.argv[1:] == ['script']:
        gen_script_controls()
        return
    if sys.argv[1:] == ['features']:
        gen_features()
        return
    if sys.argv[1:] == ['log']:
        gen_log()
        return
    os.makedirs(OUT, exist_ok=True)
    np.random.seed(0)
    with open(os.path.join(OUT, 'configs.json'), 'w') as f:
        json.dump(dict(configs=cfg_json(), numpy=np.__version__), f, indent=1)
    gen_kats()
    gen_schedule()
    gen_create()
    gen_edges()
    gen_steps()
    gen_games()
    gen_features()
    gen_log()
    gen_script_controls()
    gen_config1()
    gen_long_games()


if __name__ == '__main__':
    main()
