"""Single-game numpy port of Astro's create/step -- TEST ORACLE / CPU BASELINE.

This is the "reference CPU path" that bench.py times on the GPU box's host
cores (the reference itself cannot travel there).  It restates
astro/core.py's ``create`` (core.py:86-135) and ``step`` (core.py:215-303)
for ONE game on reference-shaped ``State`` tuples with small numpy arrays,
so its per-tick cost has the reference's shape (a few dozen numpy calls on
arrays of <= ~40 rows).  numpy's own dtype promotion reproduces the
reference's float32-at-tick-0 / float64-after behaviour, and
tests/test_oracle_golden.py pins it bit for bit against the golden
transitions.  Not imported by the product package.
"""
import collections
import itertools as it
import time

import numpy as np

Bodies = collections.namedtuple('Bodies', ('x', 'dx', 'b'))
State = collections.namedtuple('State', ('ships', 'planets', 'bullets', 'reload', 't'))


def _unit(angle):
    """(sin, cos) in float32 -- util.direction (util.py:87-92)."""
    return np.stack((np.sin(angle, dtype=np.float32), np.cos(angle, dtype=np.float32)), axis=-1)


def _field(planet_x, at, gm):
    """Planet gravity at points ``at`` (core.py:138-153)."""
    rel = planet_x[np.newaxis, :, :] - at[:, np.newaxis, :]
    inv = gm / np.maximum(1e-12, (rel ** 2).sum(axis=2))
    return (inv[:, :, np.newaxis] * rel).sum(axis=1)


def _move(x, dx, acc, dt):
    ndx = dx + acc * dt
    return x + dt * ndx, ndx


class Game:
    """Precomputed per-config constants + create/step for one game."""

    def __init__(self, config):
        self.c = config
        self.gm = config.gravity * config.planet_mass
        self.ns = 1 if config.solo else 2

    def create(self, seed=None):
        c = self.c
        rs = np.random.RandomState(c.seed if seed is None else seed)
        n = rs.randint(1, c.max_planets + 1)
        outer = c.outer_ship_position * np.sign(rs.rand(2).astype(np.float32) - 0.5)
        inner = c.inner_ship_position * _unit(2 * np.pi * rs.rand())
        if n == 1:
            ships = outer[np.newaxis] if c.solo else np.stack((outer, -outer))
        elif c.solo:
            ships = (outer if rs.rand() < 0.5 else inner)[np.newaxis]
        else:
            pick = rs.rand() < 0.5
            ships = np.stack((outer, inner) if pick else (inner, outer))
        b = 2 * np.pi * rs.rand(ships.shape[0]).astype(np.float32)
        if n == 1:
            px = np.zeros((1, 2), dtype=np.float32)
            pdx = np.zeros_like(px)
        else:
            ang = 2 * np.pi * rs.rand() + np.linspace(0, 2 * np.pi, num=n, endpoint=False)
            turn = rs.choice((-1, 1))
            px = c.planet_orbit * _unit(ang)
            pdx = np.sqrt(c.gravity * c.planet_mass * (n - 1) / 2) * _unit(ang + turn * np.pi / 2)
        empty = np.zeros((0, 2), dtype=np.float32)
        return State(ships=Bodies(ships, np.zeros_like(ships), b),
                     planets=Bodies(px, pdx, None),
                     bullets=Bodies(empty, empty.copy(), None), reload=0.0, t=0.0)

    def step(self, state, control):
        c = self.c
        sh, pl, bu = state.ships, state.planets, state.bullets
        heading = _unit(sh.b)
        acc = c.ship_thrust * (control % 2)[:, np.newaxis] * heading + _field(pl.x, sh.x, self.gm)
        turn = c.dt * c.ship_rspeed * ((control // 2) - 1)
        ns, npl, nb = sh.x.shape[0], pl.x.shape[0], bu.x.shape[0]
        pos = np.concatenate((sh.x, pl.x, bu.x))
        rad = np.concatenate((np.repeat(c.ship_radius, ns), np.repeat(c.planet_radius, npl),
                              np.zeros(nb)))
        d2 = ((pos[np.newaxis] - pos[:, np.newaxis]) ** 2).sum(axis=2)
        hit = ((d2 < (rad[np.newaxis] + rad[:, np.newaxis]) ** 2) & ~np.eye(len(rad), dtype=bool)).any(1)
        if hit[:ns].any():
            return None, 1 - 2 * hit[:ns]
        if c.max_time <= state.t + c.dt:
            return None, np.full(ns, 1 if c.solo else 0, dtype=np.float32)
        reload = state.reload + c.dt
        keep = ~hit[ns + npl:]
        bx, bdx = bu.x[keep], bu.dx[keep]
        if c.reload_time <= reload:
            bx = np.concatenate([bx, sh.x + 1.001 * c.ship_radius * heading])
            bdx = np.concatenate([bdx, sh.dx + c.bullet_speed * heading])
            reload -= c.reload_time
        sx, sdx = _move(sh.x, sh.dx, acc, c.dt)
        px, pdx = _move(pl.x, pl.dx, _field(pl.x, pl.x, self.gm), c.dt)
        nbx, nbdx = _move(bx, bdx, 0, c.dt)
        inside = ((-1 <= nbx) & (nbx <= 1)).any(axis=1)
        wrap = lambda v: ((v + 1) % 2) - 1  # noqa: E731
        nxt = State(ships=Bodies(wrap(sx), sdx, sh.b + turn),
                    planets=Bodies(wrap(px), pdx, None),
                    bullets=Bodies(nbx[inside], nbdx[inside], None),
                    reload=reload, t=state.t + c.dt)
        return nxt, np.zeros(ns, dtype=np.float32)


def run_for(config, seconds, seed=0, planets_only=0):
    """Random-action games with re-create on termination (each new game from
    the next config of generate_configs, filtered to ``planets_only``-planet
    games when set, as BatchedEnv(planets_only=...)) for about ``seconds``;
    returns (env-steps, elapsed)."""
    g = Game(config)
    rng = np.random.RandomState(seed)
    stream = np.random.RandomState(config.seed + seed)   # generate_configs stream

    class _Seeds:
        @staticmethod
        def randint(hi):
            while True:
                s = stream.randint(hi)
                if not planets_only or np.random.RandomState(s).randint(1, config.max_planets + 1) == planets_only:
                    return s
    seeds = _Seeds
    state = g.create(seeds.randint(1 << 30))
    steps = 0
    t0 = time.perf_counter()
    end = t0 + seconds
    for _ in it.count():
        ctl = rng.randint(0, 6, size=g.ns)
        state, _ = g.step(state, ctl)
        steps += 1
        if state is None:
            state = g.create(seeds.randint(1 << 30))
        if (steps & 255) == 0 and time.perf_counter() >= end:
            break
    return steps, time.perf_counter() - t0
