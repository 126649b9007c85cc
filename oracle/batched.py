"""Batched struct-of-arrays restatement of Astro's physics -- TEST ORACLE ONLY.

Restates, over N independent games held in padded arrays, exactly what the
reference computes for ONE game in

* ``step``            astro/core.py:215-303 (+ helpers _gravity :138-153,
                      _mask :156-168, _update_bodies :171-197, _collisions
                      :200-212, util.direction util.py:87-92,
                      util.wrap_unit_square util.py:145-148)
* ``create``          astro/core.py:86-135
* ``generate_configs``astro/core.py:77-83
* the float64 ``t``/``reload`` bookkeeping of core.py:257,263,280,301-302,
  as a per-tick fire/timeout schedule

including the reference's numpy dtype behaviour (numpy 2.x promotion): the
arrays ``create`` returns are float32 (planet velocities float64 when there
are >= 2 planets), so the first ``step`` of a game evaluates gravity and
collision distances in float32; every later step runs in float64.  A
one-planet game keeps its planet arrays float32 for ever.  Tick 0 is detected
from the env's tick counter, exactly as the HIP kernel does.

State values are float64 arrays; ``store='f32'`` rounds every stored value to
float32 after each step (the HIP kernel's float32 state), ``store='f64'``
keeps them (the kernel's float64 state).  Pinned against the reference's own
outputs by tests/test_oracle_golden.py.
"""
import math
from dataclasses import dataclass

import numpy as np

from . import mt19937
from .npsincos import cos32, sin32

F32 = np.float32
F64 = np.float64


# ---------------------------------------------------------------------------
# Config-derived constants and the fire/timeout schedule

@dataclass
class Params:
    config: object
    nships: int
    gm: float          # gravity * planet_mass, Python float (core.py:151)
    db: float          # dt * ship_rspeed (core.py:239)
    r2_ss: float       # (r_ship + r_ship)**2   (core.py:211)
    r2_sp: float       # (r_ship + r_planet)**2
    r2_s0: float       # (r_ship + 0)**2  ship <-> bullet
    r2_p0: float       # (r_planet + 0)**2 planet <-> bullet
    spawn_off: np.float32      # float32(1.001 * ship_radius)  (core.py:273)
    bullet_speed: np.float32   # float32(bullet_speed)         (core.py:277)
    timeout_reward: float
    fire: np.ndarray           # bool[timeout_tick]
    timeout_tick: int


def schedule(config, limit=1 << 24):
    """Fire ticks and timeout tick from the reference's float64 recurrence.

    Step call k (state after k ticks) times out iff max_time <= t_k + dt
    (core.py:257); otherwise reload_{k+1} = reload_k + dt, fire iff
    reload_time <= reload_{k+1}, then reload_{k+1} -= reload_time
    (core.py:263,267,280); t_{k+1} = t_k + dt (core.py:302)."""
    t = 0.0
    reload = 0.0
    fire = []
    ts, reloads = [], []
    for k in range(limit):
        ts.append(t)
        reloads.append(reload)
        if config.max_time <= t + config.dt:
            return np.array(fire, dtype=bool), k, np.array(ts), np.array(reloads)
        nxt = reload + config.dt
        f = config.reload_time <= nxt
        if f:
            nxt -= config.reload_time
        fire.append(f)
        reload = nxt
        t = t + config.dt
    raise ValueError('max_time / dt exceeds the schedule limit')


def make_params(config):
    rs, rp = config.ship_radius, config.planet_radius
    r = np.array([rs, rp, 0.0], dtype=F64)
    fire, tt, _, _ = schedule(config)
    return Params(
        config=config,
        nships=1 if config.solo else 2,
        gm=config.gravity * config.planet_mass,
        db=config.dt * config.ship_rspeed,
        r2_ss=float((r[0] + r[0]) ** 2),
        r2_sp=float((r[0] + r[1]) ** 2),
        r2_s0=float((r[0] + r[2]) ** 2),
        r2_p0=float((r[1] + r[2]) ** 2),
        spawn_off=F32(1.001 * rs),
        bullet_speed=F32(config.bullet_speed),
        timeout_reward=1.0 if config.solo else 0.0,
        fire=fire, timeout_tick=tt)


# ---------------------------------------------------------------------------
# Batched state

@dataclass
class Batch:
    tick: np.ndarray       # int32[N]
    nplanets: np.ndarray   # int32[N]
    nbullets: np.ndarray   # int32[N]
    ships: np.ndarray      # f64[N, S, 4]  x, y, dx, dy
    ships_b: np.ndarray    # f64[N, S]
    planets: np.ndarray    # f64[N, Pp, 4]
    bullets: np.ndarray    # f64[N, Bc, 4]
    overflow: np.ndarray   # bool[N] (sticky: a bullet was dropped for lack of room)

    @staticmethod
    def zeros(n, nships, p_pad, b_cap):
        return Batch(np.zeros(n, np.int32), np.zeros(n, np.int32), np.zeros(n, np.int32),
                     np.zeros((n, nships, 4)), np.zeros((n, nships)),
                     np.zeros((n, p_pad, 4)), np.zeros((n, b_cap, 4)), np.zeros(n, bool))

    def copy(self):
        return Batch(*(getattr(self, f).copy() for f in self.__dataclass_fields__))

    def take(self, idx):
        return Batch(*(getattr(self, f)[idx] for f in self.__dataclass_fields__))

    def put(self, idx, other):
        for f in self.__dataclass_fields__:
            getattr(self, f)[idx] = getattr(other, f)


def _gravity(T, gm, px, py, valid, x, y):
    """Field of the valid planets at K points per env, in dtype T.
    px, py: [N, P]; valid: [N, P]; x, y: [N, K] -> ax, ay [N, K].
    Summed over planets in index order (numpy's axis=1 reduction)."""
    px, py, x, y = (np.asarray(a).astype(T) for a in (px, py, x, y))
    rx = px[:, None, :] - x[:, :, None]
    ry = py[:, None, :] - y[:, :, None]
    d2 = rx * rx + ry * ry
    f = T(gm) / np.maximum(T(1e-12), d2)
    tx, ty = f * rx, f * ry
    ax = np.zeros(x.shape, T)
    ay = np.zeros(x.shape, T)
    first = np.ones(x.shape, bool)
    for j in range(px.shape[1]):
        v = valid[:, j][:, None]
        ax = np.where(v, np.where(first, tx[..., j], ax + tx[..., j]), ax)
        ay = np.where(v, np.where(first, ty[..., j], ay + ty[..., j]), ay)
        first = first & ~v
    return ax, ay


def _wrap(T, v):
    """util.wrap_unit_square in dtype T: ((v + 1) % 2) - 1, numpy floored mod."""
    v = np.asarray(v).astype(T)
    return np.remainder(v + T(1), T(2)) - T(1)


def _d2(T, ax, ay, bx, by):
    dx = np.asarray(ax).astype(T) - np.asarray(bx).astype(T)
    dy = np.asarray(ay).astype(T) - np.asarray(by).astype(T)
    return (dx * dx + dy * dy).astype(F64)


def _floor_divmod2(c):
    c = np.asarray(c, dtype=np.int64)
    return c // 2, c % 2


def step(st, control, P, store='f32'):
    """One tick for every env of ``st``.  Returns (new Batch, reward f32[N,S],
    done u8[N]) with done = 0 running, 1 ship collision, 2 timeout.  Envs that
    finish keep their input state (the caller resets them)."""
    N, S = st.ships.shape[:2]
    Pp, Bc = st.planets.shape[1], st.bullets.shape[1]
    t0 = st.tick == 0
    T0 = t0[:, None]
    pvalid = np.arange(Pp)[None, :] < st.nplanets[:, None]
    bvalid = np.arange(Bc)[None, :] < st.nbullets[:, None]
    sx, sy, sdx, sdy = (st.ships[..., i] for i in range(4))
    px, py, pdx, pdy = (st.planets[..., i] for i in range(4))
    bx, by, bdx, bdy = (st.bullets[..., i] for i in range(4))

    # ship acceleration: thrust along util.direction(b) + gravity (core.py:234-237)
    k, m = _floor_divmod2(np.asarray(control)[:, :S])
    b32 = st.ships_b.astype(F32)
    dsin, dcos = sin32(b32), cos32(b32)
    thr = P.config.ship_thrust * m
    gx64, gy64 = _gravity(F64, P.gm, px, py, pvalid, sx, sy)
    gx32, gy32 = _gravity(F32, P.gm, px, py, pvalid, sx, sy)
    ax = thr * dsin.astype(F64) + np.where(T0, gx32.astype(F64), gx64)
    ay = thr * dcos.astype(F64) + np.where(T0, gy32.astype(F64), gy64)
    dbear = P.db * (k - 1)

    # collisions on the old positions (core.py:241-251); only ship and bullet
    # flags are ever read, so only those pairs are evaluated (exact pruning)
    def dist2(a, b_, c, d):
        return np.where(t0.reshape((N,) + (1,) * (np.ndim(a) - 1)),
                        _d2(F32, a, b_, c, d), _d2(F64, a, b_, c, d))
    ship_hit = np.zeros((N, S), bool)
    for s in range(S):
        for o in range(S):
            if o != s:
                ship_hit[:, s] |= dist2(sx[:, s], sy[:, s], sx[:, o], sy[:, o]) < P.r2_ss
        ship_hit[:, s] |= (pvalid & (dist2(sx[:, s:s + 1], sy[:, s:s + 1], px, py) < P.r2_sp)).any(1)
        ship_hit[:, s] |= (bvalid & (dist2(sx[:, s:s + 1], sy[:, s:s + 1], bx, by) < P.r2_s0)).any(1)
    bullet_hit = np.zeros((N, Bc), bool)
    for j in range(Pp):
        bullet_hit |= pvalid[:, j:j + 1] & (dist2(bx, by, px[:, j:j + 1], py[:, j:j + 1]) < P.r2_p0)
    for s in range(S):
        bullet_hit |= dist2(bx, by, sx[:, s:s + 1], sy[:, s:s + 1]) < P.r2_s0

    collided = ship_hit.any(1)
    timeout = ~collided & (st.tick >= P.timeout_tick)
    done = np.where(collided, 1, np.where(timeout, 2, 0)).astype(np.uint8)
    reward = np.where(collided[:, None], np.where(ship_hit, -1.0, 1.0),
                      np.where(timeout[:, None], P.timeout_reward, 0.0)).astype(F32)

    out = st.copy()
    run = done == 0

    # ships: semi-implicit Euler + wrap, always float64 (core.py:283-288)
    ndx = sdx + ax * P.config.dt
    ndy = sdy + ay * P.config.dt
    nx = _wrap(F64, sx + P.config.dt * ndx)
    ny = _wrap(F64, sy + P.config.dt * ndy)
    nb = st.ships_b + dbear

    # planets: self-gravity (core.py:289-294)
    gpx64, gpy64 = _gravity(F64, P.gm, px, py, pvalid, px, py)
    gpx32, gpy32 = _gravity(F32, P.gm, px, py, pvalid, px, py)
    dt32 = F32(P.config.dt)
    qdx = np.where(T0, pdx + (gpx32 * dt32).astype(F64), pdx + gpx64 * P.config.dt)
    qdy = np.where(T0, pdy + (gpy32 * dt32).astype(F64), pdy + gpy64 * P.config.dt)
    qx = _wrap(F64, px + P.config.dt * qdx)
    qy = _wrap(F64, py + P.config.dt * qdy)
    one = (st.nplanets == 1)[:, None]
    # a one-planet game keeps float32 planet arrays: all float32 arithmetic
    p1dx = (pdx.astype(F32) + gpx32 * dt32)
    p1dy = (pdy.astype(F32) + gpy32 * dt32)
    p1x = _wrap(F32, px.astype(F32) + dt32 * p1dx)
    p1y = _wrap(F32, py.astype(F32) + dt32 * p1dy)
    qdx = np.where(one, p1dx.astype(F64), qdx)
    qdy = np.where(one, p1dy.astype(F64), qdy)
    qx = np.where(one, p1x.astype(F64), qx)
    qy = np.where(one, p1y.astype(F64), qy)

    # bullets: survivors in order, then one new bullet per ship (core.py:262-280),
    # then move without gravity and cull when BOTH coords leave [-1, 1]
    # (core.py:295-300, 195); float32 at tick 0, float64 after
    fire = np.zeros(N, bool)
    live = st.tick < P.timeout_tick
    fire[live] = P.fire[st.tick[live]]
    off_s = (P.spawn_off * dsin).astype(F64)
    off_c = (P.spawn_off * dcos).astype(F64)
    vel_s = (P.bullet_speed * dsin).astype(F64)
    vel_c = (P.bullet_speed * dcos).astype(F64)
    nbx = np.where(T0, (sx.astype(F32) + off_s.astype(F32)).astype(F64), sx + off_s)
    nby = np.where(T0, (sy.astype(F32) + off_c.astype(F32)).astype(F64), sy + off_c)
    nbdx = np.where(T0, (sdx.astype(F32) + vel_s.astype(F32)).astype(F64), sdx + vel_s)
    nbdy = np.where(T0, (sdy.astype(F32) + vel_c.astype(F32)).astype(F64), sdy + vel_c)

    cand_x = np.concatenate([bx, nbx], 1)
    cand_y = np.concatenate([by, nby], 1)
    cand_dx = np.concatenate([bdx, nbdx], 1)
    cand_dy = np.concatenate([bdy, nbdy], 1)
    cand_ok = np.concatenate([bvalid & ~bullet_hit, np.repeat(fire[:, None], S, 1)], 1)
    mdx = cand_dx + 0.0
    mdy = cand_dy + 0.0
    mx = cand_x + P.config.dt * mdx
    my = cand_y + P.config.dt * mdy
    mdx32 = cand_dx.astype(F32) + F32(0.0)
    mdy32 = cand_dy.astype(F32) + F32(0.0)
    mx32 = cand_x.astype(F32) + dt32 * mdx32
    my32 = cand_y.astype(F32) + dt32 * mdy32
    inb = (((-1 <= mx) & (mx <= 1)) | ((-1 <= my) & (my <= 1)))
    inb32 = (((-1 <= mx32) & (mx32 <= 1)) | ((-1 <= my32) & (my32 <= 1)))
    keep = cand_ok & np.where(T0, inb32, inb)
    mx = np.where(T0, mx32.astype(F64), mx)
    my = np.where(T0, my32.astype(F64), my)
    mdx = np.where(T0, mdx32.astype(F64), mdx)
    mdy = np.where(T0, mdy32.astype(F64), mdy)

    newb = np.zeros_like(st.bullets)
    nnew = np.zeros(N, np.int32)
    ovf = np.zeros(N, bool)
    for i in np.nonzero(run)[0]:
        sel = np.nonzero(keep[i])[0]
        if sel.size > Bc:
            ovf[i] = True
            sel = sel[:Bc]
        nnew[i] = sel.size
        newb[i, :sel.size] = np.stack([mx[i, sel], my[i, sel], mdx[i, sel], mdy[i, sel]], -1)

    r = run
    out.ships[r] = np.stack([nx, ny, ndx, ndy], -1)[r]
    out.ships_b[r] = nb[r]
    out.planets[r] = np.where(pvalid[..., None], np.stack([qx, qy, qdx, qdy], -1), 0.0)[r]
    out.bullets[r] = newb[r]
    out.nbullets[r] = nnew[r]
    out.overflow[r] |= ovf[r]
    out.tick[r] = st.tick[r] + 1
    if store == 'f32':
        for f in ('ships', 'ships_b', 'planets', 'bullets'):
            a = getattr(out, f)
            a[r] = a[r].astype(F32).astype(F64)
    return out, reward, done


# ---------------------------------------------------------------------------
# create() over a batch of seeds

def create(seeds, P, p_pad, b_cap, store='f32', nwords=96):
    """Fresh games for the given seeds (core.py:86-135), as a Batch."""
    cfg = P.config
    seeds = np.asarray(seeds, dtype=np.uint32)
    W = mt19937.words(seeds, nwords)
    S = P.nships
    out = Batch.zeros(seeds.shape[0], S, p_pad, b_cap)
    two_pi = 2 * np.pi
    for i in range(seeds.shape[0]):
        g = mt19937.Stream(W[i])
        n = g.randint(1, cfg.max_planets + 1)
        u = np.array([g.rand(), g.rand()], dtype=F64).astype(F32)
        outer = F32(cfg.outer_ship_position) * np.sign(u - F32(0.5))
        a = F32(two_pi * g.rand())
        inner = F32(cfg.inner_ship_position) * np.array([sin32(a), cos32(a)], dtype=F32)
        if n == 1 and cfg.solo:
            ships = [outer]
        elif n == 1:
            ships = [outer, -outer]
        elif cfg.solo:
            ships = [outer if g.rand() < 0.5 else inner]
        else:
            ships = [outer, inner] if g.rand() < 0.5 else [inner, outer]
        bs = [F32(two_pi) * F32(g.rand()) for _ in range(S)]
        for s in range(S):
            out.ships[i, s, 0:2] = ships[s]
            out.ships_b[i, s] = bs[s]
        out.nplanets[i] = n
        if n > 1:
            base = two_pi * g.rand()
            step_ = two_pi / n
            orient = base + np.arange(n) * step_
            reverse = -1 if g.randint(0, 2) == 0 else 1
            o32 = orient.astype(F32)
            out.planets[i, :n, 0] = F32(cfg.planet_orbit) * sin32(o32)
            out.planets[i, :n, 1] = F32(cfg.planet_orbit) * cos32(o32)
            amp = math.sqrt(cfg.gravity * cfg.planet_mass * (n - 1) / 2)
            o2 = (orient + reverse * np.pi / 2).astype(F32)
            out.planets[i, :n, 2] = amp * sin32(o2).astype(F64)
            out.planets[i, :n, 3] = amp * cos32(o2).astype(F64)
        if g.pos > nwords:
            raise RuntimeError('create consumed more words than generated')
    if store == 'f32':
        out.planets[:] = out.planets.astype(F32).astype(F64)
    return out


def stream_seeds(base_seed, n_env):
    """Per-env stream seeds: the first n_env configs of
    generate_configs(config) (core.py:77-83) -- env i's games are then
    generate_configs(config._replace(seed=stream_seeds[i]))."""
    return mt19937.generate_config_seeds(base_seed, n_env)


def game_seeds(env_stream_seeds, n_games):
    """[N, n_games] seeds of each env's successive games."""
    w = mt19937.words(env_stream_seeds, n_games).astype(np.uint64)
    return (w & np.uint64((1 << 30) - 1)).astype(np.uint32)


def filtered_game_seeds(env_stream_seeds, n_games, planets, max_planets, draws=200):
    """[N, n_games] seeds of each env's successive games when its
    generate_configs stream is filtered to games of exactly ``planets``
    planets (BatchedEnv(planets_only=...)): create()'s randint(1,
    max_planets + 1) (core.py:90) is the first word of RandomState(seed)
    masked, max_planets a power of two."""
    cand = game_seeds(env_stream_seeds, draws)                       # [N, draws]
    first = mt19937.first_words(cand).reshape(cand.shape)
    n = 1 + (first & np.uint32(max_planets - 1)).astype(np.int64)
    out = np.zeros((len(env_stream_seeds), n_games), np.uint32)
    for i in range(len(env_stream_seeds)):
        ok = cand[i][n[i] == planets]
        assert len(ok) >= n_games, 'increase draws'
        out[i] = ok[:n_games]
    return out


def filtered_game_draws(env_stream_seeds, n_games, planets, max_planets, draws):
    """Like filtered_game_seeds, plus the stream index (0-based draw number
    of RandomState(stream_seed)) each game's seed came from: [N, n_games]
    seeds, [N, n_games] draw indices."""
    cand = game_seeds(env_stream_seeds, draws)
    first = mt19937.first_words(cand).reshape(cand.shape)
    n = 1 + (first & np.uint32(max_planets - 1)).astype(np.int64)
    seeds = np.zeros((len(env_stream_seeds), n_games), np.uint32)
    idx = np.zeros((len(env_stream_seeds), n_games), np.int64)
    for i in range(len(env_stream_seeds)):
        k = np.nonzero(n[i] == planets)[0]
        assert len(k) >= n_games, 'increase draws'
        idx[i] = k[:n_games]
        seeds[i] = cand[i][idx[i]]
    return seeds, idx


def collisions_allpairs(x, r):
    """Generic all-pairs collision mask (core.py:200-212): body i is hit iff
    some other body j has |x_i - x_j|^2 < (r_i + r_j)^2 (strict, self
    excluded).  The step above evaluates only the ship and bullet rows of
    this matrix; tests cross-check the pruning against this full form."""
    x = np.asarray(x)
    r = np.asarray(r)
    d = x[None, :, :] - x[:, None, :]
    d2 = d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]
    rr = r[None, :] + r[:, None]
    hit = d2 < rr * rr
    np.fill_diagonal(hit, False)
    return hit.any(axis=1)
