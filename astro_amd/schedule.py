"""Host-side reduction of a Config to the kernel's POD parameters.

The reference keeps ``t`` and ``reload`` as float64 Python scalars and
decides timeout and firing from them each step (core.py:257, 263, 267, 280,
301-302).  Both depend only on how many steps a game has taken, so the host
replays that exact float64 recurrence once per Config and hands the kernel a
per-tick fire bitmask plus the timeout tick; the kernel keeps an int32 tick
per env instead of two float64s.  The same tables give back the exact
``t``/``reload`` of any tick for reference-shaped State exports.
"""
import math
from dataclasses import dataclass

import numpy as np

TICK_LIMIT = (1 << 22) - 1   # tick shares hdr word 0 with 10 bits of chain progress


@dataclass
class Schedule:
    fire: np.ndarray        # bool[timeout_tick]: fire on step call k
    timeout_tick: int       # first k with max_time <= t_k + dt
    t: np.ndarray           # float64[timeout_tick + 1]: t before step call k
    reload: np.ndarray      # float64[timeout_tick + 1]: reload before step call k

    def fire_bits(self):
        """uint32 words, bit (k & 31) of word k >> 5 = fire on tick k."""
        n = max(1, (self.timeout_tick + 31) // 32)
        words = np.zeros(n, dtype=np.uint64)
        k = np.nonzero(self.fire)[0]
        np.bitwise_or.at(words, k >> 5, np.left_shift(np.uint64(1), (k & 31).astype(np.uint64)))
        return words.astype(np.uint32)


def build(config):
    """Replay core.step's float64 t/reload bookkeeping (core.py:257-302)."""
    dt = config.dt
    t = 0.0
    reload = 0.0
    fire, ts, rs = [], [], []
    for k in range(TICK_LIMIT):
        ts.append(t)
        rs.append(reload)
        if config.max_time <= t + dt:
            return Schedule(np.array(fire, dtype=bool), k, np.array(ts), np.array(rs))
        nxt = reload + dt
        f = config.reload_time <= nxt
        if f:
            nxt -= config.reload_time
        fire.append(f)
        reload = nxt
        t = t + dt
    raise ValueError('max_time / dt exceeds %d ticks' % TICK_LIMIT)


def kernel_constants(config):
    """The float64/float32 constants exactly as the reference evaluates them."""
    rs, rp = float(config.ship_radius), float(config.planet_radius)
    r = np.array([rs, rp, 0.0], dtype=np.float64)   # np.repeat(...) radii, core.py:248-251
    return dict(
        gm=config.gravity * config.planet_mass,       # core.py:151
        dt=float(config.dt),
        db=config.dt * config.ship_rspeed,            # core.py:239
        thrust=float(config.ship_thrust),
        r2_ss=float((r[0] + r[0]) ** 2),              # core.py:211
        r2_sp=float((r[0] + r[1]) ** 2),
        r2_s0=float((r[0] + r[2]) ** 2),
        r2_p0=float((r[1] + r[2]) ** 2),
        gravity=float(config.gravity),
        planet_mass=float(config.planet_mass),
        spawn_off=float(np.float32(1.001 * config.ship_radius)),   # core.py:273
        bullet_speed=float(np.float32(config.bullet_speed)),      # core.py:277
        timeout_reward=1.0 if config.solo else 0.0,               # core.py:260
        outer_pos=float(np.float32(config.outer_ship_position)),  # core.py:93
        inner_pos=float(np.float32(config.inner_ship_position)),  # core.py:95
        planet_orbit=float(np.float32(config.planet_orbit)),      # core.py:119
        nships=1 if config.solo else 2,
        solo=1 if config.solo else 0,
        max_planets=int(config.max_planets),
    )


def check_config(config):
    if int(config.max_planets) != config.max_planets or config.max_planets < 1:
        raise ValueError('max_planets must be a positive integer')
    if config.max_planets > 16:
        raise ValueError('max_planets > 16 is not supported (planet slots are registers)')
    if not math.isfinite(config.dt) or config.dt <= 0:
        raise ValueError('dt must be positive')
