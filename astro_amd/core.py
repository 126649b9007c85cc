"""Drop-in single-game surface: ``create``/``step``/``roll_ships``/``play``.

Same names, arguments, return values and dtypes as astro/core.py
(create :86-135, step :215-303, roll_ships :306-327, Bots :359-374,
play :377-410), so astro/server.py (``game_start``/``game_tick``) and
astro/rl.py (``core.play`` rollouts) can call this module instead.  Every
call runs the HIP kernel on a one-env float64 BatchedEnv, which reproduces
the reference bit for bit (tests/test_gpu_parity.py): inputs are never
mutated, a finished game returns ``(None, reward)`` with an int64 reward for
a collision and a float32 reward for a timeout.

This path is latency-bound by design: by default (``ASTRO_SHIM=mapped``) the
game lives in host-mapped memory the kernel addresses directly and a tick is
one ``astro_game_step`` C call -- the State packed (in C, ``_gamestep``), one
one-wave launch on the caller's current stream, a busy-wait on the
completion word the wave stores after its last store, the next State built
(~18.7 us per core.step on MI355X); ``ASTRO_SHIM=copy``
moves a packed device arena with one H2D and one D2H copy per tick.  Bulk
simulation belongs on :class:`astro_amd.env.BatchedEnv`.
"""
import ctypes
import os
import threading

import numpy as np
import torch

from . import _lib
from .config import (Bodies, Config, DEFAULT_CONFIG, Game, SOLO_CONFIG,  # noqa: F401
                     SOLO_EASY_CONFIG, State, Tick, generate_configs, nships)
from .env import BatchedEnv

try:   # core.step's packing around astro_game_step in C (built by __graft_entry__.build)
    from . import _gamestep
except ImportError:   # the same tick with the packing in Python (_step_mapped)
    _gamestep = None
# ASTRO_SHIM_PY=1: the Python packing even when the helper is built (tests of both)
if os.environ.get('ASTRO_SHIM_PY') == '1':
    _gamestep = None

class _ShimCache(dict):
    """(config without seed, device) -> _Shim.  Emptying it also drops the
    per-tick fast path (_LAST), so a cleared shim is never used again."""

    def clear(self):
        global _LAST
        _LAST = (None, None, None, None)
        super().clear()

    def __delitem__(self, key):
        global _LAST
        _LAST = (None, None, None, None)
        super().__delitem__(key)

    def pop(self, *a):
        global _LAST
        _LAST = (None, None, None, None)
        return super().pop(*a)

    def popitem(self):
        global _LAST
        _LAST = (None, None, None, None)
        return super().popitem()


_ENVS = _ShimCache()


def clear_shims():
    """Drop every single-game shim (their arenas are freed with them)."""
    _ENVS.clear()


def _device():
    return torch.device('cuda', torch.cuda.current_device())


class _Arena:
    """The arrays of one game packed (16-byte aligned) into one buffer, with
    numpy views for the host and device addresses for AstroState.  mode
    'copy': a device buffer mirrored by a pinned host buffer (one H2D copy
    of a tick's input, one D2H copy back); mode 'mapped': page-locked host
    memory the kernels address directly (astro_host_alloc; no copies, every
    kernel access crosses PCIe)."""

    def __init__(self, lib, specs, device, mode):
        self.lib, self.mode = lib, mode
        self.layout = {}
        off = 0
        for name, shape, dt in specs:
            nbytes = int(np.prod(shape)) * np.dtype(dt).itemsize
            self.layout[name] = (off, shape, dt, nbytes)
            off = (off + nbytes + 15) // 16 * 16
        self.nbytes = off
        self.host = None
        if mode == 'mapped':
            h, d = ctypes.c_void_p(), ctypes.c_void_p()
            _lib.check(lib.astro_host_alloc(off, ctypes.byref(h), ctypes.byref(d)), 'astro_host_alloc')
            self.host, self.device = h.value, d.value
            raw = np.frombuffer((ctypes.c_uint8 * off).from_address(self.host), dtype=np.uint8)
        else:
            self.dev = torch.zeros(off, dtype=torch.uint8, device=device)
            self.pinned = torch.zeros(off, dtype=torch.uint8).pin_memory()
            self.device = self.dev.data_ptr()
            raw = self.pinned.numpy()
        raw[:] = 0
        self.views = {n: raw[o:o + nb].view(dt).reshape(shape) for n, (o, shape, dt, nb) in self.layout.items()}

    def ptr(self, name):
        return self.device + self.layout[name][0]

    def end(self, name):
        o, _, _, nb = self.layout[name]
        return o + nb

    def push(self, upto):
        """copy mode: host bytes [0, upto) to the device (stream-ordered)."""
        if self.mode == 'copy':
            self.dev[:upto].copy_(self.pinned[:upto], non_blocking=True)

    def pull(self):
        """copy mode: every byte back to the host (stream-ordered)."""
        if self.mode == 'copy':
            self.pinned.copy_(self.dev, non_blocking=True)

    def __del__(self):
        if getattr(self, 'host', None):
            self.lib.astro_host_free(ctypes.c_void_p(self.host))
            self.host = None


# The single-game arena: 'mapped' (default) = the game's arrays in host
# memory the kernel addresses directly, a tick is one astro_game_step call
# (launch + completion-word wait); ASTRO_SHIM=copy = a device arena with one
# packed H2D and one packed D2H copy per tick.  Measured on MI355X (bench.py
# `single_game`, round 5): mapped 18.7 us per core.step, copy 38 us (DESIGN.md
# section 10)
SHIM_MODE = os.environ.get('ASTRO_SHIM', 'mapped')
# the step kernel of the one-env game (every kernel gives the same results)
SHIM_KERNEL = os.environ.get('ASTRO_SHIM_KERNEL', 'auto')


class _Shim:
    """One float64 game on the device for the single-game surface: its
    arrays packed in one buffer (_Arena), a tick = the input written into
    the host view, one launch (mapped; copy mode: between one H2D and one D2H
    copy of the packed arena), one wait for an event (busy-polled: a blocking
    synchronisation wakes ~10-30 us late)."""

    def __init__(self, config, b_cap, device, mode=None):
        self.mode = mode or SHIM_MODE
        self.env = env = BatchedEnv(config, 1, device=device, b_cap=b_cap, dtype=torch.float64,
                                    auto_reset=False, use_key_table=False, kernel=SHIM_KERNEL)
        # one tick at a time: the arena is this game's input and output, and
        # in mapped mode the kernel reads it while it runs (a server's
        # request threads may call step concurrently)
        self.lock = threading.Lock()
        S, P = env.S, env.p_pad
        f8, i4 = np.float64, np.int32
        self.arena = a = _Arena(env.lib, (
            ('hdr', (1, 4), i4), ('ships', (S, 1, 4), f8), ('ships_b', (S, 1), f8), ('planets', (P, 1, 4), f8),
            ('bullets', (1, b_cap, 4), f8), ('control', (1, S), np.int8), ('fire', (2,), i4), ('seed', (1,), np.uint32),
            ('reward', (1, S), np.float32), ('done', (1,), np.uint8), ('errors', (1,), np.uint32),
            ('flag', (1,), np.uint32)),
            env.device, self.mode)
        self.in_bytes = a.end('seed')   # hdr .. seed: a tick's input
        self.event = torch.cuda.Event()
        self.h = a.views
        # the env's own state record with its arrays moved to the arena (its
        # seed stream and schedule stay the BatchedEnv's)
        st = env.state
        self.state = type(st)(ships=a.ptr('ships'), ships_b=a.ptr('ships_b'), planets=a.ptr('planets'),
                              bullets=a.ptr('bullets'), hdr=a.ptr('hdr'), stream=st.stream,
                              stream_ring=st.stream_ring, n_env=1, state_f64=1, errors=a.ptr('errors'))
        # the launch's schedule per (first tick of a game?, times out?):
        # fire word = arena 'fire', timeout tick so `timeout` holds this call
        self.params = {}
        for tick in (0, 1):
            for to in (False, True):
                p = type(env.params).from_buffer_copy(env.params)
                p.timeout_tick = tick if to else tick + 1
                p.fire_bits = a.ptr('fire')
                self.params[tick, to] = p
        # mapped mode: a whole tick is one astro_game_step call (pack, launch,
        # wait, unpack in C); the packed state goes in through `inbuf` and
        # comes back through `outbuf` (float64, the State arrays in order)
        self.tick = None
        if a.mode == 'mapped':
            n_max = 5 * S + 4 * P + 4 * b_cap
            self.inbuf = np.zeros(n_max)
            self.outbuf = np.zeros(n_max)
            t = _lib.AstroGameTick()
            t.params = env.params
            t.state = self.state
            for f in ('hdr', 'ships', 'ships_b', 'planets', 'bullets', 'control', 'fire', 'reward', 'done', 'errors'):
                setattr(t, f, a.host + a.layout[f][0])
            t.control_dev, t.fire_dev = a.ptr('control'), a.ptr('fire')
            t.reward_dev, t.done_dev = a.ptr('reward'), a.ptr('done')
            # the tick's completion word (astro_game_step waits on it)
            t.flag, t.flag_dev = a.host + a.layout['flag'][0], a.ptr('flag')
            t.in_ = self.inbuf.__array_interface__['data'][0]
            t.out = self.outbuf.__array_interface__['data'][0]
            # the caller's current stream, refreshed on every tick (step)
            self.dev_index = env.device.index if env.device.index is not None else torch.cuda.current_device()
            t.stream = _raw_stream(self.dev_index)
            self.tick = t
            self.tick_ptr = ctypes.addressof(t)
            self.game_step = env.lib.astro_game_step
            self.game_step_addr = ctypes.cast(self.game_step, ctypes.c_void_p).value

    def stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.env.device).cuda_stream)

    def sync(self):
        """Results back to the host view; wait for them (busy-poll)."""
        self.arena.pull()
        ev = self.event
        ev.record(torch.cuda.current_stream(self.env.device))
        while not ev.query():
            pass
        bits = int(self.h['errors'][0])
        if bits:
            self.h['errors'][0] = 0
            self.arena.push(self.arena.end('errors'))
            why = '; '.join(m for b, m in sorted(_lib.ERRORS.items()) if bits & b) or 'unknown'
            raise _lib.AstroError('astro_step reported device error 0x%x: %s' % (bits, why))

    def create(self, seed):
        self.h['seed'][0] = seed
        self.arena.push(self.in_bytes)
        _lib.check(self.env.lib.astro_reset(ctypes.byref(self.env.params), ctypes.byref(self.state),
                                            self.arena.ptr('seed'), None, self.stream()), 'astro_reset')
        self.sync()

    def state_of(self):
        """Reference-shaped State from the mapped arrays."""
        h = self.h
        hdr = h['hdr'].view(np.uint32)
        host = dict(ships=h['ships'].transpose(1, 0, 2), ships_b=h['ships_b'].transpose(1, 0),
                    planets=h['planets'].transpose(1, 0, 2), bullets=h['bullets'],
                    tick=hdr[:, 0] & 0x3fffff, nplanets=hdr[:, 1] & 0xff, nbullets=(hdr[:, 1] >> 16) & 0xffff,
                    flags=(hdr[:, 1] >> 8) & 0xff)
        return self.env.state_of(0, host)


# (config, device index, shim, the _ENVS dict it lives in) of the last call:
# the per-tick fast path (one tuple, read and replaced whole: thread-safe)
_LAST = (None, None, None, None)
_SHIM_LOCK = threading.Lock()


# device index -> the current hipStream_t (~0.1 us; torch's public path as a fallback)
_raw_stream = getattr(torch._C, '_cuda_getCurrentRawStream', None) or (
    lambda d: torch.cuda.current_stream(d).cuda_stream)


def _shim(config, bullets_needed):
    global _LAST
    dev = torch.cuda.current_device()
    cfg, ldev, sh, envs = _LAST
    if (cfg is config and ldev == dev and envs is _ENVS and envs and sh.env.b_cap >= bullets_needed
            and sh.mode == SHIM_MODE):
        return sh
    key = (config._replace(seed=0), torch.device('cuda', dev))
    with _SHIM_LOCK:   # (two request threads meeting a new config build one shim)
        sh = _ENVS.get(key)
        if sh is None or sh.env.b_cap < bullets_needed or sh.mode != SHIM_MODE:
            cap = 64 if sh is None else max(64, sh.env.b_cap)
            while cap < bullets_needed:
                cap *= 2
            sh = _Shim(config, cap, key[1])
            _ENVS[key] = sh
        _LAST = (config, dev, sh, _ENVS)
    return sh


def create(config):
    """Create a new game state from ``config.seed`` (core.create)."""
    seed = int(config.seed)
    if not 0 <= seed < 1 << 32:   # as np.random.RandomState(seed) (core.py:89) refuses it
        raise ValueError('Seed must be between 0 and 2**32 - 1')
    sh = _shim(config, 0)
    with sh.lock:
        sh.create(seed)
        return sh.state_of()


def step(state, control, config):
    """Advance one game by one tick (core.step).  Returns (State or None,
    reward array[nships])."""
    S = 1 if config.solo else 2
    if len(control) != S or np.ndim(control) != 1:
        raise ValueError('control must have shape (%d,)' % S)
    c0 = int(control[0])
    c1 = int(control[1]) if S == 2 else 0
    if not (-128 <= c0 <= 127 and -128 <= c1 <= 127):
        raise ValueError('control codes must fit int8')
    nb = state.bullets.x.shape[0]
    sh = _shim(config, nb + S)
    with sh.lock:
        if sh.tick is not None:
            # (each tick on the caller's current stream, as BatchedEnv's calls)
            sh.tick.stream = _raw_stream(sh.dev_index)
            if _gamestep is not None:   # packing, the C call and the next State in C
                r = _gamestep.step(sh.tick_ptr, sh.game_step_addr, state, c0, c1, config.dt, config.reload_time,
                                   config.max_time, State, Bodies)
                if r is not NotImplemented:
                    if isinstance(r, int):
                        _lib.check(r, 'astro_game_step')
                    return r
            return _step_mapped(sh, state, c0, c1, config, S, nb)
        return _step(sh, state, np.array([c0, c1][:S]), config, S, nb)


def _step_mapped(sh, state, c0, c1, config, S, nb):
    """One tick through astro_game_step: the state packed into the shim's
    input buffer, then pack / launch / wait / unpack in one C call."""
    ships, planets, bullets = state.ships, state.planets, state.bullets
    npl = planets.x.shape[0]
    if npl > sh.env.p_pad:
        raise ValueError('a state holds more planets than max_planets')
    fresh = ships.x.dtype == np.float32      # create()'s float32 arrays
    n_in = 5 * S + 4 * (npl + nb)
    np.concatenate((ships.x, ships.dx, ships.b, planets.x, planets.dx, bullets.x, bullets.dx), axis=None,
                   out=sh.inbuf[:n_in])
    # the reference's float64 bookkeeping for THIS call (core.py:257,263,267)
    t = sh.tick
    t.nplanets, t.nbullets, t.control0, t.control1 = npl, nb, c0, c1
    t.first_step = fresh
    t.fire_now = config.reload_time <= state.reload + config.dt
    t.timeout_now = config.max_time <= state.t + config.dt
    rc = sh.game_step(sh.tick_ptr)
    if rc != 0:
        _lib.check(rc, 'astro_game_step')
    done = t.done_out
    if done:
        reward = np.array(t.reward_out[:S], dtype=np.float32)
        return None, (reward.astype(np.int64) if done == 1 else reward)
    nb2 = t.out_nbullets
    o = sh.outbuf[:5 * S + 4 * (npl + nb2)].copy()
    p0, b0 = 5 * S, 5 * S + 4 * npl
    sx = o[0:2 * S].reshape(S, 2)
    sdx = o[2 * S:4 * S].reshape(S, 2)
    px = o[p0:p0 + 2 * npl].reshape(npl, 2)
    pdx = o[p0 + 2 * npl:b0].reshape(npl, 2)
    bx = o[b0:b0 + 2 * nb2].reshape(nb2, 2)
    bdx = o[b0 + 2 * nb2:b0 + 4 * nb2].reshape(nb2, 2)
    if npl == 1:              # a lone planet's arrays stay float32
        px, pdx = px.astype(np.float32), pdx.astype(np.float32)
    if fresh:                 # tick-0 bullets are float32
        bx, bdx = bx.astype(np.float32), bdx.astype(np.float32)
    reload = state.reload + config.dt
    if t.fire_now:
        reload -= config.reload_time
    new = State(ships=Bodies(x=sx, dx=sdx, b=o[4 * S:5 * S]), planets=Bodies(x=px, dx=pdx, b=None),
                bullets=Bodies(x=bx, dx=bdx, b=None), reload=reload, t=state.t + config.dt)
    return new, np.zeros(S, dtype=np.float32)


def _step(sh, state, control, config, S, nb):
    env, h = sh.env, sh.h
    # the reference's float64 bookkeeping for THIS call (core.py:257,263,267)
    timeout = config.max_time <= state.t + config.dt
    fire = config.reload_time <= state.reload + config.dt
    fresh = state.ships.x.dtype == np.float32      # create()'s float32 arrays
    tick = 0 if fresh else 1
    npl = state.planets.x.shape[0]
    if npl > env.p_pad:
        raise ValueError('a state holds more planets than max_planets')
    # the input, written straight into the memory the kernel reads
    hdr = h['hdr'].view(np.uint32)
    hdr[0, 0] = (int(hdr[0, 0]) & ~0x3fffff & 0xffffffff) | tick
    hdr[0, 1] = npl | (nb << 16)
    sx = h['ships']
    sx[:, 0, 0:2] = state.ships.x
    sx[:, 0, 2:4] = state.ships.dx
    h['ships_b'][:, 0] = state.ships.b
    h['planets'][:npl, 0, 0:2] = state.planets.x
    h['planets'][:npl, 0, 2:4] = state.planets.dx
    if nb:
        h['bullets'][0, :nb, 0:2] = state.bullets.x
        h['bullets'][0, :nb, 2:4] = state.bullets.dx
    h['control'][0] = control
    h['fire'][0] = int(fire) << tick
    a = sh.arena
    a.push(sh.in_bytes)
    rc = env.lib.astro_step(ctypes.byref(sh.params[tick, bool(timeout)]), ctypes.byref(sh.state), a.ptr('control'),
                            a.ptr('reward'), a.ptr('done'), None, 0, sh.stream())
    if rc != 0:
        _lib.check(rc, 'astro_step')
    sh.sync()
    done = int(h['done'][0])
    reward = h['reward'][0].copy()
    if done == 1:
        return None, reward.astype(np.int64)
    if done == 2:
        return None, reward.astype(np.float32)
    # the next state straight from the returned arrays (float64 after a step;
    # a lone planet's arrays stay float32; tick-0 bullets are float32)
    reload = state.reload + config.dt
    if fire:
        reload -= config.reload_time
    bdt = np.float32 if fresh else np.float64
    pdt = np.float32 if npl == 1 else np.float64
    nb2 = int(hdr[0, 1]) >> 16
    sv, pl, bl = h['ships'][:, 0], h['planets'][:npl, 0], h['bullets'][0, :nb2]
    new = State(
        ships=Bodies(x=sv[:, 0:2].copy(), dx=sv[:, 2:4].copy(), b=h['ships_b'][:, 0].copy()),
        planets=Bodies(x=pl[:, 0:2].astype(pdt), dx=pl[:, 2:4].astype(pdt), b=None),
        bullets=Bodies(x=bl[:, 0:2].astype(bdt), dx=bl[:, 2:4].astype(bdt), b=None),
        reload=reload, t=state.t + config.dt)
    return new, np.zeros(S, dtype=np.float32)


def roll_ships(state, index):
    """Ego view: rotate the ship arrays so ship ``index`` comes first
    (core.roll_ships); planets, bullets, reload and t are shared."""
    if state is None:
        return None
    s = state.ships
    return state._replace(ships=Bodies(x=np.roll(s.x, -index, 0), dx=np.roll(s.dx, -index, 0),
                                       b=np.roll(s.b, -index, 0)))


def roll_ships_batched(ships, index):
    """roll_ships for a BatchedEnv observation tensor [N, S, ...]."""
    return torch.roll(ships, -index, dims=1)


class Bot:
    """Bot protocol of core.Bot (core.py:330-356)."""

    def __call__(self, state):
        raise NotImplementedError

    def reward(self, state, reward):
        pass

    @property
    def data(self):
        return None


class Bots:
    """Per-tick bot fan-out of core.Bots (core.py:359-374)."""

    @staticmethod
    def control(bots, state):
        return np.array([bot(roll_ships(state, i)) for i, bot in enumerate(bots)])

    @staticmethod
    def reward(bots, state, reward):
        for i, bot in enumerate(bots):
            if hasattr(bot, 'reward'):
                bot.reward(roll_ships(state, i), reward[i])

    @staticmethod
    def data(bots):
        return [getattr(bot, 'data', None) for bot in bots]


def play(config, bots):
    """Play one game to the end (core.play): returns Game(config, winner, ticks)."""
    ticks = []
    state = create(config)
    while True:
        control = Bots.control(bots, state)
        prev = state
        state, reward = step(state, control, config)
        Bots.reward(bots, state, reward)
        ticks.append(Tick(state=prev, control=control, reward=reward, bot_data=Bots.data(bots)))
        if state is None:
            winner = None if np.max(reward) < 1 else int(np.argmax(reward))
            return Game(config=config, winner=winner, ticks=ticks)
