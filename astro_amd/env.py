"""BatchedEnv: N independent Astro games advanced in lockstep on one GPU.

This is the batched counterpart of the reference's per-game loop
(``core.play``, core.py:377-410 driving ``core.step``/``core.create``):
``reset()`` creates every game, ``step(control)`` advances every game by one
tick and, for games that end, starts the env's next game in the same kernel
(auto-reset).  Env i plays the games of
``generate_configs(config._replace(seed=stream_seed[i]))`` where
``stream_seed`` = the first configs of ``generate_configs(config)``
(core.py:77-83), indexed by GLOBAL env id, so a run sharded over G GPUs
(``env_offset``) plays exactly the games of a 1-GPU run.

All state lives in HBM as PyTorch tensors; ships and planets struct-of-arrays,
entity-major (a wave's lanes read contiguous rows), bullets one contiguous row
per env (the kernels walk an env's live bullets in slot order):

    ships    [S, N, 4]   x, y, dx, dy        ships_b  [S, N]
    planets  [P, N, 4]   x, y, dx, dy        bullets  [N, B, 4]
    hdr      [N, 4]      tick, nplanets | flags << 8 | nbullets << 16,
                         next game's seed | key_valid << 31 (or undrawn << 30: the
                         game's first step draws it), key[397] of its init chain
    stream   [N, 4]      seed-stream cursor + current game's seed
    stream_ring [N, 624] the stream's MT19937 state words (exact for any length)

and every call goes through libastro_hip.so (include/astro_step.h) on the
current torch stream.  There is no CPU path.
"""
import collections
import ctypes
import os

import numpy as np
import torch

from . import _lib
from . import shard as _shard
from .config import Bodies, State, nships as _nships
from . import schedule as _schedule

TICK_MASK = (1 << 22) - 1
MT_N = 624   # MT19937 state words: each env's seed stream keeps its own (stream_ring)

Observation = collections.namedtuple(
    'Observation', ('ships', 'ships_b', 'planets', 'nplanets', 'bullets', 'nbullets', 'tick'))


def _stream_ptr(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


_KEY_TABLES = {}
KEY_TABLE_SEEDS = 1 << 30


def key_table(device):
    """The per-device table of key[397] of MT19937 init_genrand for every
    30-bit seed (4 GiB, built once per process and device in ~0.1 s): it
    turns each game's 397-step seeding chain into one gather."""
    device = torch.device(device)
    key = (device.type, device.index if device.index is not None else torch.cuda.current_device())
    t = _KEY_TABLES.get(key)
    if t is None:
        lib = _lib.load()
        t = torch.empty(KEY_TABLE_SEEDS, dtype=torch.int32, device=device)
        _lib.check(lib.astro_keytable_build(t.data_ptr(), 0, KEY_TABLE_SEEDS, _stream_ptr(device)),
                   'astro_keytable_build')
        _KEY_TABLES[key] = t
    return t


QUAD_MAX_ENVS = 32768   # include/astro_step.h ASTRO_QUAD_MAX_ENVS

_TORCH_TYPESTR = {torch.float32: '<f4', torch.float64: '<f8', torch.int32: '<i4', torch.uint8: '|u1'}


class _DevBlock:
    """One astro_dev_alloc block, seen by torch through the CUDA array
    interface (the tensors keep the block alive; freed with the last)."""

    def __init__(self, lib, shape, dtype, kind):
        self.lib = lib
        n = int(np.prod(shape)) * torch.empty((), dtype=dtype).element_size()
        ptr = ctypes.c_void_p()
        _lib.check(lib.astro_dev_alloc(max(n, 16), kind, ctypes.byref(ptr)), 'astro_dev_alloc')
        self.ptr = ptr.value
        self.__cuda_array_interface__ = dict(shape=tuple(int(x) for x in shape), typestr=_TORCH_TYPESTR[dtype],
                                             data=(self.ptr, False), version=2, strides=None)

    def __del__(self):
        if getattr(self, 'ptr', None):
            self.lib.astro_dev_free(ctypes.c_void_p(self.ptr))
            self.ptr = None


def _dev_tensor(lib, shape, dtype, device, kind):
    """A zeroed device tensor in memory of the given ASTRO_MEM_* kind."""
    if kind == _lib.MEM['default'] or 0 in shape:
        return torch.zeros(shape, dtype=dtype, device=device)
    with torch.cuda.device(device):
        t = torch.as_tensor(_DevBlock(lib, shape, dtype, kind), device=device)
    if t.data_ptr() == 0 or tuple(t.shape) != tuple(shape) or t.dtype != dtype:
        raise RuntimeError('astro_dev_alloc block not seen as a %s %s tensor' % (dtype, tuple(shape)))
    return t


class BatchedEnv:
    """N lockstep games of one Config on one device.

    config     -- astro_amd.Config (same fields as astro.core.Config)
    n_env      -- envs on this device
    b_cap      -- bullet slots per env (bullets beyond are dropped and
                  counted: hdr flag bit0 + stats 'overflows')
    p_pad      -- planet slots per env (default: config.max_planets)
    dtype      -- torch.float32 (default) or torch.float64 state storage
    env_offset -- global id of env 0 (multi-GPU sharding)
    kernel     -- 'auto', 'lane' (one lane per env), 'quad' (four lanes
                  per env) or 'pair' (two); identical results, different speed
    use_key_table -- share the device's 4 GiB seeding table (see key_table);
                  False runs every game's 397-step chain inline (same results)
    planets_only -- 0, or P: each env's games are its generate_configs stream
                  filtered to the seeds whose create() draws exactly P planets
                  (config.generate_configs_filtered); max_planets must be a
                  power of two
    mem        -- memory kind of the per-step state arrays (ships, ships_b,
                  planets, bullets, hdr, reward, done): 'default' (hipMalloc),
                  'uncached' or 'finegrained' (astro_dev_alloc); default: the
                  ASTRO_MEM environment variable, else 'default'
    """

    def __init__(self, config, n_env, device=None, b_cap=32, p_pad=None,
                 dtype=torch.float32, env_offset=0, auto_reset=True, kernel='auto',
                 use_key_table=True, planets_only=0, mem=None):
        _schedule.check_config(config)
        planets_only = int(planets_only)
        if planets_only and (not 1 <= planets_only <= config.max_planets
                             or config.max_planets & (config.max_planets - 1)):
            raise ValueError('planets_only must be in [1, max_planets], max_planets a power of two')
        self.planets_only = planets_only
        if dtype not in (torch.float32, torch.float64):
            raise ValueError('dtype must be torch.float32 or torch.float64')
        self.lib = _lib.load()
        self.config = config
        self.n_env = int(n_env)
        self.S = _nships(config)
        self.p_pad = int(p_pad or config.max_planets)
        if self.p_pad < config.max_planets or self.p_pad > 16:
            raise ValueError('p_pad must be in [max_planets, 16]')
        self.b_cap = int(b_cap)
        self.dtype = dtype
        self.device = torch.device(device if device is not None else 'cuda')
        if self.device.type != 'cuda':
            raise ValueError('BatchedEnv runs on a HIP device only (got %s)' % self.device)
        self.env_offset = int(env_offset)
        self.auto_reset = bool(auto_reset)
        self.schedule = _schedule.build(config)

        N, S, dev = self.n_env, self.S, self.device
        self.mem = mem or os.environ.get('ASTRO_MEM', 'default')
        if self.mem not in _lib.MEM:
            raise ValueError('mem must be one of %s' % sorted(_lib.MEM))
        z = lambda *shape, dt=dtype: torch.zeros(shape, dtype=dt, device=dev)  # noqa: E731
        zs = lambda *shape, dt=dtype: _dev_tensor(self.lib, shape, dt, dev, _lib.MEM[self.mem])  # noqa: E731
        self.ships = zs(S, N, 4)
        self.ships_b = zs(S, N)
        self.planets = zs(self.p_pad, N, 4)
        self.bullets = zs(N, self.b_cap, 4)
        self.hdr = zs(N, 4, dt=torch.int32)
        self.reward = zs(N, S, dt=torch.float32)
        self.done = zs(N, dt=torch.uint8)
        self.errors = z(1, dt=torch.int32)   # AstroState.errors: the ASTRO_ERR_* bits a faulting launch sets
        self.stream = z(N, 4, dt=torch.int32)
        self.stream_ring = z(N, MT_N, dt=torch.int32)
        self.stats = z(max(1, (N + 15) // 16), _lib.NSTATS, dt=torch.int64)
        self.fire_bits = torch.from_numpy(self.schedule.fire_bits().view(np.int32)).to(dev)

        k = _schedule.kernel_constants(config)
        self.key_table = key_table(dev) if use_key_table else None
        self.params = _lib.AstroParams(
            p_pad=self.p_pad, b_cap=self.b_cap, timeout_tick=self.schedule.timeout_tick,
            fire_bits=self.fire_bits.data_ptr(), kernel=_lib.KERNELS[kernel], planets_only=planets_only,
            key_table=self.key_table.data_ptr() if self.key_table is not None else None, **k)
        self.state = _lib.AstroState(
            ships=self.ships.data_ptr(), ships_b=self.ships_b.data_ptr(),
            planets=self.planets.data_ptr(), bullets=self.bullets.data_ptr(),
            hdr=self.hdr.data_ptr(), stream=self.stream.data_ptr(),
            stream_ring=self.stream_ring.data_ptr(),
            n_env=N, state_f64=1 if dtype == torch.float64 else 0, errors=self.errors.data_ptr())

        self.stream_seeds = _shard.stream_seeds(config, self.env_offset, N)
        seeds_t = torch.from_numpy(self.stream_seeds.view(np.int32)).to(dev)
        _lib.check(self.lib.astro_stream_init(ctypes.byref(self.state), seeds_t.data_ptr(),
                                              _stream_ptr(dev)), 'astro_stream_init')
        torch.cuda.current_stream(dev).synchronize()

    # ------------------------------------------------------------------ calls

    def reset(self, mask=None, seeds=None):
        """core.create for every env (or those with mask != 0): from the next
        seed of each env's stream, or from explicit ``seeds`` (uint32 [N])."""
        m = None
        if mask is not None:
            m = torch.as_tensor(mask, device=self.device).to(torch.uint8).contiguous()
        s = None
        if seeds is not None:
            s = torch.as_tensor(np.asarray(seeds, dtype=np.uint32).view(np.int32)
                                if not torch.is_tensor(seeds) else seeds,
                                device=self.device).to(torch.int32).contiguous()
        _lib.check(self.lib.astro_reset(
            ctypes.byref(self.params), ctypes.byref(self.state),
            None if s is None else s.data_ptr(), None if m is None else m.data_ptr(),
            _stream_ptr(self.device)), 'astro_reset')
        self._keep = (m, s)   # keep the arguments alive until the call has run
        return self.obs()

    def step(self, control, auto_reset=None, stats=True):
        """core.step for every env.  control: int8 [N, S] device tensor (or
        anything torch.as_tensor accepts).  Returns (obs, reward f32 [N, S],
        done u8 [N]); done = 1 ship collision, 2 timeout.  Finished envs are
        re-created in the same launch when auto_reset is on."""
        c = control
        if not (torch.is_tensor(c) and c.dtype == torch.int8 and c.device == self.device
                and c.is_contiguous()):
            c = torch.as_tensor(c, device=self.device).to(torch.int8).contiguous()
        if c.shape != (self.n_env, self.S):
            raise ValueError('control must be [%d, %d], got %s' % (self.n_env, self.S, tuple(c.shape)))
        self.launch(c.data_ptr(), auto_reset, stats)
        self._ctl = c
        self._last = (self.reward, self.done)
        return self.obs(), self.reward, self.done

    def step_many(self, controls, auto_reset=None, stats=True):
        """k consecutive steps with the controls given up front (int8
        [k, N, S]): k launches of the one-tick kernel from C
        (astro_step_many).  Returns (reward f32 [k, N, S], done u8 [k, N]);
        identical to k step() calls."""
        c = controls
        if not (torch.is_tensor(c) and c.dtype == torch.int8 and c.device == self.device
                and c.is_contiguous()):
            c = torch.as_tensor(c, device=self.device).to(torch.int8).contiguous()
        if c.dim() != 3 or c.shape[1:] != (self.n_env, self.S):
            raise ValueError('controls must be [k, %d, %d], got %s' % (self.n_env, self.S, tuple(c.shape)))
        k = c.shape[0]
        reward = torch.empty(k, self.n_env, self.S, dtype=torch.float32, device=self.device)
        done = torch.empty(k, self.n_env, dtype=torch.uint8, device=self.device)
        self.launch_many(c.data_ptr(), k, reward.data_ptr(), done.data_ptr(), auto_reset, stats)
        self._last = (reward[-1], done[-1]) if k else None
        return reward, done

    def launch_many(self, control_ptr, k, reward_ptr, done_ptr, auto_reset=None, stats=True, stream=None):
        """Raw astro_step_many (no checks, no allocation): for timed loops.
        The rewards and dones go to the caller's buffers only, so info()
        raises until the next step()/step_many()/launch()/rollout()."""
        ar = self.auto_reset if auto_reset is None else bool(auto_reset)
        rc = self.lib.astro_step_many(
            ctypes.byref(self.params), ctypes.byref(self.state), control_ptr, int(k), reward_ptr, done_ptr,
            self.stats.data_ptr() if stats else None, 1 if ar else 0,
            stream if stream is not None else _stream_ptr(self.device))
        if rc != 0:
            _lib.check(rc, 'astro_step_many')
        self._last = False   # info(): the last tick's reward/done are not held here

    def launch(self, control_ptr, auto_reset=None, stats=True, stream=None):
        """Raw launch (no checks, no allocation): for timed loops/graphs."""
        ar = self.auto_reset if auto_reset is None else bool(auto_reset)
        rc = self.lib.astro_step(
            ctypes.byref(self.params), ctypes.byref(self.state), control_ptr,
            self.reward.data_ptr(), self.done.data_ptr(),
            self.stats.data_ptr() if stats else None, 1 if ar else 0,
            stream if stream is not None else _stream_ptr(self.device))
        if rc != 0:
            _lib.check(rc, 'astro_step')
        self._last = None   # info(): this launch's reward/done

    @property
    def step_kernel(self):
        """'quad' or 'lane': the kernel astro_step runs for this env batch
        (the library's AUTO rule, pick_kernel in astro_kernels.hip)."""
        k = self.params.kernel
        if self.p_pad > 8:
            return 'lane'   # (QUAD/PAIR are built for up to 8 planet slots)
        for name in ('lane', 'quad', 'pair'):
            if k == _lib.KERNELS[name]:
                return name
        if self.p_pad > 8:
            return 'lane'
        return 'quad' if self.n_env <= QUAD_MAX_ENVS else 'pair'

    # ------------------------------------------------------------ observation

    @property
    def tick(self):
        return self.hdr[:, 0] & TICK_MASK

    @property
    def nplanets(self):
        return self.hdr[:, 1] & 0xff

    @property
    def flags(self):
        return (self.hdr[:, 1] >> 8) & 0xff

    @property
    def nbullets(self):
        return (self.hdr[:, 1] >> 16) & 0xffff

    def launch_waves(self):
        """(step waves, helper waves) of one astro_step launch of this batch:
        the library's rule (launch_step in astro_kernels.hip) -- a one-tick
        auto-reset launch of at most 2,048 quad/pair step waves gets one
        helper wave per step wave (HelpBox)."""
        lpe = dict(lane=1, quad=4, pair=2)[self.step_kernel]
        sw = (self.n_env * lpe + 63) // 64
        help_ = lpe > 1 and self.auto_reset and self.n_env * lpe <= 64 * 2048
        return sw, sw if help_ else 0

    def device_errors(self, clear=True):
        """The ASTRO_ERR_* bits any launch since the last check set (0: none;
        synchronises).  Every bit means a launch detected an internal fault
        and the state it wrote is not trusted."""
        v = int(self.errors.item())
        if v and clear:
            self.errors.zero_()
        return v

    def check_errors(self):
        """Raise AstroError if a launch since the last check reported a fault."""
        v = self.device_errors()
        if v:
            why = '; '.join(m for b, m in sorted(_lib.ERRORS.items()) if v & b) or 'unknown'
            raise _lib.AstroError('astro_step reported device error 0x%x: %s' % (v, why))

    def info(self, check=False):
        """Per-env flags of the last step, launch or rollout tick (SURVEY
        section 8b's info): ``hit`` uint8 bitmask of the ships a collision hit
        (bit s: reward[s] == -1 on a collision, core.py:253-255), ``overflow``
        the env's current game has dropped a bullet for lack of b_cap,
        ``create_exhausted`` its create() needed more than 227 MT19937 words
        (never in practice).  Device ops only; ``check=True`` also raises if
        a launch reported a device fault (a host synchronisation)."""
        if check:
            self.check_errors()
        last = getattr(self, '_last', None)
        if last is False:
            raise RuntimeError('info() after a raw launch_many(): its reward/done are in the caller\'s buffers')
        reward, done = last or (self.reward, self.done)
        hit = ((reward < 0) & (done == 1)[:, None]).to(torch.uint8)
        hit = (hit << torch.arange(self.S, device=self.device, dtype=torch.uint8)[None, :]).sum(1)
        fl = self.flags
        return dict(hit=hit.to(torch.uint8), overflow=(fl & 1) != 0, create_exhausted=(fl & 2) != 0)

    @property
    def game_seed(self):
        """Config.seed of each env's current game."""
        return self.stream[:, 3]

    def obs(self):
        """Env-major views of the state (no copies): ships [N, S, 4] ..."""
        return Observation(
            ships=self.ships.permute(1, 0, 2), ships_b=self.ships_b.permute(1, 0),
            planets=self.planets.permute(1, 0, 2), nplanets=self.nplanets,
            bullets=self.bullets, nbullets=self.nbullets, tick=self.tick)

    def policy(self, policy, seed=0, tick0=0, script_args=None):
        """The AstroPolicy of a policy name: 'random' (bench.py's splitmix64
        controls keyed by GLOBAL env id and tick), 'nothing'
        (script.NothingBot), 'script' (script.ScriptBot for every ship), or
        one bot name per ship, e.g. ('nothing', 'script') -- core.Bots with
        those bots (core.py:359-363).  script_args: ScriptBot's args
        (default ScriptBot.DEFAULT_ARGS, script.py:18-21)."""
        c = self.config
        a = dict(avoid_distance=0.1, avoid_threshold=0.45)
        a.update(script_args or {})
        pol = _lib.AstroPolicy(
            seed=int(seed), tick0=int(tick0), env_offset=self.env_offset,
            script_r2=(c.planet_radius + c.ship_radius + a['avoid_distance']) ** 2,
            script_threshold=float(a['avoid_threshold']), ship_thrust=float(c.ship_thrust),
            ship_rspeed=float(c.ship_rspeed), bullet_speed=float(c.bullet_speed),
            ship_radius=float(c.ship_radius))
        if isinstance(policy, str) and policy in ('random', 'nothing'):
            pol.kind = _lib.POLICIES[policy]
            return pol
        names = [policy] * self.S if isinstance(policy, str) else list(policy)
        if len(names) != self.S or any(n not in _lib.BOTS for n in names):
            raise ValueError('policy must be random/nothing/script or one of %s per ship' % sorted(_lib.BOTS))
        pol.kind = _lib.POLICIES['bots']
        pol.bots = sum(_lib.BOTS[n] << (4 * s) for s, n in enumerate(names))
        return pol

    def controls(self, policy='script', seed=0, tick0=0, script_args=None):
        """core.Bots.control (core.py:359-363) for every env: int8 [N, S]
        controls ``policy`` (see ``policy``) picks on the current state, each
        ship on its ego view -- computed on the device (astro_controls)."""
        out = torch.empty((self.n_env, self.S), dtype=torch.int8, device=self.device)
        pol = self.policy(policy, seed, tick0, script_args)
        _lib.check(self.lib.astro_controls(ctypes.byref(self.params), ctypes.byref(self.state), ctypes.byref(pol),
                                           out.data_ptr(), _stream_ptr(self.device)), 'astro_controls')
        return out

    def rollout(self, ticks, policy='random', seed=0, tick0=0, auto_reset=None, stats=True, script_args=None):
        """``ticks`` consecutive steps in one launch (quad/pair kernels; one
        per tick for the lane kernel): exactly ``ticks`` calls of ``step``
        with the controls ``policy`` picks each tick -- a policy name (see
        ``policy``: 'random', 'nothing', 'script', or one bot per ship) or
        an int8 tensor [ticks, N, S] of controls.  Returns (reward [ticks,
        N, S], done [ticks, N])."""
        ticks = int(ticks)
        ar = self.auto_reset if auto_reset is None else bool(auto_reset)
        ctl = None
        if torch.is_tensor(policy):
            ctl = policy.to(device=self.device, dtype=torch.int8).contiguous()
            if tuple(ctl.shape) != (ticks, self.n_env, self.S):
                raise ValueError('control must be [%d, %d, %d]' % (ticks, self.n_env, self.S))
            pol = _lib.AstroPolicy(kind=_lib.POLICIES['control'])
        else:
            pol = self.policy(policy, seed, tick0, script_args)
        reward = torch.empty((ticks, self.n_env, self.S), dtype=torch.float32, device=self.device)
        done = torch.empty((ticks, self.n_env), dtype=torch.uint8, device=self.device)
        _lib.check(self.lib.astro_rollout(
            ctypes.byref(self.params), ctypes.byref(self.state), ctypes.byref(pol), ticks,
            None if ctl is None else ctl.data_ptr(), reward.data_ptr(), done.data_ptr(),
            self.stats.data_ptr() if stats else None, int(ar), _stream_ptr(self.device)), 'astro_rollout')
        self._keep_rollout = ctl
        self._last = (reward[-1], done[-1])   # info() describes the last tick
        return reward, done

    def play(self, bots, games=1, chunk=256, max_ticks=None, script_args=None):
        """core.play (core.py:377-410) batched: every env plays its next
        ``games`` games (auto-reset onto its generate_configs stream) with
        ``bots`` (one name per ship, or one name for all: 'nothing',
        'script', 'random'), ``chunk`` ticks per astro_rollout launch, from
        the envs' current states.  Returns (winner int64 [N, games]: -1 for
        None, else the index of the winning ship -- argmax of the final
        reward when its max is >= 1, core.py:409 -- and length int64
        [N, games] in ticks)."""
        N, G = self.n_env, int(games)
        winner = torch.full((N, G), -2, dtype=torch.int64, device=self.device)
        length = torch.zeros((N, G), dtype=torch.int64, device=self.device)
        got = torch.zeros(N, dtype=torch.int64, device=self.device)
        start = -self.tick.to(torch.int64)          # tick number at which each env's game began
        t = 0
        limit = max_ticks if max_ticks is not None else G * (self.schedule.timeout_tick + 1) + chunk
        while int(got.min()) < G:
            if t >= limit:
                raise RuntimeError('play: games did not finish within %d ticks' % limit)
            reward, done = self.rollout(chunk, bots, tick0=t, auto_reset=True, script_args=script_args)
            d = done != 0
            k, e = torch.nonzero(d, as_tuple=True)          # tick-major: each env's games in order
            if k.numel():
                order = torch.argsort(e * chunk + k)
                k, e = k[order], e[order]
                # rank of each finish among its env's finishes in this chunk
                first = torch.ones_like(e, dtype=torch.bool)
                first[1:] = e[1:] != e[:-1]
                idx = torch.arange(e.numel(), device=self.device)
                seg = torch.cummax(torch.where(first, idx, torch.zeros_like(idx)), 0).values
                g = got[e] + (idx - seg)
                r = reward[k, e]                              # [M, S]
                mx, am = r.max(1)
                w = torch.where(mx >= 1, am, torch.full_like(am, -1))
                prev_end = torch.where(first, start[e], t + k[torch.clamp(idx - 1, min=0)] + 1)
                ok = g < G
                winner[e[ok], g[ok]] = w[ok]
                length[e[ok], g[ok]] = (t + k + 1 - prev_end)[ok]
                last = torch.zeros(N, dtype=torch.int64, device=self.device)
                last.scatter_reduce_(0, e, t + k + 1, reduce='amax', include_self=False)
                has = torch.zeros(N, dtype=torch.bool, device=self.device)
                has[e] = True
                start = torch.where(has, last, start)
                got += torch.bincount(e, minlength=N)
            t += chunk
        return winner, length

    def features(self, rows=None, out=None):
        """Observation features of every env, as rl.ValueNetwork.get_features
        then to_batch (rl.py:36-112): float32 [N, rows, 1 + 5*S + 4], rows
        [planets, live bullets] then -1 padding; column 0 is the object type
        (0 planet, 1 bullet, -1 padding), then every ship's (x, y, dx, dy,
        norm_angle(b)/pi), then the object's (x, y, dx, dy).  rows defaults
        to p_pad + b_cap, which holds every env's objects."""
        rows = self.p_pad + self.b_cap if rows is None else int(rows)
        D = 1 + 5 * self.S + 4
        if out is None:
            out = torch.empty((self.n_env, rows, D), dtype=torch.float32, device=self.device)
        elif (tuple(out.shape) != (self.n_env, rows, D) or out.dtype != torch.float32
              or out.device != self.device or not out.is_contiguous()):
            raise ValueError('out must be a contiguous float32 [%d, %d, %d] tensor on %s'
                             % (self.n_env, rows, D, self.device))
        _lib.check(self.lib.astro_features(ctypes.byref(self.params), ctypes.byref(self.state),
                                           out.data_ptr(), rows, _stream_ptr(self.device)), 'astro_features')
        return out

    def stat_dict(self):
        v = self.stats.sum(0).cpu().tolist()
        self.check_errors()
        return dict(zip(_lib.STAT_NAMES, v))

    # ----------------------------------------------------- host import/export

    def to_host(self):
        """Every array as numpy (synchronises; raises if a launch reported a
        device fault)."""
        self.check_errors()
        return dict(ships=self.ships.permute(1, 0, 2).cpu().numpy(),
                    ships_b=self.ships_b.permute(1, 0).cpu().numpy(),
                    planets=self.planets.permute(1, 0, 2).cpu().numpy(),
                    bullets=self.bullets.cpu().numpy(),
                    tick=self.tick.cpu().numpy(), nplanets=self.nplanets.cpu().numpy(),
                    nbullets=self.nbullets.cpu().numpy(), flags=self.flags.cpu().numpy())

    def load_host(self, ships, ships_b, planets, bullets, tick, nplanets, nbullets, flags=None):
        """Overwrite the state from host arrays (env-major, like to_host).
        ``flags`` (to_host's) are the loaded games' flag bits; default 0 (a
        loaded game has dropped no bullet).  Each env's seed stream and its
        pending next game are kept."""
        dev, dt = self.device, self.dtype

        def put(dst, src):
            dst.copy_(torch.as_tensor(np.ascontiguousarray(src)).to(dt))
        put(self.ships, np.asarray(ships).transpose(1, 0, 2))
        put(self.ships_b, np.asarray(ships_b).transpose(1, 0))
        pl = np.zeros((self.n_env, self.p_pad, 4))
        pl[:, :np.asarray(planets).shape[1]] = planets
        put(self.planets, pl.transpose(1, 0, 2))
        bl = np.zeros((self.n_env, self.b_cap, 4))
        bsrc = np.asarray(bullets)
        nbmax = min(bsrc.shape[1], self.b_cap)
        bl[:, :nbmax] = bsrc[:, :nbmax]
        put(self.bullets, bl)
        nb = np.asarray(nbullets, dtype=np.int64)
        if (nb > self.b_cap).any():
            raise ValueError('a state holds more bullets than b_cap')
        old = self.hdr.cpu().numpy().view(np.uint32).astype(np.int64)
        hdr = old.copy()
        hdr[:, 0] = (old[:, 0] & ~TICK_MASK & 0xFFFFFFFF) | np.asarray(tick, np.int64)
        fl = np.zeros(self.n_env, np.int64) if flags is None else np.asarray(flags, np.int64) & 0xff
        hdr[:, 1] = np.asarray(nplanets, np.int64) | (fl << 8) | (nb << 16)
        self.hdr.copy_(torch.as_tensor(hdr.astype(np.uint32).view(np.int32)).to(dev))

    def state_of(self, i, host=None):
        """Reference-shaped State of env i (numpy, reference dtypes: float32
        arrays for a fresh game, float64 after its first step)."""
        h = host or self.to_host()
        tick = int(h['tick'][i])
        npl = int(h['nplanets'][i])
        nb = int(h['nbullets'][i])
        fresh = tick == 0
        f = np.float32 if fresh else np.float64
        ships = h['ships'][i].astype(np.float64)
        pl = h['planets'][i, :npl].astype(np.float64)
        bl = h['bullets'][i, :nb].astype(np.float64)
        pf = np.float32 if (fresh or npl == 1) else np.float64
        pdxf = np.float32 if npl == 1 else np.float64
        sch = self.schedule
        k = min(tick, sch.timeout_tick)
        return State(
            ships=Bodies(x=ships[:, 0:2].astype(f), dx=ships[:, 2:4].astype(f),
                         b=h['ships_b'][i].astype(f)),
            planets=Bodies(x=pl[:, 0:2].astype(pf), dx=pl[:, 2:4].astype(pdxf), b=None),
            bullets=Bodies(x=bl[:, 0:2].astype(f), dx=bl[:, 2:4].astype(f), b=None),
            reload=float(sch.reload[k]), t=float(sch.t[k]))
