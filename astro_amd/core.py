"""Drop-in single-game surface: ``create``/``step``/``roll_ships``/``play``.

Same names, arguments, return values and dtypes as astro/core.py
(create :86-135, step :215-303, roll_ships :306-327, Bots :359-374,
play :377-410), so astro/server.py (``game_start``/``game_tick``) and
astro/rl.py (``core.play`` rollouts) can call this module instead.  Every
call runs the HIP kernel on a one-env float64 BatchedEnv, which reproduces
the reference bit for bit (tests/test_gpu_parity.py): inputs are never
mutated, a finished game returns ``(None, reward)`` with an int64 reward for
a collision and a float32 reward for a timeout.

This path is latency-bound by design (one tiny launch + copies per tick);
bulk simulation belongs on :class:`astro_amd.env.BatchedEnv`.
"""
import numpy as np
import torch

from .config import (Bodies, Config, DEFAULT_CONFIG, Game, SOLO_CONFIG,  # noqa: F401
                     SOLO_EASY_CONFIG, State, Tick, generate_configs, nships)
from .env import BatchedEnv

_ENVS = {}


def _device():
    return torch.device('cuda', torch.cuda.current_device())


def _env(config, bullets_needed):
    key = (config._replace(seed=0), _device())
    env = _ENVS.get(key)
    if env is None or env.b_cap < bullets_needed:
        cap = 64 if env is None else env.b_cap
        while cap < bullets_needed:
            cap *= 2
        env = BatchedEnv(config, 1, device=key[1], b_cap=cap, dtype=torch.float64,
                         auto_reset=False, use_key_table=False)
        env._fire = torch.zeros(2, dtype=torch.int32, device=key[1])
        _ENVS[key] = env
    return env


def create(config):
    """Create a new game state from ``config.seed`` (core.create)."""
    seed = int(config.seed)
    if not 0 <= seed < 1 << 32:   # as np.random.RandomState(seed) (core.py:89) refuses it
        raise ValueError('Seed must be between 0 and 2**32 - 1')
    env = _env(config, 0)
    env.reset(seeds=[seed])
    return env.state_of(0)


def step(state, control, config):
    """Advance one game by one tick (core.step).  Returns (State or None,
    reward array[nships])."""
    S = nships(config)
    control = np.asarray(control)
    if control.shape != (S,):
        raise ValueError('control must have shape (%d,)' % S)
    if control.min() < -128 or control.max() > 127:
        raise ValueError('control codes must fit int8')
    nb = state.bullets.x.shape[0]
    env = _env(config, nb + S)
    # the reference's float64 bookkeeping for THIS call (core.py:257,263,267)
    timeout = config.max_time <= state.t + config.dt
    fire = config.reload_time <= state.reload + config.dt
    fresh = state.ships.x.dtype == np.float32      # create()'s float32 arrays
    tick = 0 if fresh else 1
    npl = state.planets.x.shape[0]
    pl = np.concatenate([state.planets.x, state.planets.dx], 1).astype(np.float64)[None]
    bl = np.concatenate([state.bullets.x, state.bullets.dx], 1).astype(np.float64)[None]
    sh = np.concatenate([state.ships.x, state.ships.dx], 1).astype(np.float64)[None]
    env.load_host(sh, np.asarray(state.ships.b, np.float64)[None], pl, bl,
                  [tick], [npl], [nb])
    env._fire.fill_(int(fire) << tick)
    params = type(env.params).from_buffer_copy(env.params)
    params.timeout_tick = tick if timeout else tick + 1
    params.fire_bits = env._fire.data_ptr()
    saved = env.params
    env.params = params
    try:
        env.step(torch.as_tensor(control.astype(np.int8))[None], auto_reset=False)
    finally:
        env.params = saved
    done = int(env.done[0].item())
    reward = env.reward[0].cpu().numpy()
    if done == 1:
        return None, reward.astype(np.int64)
    if done == 2:
        return None, reward.astype(np.float32)
    h = env.to_host()
    nxt = env.state_of(0, h)
    reload = state.reload + config.dt
    if fire:
        reload -= config.reload_time
    bdt = np.float32 if fresh else np.float64
    new = State(
        ships=Bodies(x=nxt.ships.x.astype(np.float64), dx=nxt.ships.dx.astype(np.float64),
                     b=nxt.ships.b.astype(np.float64)),
        planets=Bodies(x=h['planets'][0, :npl, 0:2].astype(np.float32 if npl == 1 else np.float64),
                       dx=h['planets'][0, :npl, 2:4].astype(np.float32 if npl == 1 else np.float64),
                       b=None),
        bullets=Bodies(x=nxt.bullets.x.astype(bdt), dx=nxt.bullets.dx.astype(bdt), b=None),
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
