"""Game logs in the reference's jsonlines format (core.py:413-443, util.py:13-64).

A log is one JSON line ``{"config": Config, "winner": int|None}`` followed by
one line per tick, ``Tick(state, control, reward, bot_data)``; namedtuples
carry ``"_type": "astro.core:<Name>"`` and numpy arrays are
``{"_values": [...], "_shape": [...]}``.  The type tags name the reference
module, so the reference's ``core.load_log`` and web viewer (astro.js) read
logs written here, and ``load_log`` below reads the reference's.

``record_games`` captures whole games of chosen envs of a ``BatchedEnv`` run
(states as the reference would hold them: ``BatchedEnv.state_of``) so a GPU
env can be replayed in the reference viewer.
"""
import json
import os

import numpy as np

from . import config as _config

# our namedtuples <-> the reference's type tags (core.py:11-49)
_TYPES = {name: getattr(_config, name) for name in ('Bodies', 'State', 'Config', 'Tick', 'Game')}


def to_jsonable(obj):
    """util.to_jsonable (util.py:13-30) with the reference's type tags."""
    if hasattr(obj, '_asdict'):
        d = to_jsonable(obj._asdict())
        d['_type'] = 'astro.core:' + type(obj).__name__
        return d
    if isinstance(obj, np.ndarray):
        return {'_values': obj.tolist(), '_shape': obj.shape}
    if isinstance(obj, dict):
        return {k: to_jsonable(v) for k, v in obj.items()}
    if isinstance(obj, (tuple, list)):
        return list(to_jsonable(x) for x in obj)
    return obj


def from_jsonable(obj):
    """util.from_jsonable (util.py:33-50), building astro_amd's namedtuples.
    (The reference's float64 -> float32 conversion there compares dtypes with
    ``is`` and never fires, so arrays load as float64; kept as is.)"""
    if isinstance(obj, (list, tuple)):
        return list(from_jsonable(x) for x in obj)
    if isinstance(obj, dict):
        if obj.keys() == {'_values', '_shape'}:
            return np.array(obj['_values']).reshape(obj['_shape'])
        if '_type' in obj:
            obj = dict(obj)
            module, name = obj.pop('_type').split(':')
            if module != 'astro.core' or name not in _TYPES:
                raise ValueError('unknown type tag %s:%s' % (module, name))
            return _TYPES[name](**from_jsonable(obj))
        return {k: from_jsonable(v) for k, v in obj.items()}
    return obj


def to_json(obj):
    return json.dumps(to_jsonable(obj))


def save_log(path, game):
    """core.save_log (core.py:413-426)."""
    d = os.path.dirname(path)
    if d and not os.path.isdir(d):
        os.makedirs(d)
    with open(path, 'w') as f:
        f.write(to_json(dict(config=game.config, winner=game.winner)) + '\n')
        for tick in game.ticks:
            f.write(to_json(tick) + '\n')


def load_log(path):
    """core.load_log (core.py:429-443)."""
    with open(path) as f:
        header = from_jsonable(json.loads(next(f)))
        ticks = [from_jsonable(json.loads(line)) for line in f]
    return _config.Game(config=header['config'], winner=header['winner'], ticks=ticks)


def record_games(env, env_ids, policy, max_ticks=1 << 20):
    """Play ``env`` (a BatchedEnv, auto_reset off) until each env in
    ``env_ids`` finishes its current game, and return those games as
    ``Game`` tuples (what ``core.play`` returns): per tick the state the bots
    saw, the controls, the rewards, ``bot_data`` None.

    policy -- f(env) -> int8 control tensor [N, S] on the env's device.
    """
    ids = [int(i) for i in env_ids]
    ticks = {i: [] for i in ids}
    out = {}
    S = env.S
    for _ in range(max_ticks):
        if len(out) == len(ids):
            break
        host = env.to_host()
        states = {i: env.state_of(i, host) for i in ids if i not in out}
        ctl = policy(env)
        _, rew, done = env.step(ctl, auto_reset=False)
        ctl_h = ctl.cpu().numpy()
        rew_h = rew.cpu().numpy()
        done_h = done.cpu().numpy()
        for i, st in states.items():
            d = int(done_h[i])
            if d == 1:
                reward = rew_h[i, :S].astype(np.int64)
            elif d == 2:
                reward = rew_h[i, :S].astype(np.float32)
            else:
                reward = np.zeros(S, dtype=np.float32)
            ticks[i].append(_config.Tick(state=st, control=ctl_h[i, :S].astype(np.int64), reward=reward,
                                         bot_data=[None] * S))
            if d:
                winner = None if np.max(reward) < 1 else int(np.argmax(reward))
                cfg = env.config._replace(seed=int(env.game_seed[i].item()) & 0xFFFFFFFF)
                out[i] = _config.Game(config=cfg, winner=winner, ticks=ticks[i])
    return [out[i] for i in ids if i in out]
