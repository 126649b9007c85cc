"""Scripted bots of the reference (astro/script.py:6-83), host side.

``NothingBot`` always answers control 2 (no thrust, no rotation).
``ScriptBot`` first avoids planets it is about to hit, then (two-ship games)
turns towards where the enemy will be when a bullet arrives.  Both take the
EGO view of a state (``core.roll_ships``: the bot's own ship first), as
``core.Bots.control`` hands it, and return an int control code.

Arithmetic follows the reference's numpy expressions one to one, so with the
state's own dtypes (float32 arrays for a fresh game, float64 after) a
decision is the reference's decision (tests/test_bots_logs.py
test_scriptbot_decisions_match_reference: every golden state, both ships).
For batched play use the device policies -- ``BatchedEnv.rollout(ticks,
policy)``, ``BatchedEnv.controls(policy)`` and ``BatchedEnv.play(bots)`` --
not these per-game objects.
"""
import numpy as np


def _norm_angle(b):
    return ((b + np.pi) % (2 * np.pi)) - np.pi            # util.py:125-132


def _bearing(x):
    return np.arctan2(x[..., 0], x[..., 1])               # util.py:95-103


def _mag(x):
    return np.sqrt((x ** 2).sum(axis=-1))                 # util.py:105-113


def _unit(x):
    return x / (_mag(x) + 1e-12)[..., np.newaxis]         # util.py:115-123


class NothingBot:
    """script.py:6-10."""

    def __call__(self, state):
        return 2


class ScriptBot:
    """script.py:13-83: planet avoidance, then aim at the enemy's forecast."""

    DEFAULT_ARGS = dict(avoid_distance=0.1, avoid_threshold=0.45)

    @classmethod
    def create(cls, config, args=DEFAULT_ARGS):
        return cls(args=args, config=config)

    def __init__(self, args, config):
        self.args = dict(args)
        self.config = config

    def _turn_to(self, state, target, tolerance, thrust):
        """script.py:26-35: rotate towards `target` (left 0 / right 4) unless
        within `tolerance`, then thrust (3) or idle (2)."""
        off = _norm_angle(target - state.ships.b[0])
        if off < -tolerance:
            return 0
        if tolerance < off:
            return 4
        return 3 if thrust else 2

    def _danger(self, x, dx):
        """script.py:37-62: bearing to steer for if the current course meets
        the inflated planet disc soon, else None.  (As in the reference, the
        rotation estimate uses the quadratic's linear coefficient where the
        bearing argument was meant; kept for identical decisions.)"""
        cfg = self.config
        radius = cfg.planet_radius + cfg.ship_radius
        lin = 2 * np.sum(_unit(dx) * x, axis=-1)
        const = _mag(x) ** 2 - (radius + self.args['avoid_distance']) ** 2
        det = lin ** 2 - 4 * const
        if 0 < det and 0 <= -lin + np.sqrt(det):
            distance = -lin - np.sqrt(det)
            with np.errstate(divide='ignore'):
                rotation = abs(_norm_angle(_bearing(x) - lin))
                speed = _mag(dx)
                if distance < (speed / cfg.ship_thrust + cfg.ship_rspeed / rotation) * speed:
                    return _bearing(x)
        return None

    def __call__(self, state):
        for i in range(state.planets.x.shape[0]):   # script.py:66-73
            b = self._danger(state.ships.x[0] - state.planets.x[i],
                             state.ships.dx[0] - state.planets.dx[i])
            if b is not None:
                return self._turn_to(state, b, self.args['avoid_threshold'], thrust=True)
        if self.config.solo:                         # script.py:75-77
            return 2
        cfg = self.config                            # script.py:79-88
        distance = _mag(state.ships.x[1] - state.ships.x[0])
        flight = distance / cfg.bullet_speed
        forecast = state.ships.x[1] + flight * (state.ships.dx[1] - state.ships.dx[0])
        return self._turn_to(state, _bearing(forecast - state.ships.x[0]),
                             cfg.ship_radius / distance, thrust=False)
