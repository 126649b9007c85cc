"""Reference-shaped types and presets (mirrors astro/core.py:11-83).

``Bodies``, ``State``, ``Config``, ``Tick`` and ``Game`` have the same fields
and meaning as the reference's namedtuples (core.py:11-49), and the three
presets carry the same values (core.py:52-74), so a caller written against
``astro.core`` keeps working with ``astro_amd``.
"""
import collections

import numpy as np

Bodies = collections.namedtuple('Bodies', ('x', 'dx', 'b'))

State = collections.namedtuple('State', ('ships', 'planets', 'bullets', 'reload', 't'))

Config = collections.namedtuple('Config', (
    # world
    'gravity', 'dt', 'max_time', 'reload_time', 'bullet_speed',
    'ship_thrust', 'ship_rspeed', 'ship_radius',
    # creation
    'seed', 'solo', 'outer_ship_position', 'inner_ship_position',
    'max_planets', 'planet_orbit', 'planet_mass', 'planet_radius',
))

Tick = collections.namedtuple('Tick', ('state', 'control', 'reward', 'bot_data'))

Game = collections.namedtuple('Game', ('config', 'winner', 'ticks'))

DEFAULT_CONFIG = Config(
    gravity=0.05, dt=0.02, max_time=60, reload_time=0.3, bullet_speed=1.5,
    ship_thrust=1.0, ship_rspeed=4.0, ship_radius=0.025,
    seed=42, solo=False, inner_ship_position=0.2, outer_ship_position=0.9,
    max_planets=4, planet_orbit=0.5, planet_mass=1.0, planet_radius=0.2,
)
SOLO_CONFIG = DEFAULT_CONFIG._replace(solo=True, reload_time=1000)
SOLO_EASY_CONFIG = SOLO_CONFIG._replace(max_planets=1)


def generate_configs(config):
    """Infinite stream of differently seeded copies of ``config`` (core.py:77-83):
    seed_k = RandomState(config.seed).randint(1 << 30), drawn in sequence."""
    random = np.random.RandomState(config.seed)
    while True:
        yield config._replace(seed=random.randint(1 << 30))


def create_nplanets(config, seed):
    """The number of planets create() draws for ``seed`` (core.py:90)."""
    return int(np.random.RandomState(seed).randint(1, config.max_planets + 1))


def generate_configs_filtered(config, planets):
    """generate_configs(config) restricted to the seeds whose game has exactly
    ``planets`` planets -- the game sequence of BatchedEnv(planets_only=...),
    used for BASELINE.json's fixed-planet-count workloads."""
    for cfg in generate_configs(config):
        if create_nplanets(cfg, cfg.seed) == planets:
            yield cfg


def nships(config):
    return 1 if config.solo else 2
