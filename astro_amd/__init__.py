"""astro_amd -- MI355X-native batched lockstep Astro physics.

``BatchedEnv`` (env.py) steps N independent games per GPU through one HIP
kernel (csrc/astro_kernels.hip, C-ABI include/astro_step.h); ``core``
exposes the reference's single-game create/step/play surface on top of it.
"""
from .config import (Bodies, Config, DEFAULT_CONFIG, Game, SOLO_CONFIG,  # noqa: F401
                     SOLO_EASY_CONFIG, State, Tick, generate_configs)
from .env import BatchedEnv, Observation  # noqa: F401
