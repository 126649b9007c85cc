"""ctypes binding of libastro_hip.so (include/astro_step.h).

The shared library is built in-tree by ``__graft_entry__.build()``
(hipcc --offload-arch=gfx950).  There is no fallback: if the library is
missing or its ABI version differs, every entry point raises.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# (ASTRO_LIB: another build of the same library, e.g. an A/B variant from tools/build_var.sh)
LIB_PATH = os.environ.get('ASTRO_LIB') or os.path.join(HERE, 'libastro_hip.so')
ABI_VERSION = 21

STAT_NAMES = ('bullets_in', 'bullets_out', 'resets', 'collisions', 'timeouts',
              'overflows', 'planets', 'serial_resets')
NSTATS = 8
KERNELS = {'auto': 0, 'lane': 1, 'quad': 2, 'pair': 3}
MEM = {'default': 0, 'finegrained': 1, 'uncached': 2}   # include/astro_step.h ASTRO_MEM_*
ERRORS = {1: 'a helper wave never saw its step wave post (its finished games were not re-created)',
          2: "a step wave never saw its helper's header read"}


class AstroParams(ctypes.Structure):
    _fields_ = [
        ('gm', ctypes.c_double),
        ('dt', ctypes.c_double),
        ('db', ctypes.c_double),
        ('thrust', ctypes.c_double),
        ('r2_ss', ctypes.c_double),
        ('r2_sp', ctypes.c_double),
        ('r2_s0', ctypes.c_double),
        ('r2_p0', ctypes.c_double),
        ('gravity', ctypes.c_double),
        ('planet_mass', ctypes.c_double),
        ('spawn_off', ctypes.c_float),
        ('bullet_speed', ctypes.c_float),
        ('timeout_reward', ctypes.c_float),
        ('outer_pos', ctypes.c_float),
        ('inner_pos', ctypes.c_float),
        ('planet_orbit', ctypes.c_float),
        ('nships', ctypes.c_int32),
        ('solo', ctypes.c_int32),
        ('max_planets', ctypes.c_int32),
        ('p_pad', ctypes.c_int32),
        ('b_cap', ctypes.c_int32),
        ('timeout_tick', ctypes.c_int32),
        ('fire_bits', ctypes.c_void_p),
        ('kernel', ctypes.c_int32),
        ('planets_only', ctypes.c_int32),
        ('key_table', ctypes.c_void_p),
    ]


class AstroState(ctypes.Structure):
    _fields_ = [
        ('ships', ctypes.c_void_p),
        ('ships_b', ctypes.c_void_p),
        ('planets', ctypes.c_void_p),
        ('bullets', ctypes.c_void_p),
        ('hdr', ctypes.c_void_p),
        ('stream', ctypes.c_void_p),
        ('stream_ring', ctypes.c_void_p),
        ('n_env', ctypes.c_int32),
        ('state_f64', ctypes.c_int32),
        ('errors', ctypes.c_void_p),
    ]


class AstroPolicy(ctypes.Structure):
    _fields_ = [
        ('kind', ctypes.c_int32),
        ('bots', ctypes.c_int32),
        ('seed', ctypes.c_uint64),
        ('tick0', ctypes.c_int64),
        ('env_offset', ctypes.c_int64),
        ('script_r2', ctypes.c_double),
        ('script_threshold', ctypes.c_double),
        ('ship_thrust', ctypes.c_double),
        ('ship_rspeed', ctypes.c_double),
        ('bullet_speed', ctypes.c_double),
        ('ship_radius', ctypes.c_double),
    ]


class AstroGameTick(ctypes.Structure):
    """include/astro_step.h AstroGameTick: one game's tick (astro_game_step)."""
    _fields_ = [
        ('params', AstroParams),
        ('state', AstroState),
        ('stream', ctypes.c_void_p),
        ('hdr', ctypes.c_void_p),
        ('ships', ctypes.c_void_p),
        ('ships_b', ctypes.c_void_p),
        ('planets', ctypes.c_void_p),
        ('bullets', ctypes.c_void_p),
        ('control', ctypes.c_void_p),
        ('fire', ctypes.c_void_p),
        ('reward', ctypes.c_void_p),
        ('done', ctypes.c_void_p),
        ('errors', ctypes.c_void_p),
        ('control_dev', ctypes.c_void_p),
        ('fire_dev', ctypes.c_void_p),
        ('reward_dev', ctypes.c_void_p),
        ('done_dev', ctypes.c_void_p),
        ('in_', ctypes.c_void_p),
        ('out', ctypes.c_void_p),
        ('nplanets', ctypes.c_int32),
        ('nbullets', ctypes.c_int32),
        ('control0', ctypes.c_int32),
        ('control1', ctypes.c_int32),
        ('first_step', ctypes.c_int32),
        ('fire_now', ctypes.c_int32),
        ('timeout_now', ctypes.c_int32),
        ('out_nbullets', ctypes.c_int32),
        ('done_out', ctypes.c_int32),
        ('reward_out', ctypes.c_float * 2),
        ('flag', ctypes.c_void_p),
        ('flag_dev', ctypes.c_void_p),
        ('seq', ctypes.c_uint32),
        ('reserved', ctypes.c_int32),
    ]


POLICIES = {'control': 0, 'nothing': 1, 'random': 2, 'bots': 3}
BOTS = {'nothing': 0, 'script': 1, 'random': 2}

_SYMBOLS = {
    'astro_abi_version': (ctypes.c_int, []),
    'astro_last_error': (ctypes.c_char_p, []),
    'astro_step': (ctypes.c_int, [ctypes.POINTER(AstroParams), ctypes.POINTER(AstroState),
                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                  ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]),
    'astro_step_many': (ctypes.c_int, [ctypes.POINTER(AstroParams), ctypes.POINTER(AstroState),
                                       ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]),
    'astro_reset': (ctypes.c_int, [ctypes.POINTER(AstroParams), ctypes.POINTER(AstroState),
                                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    'astro_stream_init': (ctypes.c_int, [ctypes.POINTER(AstroState), ctypes.c_void_p,
                                         ctypes.c_void_p]),
    'astro_keytable_build': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                            ctypes.c_void_p]),
    'astro_controls': (ctypes.c_int, [ctypes.POINTER(AstroParams), ctypes.POINTER(AstroState),
                                      ctypes.POINTER(AstroPolicy), ctypes.c_void_p, ctypes.c_void_p]),
    'astro_features': (ctypes.c_int, [ctypes.POINTER(AstroParams), ctypes.POINTER(AstroState),
                                      ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]),
    'astro_host_alloc': (ctypes.c_int, [ctypes.c_uint64, ctypes.POINTER(ctypes.c_void_p),
                                        ctypes.POINTER(ctypes.c_void_p)]),
    'astro_host_free': (ctypes.c_int, [ctypes.c_void_p]),
    'astro_dev_alloc': (ctypes.c_int, [ctypes.c_uint64, ctypes.c_int32, ctypes.POINTER(ctypes.c_void_p)]),
    'astro_dev_free': (ctypes.c_int, [ctypes.c_void_p]),
    'astro_game_step': (ctypes.c_int, [ctypes.c_void_p]),
    'astro_rollout': (ctypes.c_int, [ctypes.POINTER(AstroParams), ctypes.POINTER(AstroState),
                                     ctypes.POINTER(AstroPolicy), ctypes.c_int32, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32,
                                     ctypes.c_void_p]),
}

_lib = None


class AstroError(RuntimeError):
    pass


def load(path=LIB_PATH):
    """Load (once) and type the library.  Raises if it is absent or stale."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise AstroError('%s is missing: build it with `python -c "import __graft_entry__ as g; '
                         'g.build()"` (hipcc --offload-arch=gfx950)' % path)
    # torch first: the library binds to the HIP runtime already in the process
    import torch  # noqa: F401
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    ab_any = os.environ.get('ASTRO_AB_ANY_ABI') == '1'
    for name, (res, args) in _SYMBOLS.items():
        if ab_any and not hasattr(lib, name):   # (an older A/B build: entry points it predates)
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    v = lib.astro_abi_version()
    # (ASTRO_AB_ANY_ABI=1: tools/ab.py timing an older build whose structs are a
    # prefix of these -- never for results)
    if v != ABI_VERSION and not (os.environ.get('ASTRO_AB_ANY_ABI') == '1' and 12 <= v <= ABI_VERSION):
        raise AstroError('libastro_hip.so ABI %d != expected %d (rebuild)' % (v, ABI_VERSION))
    _lib = lib
    return lib


def check(rc, what):
    if rc != 0:
        msg = load().astro_last_error().decode(errors='replace')
        raise AstroError('%s failed (%d): %s' % (what, rc, msg))
