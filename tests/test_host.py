"""CPU-only checks of the boundary and the host logic (no GPU needed)."""
import ctypes
import os
import re
import subprocess
import tempfile

import numpy as np
import pytest

import __graft_entry__
from astro_amd import _lib, schedule, shard
from astro_amd.config import DEFAULT_CONFIG, SOLO_CONFIG, generate_configs
from oracle import batched
from tests import golden_io as gio

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, 'include', 'astro_step.h')


@pytest.fixture(scope='module')
def lib():
    __graft_entry__.build()
    return _lib.load()


def _declared_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(r'^\s*(?:const\s+)?\w+\s*\*?\s*(astro_\w+)\s*\(', text, re.M)))


def test_library_exports_every_header_symbol(lib):
    names = _declared_functions()
    assert set(names) == {'astro_abi_version', 'astro_last_error', 'astro_step', 'astro_step_many', 'astro_reset',
                          'astro_stream_init', 'astro_keytable_build', 'astro_features', 'astro_rollout',
                          'astro_controls', 'astro_host_alloc', 'astro_host_free', 'astro_dev_alloc',
                          'astro_dev_free', 'astro_game_step'}
    out = subprocess.check_output(['nm', '-D', '--defined-only', _lib.LIB_PATH], text=True)
    exported = set(re.findall(r' T (astro_\w+)$', out, re.M))
    assert set(names) <= exported
    for n in names:
        getattr(lib, n)
    assert lib.astro_abi_version() == _lib.ABI_VERSION


def test_ctypes_struct_layout_matches_header():
    """sizeof/offsetof of the C structs (gcc on include/astro_step.h) equal
    the ctypes mirrors'."""
    lines = ['#include <stddef.h>', '#include <stdio.h>', '#include "astro_step.h"', 'int main(void){']
    expect = []
    cname = {'in_': 'in'}   # (ctypes field names that are Python keywords)
    for st in (_lib.AstroParams, _lib.AstroState, _lib.AstroPolicy, _lib.AstroGameTick):
        lines.append('printf("%%zu\\n", sizeof(%s));' % st.__name__)
        expect.append(ctypes.sizeof(st))
        for f, _ in st._fields_:
            lines.append('printf("%%zu\\n", offsetof(%s, %s));' % (st.__name__, cname.get(f, f)))
            expect.append(getattr(st, f).offset)
    lines.append('return 0;}')
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, 'layout.c')
        exe = os.path.join(d, 'layout')
        open(src, 'w').write('\n'.join(lines))
        subprocess.check_call(['gcc', '-std=c99', '-I', os.path.dirname(HEADER), src, '-o', exe])
        got = [int(x) for x in subprocess.check_output([exe], text=True).split()]
    assert got == expect


def test_game_step_validation_without_gpu(lib):
    """astro_game_step (the single-game tick) rejects a bad record before
    touching the arena or the device."""
    assert lib.astro_game_step(None) == -91
    t = _lib.AstroGameTick()
    t.params = _lib.AstroParams(nships=2, solo=0, p_pad=4, max_planets=4, b_cap=64)
    t.state = _lib.AstroState(n_env=1, state_f64=1)
    t.nplanets, t.nbullets = 5, 0
    assert lib.astro_game_step(ctypes.byref(t)) == -92 and b'nplanets' in lib.astro_last_error()
    t.nplanets, t.nbullets = 3, 65
    assert lib.astro_game_step(ctypes.byref(t)) == -93
    t.nbullets = 0
    t.state.n_env = 2
    assert lib.astro_game_step(ctypes.byref(t)) == -94


def test_argument_validation_without_gpu(lib):
    """Bad arguments are rejected before any HIP call, with a message."""
    p = _lib.AstroParams(nships=3, solo=0, p_pad=4, max_planets=4, b_cap=32)
    s = _lib.AstroState(n_env=4)
    rc = lib.astro_step(ctypes.byref(p), ctypes.byref(s), None, None, None, None, 0, None)
    assert rc == -11 and b'nships' in lib.astro_last_error()
    p.nships = 2
    p.p_pad = 17
    rc = lib.astro_step(ctypes.byref(p), ctypes.byref(s), None, None, None, None, 0, None)
    assert rc == -13
    rc = lib.astro_step_many(ctypes.byref(p), ctypes.byref(s), None, -1, None, None, None, 0, None)
    assert rc == -35 and b'k must be' in lib.astro_last_error()
    assert lib.astro_step_many(ctypes.byref(p), ctypes.byref(s), None, 0, None, None, None, 0, None) == 0
    rc = lib.astro_step_many(ctypes.byref(p), ctypes.byref(s), None, 3, None, None, None, 0, None)
    assert rc == -13   # checked as astro_step is
    p.p_pad = 4
    p.planets_only = 5   # > max_planets
    assert lib.astro_step(ctypes.byref(p), ctypes.byref(s), None, None, None, None, 0, None) == -19
    p.max_planets, p.planets_only = 3, 2   # max_planets not a power of two
    assert lib.astro_step(ctypes.byref(p), ctypes.byref(s), None, None, None, None, 0, None) == -19
    assert b'power of two' in lib.astro_last_error()
    p.max_planets, p.planets_only = 4, 0
    p.kernel = 4
    assert lib.astro_step(ctypes.byref(p), ctypes.byref(s), None, None, None, None, 0, None) == -18
    p.kernel = 0
    s.n_env = -1
    assert lib.astro_reset(ctypes.byref(p), ctypes.byref(s), None, None, None) == -3
    s.n_env = 0   # empty batch: a no-op that never touches the device
    assert lib.astro_step(ctypes.byref(p), ctypes.byref(s), None, None, None, None, 0, None) == 0
    assert lib.astro_stream_init(ctypes.byref(s), None, None) == 0
    assert lib.astro_step(None, ctypes.byref(s), None, None, None, None, 0, None) == -10
    assert lib.astro_features(ctypes.byref(p), ctypes.byref(s), None, 0, None) == 0   # empty batch
    s.n_env = 4
    assert lib.astro_features(ctypes.byref(p), ctypes.byref(s), None, 36, None) == -4  # arrays NULL
    pol = _lib.AstroPolicy(kind=4)
    s.n_env = 0
    assert lib.astro_rollout(ctypes.byref(p), ctypes.byref(s), ctypes.byref(pol), 4, None, None, None,
                             None, 0, None) == -71
    pol.kind = 3            # BOTS with an unknown bot for ship 1
    pol.bots = 1 | (7 << 4)
    assert lib.astro_rollout(ctypes.byref(p), ctypes.byref(s), ctypes.byref(pol), 4, None, None, None,
                             None, 0, None) == -75
    assert lib.astro_controls(ctypes.byref(p), ctypes.byref(s), ctypes.byref(pol), None, None) == -75
    pol.bots = 1 | (2 << 4)
    assert lib.astro_controls(ctypes.byref(p), ctypes.byref(s), ctypes.byref(pol), None, None) == 0
    pol.kind = 0            # a control array is not a policy for astro_controls
    assert lib.astro_controls(ctypes.byref(p), ctypes.byref(s), ctypes.byref(pol), None, None) == -71
    pol.kind = 2
    assert lib.astro_rollout(ctypes.byref(p), ctypes.byref(s), ctypes.byref(pol), 0, None, None, None,
                             None, 0, None) == -72
    h, d = ctypes.c_void_p(), ctypes.c_void_p()
    assert lib.astro_host_alloc(0, ctypes.byref(h), ctypes.byref(d)) == -81
    assert lib.astro_host_alloc(64, None, None) == -80
    assert lib.astro_host_free(None) == 0
    assert lib.astro_dev_alloc(0, 0, ctypes.byref(d)) == -81
    assert lib.astro_dev_alloc(64, 0, None) == -82
    assert lib.astro_dev_alloc(64, 3, ctypes.byref(d)) == -83
    assert lib.astro_dev_free(None) == 0
    assert lib.astro_keytable_build(None, 0, 16, None) == -50
    assert lib.astro_keytable_build(ctypes.c_void_p(16), (1 << 30) - 8, 16, None) == -51


def test_schedule_matches_oracle_and_golden():
    sched = gio.load_json('schedule.json')
    for name, s in sched.items():
        cfg = DEFAULT_CONFIG._replace(**s['config'])
        sc = schedule.build(cfg)
        assert sc.timeout_tick == s['timeout_tick']
        bits = sc.fire_bits()
        fired = [k for k in range(sc.timeout_tick) if (bits[k >> 5] >> (k & 31)) & 1]
        assert fired == s['fire_ticks'], name
        assert sc.t[:50].tolist() == s['t'] and sc.reload[:50].tolist() == s['reload']


def test_kernel_constants_match_oracle():
    for cfg in gio.configs().values():
        k = schedule.kernel_constants(cfg)
        P = batched.make_params(cfg)
        for f in ('gm', 'db', 'r2_ss', 'r2_sp', 'r2_s0', 'r2_p0'):
            assert k[f] == getattr(P, f), f
        assert np.float32(k['spawn_off']) == P.spawn_off
        assert np.float32(k['bullet_speed']) == P.bullet_speed
        assert k['nships'] == P.nships


def test_generate_configs_matches_golden():
    z = gio.load('generate_configs.npz')
    import itertools as it
    for key in z.files:
        seed = int(key.split('_', 1)[1])
        got = [c.seed for c in it.islice(generate_configs(DEFAULT_CONFIG._replace(seed=seed)), 300)]
        assert got == z[key].tolist()


def test_presets_match_reference_values():
    cfgs = gio.configs()
    assert cfgs['default'] == DEFAULT_CONFIG
    assert cfgs['solo'] == SOLO_CONFIG


@pytest.mark.parametrize('n,world', [(524288, 8), (1048576, 8), (65536, 1), (1001, 4), (3, 8)])
def test_shard_ranges_partition(n, world):
    seen = []
    for r in range(world):
        off, cnt = shard.shard(n, r, world)
        seen.extend(range(off, off + cnt))
    assert seen == list(range(n))


def test_wrap_formula_matches_numpy_remainder():
    """The kernel's wrap (x - 2 trunc(x/2), +2 if negative, +0 if zero, -1) equals numpy's
    ((x + 1) % 2) - 1 (util.py:148) on random and edge values."""
    rng = np.random.default_rng(5)
    x = np.concatenate([rng.uniform(-3, 3, 100000), rng.uniform(-1e-15, 1e-15, 1000),
                        [-1.0, 1.0, 3.0, -3.0, 0.0, -0.0, 1 - 2 ** -53, -1 + 2 ** -53, 2.0 ** -1074]])
    v = x + 1.0
    m = v - 2.0 * np.trunc(v * 0.5)
    m = np.where(m < 0, m + 2.0, m)
    m = np.where(m == 0, 0.0, m)
    mine = m - 1.0
    ref = ((x + 1) % 2) - 1
    assert (mine.view(np.int64) == ref.view(np.int64)).all()
    x32 = x.astype(np.float32)
    v = x32 + np.float32(1)
    m = v - np.float32(2) * np.trunc(v * np.float32(0.5))
    m = np.where(m < 0, m + np.float32(2), m).astype(np.float32)
    m = np.where(m == 0, np.float32(0), m).astype(np.float32)
    assert ((m - np.float32(1)).view(np.int32) == (((x32 + 1) % 2) - 1).view(np.int32)).all()


def test_kernel_choice_mirrors_header():
    """BatchedEnv.step_kernel's AUTO rule uses the header's quad/lane crossover."""
    from astro_amd import env as _env
    hdr = open(os.path.join(os.path.dirname(__graft_entry__.__file__), 'include', 'astro_step.h')).read()
    n = int(re.search(r'#define ASTRO_QUAD_MAX_ENVS (\d+)', hdr).group(1))
    assert _env.QUAD_MAX_ENVS == n


def test_filtered_stream_oracle_matches_numpy():
    """oracle.batched.filtered_game_seeds == config.generate_configs_filtered
    (numpy RandomState draws create()'s planet count, core.py:90)."""
    import itertools
    from oracle import batched
    from astro_amd.config import generate_configs_filtered
    ss = batched.stream_seeds(42, 4)
    got = batched.filtered_game_seeds(ss, 6, 3, 4)
    for i in range(4):
        want = [c.seed for c in itertools.islice(
            generate_configs_filtered(DEFAULT_CONFIG._replace(seed=int(ss[i])), 3), 6)]
        assert list(got[i]) == want


def test_planets_only_validation():
    """planets_only needs 1 <= P <= max_planets and max_planets a power of two
    (one MT word decides create()'s count); checked before any device work."""
    import pytest as _pytest
    from astro_amd import BatchedEnv
    with _pytest.raises(ValueError):
        BatchedEnv(DEFAULT_CONFIG._replace(max_planets=3), 4, device='cuda:0', planets_only=2)
    with _pytest.raises(ValueError):
        BatchedEnv(DEFAULT_CONFIG, 4, device='cuda:0', planets_only=5)


def test_mtstream_ring_algorithm_matches_numpy():
    """The kernel's MTStream (astro_kernels.hip): cursor (x_k, x_{k+397}, k)
    + a 624-word ring, one word per draw, restated here line for line --
    equals numpy's RandomState(seed) for 2,000 outputs (past 227, where the
    lazy init-key form ends, and past 624 and 1,248, whole twists)."""
    M32 = 0xFFFFFFFF

    def key_next(prev, idx):
        return (1812433253 * (prev ^ (prev >> 30)) + idx) & M32

    def temper(y):
        y ^= y >> 11
        y ^= (y << 7) & 0x9d2c5680
        y ^= (y << 15) & 0xefc60000
        return y ^ (y >> 18)

    for seed in (0, 42, 5489, (1 << 32) - 1):
        a, b, k = seed, seed, 0
        for i in range(1, 398):
            b = key_next(b, i)
        ring = [None] * 624
        out = []
        for _ in range(2000):
            k1 = k + 1
            r1 = ring[k1 % 624] if k1 >= 624 else 0
            rb = ring[(k1 - 227) % 624] if k1 >= 227 else 0
            x1 = key_next(a, k1) if k1 < 624 else r1
            y = (a & 0x80000000) | (x1 & 0x7fffffff)
            z = b ^ (y >> 1) ^ (0x9908b0df if x1 & 1 else 0)
            ring[k % 624] = z
            b = key_next(b, k1 + 397) if k1 < 227 else rb
            a, k = x1, k1
            out.append(temper(z))
        ref = np.random.RandomState(seed).randint(0, 1 << 32, size=2000, dtype=np.uint64)
        assert out == [int(v) for v in ref]


def test_first_words_and_long_filtered_streams_match_numpy():
    """oracle.mt19937.first_words (create()'s planet-count word, core.py:90)
    and filtered_game_draws over 1,500 stream draws == numpy itself."""
    import itertools
    from oracle import mt19937
    from astro_amd.config import generate_configs_filtered
    seeds = np.array([0, 1, 42, 5489, 123456789, (1 << 30) - 1, (1 << 32) - 1])
    ref = [np.random.RandomState(int(s)).randint(0, 1 << 32, dtype=np.uint64) for s in seeds]
    assert list(mt19937.first_words(seeds)) == [int(r) for r in ref]
    ss = batched.stream_seeds(7, 3)
    got, idx = batched.filtered_game_draws(ss, 300, 3, 4, 1500)
    for i in range(3):
        want = [c.seed for c in itertools.islice(
            generate_configs_filtered(DEFAULT_CONFIG._replace(seed=int(ss[i])), 3), 300)]
        assert list(got[i]) == want
    assert idx.max() > 1000


def test_gamestep_packing_without_gpu():
    """astro_amd/_gamestep (core.step's packing around astro_game_step, in C)
    against a stand-in for the tick: it packs the State into the record's
    input in the shim's order, sets the call's fields from the reference's
    float64 bookkeeping, and builds the next State from the output with the
    shim's dtypes (float32 bullets at a game's first tick, float32 planets
    for a lone planet) -- or (None, int64 reward) on a collision."""
    import numpy as np
    from astro_amd import core
    from astro_amd.config import Bodies, State
    gs = core._gamestep
    if gs is None:
        import __graft_entry__ as g
        g.build_gamestep()
        from astro_amd import _gamestep as gs
    S, P, B = 2, 4, 8
    t = _lib.AstroGameTick()
    t.params = _lib.AstroParams(nships=S, solo=0, p_pad=P, max_planets=P, b_cap=B)
    inbuf, outbuf = np.zeros(5 * S + 4 * P + 4 * B), np.zeros(5 * S + 4 * P + 4 * B)
    t.in_ = inbuf.__array_interface__['data'][0]
    t.out = outbuf.__array_interface__['data'][0]
    seen = {}

    @ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p)
    def tick(ptr):   # the next state = the input + 1, two bullets fewer
        r = _lib.AstroGameTick.from_address(ptr)
        seen.update(np=r.nplanets, nb=r.nbullets, c=(r.control0, r.control1), first=r.first_step, fire=r.fire_now,
                    timeout=r.timeout_now)
        n = 5 * S + 4 * (r.nplanets + r.nbullets)
        outbuf[:n] = inbuf[:n] + 1
        r.out_nbullets = r.nbullets
        r.done_out = 0
        return 0
    fn = ctypes.cast(tick, ctypes.c_void_p).value
    f32 = np.float32
    st = State(Bodies(np.arange(4, dtype=f32).reshape(2, 2), np.zeros((2, 2), f32), np.array([0.5, 1.5], f32)),
               Bodies(np.ones((1, 2), f32), np.zeros((1, 2), f32), None),
               Bodies(np.zeros((3, 2), f32), np.full((3, 2), 2, f32), None), 0.0, 0.0)
    new, rw = gs.step(ctypes.addressof(t), fn, st, 3, 4, 0.01, 0.005, 1.0, State, Bodies)
    assert seen == dict(np=1, nb=3, c=(3, 4), first=1, fire=1, timeout=0)
    assert new.ships.x.dtype == np.float64 and np.array_equal(new.ships.x, st.ships.x + 1)
    assert np.array_equal(new.ships.b, st.ships.b + 1) and new.ships.b.shape == (2,)
    assert new.planets.x.dtype == np.float32 and new.planets.b is None      # a lone planet stays float32
    assert new.bullets.x.dtype == np.float32 and new.bullets.x.shape == (3, 2)   # first tick: float32 bullets
    assert np.array_equal(new.bullets.dx, st.bullets.dx + 1)
    assert new.reload == 0.0 + 0.01 - 0.005 and new.t == 0.01 and type(new.t) is float
    assert rw.dtype == np.float32 and not rw.any()
    # float64 state, two planets: float64 out; a non-contiguous array -> the Python path
    st2 = new._replace(ships=new.ships._replace(x=np.asfortranarray(np.ones((2, 3)))[:, :2]))
    assert gs.step(ctypes.addressof(t), fn, st2, 0, 0, 0.01, 0.005, 1.0, State, Bodies) is NotImplemented

    @ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p)
    def hit(ptr):
        r = _lib.AstroGameTick.from_address(ptr)
        r.done_out, r.reward_out[0], r.reward_out[1] = 1, -1.0, 1.0
        return 0
    none, rw = gs.step(ctypes.addressof(t), ctypes.cast(hit, ctypes.c_void_p).value, new, 0, 0, 0.01, 0.005, 1.0,
                       State, Bodies)
    assert none is None and rw.dtype == np.int64 and list(rw) == [-1, 1]

    @ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p)
    def bad(ptr):
        return -90
    assert gs.step(ctypes.addressof(t), ctypes.cast(bad, ctypes.c_void_p).value, new, 0, 0, 0.01, 0.005, 1.0,
                   State, Bodies) == -90


def test_exact_fmod_identity():
    """The kernel's exact_fmod (astro_kernels.hip, used by util.norm_angle on
    the device): q = trunc(fl(x / y)), r = fma(-q, y, x), then +-y when r
    has the other sign than x.  With exact rationals: x - q*y is exactly
    representable (so the fma returns it), the corrected sum is exactly
    representable (so the add returns it), and the result is np.fmod's,
    for float64 and float32, on random bearings and on x next to multiples
    of 2 pi (where x / y rounds up to an integer)."""
    from fractions import Fraction
    rng = np.random.RandomState(7)
    for dt in (np.float64, np.float32):
        y = dt(6.283185307179586)
        xs = list(rng.uniform(-3e4, 3e4, 4000).astype(dt))
        for k in range(-400, 400):
            m = dt(k) * y
            xs += [np.nextafter(m, dt(np.inf)), np.nextafter(m, dt(-np.inf)), m]
        fy = Fraction(float(y))
        for x in xs:
            x = dt(x)
            q = np.trunc(dt(x / y))                           # correctly rounded division, trunc
            exact = Fraction(float(x)) - Fraction(float(q)) * fy
            r = dt(float(exact))
            assert Fraction(float(r)) == exact, (dt, x)       # the fma is exact
            if (x >= 0 and r < 0) or (x < 0 and r > 0):
                s_exact = exact + (fy if x >= 0 else -fy)
                r = dt(float(s_exact))
                assert Fraction(float(r)) == s_exact, (dt, x)  # the correction is exact
            want = np.fmod(x, y)
            assert r == want, (dt, x, r, want)


def test_shim_cache_clear_drops_the_fast_path():
    """Emptying the single-game shim cache (clear_shims, or any clear/pop/
    del on it) also drops the per-tick fast path (_LAST), so a cleared
    shim's arena is never used again."""
    from astro_amd import core
    saved = dict(core._ENVS)
    try:
        for drop in (lambda c: c.clear(), lambda c: c.pop('k'), lambda c: c.__delitem__('k'), lambda c: c.popitem()):
            core._ENVS['k'] = object()
            core._LAST = ('cfg', 0, object(), core._ENVS)
            drop(core._ENVS)
            assert core._LAST == (None, None, None, None)
        core._LAST = ('cfg', 0, object(), core._ENVS)
        core.clear_shims()
        assert core._LAST == (None, None, None, None) and not core._ENVS
    finally:
        core._ENVS.update(saved)
