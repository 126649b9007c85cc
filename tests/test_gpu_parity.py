"""HIP kernel parity: libastro_hip.so (via BatchedEnv) vs the reference's
golden outputs and vs the CPU oracle.  Needs an MI355X.

Bars
  * float64 state: bit-exact to the reference (create, teacher-forced steps,
    whole free-running games).
  * float32 state: every stored value == float32(reference value computed
    from the same float32 input state); integer flags/counts/done exact.
"""
import numpy as np
import pytest
import torch

from oracle import batched
from tests import golden_io as gio

pytestmark = pytest.mark.gpu

CFG = gio.configs()


KERNELS = ['lane', 'quad', 'pair']
# True: the one-tick instances that count (stats rows); False: the same
# instances built without the counters -- what a caller passing no stats
# buffer runs, and what bench.py times and the single-game shim runs
STATS = [False, True]


def _env(cfg, n, dtype=torch.float64, b_cap=64, p_pad=8, auto_reset=False, kernel='auto'):
    from astro_amd import BatchedEnv
    return BatchedEnv(cfg, n, device='cuda:0', b_cap=b_cap, p_pad=p_pad, dtype=dtype,
                      auto_reset=auto_reset, kernel=kernel)


def _host_batch(env):
    h = env.to_host()
    return batched.Batch(h['tick'].astype(np.int32), h['nplanets'].astype(np.int32),
                         h['nbullets'].astype(np.int32), h['ships'].astype(np.float64),
                         h['ships_b'].astype(np.float64), h['planets'].astype(np.float64),
                         h['bullets'].astype(np.float64), (h['flags'] & 1).astype(bool))


def _assert_same(tag, got, want, run, rounding):
    """got: Batch from the GPU; want: oracle/reference Batch (float64 values)."""
    r = (lambda a: a.astype(np.float32).astype(np.float64)) if rounding else (lambda a: a)
    assert (got.nbullets[run] == want.nbullets[run]).all(), tag
    assert (got.tick[run] == want.tick[run]).all(), tag
    assert np.array_equal(got.ships[run], r(want.ships[run])), tag
    assert np.array_equal(got.ships_b[run], r(want.ships_b[run])), tag
    pv = (np.arange(got.planets.shape[1])[None, :] < got.nplanets[:, None]) & run[:, None]
    assert np.array_equal(got.planets[pv], r(want.planets[pv])), tag
    bv = (np.arange(got.bullets.shape[1])[None, :] < got.nbullets[:, None]) & run[:, None]
    assert np.array_equal(got.bullets[bv], r(want.bullets[bv])), tag


# ------------------------------------------------------------------- create

@pytest.mark.parametrize('dtype', [torch.float64, torch.float32])
@pytest.mark.parametrize('name', sorted(CFG))
def test_create_matches_reference(name, dtype):
    z = gio.load('create.npz')
    cfg = CFG[name]
    seeds = z[name + '__seed']
    env = _env(cfg, seeds.size, dtype=dtype, b_cap=4)
    env.reset(seeds=seeds)
    h = env.to_host()
    S = env.S
    npl = z[name + '__nplanets']
    assert (h['nplanets'] == npl).all() and (h['tick'] == 0).all() and (h['nbullets'] == 0).all()
    assert np.array_equal(h['ships'][..., 0:2].astype(np.float32), z[name + '__ships_x'][:, :S])
    assert not h['ships'][..., 2:4].any()
    assert np.array_equal(h['ships_b'].astype(np.float32), z[name + '__ships_b'][:, :S])
    pv = np.arange(8)[None, :] < npl[:, None]
    assert np.array_equal(h['planets'][..., 0:2][pv].astype(np.float32), z[name + '__planets_x'][pv])
    want_dx = z[name + '__planets_dx'][pv]
    if dtype == torch.float32:
        want_dx = want_dx.astype(np.float32)
    assert np.array_equal(h['planets'][..., 2:4][pv], want_dx)
    assert (env.game_seed.cpu().numpy().view(np.uint32) == seeds).all()


def test_seed_streams_follow_generate_configs():
    """Env i's k-th game seed == k-th config of
    generate_configs(config._replace(seed=stream_seed_i)) (core.py:77-83)."""
    cfg = CFG['default']
    env = _env(cfg, 300, dtype=torch.float32)
    ss = batched.stream_seeds(cfg.seed, 300)
    assert (env.stream_seeds == ss).all()
    want = batched.game_seeds(ss, 5)
    for k in range(5):
        env.reset()
        assert (env.game_seed.cpu().numpy().view(np.uint32) == want[:, k]).all()


@pytest.mark.parametrize('stats', STATS)
@pytest.mark.parametrize('kernel', KERNELS)
@pytest.mark.parametrize('fast_end', [False, True])
def test_planets_only_streams(kernel, fast_end, stats):
    """planets_only=3 (BASELINE.json's "3 planets" workloads): every game an
    env plays, through reset() and auto-reset alike, is the next seed of its
    generate_configs stream whose create() draws 3 planets, and the game is
    that seed's reference game (bit-exact vs the oracle's create + step).
    fast_end: huge planets end most games at their first step, before any
    step has checked the next pending seed -- the resets' own seed walk."""
    cfg = CFG['default']
    if fast_end:
        cfg = cfg._replace(planet_radius=0.45)
    P = batched.make_params(cfg)
    n, ticks = 1000, 150 if not fast_end else 25
    from astro_amd import BatchedEnv
    env = BatchedEnv(cfg, n, device='cuda:0', b_cap=32, planets_only=3, kernel=kernel)
    env.reset()
    seeds = batched.filtered_game_seeds(env.stream_seeds, 12 if not fast_end else 30, 3, cfg.max_planets, draws=220)
    assert (env.game_seed.cpu().numpy().view(np.uint32) == seeds[:, 0]).all()
    games = np.ones(n, np.int64)
    rng = np.random.RandomState(2)
    for t in range(ticks):
        B = _host_batch(env)
        assert (B.nplanets == 3).all(), t
        ctl = rng.randint(0, 6, size=(n, 2)).astype(np.int8)
        want, wrew, wdone = batched.step(B, ctl, P, store='f32')
        fin = np.nonzero(wdone)[0]
        if fin.size:
            fresh = batched.create(seeds[fin, games[fin]], P, p_pad=env.p_pad, b_cap=32, store='f32')
            want.put(fin, fresh)
            games[fin] += 1
        _, rew, done = env.step(torch.from_numpy(ctl).cuda(), stats=stats)
        assert (done.cpu().numpy() == wdone).all(), t
        assert np.array_equal(rew.cpu().numpy(), wrew), t
        got = _host_batch(env)
        _assert_same('planets_only t=%d' % t, got, want, np.ones(n, bool), rounding=True)
        assert (env.game_seed.cpu().numpy().view(np.uint32) == seeds[np.arange(n), games - 1]).all(), t
    assert games.max() > 2


@pytest.mark.parametrize('stats', STATS)
@pytest.mark.parametrize('kernel', KERNELS)
def test_config2_exact_vs_oracle(kernel, stats):
    """BASELINE.json config 2 as bench.py runs it: 4,096 envs,
    DEFAULT_CONFIG with reload_time=1000 (no bullets), 2 ships, games
    filtered to 3 planets, auto-reset -- 200 ticks, every tick equal to the
    oracle stepped from the kernel's own float32 input state, every new game
    the oracle's create() of the stream's next 3-planet seed."""
    cfg = CFG['default']._replace(reload_time=1000)
    P = batched.make_params(cfg)
    n, ticks = 4096, 200
    from astro_amd import BatchedEnv
    env = BatchedEnv(cfg, n, device='cuda:0', b_cap=32, p_pad=4, planets_only=3, kernel=kernel)
    env.reset()
    seeds = batched.filtered_game_seeds(env.stream_seeds, 16, 3, cfg.max_planets, draws=220)
    games = np.ones(n, np.int64)
    rng = np.random.RandomState(22)
    for t in range(ticks):
        B = _host_batch(env)
        assert (B.nplanets == 3).all() and (B.nbullets == 0).all(), t
        ctl = rng.randint(0, 6, size=(n, 2)).astype(np.int8)
        want, wrew, wdone = batched.step(B, ctl, P, store='f32')
        fin = np.nonzero(wdone)[0]
        if fin.size:
            want.put(fin, batched.create(seeds[fin, games[fin]], P, p_pad=env.p_pad, b_cap=32, store='f32'))
            games[fin] += 1
        _, rew, done = env.step(torch.from_numpy(ctl).cuda(), stats=stats)
        assert (done.cpu().numpy() == wdone).all(), t
        assert np.array_equal(rew.cpu().numpy(), wrew), t
        _assert_same('c2 t=%d' % t, _host_batch(env), want, np.ones(n, bool), rounding=True)
    assert games.max() > 1
    st = env.stat_dict()
    if stats:
        assert st['bullets_in'] == 0 and st['resets'] == int((games - 1).sum()) > 0
    else:   # (the counter-free instance leaves the stats rows alone)
        assert not any(st.values())


# ------------------------------------------------- teacher-forced transitions

@pytest.mark.parametrize('stats', STATS)
@pytest.mark.parametrize('kernel', KERNELS)
@pytest.mark.parametrize('dtype', [torch.float64, torch.float32])
@pytest.mark.parametrize('fname', ['steps.npz', 'edge_steps.npz'])
def test_step_teacher_forced_vs_reference(fname, dtype, kernel, stats):
    tr = gio.Transitions(fname)
    for name, idx in tr.groups():
        cfg = CFG[name]
        S = 1 if cfg.solo else 2
        bcap = tr.max_bullets(idx) + 2
        B = tr.batch_in(idx, S, b_cap=bcap)
        env = _env(cfg, idx.size, dtype=dtype, b_cap=bcap, kernel=kernel)
        env.load_host(B.ships, B.ships_b, B.planets, B.bullets, B.tick, B.nplanets, B.nbullets)
        ctl = tr.z['control'][idx, :S].astype(np.int8)
        _, rew, done = env.step(torch.from_numpy(ctl).cuda(), auto_reset=False, stats=stats)
        E, erew, edone = tr.expected(idx, S, b_cap=bcap)
        done = done.cpu().numpy()
        assert (done == edone).all(), name
        assert np.array_equal(rew.cpu().numpy(), erew.astype(np.float32)), name
        _assert_same('%s/%s' % (fname, name), _host_batch(env), E, done == 0,
                     rounding=dtype == torch.float32)


@pytest.mark.parametrize('kernel', KERNELS)
@pytest.mark.parametrize('dtype', [torch.float64, torch.float32])
def test_planets_only_handmade_states(dtype, kernel):
    """With planets_only=3 the step kernels do not read planet slots >= 3 (a
    filtered game never has a planet there); a hand-made state that does --
    here the reference's own 1-4 planet transitions -- must still step
    exactly: the kernel reads those slots once the header says so."""
    tr = gio.Transitions('steps.npz')
    idx = [i for name, i in tr.groups() if name == 'default'][0]
    cfg = CFG['default']
    bcap = tr.max_bullets(idx) + 2
    B = tr.batch_in(idx, 2, p_pad=4, b_cap=bcap)
    assert (B.nplanets == 4).any() and (B.nplanets < 4).any()
    from astro_amd import BatchedEnv
    env = BatchedEnv(cfg, idx.size, device='cuda:0', b_cap=bcap, p_pad=4, dtype=dtype, auto_reset=False,
                     kernel=kernel, planets_only=3)
    env.load_host(B.ships, B.ships_b, B.planets, B.bullets, B.tick, B.nplanets, B.nbullets)
    ctl = tr.z['control'][idx, :2].astype(np.int8)
    _, rew, done = env.step(torch.from_numpy(ctl).cuda(), auto_reset=False)
    E, erew, edone = tr.expected(idx, 2, p_pad=4, b_cap=bcap)
    done = done.cpu().numpy()
    assert (done == edone).all()
    assert np.array_equal(rew.cpu().numpy(), erew.astype(np.float32))
    _assert_same('planets_only handmade', _host_batch(env), E, done == 0, rounding=dtype == torch.float32)


# ------------------------------------------------------- free-running games

@pytest.mark.parametrize('kernel', KERNELS)
def test_whole_games_float64_bit_exact(kernel):
    """Every golden game replayed from create(seed) with its open-loop
    controls: every tick's ship state, bullet count, the game length and the
    outcome match the reference bit for bit."""
    games = gio.games()
    by_cfg = {}
    for g in games:
        by_cfg.setdefault(g['cfg'], []).append(g)
    for name, gs in by_cfg.items():
        cfg = CFG[name]
        S = 1 if cfg.solo else 2
        env = _env(cfg, len(gs), dtype=torch.float64, b_cap=512, kernel=kernel)
        env.reset(seeds=np.array([g['seed'] for g in gs], dtype=np.uint32))
        T = max(g['ships'].shape[0] for g in gs)
        alive = np.ones(len(gs), bool)
        for t in range(T):
            h = env.to_host()
            for k, g in enumerate(gs):
                if alive[k]:
                    assert np.array_equal(h['ships'][k], g['ships'][t, :S, 0:4]), (name, g['gid'], t)
                    assert np.array_equal(h['ships_b'][k], g['ships'][t, :S, 4]), (name, g['gid'], t)
                    assert h['nbullets'][k] == g['nbullets'][t], (name, g['gid'], t)
            ctl = np.full((len(gs), S), 2, np.int8)
            for k, g in enumerate(gs):
                if alive[k]:
                    ctl[k] = g['controls'][t]
            _, rew, done = env.step(torch.from_numpy(ctl).cuda(), auto_reset=False)
            done = done.cpu().numpy()
            rew = rew.cpu().numpy()
            for k, g in enumerate(gs):
                if not alive[k]:
                    continue
                last = t == g['ships'].shape[0] - 1
                assert bool(done[k]) == last, (name, g['gid'], t)
                if last:
                    assert done[k] == g['done'] and np.array_equal(rew[k], g['reward'][:S])
                    alive[k] = False
        assert not alive.any()


# ----------------------------------------- batched run vs oracle, auto-reset

@pytest.mark.parametrize('stats', STATS)
@pytest.mark.parametrize('kernel', KERNELS)
@pytest.mark.parametrize('name,n,ticks,bcap', [('default', 4096, 60, 32), ('mp8', 2000, 40, 32),
                                              ('rapid', 517, 30, 6), ('solo', 701, 40, 32),
                                              ('rapid', 77, 70, 100)])
def test_batched_auto_reset_vs_oracle(name, n, ticks, bcap, kernel, stats):
    """N envs with auto-reset, float32 state: every tick equals the oracle
    stepped from the kernel's own input state, resets draw the right seeds
    and create the right games, overflow (small b_cap) is counted alike.
    stats=False: the counter-free build, the one bench.py times."""
    _auto_reset_vs_oracle(CFG[name], name, n, ticks, bcap, kernel, stats)


@pytest.mark.parametrize('kernel', KERNELS)
def test_irregular_fire_schedule(kernel):
    """A config whose fire schedule is not periodic (reload_time 0.33: the
    host's float64 reload recurrence, core.py:262-280, fires on ticks 1, 2,
    4, 5, ... not every k-th) against the oracle."""
    from astro_amd import schedule
    cfg = CFG['default']._replace(reload_time=0.33)
    k = np.nonzero(schedule.build(cfg).fire)[0]
    assert len(set(np.diff(k[:200]).tolist())) > 1
    _auto_reset_vs_oracle(cfg, 'reload0.33', 600, 60, 32, kernel)


def _auto_reset_vs_oracle(cfg, name, n, ticks, bcap, kernel, stats=True):
    P = batched.make_params(cfg)
    env = _env(cfg, n, dtype=torch.float32, b_cap=bcap, auto_reset=True, kernel=kernel)
    env.reset()
    seeds = batched.game_seeds(env.stream_seeds, 64)
    games = np.ones(n, np.int64)          # game 0 was created by reset()
    rng = np.random.RandomState(1)
    max_wave_bullets = 0   # live bullets of 16 consecutive envs (a quad-kernel wave) at a step's start
    saw_overflow = False
    for t in range(ticks):
        B = _host_batch(env)
        ctl = rng.randint(0, 6, size=(n, env.S)).astype(np.int8)
        want, wrew, wdone = batched.step(B, ctl, P, store='f32')
        fin = np.nonzero(wdone)[0]
        if fin.size:
            fresh = batched.create(seeds[fin, games[fin]], P, p_pad=env.p_pad, b_cap=bcap, store='f32')
            want.put(fin, fresh)
            games[fin] += 1
        _, rew, done = env.step(torch.from_numpy(ctl).cuda(), stats=stats)
        done = done.cpu().numpy()
        assert (done == wdone).all(), t
        assert np.array_equal(rew.cpu().numpy(), wrew), t
        got = _host_batch(env)
        _assert_same('%s t=%d' % (name, t), got, want, np.ones(n, bool), rounding=True)
        assert (got.overflow == want.overflow).all(), t
        saw_overflow |= bool(want.overflow.any())
        nb16 = np.pad(B.nbullets, (0, -n % 16)).reshape(-1, 16).sum(1)
        max_wave_bullets = max(max_wave_bullets, int(nb16.max()))
    assert games.max() > 1
    st = env.stat_dict()
    if stats:
        assert st['resets'] == int((games - 1).sum())
    else:   # (the counter-free instance leaves the stats rows alone)
        assert not any(st.values())
    if name == 'rapid' and bcap < 10:
        assert saw_overflow and (st['overflows'] > 0 or not stats)
    if bcap > 64:   # the quad kernel indexes a wave's bullets in windows of 1024
        assert max_wave_bullets > 1024


# ------------------------------------------------------- shapes / edge cases

@pytest.mark.parametrize('kernel', KERNELS)
@pytest.mark.parametrize('n', [1, 15, 17, 63, 65, 1000])
def test_ragged_env_counts(n, kernel):
    cfg = CFG['default']
    env = _env(cfg, n, dtype=torch.float32, b_cap=32, auto_reset=True, kernel=kernel)
    env.reset()
    P = batched.make_params(cfg)
    B = _host_batch(env)
    ctl = np.random.RandomState(n).randint(0, 6, size=(n, 2)).astype(np.int8)
    want, wrew, wdone = batched.step(B, ctl, P, store='f32')
    _, rew, done = env.step(torch.from_numpy(ctl).cuda(), auto_reset=False)
    assert (done.cpu().numpy() == wdone).all()
    _assert_same('n=%d' % n, _host_batch(env), want, wdone == 0, rounding=True)


@pytest.mark.parametrize('kernel', KERNELS)
def test_zero_envs_is_a_noop(kernel):
    cfg = CFG['default']
    env = _env(cfg, 0, dtype=torch.float32, kernel=kernel)
    env.reset()
    env.step(torch.zeros((0, 2), dtype=torch.int8, device='cuda'))
    torch.cuda.synchronize()


def test_bad_arguments_raise():
    from astro_amd import _lib
    cfg = CFG['default']
    env = _env(cfg, 8, dtype=torch.float32)
    with pytest.raises(ValueError):
        env.step(torch.zeros((8, 3), dtype=torch.int8, device='cuda'))
    bad = type(env.params).from_buffer_copy(env.params)
    bad.nships = 3
    env.params, good = bad, env.params
    with pytest.raises(_lib.AstroError):
        env.step(torch.zeros((8, 2), dtype=torch.int8, device='cuda'))
    env.params = good


# ------------------------------------------------ size-independent properties

def test_full_size_determinism_and_shard_invariance():
    """65,536 envs (BASELINE config 3): two identical runs agree bit for bit,
    and two half-size shards with global env ids reproduce the full run."""
    cfg = CFG['default']
    n, ticks = 65536, 200
    g = torch.Generator(device='cuda').manual_seed(0)
    ctls = torch.randint(0, 6, (ticks, n, 2), generator=g, device='cuda', dtype=torch.int8)

    def run(offset, count, kernel='auto'):
        from astro_amd import BatchedEnv
        env = BatchedEnv(cfg, count, device='cuda:0', b_cap=32, env_offset=offset, kernel=kernel)
        env.reset()
        for t in range(ticks):
            env.step(ctls[t, offset:offset + count].contiguous())
        return env
    a = run(0, n)
    b = run(0, n)
    c = run(0, n, kernel='lane')
    d = run(0, n, kernel='quad')
    e = run(0, n, kernel='pair')
    for f in ('ships', 'ships_b', 'planets', 'bullets', 'hdr', 'stream'):
        assert torch.equal(getattr(a, f), getattr(e, f)), f
    for f in ('ships', 'ships_b', 'planets', 'bullets', 'hdr', 'stream'):
        assert torch.equal(getattr(a, f), getattr(c, f)), f
        assert torch.equal(getattr(a, f), getattr(d, f)), f
    for f in ('ships', 'ships_b', 'planets', 'bullets', 'hdr', 'stream'):
        assert torch.equal(getattr(a, f), getattr(b, f)), f
    lo = run(0, n // 2)
    hi = run(n // 2, n // 2)
    assert torch.equal(torch.cat([lo.hdr, hi.hdr]), a.hdr)
    assert torch.equal(torch.cat([lo.stream, hi.stream]), a.stream)
    assert torch.equal(torch.cat([lo.ships, hi.ships], 1), a.ships)
    nb = a.nbullets
    assert int(nb.max()) <= 32 and int(a.nplanets.min()) >= 1 and int(a.nplanets.max()) <= 4
    st = a.stat_dict()
    assert st['resets'] == st['collisions'] + st['timeouts'] > 0


def test_config4_eight_shards_compose():
    """BASELINE.json config 4's sharding on one GPU: 8 BatchedEnv shards of
    65,536 envs (env_offset = rank * 65,536, as bench.py's ranks) stepped
    200 ticks equal one 524,288-env run bit for bit -- headers, stream
    cursors and rings, ships, planets, bullets.  (The shards' launches, two
    step waves per SIMD, create their finished games' next ones on helper
    waves -- HelpBox in the kernel -- the full run's step waves create their
    own: the two paths must agree.)"""
    cfg = CFG['default']
    n, G, ticks = 65536, 8, 200
    from astro_amd import BatchedEnv
    g = torch.Generator(device='cuda').manual_seed(4)
    ctls = torch.randint(0, 6, (ticks, n * G, 2), generator=g, device='cuda', dtype=torch.int8)
    full = BatchedEnv(cfg, n * G, device='cuda:0', b_cap=32, p_pad=4, planets_only=3)
    full.reset()
    for t in range(ticks):
        full.step(ctls[t])
    for r in range(G):
        env = BatchedEnv(cfg, n, device='cuda:0', b_cap=32, p_pad=4, planets_only=3, env_offset=r * n)
        env.reset()
        for t in range(ticks):
            env.step(ctls[t, r * n:(r + 1) * n].contiguous())
        sl = slice(r * n, (r + 1) * n)
        assert torch.equal(env.hdr, full.hdr[sl]), r
        assert torch.equal(env.stream, full.stream[sl]), r
        assert torch.equal(env.stream_ring, full.stream_ring[sl]), r
        assert torch.equal(env.ships, full.ships[:, sl]), r
        assert torch.equal(env.ships_b, full.ships_b[:, sl]), r
        assert torch.equal(env.planets, full.planets[:, sl]), r
        assert torch.equal(env.bullets, full.bullets[sl]), r
        del env
    assert int(full.stat_dict()['resets']) > 0


def test_config5_full_size_instances_agree():
    """BASELINE config 5 per GPU exactly as bench.py's c5 runs it: 131,072
    envs, max_planets 8 (1-8 planets, p_pad 8), bullets on, auto-reset, 200
    ticks.  The instance the bench times -- AUTO = pair kernel WITHOUT helper
    waves (4,096 step waves, more than two per SIMD) -- equals two 65,536-env
    shards (pair kernel WITH helper waves) and the lane kernel, bit for bit,
    on every array (headers, stream cursors and rings, ships, planets,
    bullets).  (create() draws the planet count from the seed's first word,
    core.py:90: the batch holds every count 1..8.)"""
    from astro_amd import BatchedEnv
    cfg = CFG['default']._replace(max_planets=8)
    n, ticks = 131072, 200
    g = torch.Generator(device='cuda').manual_seed(5)
    ctls = torch.randint(0, 6, (ticks, n, 2), generator=g, device='cuda', dtype=torch.int8)

    def run(offset, count, kernel='auto'):
        env = BatchedEnv(cfg, count, device='cuda:0', b_cap=32, p_pad=8, env_offset=offset, kernel=kernel)
        env.reset()
        for t in range(ticks):
            env.launch(ctls[t, offset:offset + count].contiguous().data_ptr())
        torch.cuda.synchronize()
        env.check_errors()
        return env
    full = run(0, n)
    assert full.step_kernel == 'pair' and full.launch_waves() == (4096, 0)
    np_ = full.nplanets
    assert int(np_.min()) == 1 and int(np_.max()) == 8
    st = full.stat_dict()
    assert st['resets'] > 10000 and st['bullets_in'] > 0
    arrays = ('hdr', 'stream', 'stream_ring', 'bullets')      # [N, ...]
    slot_major = ('ships', 'ships_b', 'planets')              # [slot, N, ...]
    for r in range(2):
        half = run(r * (n // 2), n // 2)
        assert half.launch_waves() == (2048, 2048)
        sl = slice(r * (n // 2), (r + 1) * (n // 2))
        for f in arrays:
            assert torch.equal(getattr(half, f), getattr(full, f)[sl]), (r, f)
        for f in slot_major:
            assert torch.equal(getattr(half, f), getattr(full, f)[:, sl]), (r, f)
        del half
    lane = run(0, n, kernel='lane')
    for f in arrays + slot_major:
        assert torch.equal(getattr(lane, f), getattr(full, f)), f


@pytest.mark.parametrize('stats', STATS)
@pytest.mark.parametrize('kernel', KERNELS)
@pytest.mark.parametrize('tick', [0, 7])
def test_near_threshold_collisions_exact(tick, kernel, stats):
    """Bodies placed within +-2e-4 (relative) of every collision threshold
    (ship-ship, ship-planet, ship-bullet, bullet-planet), at tick 0 (float32
    distances) and later (float64): hit flags, rewards and bullet survival
    equal the oracle's exactly -- the kernel's float32 prefilter + guard band
    must never decide a case the exact arithmetic decides differently."""
    cfg = CFG['default']
    P = batched.make_params(cfg)
    n, bcap = 4096, 8
    rng = np.random.RandomState(11 + tick)
    B = batched.Batch.zeros(n, 2, 4, bcap)
    B.tick[:] = tick
    B.nplanets[:] = rng.randint(1, 5, n)
    B.planets[..., 0:2] = rng.uniform(-0.6, 0.6, (n, 4, 2))
    B.planets[..., 2:4] = rng.uniform(-0.1, 0.1, (n, 4, 2))
    B.ships[..., 0:2] = rng.uniform(-0.9, 0.9, (n, 2, 2))
    B.ships[..., 2:4] = rng.uniform(-0.2, 0.2, (n, 2, 2))
    B.ships_b[:] = rng.uniform(-7, 7, (n, 2))

    def around(c, r2):
        ang = rng.uniform(0, 2 * np.pi, c.shape[:-1])
        rad = np.sqrt(r2) * (1 + rng.uniform(-2e-4, 2e-4, c.shape[:-1]))
        return c + np.stack([np.cos(ang), np.sin(ang)], -1) * rad[..., None]
    kind = rng.randint(0, 3, n)
    # ship 0 near planet 0 / near ship 1 / free
    B.ships[kind == 0, 0, 0:2] = around(B.planets[kind == 0, 0, 0:2], P.r2_sp)
    B.ships[kind == 1, 0, 0:2] = around(B.ships[kind == 1, 1, 0:2], P.r2_ss)
    nb = rng.randint(0, bcap + 1, n)
    B.nbullets[:] = nb
    for k in range(bcap):
        tgt = rng.randint(0, 2, n)
        c = np.where(tgt[:, None] == 0, B.planets[:, 0, 0:2], B.ships[:, 1, 0:2])
        r2 = np.where(tgt == 0, P.r2_p0, P.r2_s0)
        B.bullets[:, k, 0:2] = around(c, r2)
        B.bullets[:, k, 2:4] = rng.uniform(-1.5, 1.5, (n, 2))
    for f in ('ships', 'ships_b', 'planets', 'bullets'):
        a = getattr(B, f)
        a[:] = a.astype(np.float32).astype(np.float64)
    env = _env(cfg, n, dtype=torch.float32, b_cap=bcap, p_pad=4, kernel=kernel)
    env.load_host(B.ships, B.ships_b, B.planets, B.bullets, B.tick, B.nplanets, B.nbullets)
    ctl = rng.randint(0, 6, size=(n, 2)).astype(np.int8)
    want, wrew, wdone = batched.step(B, ctl, P, store='f32')
    _, rew, done = env.step(torch.from_numpy(ctl).cuda(), auto_reset=False, stats=stats)
    done = done.cpu().numpy()
    assert (done == wdone).all()
    assert np.array_equal(rew.cpu().numpy(), wrew)
    _assert_same('near-threshold tick=%d' % tick, _host_batch(env), want, wdone == 0, rounding=True)
    assert 0.05 < (wdone == 1).mean() < 0.95   # both outcomes well represented


def test_key_table_matches_mt_init_chain():
    """The device seeding table holds key[397] of init_genrand for every
    30-bit seed: spot-check against the oracle's MT19937 restatement."""
    from astro_amd.env import key_table
    from oracle import mt19937
    t = key_table('cuda:0')
    rng = np.random.RandomState(3)
    seeds = np.concatenate([[0, 1, 42, (1 << 30) - 1], rng.randint(0, 1 << 30, 2000)]).astype(np.uint64)
    want = mt19937.init_genrand(seeds)[:, 397].astype(np.uint32)
    got = t[torch.from_numpy(seeds.astype(np.int64)).cuda()].cpu().numpy().view(np.uint32)
    assert (got == want).all()


@pytest.mark.parametrize('kernel', KERNELS)
def test_without_key_table_identical(kernel):
    """use_key_table=False (inline 397-step chains) gives the same games."""
    from astro_amd import BatchedEnv
    cfg = CFG['default']
    n, ticks = 2048, 120
    g = torch.Generator(device='cuda').manual_seed(5)
    ctls = torch.randint(0, 6, (ticks, n, 2), generator=g, device='cuda', dtype=torch.int8)
    envs = [BatchedEnv(cfg, n, device='cuda:0', use_key_table=u, kernel=kernel) for u in (True, False)]
    for e in envs:
        e.reset()
        for t in range(ticks):
            e.step(ctls[t])
    for f in ('ships', 'ships_b', 'planets', 'bullets', 'stream'):
        assert torch.equal(getattr(envs[0], f), getattr(envs[1], f)), f
    assert torch.equal(envs[0].hdr[:, 1], envs[1].hdr[:, 1])
    assert envs[0].stat_dict()['resets'] > 0


# ------------------------------------------------- observation features

@pytest.mark.parametrize('dtype', [torch.float64, torch.float32])
def test_features_match_reference(dtype):
    """astro_features on every golden input state == rl.ValueNetwork
    .get_features of the reference, bit for bit (float32 state: the golden
    inputs are float32-valued, so the stored values are identical), with
    to_batch's -1 padding after each env's objects."""
    tr = gio.Transitions('steps.npz')
    fx = gio.Features()
    for name, idx in tr.groups():
        cfg = CFG[name]
        S = 1 if cfg.solo else 2
        bcap = tr.max_bullets(idx) + 2
        B = tr.batch_in(idx, S, b_cap=bcap)
        env = _env(cfg, idx.size, dtype=dtype, b_cap=bcap)
        env.load_host(B.ships, B.ships_b, B.planets, B.bullets, B.tick, B.nplanets, B.nbullets)
        got = env.features().cpu().numpy()
        assert got.shape == (idx.size, env.p_pad + bcap, 1 + 5 * S + 4)
        for r, i in enumerate(idx):
            want = fx.of(i)
            assert np.array_equal(got[r, :want.shape[0]].view(np.uint32), want.view(np.uint32)), (name, i)
            assert (got[r, want.shape[0]:] == -1).all(), (name, i)


def test_features_batched_run_vs_oracle():
    """Features of a float32 auto-reset run (fresh games at tick 0 every
    step) == the oracle's, each tick; a cut `rows` keeps the first objects."""
    from oracle import features
    cfg = CFG['rapid']
    n = 999
    env = _env(cfg, n, dtype=torch.float32, b_cap=24, p_pad=4, auto_reset=True)
    env.reset()
    rng = np.random.RandomState(5)
    for t in range(25):
        B = _host_batch(env)
        rows = env.p_pad + env.b_cap
        assert np.array_equal(env.features().cpu().numpy(), features.batched(B, env.S, rows)), t
        if t % 8 == 3:
            assert np.array_equal(env.features(rows=5).cpu().numpy(), features.batched(B, env.S, 5)), t
        ctl = rng.randint(0, 6, size=(n, env.S)).astype(np.int8)
        env.step(torch.from_numpy(ctl).cuda())
    out = torch.empty((n, 28, 15), dtype=torch.float32, device='cuda:0')
    assert env.features(out=out) is out
    with pytest.raises(ValueError):
        env.features(out=torch.empty((n, 27, 15), dtype=torch.float32, device='cuda:0'))


# ------------------------------------------------------- K-tick rollouts

@pytest.mark.parametrize('kernel', KERNELS)
@pytest.mark.parametrize('dtype', [torch.float32, torch.float64])
def test_rollout_equals_stepping(kernel, dtype):
    """rollout(K, controls) == K calls of step(controls[k]) bit for bit: every
    state array, reward and done, auto-reset included (the quad kernel runs
    the K ticks in one launch)."""
    cfg = CFG['rapid']
    n, K = 700, 37
    a = _env(cfg, n, dtype=dtype, b_cap=24, p_pad=4, auto_reset=True, kernel=kernel)
    b = _env(cfg, n, dtype=dtype, b_cap=24, p_pad=4, auto_reset=True, kernel=kernel)
    a.reset()
    b.reset()
    ctl = torch.from_numpy(np.random.RandomState(3).randint(0, 6, size=(K, n, 2)).astype(np.int8)).cuda()
    rew, done = a.rollout(K, ctl)
    for k in range(K):
        _, r, d = b.step(ctl[k])
        assert torch.equal(rew[k], r) and torch.equal(done[k], d), k
    for f in ('ships', 'ships_b', 'planets', 'bullets', 'hdr', 'stream'):
        assert torch.equal(getattr(a, f), getattr(b, f)), f
    assert a.stat_dict() == b.stat_dict()


RESIDENT_CASES = {
    # (config, b_cap, p_pad, planets_only, auto_reset, ticks)
    'overflow_no_reset': (CFG['rapid'], 6, 4, 0, False, 30),
    'c3_filtered_long': (CFG['default'], 32, 4, 3, True, 150),
    'eight_slots': (None, 16, 8, 0, True, 60),
    'solo': (CFG['solo'], 8, 4, 0, True, 40),
}


@pytest.mark.parametrize('kernel', ['quad', 'pair'])
@pytest.mark.parametrize('case', sorted(RESIDENT_CASES))
def test_resident_rollout_equals_stepping(kernel, case):
    """The resident rollout (float32 state, b_cap <= 32: the env state held
    on chip for the launch's K ticks) == K astro_step launches bit for bit on
    every state array -- dead bullet slots and padded planet slots included
    -- and the same statistics: with bullets dropped for lack of b_cap and
    no auto-reset (finished games re-stepped), on the 3-planet-filtered c3
    workload long enough for every game's pending-seed checks and draws, and
    with 8 planet slots (1-8 planets)."""
    from astro_amd import BatchedEnv
    cfg, b_cap, p_pad, only, ar, K = RESIDENT_CASES[case]
    if cfg is None:
        cfg = CFG['default']._replace(max_planets=8)
    n = 1500
    envs = [BatchedEnv(cfg, n, device='cuda:0', b_cap=b_cap, p_pad=p_pad, dtype=torch.float32,
                       auto_reset=ar, kernel=kernel, planets_only=only, env_offset=77) for _ in range(2)]
    for e in envs:
        e.reset()
        e.rollout(25, 'random', tick0=1 << 20, auto_reset=True)   # games of several ages first
    a, b = envs
    ctl = torch.from_numpy(np.random.RandomState(11).randint(0, 6, size=(K, n, a.S)).astype(np.int8)).cuda()
    rew, done = a.rollout(K, ctl, auto_reset=ar)
    for k in range(K):
        _, r, d = b.step(ctl[k], auto_reset=ar)
        assert torch.equal(rew[k], r) and torch.equal(done[k], d), k
    for f in ('ships', 'ships_b', 'planets', 'bullets', 'hdr', 'stream', 'stream_ring'):
        assert torch.equal(getattr(a, f), getattr(b, f)), f
    assert a.stat_dict() == b.stat_dict()
    assert int(done.ne(0).sum()) > 0
    if case == 'overflow_no_reset':
        assert int(((a.flags & 1) != 0).sum()) > 0   # bullets were dropped


@pytest.mark.parametrize('kernel', ['quad', 'pair'])
def test_resident_rollout_vs_oracle(kernel):
    """The resident rollout (astro_rollout_res_kernel: float32 state, b_cap
    <= 32, at most 2,048 waves, a control array -- the instance bench.py's
    rollout line runs) on the c3 workload (3-planet filtered streams,
    auto-reset), against the oracle directly: K = 90 ticks in ONE launch,
    free-running numpy ticks (batched.step, float32 stores) with each
    finished env re-created from its stream's next 3-planet seed; every
    tick's reward and done compared, then the whole final state."""
    from astro_amd import BatchedEnv
    cfg = CFG['default']
    P = batched.make_params(cfg)
    n, K = 1000, 90
    env = BatchedEnv(cfg, n, device='cuda:0', b_cap=32, p_pad=4, dtype=torch.float32, auto_reset=True,
                     kernel=kernel, planets_only=3, env_offset=321)
    env.reset()
    seeds = batched.filtered_game_seeds(env.stream_seeds, 8, 3, cfg.max_planets, draws=220)
    assert (env.game_seed.cpu().numpy().view(np.uint32) == seeds[:, 0]).all()
    B = _host_batch(env)             # the oracle's start state
    ctl = np.random.RandomState(6).randint(0, 6, size=(K, n, 2)).astype(np.int8)
    rew, done = env.rollout(K, torch.from_numpy(ctl).cuda(), stats=False)
    rew, done = rew.cpu().numpy(), done.cpu().numpy()
    games = np.ones(n, np.int64)
    for k in range(K):
        B, wrew, wdone = batched.step(B, ctl[k], P, store='f32')
        fin = np.nonzero(wdone)[0]
        if fin.size:
            B.put(fin, batched.create(seeds[fin, games[fin]], P, p_pad=4, b_cap=32, store='f32'))
            games[fin] += 1
        assert (done[k] == wdone).all(), k
        assert np.array_equal(rew[k], wrew), k
    _assert_same('resident rollout, final', _host_batch(env), B, np.ones(n, bool), rounding=True)
    assert (env.game_seed.cpu().numpy().view(np.uint32) == seeds[np.arange(n), games - 1]).all()
    assert games.max() > 2 and int((B.nbullets > 0).sum()) > n // 2


PLAIN_CASES = {
    # (kernel, auto_reset, n_env, p_pad, state dtype): every one-tick quad/pair
    # instance -- with helper waves (auto-reset, <= 2,048 waves) and without
    'quad_helpers': ('quad', True, 1500, 4, torch.float32),
    'pair_helpers': ('pair', True, 1500, 4, torch.float32),
    'pair_helpers_8': ('pair', True, 1500, 8, torch.float32),
    'pair_helpers_f64': ('pair', True, 1500, 4, torch.float64),
    'quad_plain': ('quad', False, 1500, 4, torch.float32),
    'pair_plain_8': ('pair', False, 1500, 8, torch.float32),
    'pair_large_resets': ('pair', True, 70000, 4, torch.float32),
    'quad_large_resets': ('quad', True, 40000, 8, torch.float32),
    'pair_large_8_resets': ('pair', True, 70000, 8, torch.float32),   # config 5's instance
}


@pytest.mark.parametrize('case', sorted(PLAIN_CASES))
def test_plain_instance_equals_counting(case):
    """A launch without a stats buffer runs the one-tick instance built
    without the counters (STATS = false); stepping with it == stepping with
    the counting instance, bit for bit on every state array, reward and done
    (the counting instance is the one the oracle tests check)."""
    from astro_amd import BatchedEnv
    kernel, ar, n, p_pad, dt = PLAIN_CASES[case]
    cfg = CFG['rapid'] if p_pad == 4 else CFG['default']._replace(max_planets=8)
    envs = [BatchedEnv(cfg, n, device='cuda:0', b_cap=24, p_pad=p_pad, dtype=dt, auto_reset=ar, kernel=kernel,
                       env_offset=5) for _ in range(2)]
    for e in envs:
        e.reset()
        e.rollout(20, 'random', tick0=1 << 21, auto_reset=True)   # games of several ages
    a, b = envs
    K = 40
    ctl = torch.from_numpy(np.random.RandomState(17).randint(0, 6, size=(K, n, a.S)).astype(np.int8)).cuda()
    n_done = 0
    for k in range(K):
        _, ra, da = a.step(ctl[k], stats=True)
        _, rb, db = b.step(ctl[k], stats=False)
        assert torch.equal(ra, rb) and torch.equal(da, db), k
        n_done += int(da.ne(0).sum())
    for f in ('ships', 'ships_b', 'planets', 'bullets', 'hdr', 'stream', 'stream_ring'):
        assert torch.equal(getattr(a, f), getattr(b, f)), f
    assert n_done > 0


@pytest.mark.parametrize('kernel', KERNELS)
def test_step_many_equals_stepping(kernel):
    """step_many(controls [K, N, S]) (astro_step_many: K one-tick launches
    issued from C) == K calls of step(controls[k]) bit for bit, auto-reset
    and the helper-wave instance included; K = 0 changes nothing."""
    cfg = CFG['rapid']
    n, K = 700, 23
    a = _env(cfg, n, dtype=torch.float32, b_cap=24, p_pad=4, auto_reset=True, kernel=kernel)
    b = _env(cfg, n, dtype=torch.float32, b_cap=24, p_pad=4, auto_reset=True, kernel=kernel)
    a.reset()
    b.reset()
    ctl = torch.from_numpy(np.random.RandomState(5).randint(0, 6, size=(K, n, 2)).astype(np.int8)).cuda()
    r0, d0 = a.step_many(ctl[:0])
    assert r0.shape == (0, n, 2) and d0.shape == (0, n)
    rew, done = a.step_many(ctl)
    for k in range(K):
        _, r, d = b.step(ctl[k])
        assert torch.equal(rew[k], r) and torch.equal(done[k], d), k
    for f in ('ships', 'ships_b', 'planets', 'bullets', 'hdr', 'stream'):
        assert torch.equal(getattr(a, f), getattr(b, f)), f
    assert a.stat_dict() == b.stat_dict()
    a.check_errors()


@pytest.mark.parametrize('kernel', KERNELS)
def test_rollout_device_policies(kernel):
    """The on-device RANDOM policy draws bench.py's controls (global env id,
    tick); NOTHING is script.NothingBot's constant 2."""
    import bench
    cfg = CFG['default']
    n, K, off = 513, 12, 1000
    from astro_amd import BatchedEnv
    a = BatchedEnv(cfg, n, device='cuda:0', b_cap=32, env_offset=off, kernel=kernel)
    b = BatchedEnv(cfg, n, device='cuda:0', b_cap=32, env_offset=off, kernel=kernel)
    a.reset()
    b.reset()
    rew, done = a.rollout(K, 'random', seed=0, tick0=5)
    host = torch.from_numpy(bench.controls(off, n, 2, 5 + K)[5:]).cuda()
    rew_b, done_b = b.rollout(K, host)
    assert torch.equal(rew, rew_b) and torch.equal(done, done_b)
    assert torch.equal(a.ships, b.ships) and torch.equal(a.bullets, b.bullets)
    rew, done = a.rollout(K, 'nothing')
    rew_b, done_b = b.rollout(K, torch.full((K, n, 2), 2, dtype=torch.int8, device='cuda:0'))
    assert torch.equal(rew, rew_b) and torch.equal(done, done_b) and torch.equal(a.planets, b.planets)


def test_step_info_flags():
    """BatchedEnv.info(): the hit bitmask of a collision step equals the
    reference's 1 - 2 * hit rewards (core.py:253-255), and the overflow flag
    of each env equals the oracle's dropped-bullet flag (small b_cap)."""
    cfg = CFG['rapid']
    P = batched.make_params(cfg)
    n = 517
    env = _env(cfg, n, dtype=torch.float32, b_cap=6, auto_reset=False)
    env.reset()
    rng = np.random.RandomState(3)
    saw_hit = saw_over = False
    for t in range(40):
        B = _host_batch(env)
        ctl = rng.randint(0, 6, size=(n, 2)).astype(np.int8)
        want, wrew, wdone = batched.step(B, ctl, P, store='f32')
        env.step(torch.from_numpy(ctl).cuda(), auto_reset=False)
        info = env.info()
        hit = info['hit'].cpu().numpy()
        coll = wdone == 1
        want_hit = ((wrew < 0) & coll[:, None]).astype(np.uint8) @ np.array([1, 2], np.uint8)
        assert np.array_equal(hit, want_hit), t
        run = wdone == 0
        assert np.array_equal(info['overflow'].cpu().numpy()[run], want.overflow[run]), t
        assert not info['create_exhausted'].cpu().numpy().any()
        saw_hit |= bool(hit.any())
        saw_over |= bool(want.overflow[run].any())
        if (~run).any():
            env.reset(mask=torch.from_numpy((~run).astype(np.uint8)).cuda())
    assert saw_hit and saw_over
