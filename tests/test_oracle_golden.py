"""Pin the CPU oracle against the reference's own outputs (golden fixtures).

Everything here runs on the CPU ("not gpu").  Bar: bit-exact.  The fixtures
were produced by tools/gen_golden.py running /root/reference/astro itself."""
import numpy as np
import pytest

from oracle import batched, mt19937, npsincos
from tests import golden_io as gio

CFG = gio.configs()


# --------------------------------------------------------------------- KATs

def test_kat_collisions():
    # reference test_core.py:6-17 (as data)
    k = gio.load_json('kat.json')['collisions']
    assert batched.collisions_allpairs(k['x'], k['r']).tolist() == k['out'] == [False, True, True, True]


def test_kat_direction_bits():
    # util.direction (util.py:87-92) float32 output, bit for bit
    k = gio.load_json('kat.json')
    d = k['direction']
    b = np.asarray(d['b'])
    got = np.stack([npsincos.sin32(b.astype(np.float32)), npsincos.cos32(b.astype(np.float32))], -1)
    np.testing.assert_allclose(got, d['out'], atol=1e-6)   # test_util.py:59-64
    df = k['direction_f32']
    b = np.asarray(df['b']).astype(np.float32)
    got = np.stack([npsincos.sin32(b), npsincos.cos32(b)], -1)
    assert (got.view(np.uint32) == np.asarray(df['out_bits'], dtype=np.uint32)).all()


def test_npsincos_matches_numpy_exhaustive_sample():
    rng = np.random.default_rng(7)
    for scale in (1.0, 8.0, 300.0, 70000.0):
        x = rng.uniform(-scale, scale, 400_000).astype(np.float32)
        for mine, ref in ((npsincos.sin32, np.sin), (npsincos.cos32, np.cos)):
            assert (mine(x).view(np.int32) == ref(x, dtype=np.float32).view(np.int32)).all()


def test_kat_wrap():
    k = gio.load_json('kat.json')
    for key in ('wrap_unit_square', 'wrap_random'):
        x = np.asarray(k[key]['x'])
        got = batched._wrap(np.float64, x)
        assert np.array_equal(got, np.asarray(k[key]['out']))


# ----------------------------------------------------------- MT19937 / seeds

def test_mt19937_words_match_numpy():
    seeds = [0, 1, 42, 5489, 123456789, (1 << 31) + 7, (1 << 32) - 1]
    w = mt19937.words(seeds, 1300)
    for i, s in enumerate(seeds):
        ref = np.random.RandomState(s).randint(0, 1 << 32, size=1300, dtype=np.uint64)
        assert (w[i] == ref.astype(np.uint32)).all()


def test_generate_configs_golden():
    z = gio.load('generate_configs.npz')
    for key in z.files:
        seed = int(key.split('_', 1)[1])
        assert (mt19937.generate_config_seeds(seed, 300) == z[key]).all()


# ------------------------------------------------------------------ schedule

def test_schedule_golden():
    sched = gio.load_json('schedule.json')
    for name, s in sched.items():
        cfg = CFG['default']._replace(**s['config'])
        fire, tt, ts, reloads = batched.schedule(cfg)
        assert tt == s['timeout_tick'], name
        assert np.nonzero(fire)[0].tolist() == s['fire_ticks'], name
        assert ts[:50].tolist() == s['t'] and reloads[:50].tolist() == s['reload']
        assert ts[-1] == s['t_last']


# -------------------------------------------------------------------- create

@pytest.mark.parametrize('name', sorted(CFG))
def test_create_golden(name):
    z = gio.load('create.npz')
    cfg = CFG[name]
    P = batched.make_params(cfg)
    seeds = z[name + '__seed']
    B = batched.create(seeds, P, p_pad=8, b_cap=4, store='f64')
    S = P.nships
    assert (B.nplanets == z[name + '__nplanets']).all()
    assert np.array_equal(B.ships[..., 0:2].astype(np.float32), z[name + '__ships_x'][:, :S])
    assert np.array_equal(B.ships[..., 2:4], z[name + '__ships_dx'][:, :S])
    assert np.array_equal(B.ships_b.astype(np.float32), z[name + '__ships_b'][:, :S])
    assert np.array_equal(B.planets[..., 0:2].astype(np.float32), z[name + '__planets_x'])
    # planet velocities are float64 in the reference: compare the float64 values
    assert np.array_equal(B.planets[..., 2:4], z[name + '__planets_dx'])
    assert (B.nbullets == 0).all() and (B.tick == 0).all()


# ------------------------------------------------- teacher-forced transitions

def _compare(tag, got, rew, done, E, erew, edone):
    assert (done == edone).all(), tag
    assert np.array_equal(rew, erew.astype(np.float32)), tag
    run = edone == 0
    assert (got.nbullets[run] == E.nbullets[run]).all(), tag
    assert np.array_equal(got.ships[run], E.ships[run]), tag
    assert np.array_equal(got.ships_b[run], E.ships_b[run]), tag
    pv = (np.arange(got.planets.shape[1])[None, :] < got.nplanets[:, None]) & run[:, None]
    assert np.array_equal(got.planets[pv], E.planets[pv]), tag
    bv = (np.arange(got.bullets.shape[1])[None, :] < got.nbullets[:, None]) & run[:, None]
    assert np.array_equal(got.bullets[bv], E.bullets[bv]), tag


@pytest.mark.parametrize('fname', ['steps.npz', 'edge_steps.npz'])
def test_step_teacher_forced_bit_exact(fname):
    """Oracle step (float64 arithmetic) == reference step on the same
    (float32-valued) input states, bit for bit, including the tick-0 float32
    paths, 1..8 planets, bullets, rewards and done causes."""
    tr = gio.Transitions(fname)
    total = 0
    for name, idx in tr.groups():
        cfg = CFG[name]
        P = batched.make_params(cfg)
        S = P.nships
        B = tr.batch_in(idx, S)
        got, rew, done = batched.step(B, tr.z['control'][idx], P, store='f64')
        E, erew, edone = tr.expected(idx, S, b_cap=B.bullets.shape[1])
        _compare('%s/%s' % (fname, name), got, rew, done, E, erew, edone)
        total += idx.size
    assert total == tr.n


# ------------------------------------------------------- free-running games

def test_games_free_running_float64_bit_exact():
    """Whole games from create(seed) under the recorded open-loop controls:
    the float64 oracle reproduces every ship state of every tick, the game
    length, the bullet counts and the outcome."""
    for g in gio.games():
        cfg = CFG[g['cfg']]._replace(seed=int(g['seed']))
        P = batched.make_params(cfg)
        S = P.nships
        st = batched.create([g['seed']], P, p_pad=8, b_cap=512, store='f64')
        ticks = g['ships'].shape[0]
        for t in range(ticks):
            assert np.array_equal(st.ships[0], g['ships'][t, :S, 0:4]), (g['gid'], t)
            assert np.array_equal(st.ships_b[0], g['ships'][t, :S, 4]), (g['gid'], t)
            n = st.nplanets[0]
            assert np.array_equal(st.planets[0, :n], g['planets'][t, :n]), (g['gid'], t)
            assert st.nbullets[0] == g['nbullets'][t], (g['gid'], t)
            ctl = np.zeros((1, 2), np.int64)
            ctl[0, :S] = g['controls'][t]
            st, rew, done = batched.step(st, ctl, P, store='f64')
            if t < ticks - 1:
                assert done[0] == 0
        assert done[0] == g['done'], g['gid']
        assert np.array_equal(rew[0], g['reward'][:S].astype(np.float32))


# ------------------------------------------------------- single-game port

def _state_from_row(tr, i, S):
    from oracle import port
    z = tr.z
    fl = int(z['dtype_flags'][i])
    sf = np.float32 if fl & 1 else np.float64
    pxf = np.float32 if fl & 2 else np.float64
    pdf = np.float32 if fl & 4 else np.float64
    bf = np.float32 if fl & 8 else np.float64
    sh = z['in_ships'][i, :S]
    n = z['nplanets'][i]
    pl = z['in_planets'][i, :n]
    off = z['in_bullets_off']
    bl = z['in_bullets'][off[i]:off[i + 1]]
    return port.State(ships=port.Bodies(sh[:, 0:2].astype(sf), sh[:, 2:4].astype(sf), sh[:, 4].astype(sf)),
                      planets=port.Bodies(pl[:, 0:2].astype(pxf), pl[:, 2:4].astype(pdf), None),
                      bullets=port.Bodies(bl[:, 0:2].astype(bf), bl[:, 2:4].astype(bf), None),
                      reload=0.0, t=0.0)


def test_port_step_teacher_forced_bit_exact():
    """The single-game CPU port (timed CPU baseline) == reference, on every
    golden transition; reload/t come from the schedule of the tick."""
    from oracle import port
    tr = gio.Transitions('steps.npz')
    for name, idx in tr.groups():
        cfg = CFG[name]
        g = port.Game(cfg)
        S = g.ns
        _, _, ts, reloads = batched.schedule(cfg)
        for i in idx[::3]:
            st = _state_from_row(tr, i, S)
            k = int(tr.z['tick'][i])
            st = st._replace(t=float(ts[k]), reload=float(reloads[k]))
            out, rew = g.step(st, tr.z['control'][i, :S].astype(np.int64))
            done = tr.z['out_done'][i]
            assert (out is None) == (done != 0)
            assert np.array_equal(rew, tr.z['out_reward'][i, :S])
            if out is None:
                continue
            assert np.array_equal(out.ships.x, tr.z['out_ships'][i, :S, 0:2])
            assert np.array_equal(out.ships.b, tr.z['out_ships'][i, :S, 4])
            n = tr.z['nplanets'][i]
            assert np.array_equal(out.planets.dx, tr.z['out_planets'][i, :n, 2:4])
            off = tr.z['out_bullets_off']
            assert np.array_equal(out.bullets.x, tr.z['out_bullets'][off[i]:off[i + 1], 0:2])


def test_port_create_bit_exact():
    from oracle import port
    z = gio.load('create.npz')
    for name in ('default', 'mp8', 'solo'):
        g = port.Game(CFG[name])
        for k, seed in enumerate(z[name + '__seed'][:64]):
            s = g.create(int(seed))
            n = s.planets.x.shape[0]
            assert np.array_equal(s.ships.x, z[name + '__ships_x'][k, :g.ns])
            assert np.array_equal(s.planets.dx, z[name + '__planets_dx'][k, :n])


# ------------------------------------------------- observation features

def test_features_golden_bit_exact():
    """oracle.features.get_features == rl.ValueNetwork.get_features
    (rl.py:43-72) on all 8,812 golden input states, bit for bit (float32
    bearings at tick 0, float64 after)."""
    from oracle import features
    tr = gio.Transitions('steps.npz')
    fx = gio.Features()
    for i in range(tr.n):
        S = int(tr.z['nships'][i])
        got = features.get_features(_state_from_row(tr, i, S))
        want = fx.of(i)
        assert got.shape == want.shape and got.dtype == np.float32
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), i


def test_features_to_batch_golden():
    """to_batch (rl.py:75-99): -1 padding to the longest member."""
    from oracle import features
    tr = gio.Transitions('steps.npz')
    fx = gio.Features()
    for idx, want in fx.batches():
        got = features.to_batch([fx.of(int(i)) for i in idx])
        assert np.array_equal(got, want)
    with pytest.raises(ValueError):
        features.to_batch([np.zeros((2, 15), np.float32), np.zeros((2, 10), np.float32)])


def test_features_batched_equals_per_state():
    """The batched form (what the kernel is checked against) agrees with the
    per-state restatement on a golden group, padding included."""
    from oracle import features
    tr = gio.Transitions('steps.npz')
    fx = gio.Features()
    for name, idx in tr.groups():
        S = 1 if CFG[name].solo else 2
        idx = idx[:200]
        B = tr.batch_in(idx, S)
        rows = 8 + B.bullets.shape[1]
        got = features.batched(B, S, rows)
        for r, i in enumerate(idx):
            want = fx.of(i)
            assert np.array_equal(got[r, :want.shape[0]], want), (name, i)
            assert (got[r, want.shape[0]:] == -1).all()
