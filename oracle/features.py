"""Observation features of Astro states -- TEST ORACLE ONLY.

Restates rl.ValueNetwork.get_features / to_batch (astro/rl.py:36-112), the
observation a batched policy consumes, with the reference's numpy dtype
behaviour: the bearing feature util.norm_angle(b) / pi (util.py:125-132) is
evaluated in the dtype of the ships' arrays (float32 for create()'s fresh
state, float64 after a step) and every feature is stored as float32.

* ``get_features(state)``     one reference-shaped State -> float32 [P + B, D]
* ``to_batch(features)``      list of those -> [len, max rows, D], -1 padding
* ``batched(B, S, rows)``     an oracle ``batched.Batch`` (float64 values,
                              tick 0 = float32 ships) -> float32 [N, rows, D],
                              what astro_features writes

Pinned against the reference's own outputs (tests/golden/features.npz, made by
tools/gen_golden.py) in tests/test_oracle_golden.py.  Not imported by the
product package.
"""
import numpy as np


def _norm_angle_over_pi(b):
    """util.norm_angle(b) / np.pi in b's own dtype (numpy 2 promotion: the
    Python-float constants take the array's dtype)."""
    return (((b + np.pi) % (2 * np.pi)) - np.pi) / np.pi


def feature_dim(nships):
    return 1 + 5 * nships + 4


def get_features(state):
    """rl.ValueNetwork.get_features (rl.py:43-72): rows [planets, bullets];
    columns [type (0 planet / 1 bullet), ships (x, y, dx, dy, b') * S, object
    (x, y, dx, dy)]."""
    S = state.ships.x.shape[0]
    P = state.planets.x.shape[0]
    B = state.bullets.x.shape[0]
    out = np.zeros((P + B, feature_dim(S)), dtype=np.float32)
    out[P:, 0] = 1
    ships = np.concatenate((state.ships.x, state.ships.dx,
                            _norm_angle_over_pi(state.ships.b[:, np.newaxis])), axis=1)
    out[:, 1:1 + 5 * S] = ships.flatten()
    out[:P, 1 + 5 * S:] = np.concatenate((state.planets.x, state.planets.dx), axis=1)
    out[P:, 1 + 5 * S:] = np.concatenate((state.bullets.x, state.bullets.dx), axis=1)
    return out


def to_batch(features):
    """rl.ValueNetwork.to_batch (rl.py:75-99): pad rows with -1."""
    if any(f.shape[1] != features[0].shape[1] for f in features):
        raise ValueError('feature dimensions differ (solo and non-solo games mixed)')
    rows = max(f.shape[0] for f in features)
    out = np.full((len(features), rows, features[0].shape[1]), -1, dtype=np.float32)
    for k, f in enumerate(features):
        out[k, :f.shape[0]] = f
    return out


def batched(B, nships, rows):
    """Features of every env of a batched.Batch, padded/cut to ``rows``:
    what the HIP astro_features writes for the same stored state."""
    N = B.tick.shape[0]
    S = nships
    out = np.full((N, rows, feature_dim(S)), -1, dtype=np.float32)
    for i in range(N):
        t0 = B.tick[i] == 0
        sd = np.float32 if t0 else np.float64
        npl, nb = int(B.nplanets[i]), int(B.nbullets[i])
        f = np.zeros((npl + nb, feature_dim(S)), dtype=np.float32)
        f[npl:, 0] = 1
        sh = B.ships[i, :S]
        ships = np.concatenate((sh[:, 0:4].astype(sd),
                                _norm_angle_over_pi(B.ships_b[i, :S].astype(sd))[:, np.newaxis]), axis=1)
        f[:, 1:1 + 5 * S] = ships.flatten()
        f[:npl, 1 + 5 * S:] = B.planets[i, :npl]
        f[npl:, 1 + 5 * S:] = B.bullets[i, :nb]
        k = min(rows, npl + nb)
        out[i, :k] = f[:k]
    return out
