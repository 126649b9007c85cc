"""Load the committed golden fixtures (tests/golden/) into oracle Batches.

The fixtures were written by tools/gen_golden.py from the reference itself;
this module only reads data (npz with allow_pickle=False, json)."""
import json
import os

import numpy as np

from astro_amd.config import Config
from oracle import batched

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def configs():
    with open(os.path.join(GOLDEN, 'configs.json')) as f:
        raw = json.load(f)['configs']
    return {k: Config(**v) for k, v in raw.items()}


def load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def load_json(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


class Transitions:
    """Teacher-forced (state_in, control) -> reference output records."""

    def __init__(self, fname):
        z = load(fname)
        self.z = {k: z[k] for k in z.files}
        self.n = self.z['tick'].shape[0]
        self.cfg_names = [str(x) for x in self.z['cfg_names']]

    def groups(self):
        """Yield (cfg_name, row indices) per config."""
        for ci, name in enumerate(self.cfg_names):
            idx = np.nonzero(self.z['cfg'] == ci)[0]
            if idx.size:
                yield name, idx

    def max_bullets(self, idx):
        z = self.z
        nin = np.diff(z['in_bullets_off'])[idx]
        nout = np.diff(z['out_bullets_off'])[idx]
        return int(max(nin.max(initial=0), nout.max(initial=0)))

    def batch_in(self, idx, nships, p_pad=8, b_cap=None):
        z = self.z
        if b_cap is None:
            b_cap = max(self.max_bullets(idx), 1)
        B = batched.Batch.zeros(idx.size, nships, p_pad, b_cap)
        B.tick[:] = z['tick'][idx]
        B.nplanets[:] = z['nplanets'][idx]
        B.ships[:] = z['in_ships'][idx, :nships, 0:4]
        B.ships_b[:] = z['in_ships'][idx, :nships, 4]
        B.planets[:] = z['in_planets'][idx, :p_pad]
        off = z['in_bullets_off']
        for r, i in enumerate(idx):
            nb = off[i + 1] - off[i]
            B.nbullets[r] = nb
            B.bullets[r, :nb] = z['in_bullets'][off[i]:off[i + 1]]
        return B

    def expected(self, idx, nships, p_pad=8, b_cap=None):
        """Reference outputs as a Batch (+ reward, done)."""
        z = self.z
        if b_cap is None:
            b_cap = max(self.max_bullets(idx), 1)
        E = batched.Batch.zeros(idx.size, nships, p_pad, b_cap)
        E.ships[:] = z['out_ships'][idx, :nships, 0:4]
        E.ships_b[:] = z['out_ships'][idx, :nships, 4]
        E.planets[:] = z['out_planets'][idx, :p_pad]
        E.nplanets[:] = z['nplanets'][idx]
        off = z['out_bullets_off']
        for r, i in enumerate(idx):
            nb = off[i + 1] - off[i]
            E.nbullets[r] = nb
            E.bullets[r, :nb] = z['out_bullets'][off[i]:off[i + 1]]
        E.tick[:] = z['tick'][idx] + 1
        return E, z['out_reward'][idx, :nships], z['out_done'][idx]


def games():
    z = load('games.npz')
    idx = load_json('games.json')
    out = []
    for g in idx:
        key = 'g%03d' % g['gid']
        g = dict(g)
        for f in ('seed', 'controls', 'ships', 'planets', 'nbullets', 'reward'):
            g[f] = z[key + '__' + f]
        out.append(g)
    return out


class Features:
    """rl.ValueNetwork.get_features of every input state of steps.npz, and a
    few to_batch results (tools/gen_golden.py: gen_features)."""

    def __init__(self):
        z = load('features.npz')
        self.z = {k: z[k] for k in z.files}

    def of(self, i):
        z = self.z
        a, b = z['features_off'][i], z['features_off'][i + 1]
        return z['features'][a:b, :z['dims'][i]]

    def batches(self):
        k = 0
        while 'batch_%d' % k in self.z:
            yield self.z['batch_idx_%d' % k], self.z['batch_%d' % k]
            k += 1
