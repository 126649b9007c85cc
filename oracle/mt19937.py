"""Restated numpy legacy MT19937 ``RandomState`` (numpy 2.2.6) -- TEST ORACLE ONLY.

The reference draws every random number of ``create`` (astro/core.py:86-135)
and of ``generate_configs`` (astro/core.py:77-83) from
``np.random.RandomState(int_seed)``.  That is a third-party algorithm (numpy,
pinned version 2.2.6 in configs.json), restated here from its published
definition:

* seeding  = Matsumoto-Nishimura ``init_genrand``:
             ``mt[0] = s; mt[i] = 1812433253*(mt[i-1] ^ (mt[i-1] >> 30)) + i``
* output i = tempered word i of the twisted state (624-word blocks)
* ``rand()``      = ``((a >> 5) * 2**26 + (b >> 6)) / 2**53``, two words
* ``randint(lo, hi)`` (legacy, int64, range < 2**32) = masked rejection:
  ``mask`` = smallest 2**k-1 >= hi-1-lo, draw ``w & mask`` until <= range;
  range 0 draws nothing
* ``choice((a, b))`` = ``randint(0, 2)``

Everything is vectorised over a batch of seeds (uint64 arithmetic, masked to
32 bits).  tests/test_oracle_golden.py pins it against numpy itself and
against the reference's create/generate_configs fixtures.
"""
import numpy as np

N = 624
M = 397
MATRIX_A = np.uint64(0x9908B0DF)
UPPER = np.uint64(0x80000000)
LOWER = np.uint64(0x7FFFFFFF)
MASK32 = np.uint64(0xFFFFFFFF)


def init_genrand(seeds):
    """[K] seeds -> [K, 624] initial key (before the first twist)."""
    s = np.asarray(seeds, dtype=np.uint64) & MASK32
    key = np.empty((s.shape[0], N), dtype=np.uint64)
    key[:, 0] = s
    for i in range(1, N):
        prev = key[:, i - 1]
        key[:, i] = (np.uint64(1812433253) * (prev ^ (prev >> np.uint64(30))) + np.uint64(i)) & MASK32
    return key


def twist(key):
    """One full MT19937 regeneration of a [K, 624] state (returns a copy)."""
    mt = key.copy()
    for kk in range(N):
        y = (mt[:, kk] & UPPER) | (mt[:, (kk + 1) % N] & LOWER)
        mag = np.where((y & np.uint64(1)) != 0, MATRIX_A, np.uint64(0))
        mt[:, kk] = mt[:, (kk + M) % N] ^ (y >> np.uint64(1)) ^ mag
    return mt


def temper(y):
    y = np.asarray(y, dtype=np.uint64)
    y = y ^ (y >> np.uint64(11))
    y = y ^ ((y << np.uint64(7)) & np.uint64(0x9D2C5680))
    y = y ^ ((y << np.uint64(15)) & np.uint64(0xEFC60000))
    y = y ^ (y >> np.uint64(18))
    return y & MASK32


def words(seeds, count):
    """First ``count`` raw 32-bit outputs of RandomState(seed) -> [K, count] uint32."""
    mt = init_genrand(seeds)
    out = []
    have = 0
    while have < count:
        mt = twist(mt)
        out.append(temper(mt))
        have += N
    return np.concatenate(out, axis=1)[:, :count].astype(np.uint32)


def first_words(seeds):
    """Output 0 of RandomState(seed) for each seed -> [K] uint32: it needs
    only init-key words 0, 1 and 397 (the 397-step chain, no 624-word state)."""
    s = np.asarray(seeds, dtype=np.uint64).reshape(-1) & MASK32
    k1 = (np.uint64(1812433253) * (s ^ (s >> np.uint64(30))) + np.uint64(1)) & MASK32
    v = k1.copy()
    for i in range(2, M + 1):
        v = (np.uint64(1812433253) * (v ^ (v >> np.uint64(30))) + np.uint64(i)) & MASK32
    y = (s & UPPER) | (k1 & LOWER)
    mag = np.where((y & np.uint64(1)) != 0, MATRIX_A, np.uint64(0))
    return temper(v ^ (y >> np.uint64(1)) ^ mag).astype(np.uint32)


class Stream:
    """A cursor over one seed's raw words with the legacy draw rules."""

    def __init__(self, word_row):
        self.w = [int(x) for x in word_row]
        self.pos = 0

    def next32(self):
        v = self.w[self.pos]
        self.pos += 1
        return v

    def rand(self):
        a = self.next32() >> 5
        b = self.next32() >> 6
        return (a * 67108864.0 + b) / 9007199254740992.0

    def randint(self, lo, hi):
        rng = hi - 1 - lo
        if rng == 0:
            return lo
        mask = rng
        for sh in (1, 2, 4, 8, 16):
            mask |= mask >> sh
        while True:
            v = self.next32() & mask
            if v <= rng:
                return lo + v


def generate_config_seeds(seed, count):
    """The ``seed`` fields yielded by ``generate_configs`` (core.py:77-83):
    ``RandomState(seed).randint(1 << 30)`` per config = one masked word each."""
    w = words([seed], count)[0].astype(np.uint64)
    return (w & np.uint64((1 << 30) - 1)).astype(np.uint32)
