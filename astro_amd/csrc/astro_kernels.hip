// astro_kernels.hip -- MI355X (gfx950) batched lockstep Astro physics.
//
// State is struct-of-arrays, entity-major ([slot][env]) for ships and planets
// (a wave's load of slot s of its envs is one contiguous, coalesced dwordx4
// stretch) and one contiguous row per env for bullets.  One step kernel in
// three lane layouts, identical results:
//   * astro_step_kernel            -- one lane per env (64 envs per wave);
//                                     registers only, no LDS;
//   * astro_step_quad_kernel<.., 4> -- four lanes per env (16 envs per wave),
//   * astro_step_quad_kernel<.., 2> -- two lanes per env (32 envs per wave):
//     ships and planets move inside an env's lanes by DPP broadcasts; the
//     wave's live bullets are numbered densely (DPP scan) and indexed through
//     LDS, one bullet per lane per round; the env's bodies for the bullet
//     pass and the auto-reset's MT19937 init chains are staged in LDS (one
//     private LDS set per wave, wave-scoped sync only).
// Auto-reset runs inside the step (the finished envs' next games, created
// wave-cooperatively); each env's generate_configs stream is an exact
// MT19937 of any length (MTStream: cursor + the env's 624-word ring).  A
// one-tick launch of at most two step waves per SIMD gives each step wave a
// helper wave in its workgroup (HelpBox): the helper makes the envs' next
// games' MT19937 chains and -- pair instance -- their planet updates while
// the step wave steps, then stores the survivors' planets and creates the
// finished envs' next games once the step wave posts which envs finished.

// What is computed is exactly astro/core.py's step (core.py:215-303) and
// create (core.py:86-135), including the reference's numpy dtype behaviour:
//   * the first step of a game (tick 0) sees create()'s float32 arrays, so
//     gravity, collision distances and tick-0 bullets run in float32;
//   * every later step runs in float64 (numpy 2.x promotes the state);
//   * a one-planet game keeps float32 planet arrays for ever;
//   * util.direction (util.py:87-92) is numpy's own float32 sin/cos
//     algorithm (np_sincosf below), so directions match numpy bit for bit.
// The file is compiled with -ffp-contract=off: numpy never fuses a*b+c, and
// neither may we, except where numpy's sin/cos itself uses an FMA.
//
// With float64 state the kernel therefore reproduces the reference bit for
// bit; with float32 state every stored value is the float32 rounding of the
// reference's value computed from the same (float32) input state.

#include <hip/hip_runtime.h>

#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>

#include <map>
#include <mutex>
#include <type_traits>
#include <utility>

#include "astro_step.h"

namespace {

// ---------------------------------------------------------------------------
// storage vectors (16-byte aligned; a D4 is two dwordx4)

struct alignas(16) F4 { float x, y, z, w; };
struct alignas(16) D4 { double x, y, z, w; };

// 16 bytes at base + 16 i through a global (not flat) pointer: for an address
// chosen between arrays at run time (a flat load would make the compiler
// wait for every load before it, flat ones completing out of order)
__device__ __forceinline__ uint4 load_u4_global(uintptr_t base, size_t i) {
    typedef unsigned v4u __attribute__((ext_vector_type(4)));
    const v4u v = *reinterpret_cast<const __attribute__((address_space(1))) v4u *>(base + 16 * i);
    return make_uint4(v.x, v.y, v.z, v.w);
}

template <typename T> struct Store;
template <> struct Store<float> { using V = F4; };
template <> struct Store<double> { using V = D4; };


// A state store of the step: nontemporal (the next launch reads it from
// HBM anyway; streamed, the stores leave L2 to the launch's loads: c3 11.88
// -> 11.77 us, c5 32.03 -> 31.72 us, c2 even, profiles/round4/ab_nt_stores.jsonl).
// A/B build -DASTRO_TEMPORAL_STORES: plain stores
template <typename X>
__device__ __forceinline__ void st_out(X *p, const X &v) {
#ifndef ASTRO_TEMPORAL_STORES
    if constexpr (sizeof(X) == 16 && alignof(X) == 16) {
        typedef unsigned v4u __attribute__((ext_vector_type(4)));
        __builtin_nontemporal_store(*reinterpret_cast<const v4u *>(&v), reinterpret_cast<v4u *>(p));
    } else if constexpr (sizeof(X) == 32) {
        typedef unsigned v4u __attribute__((ext_vector_type(4)));
        __builtin_nontemporal_store(reinterpret_cast<const v4u *>(&v)[0], reinterpret_cast<v4u *>(p));
        __builtin_nontemporal_store(reinterpret_cast<const v4u *>(&v)[1], reinterpret_cast<v4u *>(p) + 1);
    } else if constexpr (sizeof(X) == 8) {
        __builtin_nontemporal_store(*reinterpret_cast<const unsigned long long *>(&v),
                                    reinterpret_cast<unsigned long long *>(p));
    } else if constexpr (sizeof(X) == 4) {
        __builtin_nontemporal_store(*reinterpret_cast<const unsigned *>(&v), reinterpret_cast<unsigned *>(p));
    } else {
        *p = v;
    }
#else
    *p = v;
#endif
}

// ---------------------------------------------------------------------------
// numpy 2.x float32 sin/cos (loops_trigonometric.dispatch.cpp): Cody-Waite
// reduction + minimax polynomials, every multiply-add fused as numpy's
// MulAdd is.  Bit-exact to np.sin/np.cos(x, dtype=float32) for
// |x| <= 71476.0625 (cos) / 117435.992 (sin); beyond, numpy falls back to
// libm and so do we (ocml), which is the only place we may differ.  A game's
// bearing changes by at most dt*ship_rspeed per tick, so it stays in range
// for any max_time/dt below ~8.9e5 ticks at the default speed.

__device__ __forceinline__ void np_sincosf(float x, float &s_out, float &c_out) {
    const float two_over_pi = 0x1.45f306p-1f;
    const float pio2_hi = -0x1.921fb0p+00f;
    const float pio2_med = -0x1.5110b4p-22f;
    const float pio2_lo = -0x1.846988p-48f;
    const float magic = 0x1.800000p+23f;
    float q = __builtin_fmaf(x, two_over_pi, magic) - magic;
    float r = __builtin_fmaf(q, pio2_hi, x);
    r = __builtin_fmaf(q, pio2_med, r);
    r = __builtin_fmaf(q, pio2_lo, r);
    float r2 = r * r;
    float c = __builtin_fmaf(0x1.98e616p-16f, r2, -0x1.6c06dcp-10f);
    c = __builtin_fmaf(c, r2, 0x1.55553cp-5f);
    c = __builtin_fmaf(c, r2, -0x1.000000p-1f);
    c = __builtin_fmaf(c, r2, 0x1.000000p+0f);
    float s = __builtin_fmaf(0x1.7d3bbcp-19f, r2, -0x1.a06bbap-13f);
    s = __builtin_fmaf(s, r2, 0x1.11119ap-07f);
    s = __builtin_fmaf(s, r2, -0x1.555556p-03f);
    s = __builtin_fmaf(s, r2, 0.0f);
    s = __builtin_fmaf(s, r, r);
    const int iq = (int)q;
    float sv = (iq & 1) ? c : s;
    if (iq & 2) sv = 0.0f - sv;
    const int iq1 = iq + 1;
    float cv = (iq1 & 1) ? c : s;
    if (iq1 & 2) cv = 0.0f - cv;
    const float ax = __builtin_fabsf(x);
    if (ax > 117435.992f) sv = sinf(x);
    if (ax > 71476.0625f) cv = cosf(x);
    s_out = sv;
    c_out = cv;
}

// util.wrap_unit_square (util.py:145-148): ((v + 1) % 2) - 1 with numpy's
// floored remainder (npy_divmod: fmod, then +2 when negative, +0 when
// zero).  fmod(x, 2) == x - 2*trunc(x/2) EXACTLY for finite x: x/2 and
// 2*trunc are exact, and x - 2t is exact by Sterbenz (2t and x share sign,
// |2t| <= |x| < |2t| + 2).  Five instructions instead of ocml's fmod loop.
template <typename C>
__device__ __forceinline__ C wrap_unit(C v) {
    const C x = v + C(1);
    C m = x - C(2) * trunc(x * C(0.5));
    m = m < C(0) ? m + C(2) : m;
    m = m == C(0) ? C(0) : m;
    return m - C(1);
}

// gm / d2 (IEEE, correctly rounded) as LLVM lowers an f64 division on
// AMDGPU -- rcp, two Newton steps, quotient and one residual correction --
// minus v_div_scale / v_div_fmas scaling and v_div_fixup, which are
// identities when neither operand nor the quotient is near the exponent
// limits.  Here d2 = max(1e-12, |r|^2) with |r| <= 2*sqrt(2) for live bodies
// (and garbage, selected away, for padding) and gm is a normal constant, so
// results are bit-identical to `/` (checked on 6.7e7 random operand pairs on
// MI355X: 0 mismatches) at 3 fewer instructions, two of them quarter rate.
__device__ __forceinline__ double div_gravity(double n, double d) {
    const double r0 = __builtin_amdgcn_rcp(d);
    const double e0 = __builtin_fma(-d, r0, 1.0);
    const double r1 = __builtin_fma(r0, e0, r0);
    const double e1 = __builtin_fma(-d, r1, 1.0);
    const double r2 = __builtin_fma(r1, e1, r1);
    const double q0 = n * r2;
    const double rem = __builtin_fma(-d, q0, n);
    return __builtin_fma(rem, r2, q0);
}
__device__ __forceinline__ float div_gravity(float n, float d) { return n / d; }   // tick 0: as the compiler does it

// np.maximum(1e-12, d2): NaN-propagating max
template <typename C>
__device__ __forceinline__ C max_floor(C d2) {
    const C k = C(1e-12);
    return d2 < k ? k : d2;
}

// _gravity (core.py:138-153) at one point: sum over planets in index order,
// field = gm / max(1e-12, |r|^2) * r  (a 1/r law in 2-D: no sqrt)
template <typename C, int PMAX>
__device__ __forceinline__ void field(const double (&px)[PMAX], const double (&py)[PMAX], int np,
                                      double x, double y, double gm, C &gx, C &gy, bool last = true,
                                      int np_uni = 0) {
    // every slot is evaluated (padded slots hold a copy of planet 0) and the
    // sum selects: a per-planet branch costs more than the arithmetic when
    // some lane of the wave has all PMAX planets anyway.  `last` (wave-
    // uniform) false says no lane has PMAX planets: the last slot is skipped.
    // np_uni > 0 (wave-uniform): every lane has np_uni planets, no selects
    C ax = C(0), ay = C(0);
    if (np_uni > 0) {
#pragma unroll
        for (int j = 0; j < PMAX; ++j) {
            if (j >= np_uni) break;
            const C rx = C(px[j]) - C(x);
            const C ry = C(py[j]) - C(y);
            const C d2 = rx * rx + ry * ry;
            const C f = div_gravity(C(gm), max_floor(d2));
            const C tx = f * rx, ty = f * ry;
            ax = j == 0 ? tx : ax + tx;
            ay = j == 0 ? ty : ay + ty;
        }
        gx = ax;
        gy = ay;
        return;
    }
#pragma unroll
    for (int j = 0; j < PMAX; ++j) {
        if (j == PMAX - 1 && j > 0 && !last) break;
        const C rx = C(px[j]) - C(x);
        const C ry = C(py[j]) - C(y);
        const C d2 = rx * rx + ry * ry;
        const C f = div_gravity(C(gm), max_floor(d2));
        const C tx = f * rx, ty = f * ry;
        if (j == 0) {
            ax = tx;
            ay = ty;
        } else {
            ax = j < np ? ax + tx : ax;
            ay = j < np ? ay + ty : ay;
        }
    }
    gx = ax;
    gy = ay;
}

// Collision test |a - b|^2 < r2 of _collisions (core.py:210-212), exact,
// branch-free.  At tick 0 the reference evaluates the distance in float32
// (create's float32 arrays) and that float32 value IS the answer; float
// d < double r2 <=> d <= t0_max, the largest float below r2.  Later it uses
// float64: the float32 distance of the same inputs is within ~3e-7 relative
// (well inside the 1e-4 guard, which also covers float64 state rounded to
// float32); a distance inside the guard band is flagged ambiguous and the
// caller redoes its tests in float64 (a rare, whole-bullet slow path).
struct Guard {
    float lo, hi, t0_max;
    double r2;
    __device__ explicit Guard(double r2_) : r2(r2_) {
        lo = float(r2 * (1.0 - 1e-4));
        hi = float(r2 * (1.0 + 1e-4));
        float f = float(r2);                       // round to nearest (r2 > 0)
        if (double(f) >= r2) f = __int_as_float(__float_as_int(f) - 1);
        t0_max = f;
    }
};

// The common-case test against the uniform thresholds (SGPRs): hit <=>
// d2 < lo; a d2 inside [lo, hi] is ambiguous.  Tick 0 is not decided here:
// callers flag tick-0 lanes ambiguous and decide them on the exact path.
// Invalid operands are parked at FAR_POS / -FAR_POS: their d2 is +inf, which
// neither hits nor lands in the band.
constexpr float FAR_POS = 1e30f;

__device__ __forceinline__ bool near32(float ax, float ay, float bx, float by, const Guard &g, bool &amb) {
    const float dx = ax - bx;
    const float dy = ay - by;
    const float d2 = dx * dx + dy * dy;
    amb |= (d2 >= g.lo) & (d2 <= g.hi);
    return d2 < g.lo;
}

// The same test on a lane that may be at tick 0: there the reference's own
// distance IS this float32 one (create()'s float32 arrays; closer_exact's
// float(a) - float(b) of the same values, no fma), so tick 0 is decided here
// against the largest float below r^2 and never goes to the exact path.
__device__ __forceinline__ bool near32_t0(float ax, float ay, float bx, float by, const Guard &g, bool &amb,
                                          bool t0) {
    const float dx = ax - bx;
    const float dy = ay - by;
    const float d2 = dx * dx + dy * dy;
    amb |= !t0 & (d2 >= g.lo) & (d2 <= g.hi);
    return t0 ? d2 <= g.t0_max : d2 < g.lo;
}

// the exact test of the ambiguous path: at tick 0 the float32 distance of
// create()'s float32 arrays, later float64
__device__ __forceinline__ bool closer_exact(double ax, double ay, double bx, double by, const Guard &g, bool t0) {
    if (t0) {
        const float dx = float(ax) - float(bx);
        const float dy = float(ay) - float(by);
        return dx * dx + dy * dy <= g.t0_max;
    }
    const double dx = ax - bx;
    const double dy = ay - by;
    return dx * dx + dy * dy < g.r2;
}

// Planet-on-planet gravity (core.py:291) for every planet i < np, in the
// reference's summation order (j = 0..np-1, self term +0.0 included).  The
// pair (i, j) and (j, i) share d2 bit for bit and their terms are exact
// negatives, so each gm / max(1e-12, d2) is computed once: np(np-1)/2
// divisions instead of np^2.
template <typename C, int PMAX>
__device__ __forceinline__ void planet_field(const double (&px)[PMAX], const double (&py)[PMAX], int np,
                                             double gm, C (&gx)[PMAX], C (&gy)[PMAX]) {
    if constexpr (PMAX > 8) {
        // a 16x16 table of pair factors would not fit in registers: direct form
#pragma unroll
        for (int i = 0; i < PMAX; ++i) {
            if (i < np) field<C, PMAX>(px, py, np, px[i], py[i], gm, gx[i], gy[i]);
        }
        return;
    }
    C f[PMAX][PMAX];
#pragma unroll
    for (int i = 0; i < PMAX; ++i) {
#pragma unroll
        for (int j = i + 1; j < PMAX; ++j) {
            const C rx = C(px[j]) - C(px[i]);
            const C ry = C(py[j]) - C(py[i]);
            f[i][j] = div_gravity(C(gm), max_floor(rx * rx + ry * ry));
        }
    }
#pragma unroll
    for (int i = 0; i < PMAX; ++i) {
        C ax = C(0), ay = C(0);
#pragma unroll
        for (int j = 0; j < PMAX; ++j) {
            C tx, ty;
            if (j == i) {
                tx = C(0);
                ty = C(0);
            } else {
                const C rx = C(px[j]) - C(px[i]);
                const C ry = C(py[j]) - C(py[i]);
                const C fij = j > i ? f[i][j] : f[j][i];
                tx = fij * rx;
                ty = fij * ry;
            }
            if (j == 0) {
                ax = tx;
                ay = ty;
            } else {
                ax = j < np ? ax + tx : ax;
                ay = j < np ? ay + ty : ay;
            }
        }
        gx[i] = ax;
        gy[i] = ay;
    }
}

// ---------------------------------------------------------------------------
// numpy legacy MT19937 (RandomState(int)), first 227 outputs, lazily: output
// i needs init-key words i, i+1 and i+397 only, so two cursors over the
// init_genrand recurrence replace the 624-word state (12 bytes, not 2.5 KB).

__device__ __forceinline__ uint32_t mt_key_next(uint32_t prev, uint32_t idx) {
    return 1812433253u * (prev ^ (prev >> 30)) + idx;
}

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

// key[to] of init_genrand given key[from] = v: the 397-step sequential chain
// every RandomState(seed) pays before its first output.  Each step is a
// dependent xor-shift + v_mul_lo_u32 + add, ~50 cycles of latency on gfx950,
// so a whole chain is ~9 us for a lone lane -- hence the key table below.
__device__ __forceinline__ uint32_t mt_key_at(uint32_t v, uint32_t from, uint32_t to) {
    for (uint32_t k = from + 1; k <= to; ++k) v = mt_key_next(v, k);
    return v;
}

constexpr uint32_t MT_PROLOGUE = 397;

// hdr word 0 = tick; word 2 = pending seed | KEY_VALID (word 3 then holds
// key[397] of the pending seed), or UNDRAWN: a reset leaves the next game's
// seed in the stream, for the env's first step (or its helper) to draw off
// the reset path.  The words a step rewrites for a surviving
// env are split: 0-1 (tick, counts) by the step wave, 2-3 (pending seed and
// key) by whoever checks the pending seed -- the step wave, or its helper
constexpr int TICK_BITS = 22;
constexpr uint32_t TICK_MASK = (1u << TICK_BITS) - 1;
constexpr uint32_t KEY_VALID = 1u << 31;
constexpr uint32_t UNDRAWN = 1u << 30;
constexpr uint32_t SEED_MASK = (1u << 30) - 1;   // generate_configs seeds are randint(1 << 30)

struct MTLazy {
    uint32_t a;  // key[i]
    uint32_t b;  // key[i + 397]
    uint32_t i;

    __device__ void seed(uint32_t s) { seed_from(s, mt_key_at(s, 0, 397)); }
    // seed with key[397] already known (the amortised prologue below)
    __device__ void seed_from(uint32_t s, uint32_t key397) {
        a = s;
        b = key397;
        i = 0;
    }
    __device__ bool ok() const { return i < 227; }
    __device__ uint32_t next() {
        const uint32_t a1 = mt_key_next(a, i + 1);
        const uint32_t y = (a & 0x80000000u) | (a1 & 0x7fffffffu);
        const uint32_t tw = b ^ (y >> 1) ^ ((a1 & 1u) ? 0x9908b0dfu : 0u);
        b = mt_key_next(b, i + 398);
        a = a1;
        ++i;
        return mt_temper(tw);
    }
    // RandomState.rand(): 53-bit double from two words
    __device__ double rand() {
        const uint32_t hi = next() >> 5;
        const uint32_t lo = next() >> 6;
        return (double(hi) * 67108864.0 + double(lo)) / 9007199254740992.0;
    }
    // legacy RandomState.randint(lo, hi): masked rejection, nothing drawn
    // for a single-value range
    __device__ int randint(int lo, int hi) {
        const uint32_t rng = uint32_t(hi - 1 - lo);
        if (rng == 0) return lo;
        uint32_t mask = rng;
        mask |= mask >> 1;
        mask |= mask >> 2;
        mask |= mask >> 4;
        mask |= mask >> 8;
        mask |= mask >> 16;
        uint32_t v;
        do {
            v = next() & mask;
        } while (v > rng && ok());
        return lo + int(v);
    }
};

// An env's generate_configs stream (core.py:77-83) is ONE RandomState drawn
// for as long as the env plays, so past output 226 the lazy form above no
// longer holds: output k of MT19937 is
//     x_{k+624} = x_{k+397} ^ twist(x_k, x_{k+1})      (x_0..x_623 = init key)
// and from k = 227 on x_{k+397} is an output the generator already made.
// MTStream keeps the cursor (x_k, x_{k+397}, k) and the env's last 624 twisted
// words in a ring (ring[j % 624] = x_{j+624}, written by draw j): words
// 0..226 come from the init chain as in MTLazy, later ones from the ring --
// the standard one-word-at-a-time MT19937, exact for any length.  A draw's
// ring loads depend on k only, never on the word being made, so they are
// issued first.  Draws are rare (one per game, plus planets_only rejections)
// and the ring is 2.5 KB per env, written one word per draw.
constexpr uint32_t MT_N = 624;
constexpr uint32_t MT_LAZY = MT_N - MT_PROLOGUE;   // 227: outputs with x_{k+397} still in the init key

struct MTStream {
    uint32_t a;      // x_k
    uint32_t b;      // x_{k+397}
    uint32_t k;
    uint32_t *ring;  // the env's [624] words

    __device__ uint32_t next() {
        const uint32_t k1 = k + 1u;
        uint32_t x1, nb;
        if (k1 < MT_LAZY) {   // x_{k+1} and x_{k+398} still in the init key: no memory
            x1 = mt_key_next(a, k1);
            nb = mt_key_next(b, k1 + MT_PROLOGUE);
        } else {
            const uint32_t r1 = k1 >= MT_N ? ring[k1 % MT_N] : 0u;   // x_{k+1} = x_{(k+1-624)+624}
            nb = ring[(k1 - MT_LAZY) % MT_N];                        // x_{k+398}, made by draw k-226
            x1 = k1 < MT_N ? mt_key_next(a, k1) : r1;
            // consume the loads here: a use after the join would put the
            // wait for them (vmcnt, which also counts every store and
            // prefetch in flight) on the lazy path too
            asm volatile("" ::"v"(x1), "v"(nb));
        }
        const uint32_t y = (a & 0x80000000u) | (x1 & 0x7fffffffu);
        const uint32_t z = b ^ (y >> 1) ^ ((x1 & 1u) ? 0x9908b0dfu : 0u);
        ring[k % MT_N] = z;
        b = nb;
        a = x1;
        k = k1;
        return mt_temper(z);
    }
};

__device__ __forceinline__ uint32_t *stream_ring_of(const AstroState &st, int i) {
    return st.stream_ring + size_t(i) * MT_N;
}

// key[397] of RandomState(seed)'s init chain: one gather from the device
// table (every 30-bit seed, built once by astro_keytable_build) or, without
// a table / for a wider explicit seed, the chain itself.
__device__ __forceinline__ uint32_t key397_of(const AstroParams &p, uint32_t seed) {
    if (p.key_table && seed <= SEED_MASK) return p.key_table[seed];
    return mt_key_at(seed, 0, MT_PROLOGUE);
}

// planets_only (AstroParams): the number of planets create() draws for
// `seed` -- randint(1, max_planets + 1) on RandomState(seed)'s first word,
// which alone decides it when max_planets is a power of two (checked on the
// host) -- and whether the seed's game passes the filter.
__device__ __forceinline__ int first_nplanets(const AstroParams &p, uint32_t seed, uint32_t key397) {
    const uint32_t a1 = mt_key_next(seed, 1u);
    const uint32_t y = (seed & 0x80000000u) | (a1 & 0x7fffffffu);
    const uint32_t w = mt_temper(key397 ^ (y >> 1) ^ ((a1 & 1u) ? 0x9908b0dfu : 0u));
    return 1 + int(w & uint32_t(p.max_planets - 1));
}
__device__ __forceinline__ bool seed_passes(const AstroParams &p, uint32_t seed, uint32_t key397) {
    return p.planets_only == 0 || first_nplanets(p, seed, key397) == p.planets_only;
}

constexpr double TWO_PI = 6.283185307179586;  // 2 * np.pi
constexpr double PI = 3.141592653589793;      // np.pi

// ---------------------------------------------------------------------------
// The random draws of create() (core.py:88-116), in the reference's order:
// randint(1, max_planets + 1), rand(2) (outer), rand() (inner), rand() (ship
// choice, only with > 1 planet), rand(S) (bearings), then with > 1 planet
// rand() (orientation) and choice((-1, 1)) = randint(0, 2).

template <int S>
struct CreateDraws {
    int n;
    double u_out[2], u_inner, u_choice, u_bear[S], u_base;
    int reverse;
    bool exhausted;   // the seed's first 227 outputs did not suffice
};

__device__ __forceinline__ double rand53(uint32_t hi, uint32_t lo) {   // RandomState.rand() of two words
    return (double(hi >> 5) * 67108864.0 + double(lo >> 6)) / 9007199254740992.0;
}

// The integer half of create(): randint(1, max_planets + 1) draws whole
// words until one passes the mask (once, for max_planets a power of two);
// every later draw sits at a fixed offset from the accepted word given
// n > 1 or not, so the remaining 11 + 2S words are produced straight-line.
// Called with uniform arguments (one env at a time, see next_game_scalar)
// this all runs on the scalar unit.
template <int S>
struct CreateWords {
    static constexpr int CW = 11 + 2 * S;
    int n;
    uint32_t w[CW];
    bool exhausted;   // the seed's first 227 words did not suffice
};

template <int S>
__device__ __forceinline__ CreateWords<S> create_words(const AstroParams &p, uint32_t seed, uint32_t key397) {
    constexpr int CW = CreateWords<S>::CW;
    CreateWords<S> cw;
    MTLazy g;
    g.seed_from(seed, key397);
    cw.n = g.randint(1, p.max_planets + 1);
    uint32_t a = g.a, b = g.b;
    const uint32_t i0 = g.i;
#pragma unroll
    for (int k = 0; k < CW; ++k) {
        const uint32_t a1 = mt_key_next(a, i0 + uint32_t(k + 1));
        const uint32_t y = (a & 0x80000000u) | (a1 & 0x7fffffffu);
        const uint32_t tw = b ^ (y >> 1) ^ ((a1 & 1u) ? 0x9908b0dfu : 0u);
        b = mt_key_next(b, i0 + uint32_t(k + 398));
        a = a1;
        cw.w[k] = mt_temper(tw);
    }
    const uint32_t used = i0 + uint32_t(cw.n > 1 ? CW : 6 + 2 * S);
    cw.exhausted = used >= 227u || !g.ok();   // MTLazy: valid for the first 227 words
    return cw;
}

// The float half: the draws as RandomState.rand() values.  (Both word
// layouts are converted and the results selected: selecting between array
// elements would index the array in memory.)
template <int S>
__device__ __forceinline__ CreateDraws<S> create_draws(const CreateWords<S> &cw) {
    const uint32_t *w = cw.w;
    CreateDraws<S> d;
    d.n = cw.n;
    const bool many = d.n > 1;
    d.u_out[0] = rand53(w[0], w[1]);
    d.u_out[1] = rand53(w[2], w[3]);
    d.u_inner = rand53(w[4], w[5]);
    d.u_choice = many ? rand53(w[6], w[7]) : 1.0;
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const double u_many = rand53(w[8 + 2 * s], w[9 + 2 * s]);
        const double u_one = rand53(w[6 + 2 * s], w[7 + 2 * s]);
        d.u_bear[s] = many ? u_many : u_one;
    }
    d.u_base = many ? rand53(w[8 + 2 * S], w[9 + 2 * S]) : 0.0;
    d.reverse = many && (w[10 + 2 * S] & 1u) == 0 ? -1 : 1;   // choice((-1, 1)) = randint(0, 2)
    d.exhausted = cw.exhausted;
    return d;
}

// ---------------------------------------------------------------------------
// Where create() puts a new game.  GlobalSink: the state arrays in HBM (every
// launch but the resident rollout); the resident rollout's sinks put it in
// LDS (a reset pass) or in the env's own registers (the serial create).
template <typename T>
struct GlobalSink {
    using V = typename Store<T>::V;
    const AstroState &st;
    __device__ void ship(int s, int ie, const V &v, T b) const {
        reinterpret_cast<V *>(st.ships)[size_t(s) * size_t(st.n_env) + ie] = v;
        reinterpret_cast<T *>(st.ships_b)[size_t(s) * size_t(st.n_env) + ie] = b;
    }
    // planet slot j (the caller's m-th slot of its part)
    __device__ void planet(int j, int m, int ie, const V &v) const {
        (void)m;
        reinterpret_cast<V *>(st.planets)[size_t(j) * size_t(st.n_env) + ie] = v;
    }
    __device__ void header(int ie, const int4 &h) const { reinterpret_cast<int4 *>(st.hdr)[ie] = h; }
    __device__ void stream_seed(int ie, uint32_t seed) const { st.stream[4 * size_t(ie) + 3] = seed; }
    __device__ GlobalSink for_row(int) const { return *this; }   // (a reset pass's row r)
};

// ---------------------------------------------------------------------------
// create() (core.py:86-135) for env i from `seed`; writes the env's slots.
// NPART lanes may share one env: each runs the (cheap, serial) random draws
// and writes ships s and planets j with s, j = part mod NPART, so the
// trigonometry of the planets runs in parallel.

template <typename T, int S, int PMAX, int NPART = 1, class Sink = GlobalSink<T>>
__device__ int create_env(const AstroParams &p, const Sink &sink, int i, const CreateDraws<S> &d,
                          int &flags_out, int part = 0) {
    using V = typename Store<T>::V;

    int n = d.n;
    // outer = outer_ship_position * sign(rand(2).astype(float32) - 0.5)
    const float u0 = float(d.u_out[0]) - 0.5f;
    const float u1 = float(d.u_out[1]) - 0.5f;
    const float o0 = p.outer_pos * (u0 > 0.0f ? 1.0f : (u0 < 0.0f ? -1.0f : 0.0f));
    const float o1 = p.outer_pos * (u1 > 0.0f ? 1.0f : (u1 < 0.0f ? -1.0f : 0.0f));
    // inner = inner_ship_position * direction(2 pi rand())
    float is, ic;
    np_sincosf(float(TWO_PI * d.u_inner), is, ic);
    const float i0 = p.inner_pos * is, i1 = p.inner_pos * ic;
    float shx[2], shy[2];
    const bool outer_first = d.u_choice < 0.5;
    if (n == 1) {
        shx[0] = o0;
        shy[0] = o1;
        shx[1] = -o0;
        shy[1] = -o1;
    } else if (S == 1) {
        shx[0] = outer_first ? o0 : i0;
        shy[0] = outer_first ? o1 : i1;
        shx[1] = shy[1] = 0.0f;
    } else {
        shx[0] = outer_first ? o0 : i0;
        shy[0] = outer_first ? o1 : i1;
        shx[1] = outer_first ? i0 : o0;
        shy[1] = outer_first ? i1 : o1;
    }
    // b = 2 pi * rand(S).astype(float32)   (float32 product)
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const float b = 6.2831855f * float(d.u_bear[s]);
        V v;
        v.x = T(shx[s]);
        v.y = T(shy[s]);
        v.z = T(0);
        v.w = T(0);
        if (s % NPART == part) sink.ship(s, i, v, T(b));
    }
    if (n == 1) {
        V v;
        v.x = v.y = v.z = v.w = T(0);
        if (part == 0) sink.planet(0, 0, i, v);
    } else {
        const double base = TWO_PI * d.u_base;
        const double stp = TWO_PI / double(n);
        const int reverse = d.reverse;
        const double amp = sqrt(p.gravity * p.planet_mass * double(n - 1) / 2.0);
        const double turn = double(reverse) * PI / 2.0;
#pragma unroll
        for (int m = 0; m < (PMAX + NPART - 1) / NPART; ++m) {
            const int j = part + NPART * m;
            if (j >= n || j >= PMAX) continue;
            const double orient = base + double(j) * stp;
            float ps, pc, vs, vc;
            np_sincosf(float(orient), ps, pc);
            np_sincosf(float(orient + turn), vs, vc);
            V v;
            v.x = T(p.planet_orbit * ps);
            v.y = T(p.planet_orbit * pc);
            v.z = T(amp * double(vs));
            v.w = T(amp * double(vc));
            sink.planet(j, m, i, v);
        }
    }
    if (n > PMAX) n = PMAX;
    flags_out = d.exhausted ? 2 : 0;
    return n;
}

// Env i's generate_configs stream (core.py:77-83): RandomState(stream_seed)
// .randint(1 << 30) = one masked MT word per game.  The stream record holds
// the MTStream cursor (x_k, x_{k+397}, k; the ring beside it) and the CURRENT
// game's seed; the next game's seed is drawn by the game's first step (hdr .z
// is UNDRAWN until then) and lives in hdr (.z) with key[397] of its init
// chain (.w, valid with KEY_VALID), so a reset can start creating before the
// cold stream record arrives and never touches the cursor itself.

// Start env i's next game: its seed was drawn one game ahead (hdr word 2) and
// key[397] of that seed fetched from the key table by an earlier step (hdr
// word 3, valid when KEY_VALID) -- unless the game ended at its first step
// (UNDRAWN: draw it here); create.  The following seed is drawn, and its key
// gathered, by the NEXT step, off this path.
// Everything integer about an env's next game: the create() words of its
// pending seed and the stream cursor advanced by one game (core.py:83).
template <int S>
struct NextGame {
    uint32_t seed;         // the game's seed (the pending seed, or with
                           // planets_only the first of the stream to pass)
    CreateWords<S> words;
    uint32_t ca, cb, ci;   // advanced cursor
    bool exhausted;        // create() ran past the 227 words MTLazy covers
};

// (key397 of the pending seed is either known or, have_key false, run here)
template <int S>
__device__ __forceinline__ NextGame<S> next_game(const AstroParams &p, uint32_t pend_seed, uint32_t key397,
                                                 bool have_key, bool undrawn, const uint4 &c, uint32_t *ring) {
    NextGame<S> ng;
    MTStream g{c.x, c.y, c.z, ring};
    if (undrawn) pend_seed = g.next() & SEED_MASK;
    if (!have_key || undrawn) key397 = key397_of(p, pend_seed);
    // planets_only: the pending seed may not have been checked yet (a game
    // shorter than the steps that check one candidate each): walk the
    // stream here, synchronously
    while (!seed_passes(p, pend_seed, key397)) {
        pend_seed = g.next() & SEED_MASK;
        key397 = key397_of(p, pend_seed);
    }
    ng.seed = pend_seed;
    ng.words = create_words<S>(p, pend_seed, key397);
    ng.exhausted = ng.words.exhausted;
    ng.ca = g.a;
    ng.cb = g.b;
    ng.ci = g.k;
    return ng;
}

// Start env i's next game from its NextGame: create (the float half), then
// the stream record and header (part 0).
template <typename T, int S, int PMAX, int NPART = 1, class Sink = GlobalSink<T>>
__device__ __forceinline__ void restart_env(const AstroParams &p, const AstroState &st, int i,
                                            const NextGame<S> &ng, int part, const Sink &sink) {
    int cf = 0;
    const int n = create_env<T, S, PMAX, NPART, Sink>(p, sink, i, create_draws<S>(ng.words), cf, part);
    if (part != 0) return;
    reinterpret_cast<uint4 *>(st.stream)[i] = make_uint4(ng.ca, ng.cb, ng.ci, ng.seed);
    const int flags = (ng.exhausted || cf) ? 2 : 0;
    sink.header(i, make_int4(0, n | (flags << 8), int(UNDRAWN), 0));
}

// The pending seed at the end of a step (the lane holding the env's header):
// an UNDRAWN one is drawn (cursor c); key[397] of a pending seed is gathered
// by the first step that finds it missing (KEY_VALID); with planets_only,
// that step also checks the seed and, if its game has the wrong number of
// planets, draws the stream's next one instead for the following step to
// check -- one candidate per step, off the reset path.  Returns the
// KEY_VALID bit for the header.  (The draws do not depend on the key table:
// the stream cursor evolves identically with and without it.)
__device__ __forceinline__ uint32_t check_pending(const AstroParams &p, const AstroState &st, int i, bool key_valid,
                                                  bool undrawn, const uint4 &c, uint32_t &seed, uint32_t &key) {
    if (key_valid) return KEY_VALID;
    if (!undrawn) {
        if (!p.key_table) return 0u;
        if (seed_passes(p, seed, key)) return KEY_VALID;
    }
    MTStream g{c.x, c.y, c.z, stream_ring_of(st, i)};
    seed = g.next() & SEED_MASK;
    key = 0u;
    reinterpret_cast<uint4 *>(st.stream)[i] = make_uint4(g.a, g.b, g.k, c.w);
    return 0u;
}

__device__ __forceinline__ uint32_t wave_sum32(uint32_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// ---------------------------------------------------------------------------
// the step kernel

// Diagnostic build only (-DASTRO_STAMPS, tools/sweep.py --stamps): s_memtime
// at section boundaries, lane 0 stores them over the stats rows.  Never in
// the shipped library.
#ifdef ASTRO_STAMPS
#define STAMP(k)                                                                         \
    do {                                                                                 \
        __builtin_amdgcn_sched_barrier(0);                                               \
        unsigned long long t_;                                                           \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");        \
        __builtin_amdgcn_sched_barrier(0);                                               \
        stamp_[k] = t_;                                                                  \
        if (k == 0 || k == 11) {   /* 100 MHz wall clock too: shader clock = ratio */      \
            asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
            stamp_[k == 0 ? 12 : 13] = t_;                                                \
        }                                                                                \
    } while (0)
constexpr int NSTAMP = 36;   // 0-13 step sections, 14-15 placement, 16-19 reset pass, 20-31 helper wave,
                              // 32-35 the helper's last reset pass (its 16-19)
// helper-wave stamps: s_memrealtime (HSTAMP_R) and s_memtime (HSTAMP_T) into stamp_[k]
#define HSTAMP_R(k) asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(stamp_[k])::"memory")
#define HSTAMP_T(k)                                                                                   \
    do {                                                                                              \
        __builtin_amdgcn_sched_barrier(0);                                                            \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(stamp_[k])::"memory");          \
        __builtin_amdgcn_sched_barrier(0);                                                            \
    } while (0)
#else
#define HSTAMP_R(k) \
    do {            \
    } while (0)
#define HSTAMP_T(k) \
    do {            \
    } while (0)
#define STAMP(k) \
    do {         \
    } while (0)
#endif
#ifdef ASTRO_STAMPS
#define STAMP_ARG , unsigned long long *stamp_
#define STAMP_PASS , stamp_
#else
#define STAMP_ARG
#define STAMP_PASS
#endif

constexpr int BLOCK = 64;

// Where a launch's controls come from and how many ticks it runs
// (astro_step: one tick of a control array; astro_rollout: K ticks of a
// control array or of an on-device policy).
struct TickDriver {
    const int8_t *control;   // ASTRO_POLICY_CONTROL: int8 [ticks][n_env][nships]
    int32_t policy;          // ASTRO_POLICY_*
    int32_t ticks;           // >= 1 (the lane kernel runs 1 per launch)
    uint64_t seed;           // ASTRO_POLICY_RANDOM
    int64_t tick0;           // ASTRO_POLICY_RANDOM: number of the launch's first tick
    int64_t env_offset;      // ASTRO_POLICY_RANDOM: global id of env 0
    int32_t bots;            // ASTRO_POLICY_BOTS: ship s's bot = (bots >> 4s) & 15
    double script_r2, script_threshold, ship_thrust, ship_rspeed, bullet_speed, ship_radius;
    uint32_t *flag;          // astro_game_step: the completion word the one wave stores flag_seq to
    uint32_t flag_seq;
    int32_t late_block;      // > 0: blocks from here on are the grid's last, partial round (late_block_of)
};

__device__ __forceinline__ int ship_bot(const TickDriver &d, int s) {
    return d.policy == ASTRO_POLICY_BOTS ? (d.bots >> (4 * s)) & 15
         : d.policy == ASTRO_POLICY_RANDOM ? int(ASTRO_BOT_RANDOM) : int(ASTRO_BOT_NOTHING);
}

// Control of ship s of env i at tick kt of the launch.  RANDOM is uniform in
// [0, 6) from splitmix64(global ship id, tick) -- bench.py's `controls`.  A
// ScriptBot ship gets 2 here; its decision needs the state (script_control).
template <int S>
__device__ __forceinline__ int tick_control(const TickDriver &d, int i, int s, size_t n_env, int kt) {
    if (d.policy == ASTRO_POLICY_CONTROL) return int(d.control[(size_t(kt) * n_env + size_t(i)) * S + s]);
    if (ship_bot(d, s) == ASTRO_BOT_RANDOM) {
        const uint64_t id = uint64_t(d.env_offset + i) * uint64_t(S) + uint64_t(s);
        uint64_t z = id * 0x9E3779B97F4A7C15ull + uint64_t(d.tick0 + kt + 1) * 0xD1B54A32D192ED03ull + d.seed;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        return int(((z >> 32) * 6ull) >> 32);
    }
    return 2;   // script.NothingBot
}

// ---------------------------------------------------------------------------
// script.ScriptBot (script.py:13-91) on the bot's ego view (core.roll_ships:
// its own ship first), in the precision numpy evaluates it for the state's
// dtypes (NEP 50: Python-float constants take the array's dtype):
//   X -- ship positions, velocities and bearings, and ship - planet
//        positions: float32 at a game's first tick (create()'s arrays),
//        float64 after;
//   V -- ship - planet velocities: float32 only at the first tick of a
//        one-planet game (its planet's dx is float32 for ever), else float64.
// Scalar ** 2 in the reference is pow(x, 2); x * x here (they differ only
// where pow is not correctly rounded).

// fmod(x, y) for finite x and y > 0 with |x / y| < 2^24 (float) / 2^53
// (double), exactly, in five instructions instead of ocml's fmod: q =
// trunc(x / y) is the true quotient's integer part or, when x / y rounded up
// to the next integer, one more in magnitude (the division is correctly
// rounded, so never one less); x - q y is then a multiple of y's last mantissa
// bit smaller than y in magnitude -- exactly representable -- so the fma
// returns it exactly, and the correction by +-y is an add whose exact result
// (the true remainder) is representable too.  (tests/test_host.py checks the
// argument with exact rationals.)
template <typename C>
__device__ __forceinline__ C exact_fmod(C x, C y) {
    const C q = trunc(x / y);
    C r = __builtin_fma(-q, y, x);
    r = x >= C(0) ? (r < C(0) ? r + y : r) : (r > C(0) ? r - y : r);
    return r;
}
__device__ __forceinline__ float exact_fmod(float x, float y) {
    const float q = truncf(x / y);
    float r = __builtin_fmaf(-q, y, x);
    r = x >= 0.0f ? (r < 0.0f ? r + y : r) : (r > 0.0f ? r - y : r);
    return r;
}

// util.norm_angle (util.py:125-132): ((b + pi) % (2 pi)) - pi with numpy's
// floored remainder (npy_divmod: fmod, + divisor when the signs differ, +0
// for a zero result), in C
template <typename C>
__device__ __forceinline__ C np_norm_angle(C b) {
    const C pi = C(3.141592653589793);          // np.pi (float32: 3.1415927f)
    const C two_pi = C(6.283185307179586);      // 2 * np.pi
    const C x = b + pi;
    // (|x| < 2^24 * 2 pi: bearings change by at most dt * ship_rspeed per tick)
    C m = exact_fmod(x, two_pi);
    m = m != C(0) ? (m < C(0) ? m + two_pi : m) : C(0);
    return m - pi;
}

__device__ __forceinline__ float np_atan2(float y, float x) { return atan2f(y, x); }
__device__ __forceinline__ double np_atan2(double y, double x) { return atan2(y, x); }

// ScriptBot._fly_to (script.py:26-35); t is a value of the angle's dtype
template <typename C>
__device__ __forceinline__ int fly_to(C target, C bearing, C t, bool fwd) {
    const C angle = np_norm_angle<C>(target - bearing);
    if (angle < -t) return 0;   // rotate left
    if (t < angle) return 4;    // rotate right
    return fwd ? 3 : 2;
}

// ScriptBot._danger (script.py:37-62) for one planet: true with the bearing
// to steer for when the course meets the inflated planet soon.  (As in the
// reference, `b` is rebound to the quadratic's linear coefficient before the
// rotation estimate uses it.)
template <typename X, typename V>
__device__ __forceinline__ bool script_danger(const TickDriver &d, X rx, X ry, V rvx, V rvy, X &steer) {
    using L = typename std::conditional<(sizeof(X) >= sizeof(V)), X, V>::type;
    const V speed = sqrt(rvx * rvx + rvy * rvy);            // util.mag(dx)
    const V den = speed + V(1e-12);                          // util.norm(dx)
    const V nx = rvx / den, ny = rvy / den;
    const L lin = L(2) * (L(nx) * L(rx) + L(ny) * L(ry));   // 2 * util.dot(norm(dx), x)
    const X mag = sqrt(rx * rx + ry * ry);
    const X c = mag * mag - X(d.script_r2);
    const L det = lin * lin - L(X(4) * c);
    if (!(L(0) < det)) return false;
    const L sq = sqrt(det);
    if (!(L(0) <= -lin + sq)) return false;
    const L distance = -lin - sq;
    const X bx = np_atan2(rx, ry);                           // util.bearing(x)
    const L rotation = fabs(np_norm_angle<L>(L(bx) - lin));
    const L reach = (L(speed / V(d.ship_thrust)) + L(d.ship_rspeed) / rotation) * L(speed);
    if (!(distance < reach)) return false;
    steer = bx;
    return true;
}

// ScriptBot.__call__ (script.py:64-91): (m*) the bot's own ship, (e*) the
// other ship (two-ship games), planets j < np
template <typename X, typename V, int S, int PMAX>
__device__ __forceinline__ int script_decide(const TickDriver &d, bool solo, int np, const double (&px)[PMAX],
                                          const double (&py)[PMAX], const double (&pdx)[PMAX],
                                          const double (&pdy)[PMAX], double mx, double my, double mdx,
                                          double mdy, double mb, double ex, double ey, double edx, double edy) {
    for (int j = 0; j < PMAX; ++j) {   // don't crash into planets (in index order)
        X steer;
        if (j < np && script_danger<X, V>(d, X(mx) - X(px[j]), X(my) - X(py[j]), V(mdx) - V(pdx[j]),
                                          V(mdy) - V(pdy[j]), steer))
            return fly_to<X>(steer, X(mb), X(d.script_threshold), true);
    }
    if (S == 1 || solo) return 2;      // no enemy to aim for
    // aim for the enemy: where it will be when a bullet gets there
    const X dx = X(ex) - X(mx), dy = X(ey) - X(my);
    const X distance = sqrt(dx * dx + dy * dy);
    const X flight = distance / X(d.bullet_speed);
    const X fx = X(ex) + flight * (X(edx) - X(mdx));
    const X fy = X(ey) + flight * (X(edy) - X(mdy));
    return fly_to<X>(np_atan2(fx - X(mx), fy - X(my)), X(mb), X(d.ship_radius) / distance, false);
}

// dtype dispatch: X float32 at tick 0, V float32 at tick 0 of a one-planet game
template <int S, int PMAX>
__device__ __forceinline__ int script_control(const TickDriver &d, bool solo, bool t0, int np,
                                              const double (&px)[PMAX], const double (&py)[PMAX],
                                              const double (&pdx)[PMAX], const double (&pdy)[PMAX], double mx,
                                              double my, double mdx, double mdy, double mb, double ex, double ey,
                                              double edx, double edy) {
    if (!t0)
        return script_decide<double, double, S, PMAX>(d, solo, np, px, py, pdx, pdy, mx, my, mdx, mdy, mb, ex, ey,
                                                      edx, edy);
    if (np == 1)
        return script_decide<float, float, S, PMAX>(d, solo, np, px, py, pdx, pdy, mx, my, mdx, mdy, mb, ex, ey,
                                                    edx, edy);
    return script_decide<float, double, S, PMAX>(d, solo, np, px, py, pdx, pdy, mx, my, mdx, mdy, mb, ex, ey,
                                                 edx, edy);
}
constexpr int BCHUNK = 8;  // bullets loaded per batch: 8 loads in flight per lane

// One bullet pass in precision C (float at tick 0, double after): collide
// every live bullet with the OLD planets and ships (core.py:241-251), drop the
// hit ones (core.py:264-266), move the rest without gravity and cull those
// with BOTH coordinates outside [-1, 1] (core.py:295-300, 195), compacting in
// order, in place (slot written <= slot read).
template <typename C, typename T, int S, int PMAX>
__device__ __forceinline__ void bullet_pass(const AstroParams &p, typename Store<T>::V *bullets, size_t BC, int i,
                                            int nb, int np, const double (&px)[PMAX], const double (&py)[PMAX],
                                            const double (&sx)[S], const double (&sy)[S],
                                            typename Store<T>::V (&cur)[BCHUNK], bool (&hit)[S], int &w,
                                            int &dropped, bool t0) {
    using V = typename Store<T>::V;
    const C dt = C(p.dt);
    const Guard gp(p.r2_p0), gs(p.r2_s0);
    float pxf[PMAX], pyf[PMAX], sxf[S], syf[S];   // float32 copies, padding parked far away
#pragma unroll
    for (int j = 0; j < PMAX; ++j) {
        pxf[j] = j < np ? float(px[j]) : -FAR_POS;
        pyf[j] = j < np ? float(py[j]) : -FAR_POS;
    }
#pragma unroll
    for (int s = 0; s < S; ++s) {
        sxf[s] = float(sx[s]);
        syf[s] = float(sy[s]);
    }
    for (int base = 0; base < nb; base += BCHUNK) {
        // prefetch the next chunk before working on this one (slots read
        // ahead are never below the write cursor: w <= slot being read)
        V nxt[BCHUNK];
        if (base + BCHUNK < nb) {
#pragma unroll
            for (int u = 0; u < BCHUNK; ++u) {
                const int k = base + BCHUNK + u < nb ? base + BCHUNK + u : 0;
                nxt[u] = bullets[size_t(i) * BC + k];
            }
        }
#pragma unroll
        for (int u = 0; u < BCHUNK; ++u) {
            // branch-free: every slot of the chunk is evaluated (slots past nb
            // hold a copy of slot 0); only the store and the rare exact
            // recheck are conditional
            const bool valid = base + u < nb;
            const double x = double(cur[u].x), y = double(cur[u].y);
            const float xf = valid ? float(cur[u].x) : FAR_POS, yf = valid ? float(cur[u].y) : FAR_POS;
            bool bh = false, amb = false, hs[S];
#pragma unroll
            for (int j = 0; j < PMAX; ++j) bh |= near32(xf, yf, pxf[j], pyf[j], gp, amb);
#pragma unroll
            for (int s = 0; s < S; ++s) hs[s] = near32(xf, yf, sxf[s], syf[s], gs, amb);
            amb |= t0 & valid;
            if (__any(amb)) {   // some lane within 1e-4 of a threshold (or at tick 0): exact tests
                bool bh64 = false, hs64[S];
#pragma unroll
                for (int j = 0; j < PMAX; ++j) bh64 |= (j < np) & closer_exact(x, y, px[j], py[j], gp, t0);
#pragma unroll
                for (int s = 0; s < S; ++s) hs64[s] = closer_exact(x, y, sx[s], sy[s], gs, t0);
                bh = amb ? bh64 : bh;
#pragma unroll
                for (int s = 0; s < S; ++s) hs[s] = amb ? hs64[s] : hs[s];
            }
#pragma unroll
            for (int s = 0; s < S; ++s) {
                bh |= hs[s];
                hit[s] |= hs[s];
            }
            const C ndx = C(cur[u].z) + C(0), ndy = C(cur[u].w) + C(0);
            const C nx = C(x) + dt * ndx, ny = C(y) + dt * ndy;
            const bool keep = valid & !bh & ((C(-1) <= nx && nx <= C(1)) || (C(-1) <= ny && ny <= C(1)));
            const bool fits = w < p.b_cap;
            if (keep & fits) {
                V v;
                v.x = T(nx);
                v.y = T(ny);
                v.z = T(ndx);
                v.w = T(ndy);
                bullets[size_t(i) * BC + w] = v;
            }
            // counters as arithmetic: a conditional ++ of one of two locals
            // is folded into a store through a selected pointer, which sends
            // both to scratch memory
            w += int(keep & fits);
            dropped += int(keep & !fits);
        }
#pragma unroll
        for (int u = 0; u < BCHUNK; ++u) cur[u] = nxt[u];
    }
}

// New bullet of one ship (core.py:267-279) moved and culled like the others.
template <typename C, typename T>
__device__ __forceinline__ void spawn(const AstroParams &p, typename Store<T>::V *bullets, size_t BC, int i,
                                      double sx, double sy, double sdx, double sdy, float ds, float dc, int &w,
                                      int &dropped) {
    using V = typename Store<T>::V;
    const float os = p.spawn_off * ds, oc = p.spawn_off * dc;
    const float vs = p.bullet_speed * ds, vc = p.bullet_speed * dc;
    const C bx = C(sx) + C(os), by = C(sy) + C(oc);
    const C bdx = (C(sdx) + C(vs)) + C(0), bdy = (C(sdy) + C(vc)) + C(0);
    const C dt = C(p.dt);
    const C nx = bx + dt * bdx, ny = by + dt * bdy;
    const bool keep = (C(-1) <= nx && nx <= C(1)) || (C(-1) <= ny && ny <= C(1));
    const bool fits = w < p.b_cap;
    if (keep && fits) {
        V v;
        v.x = T(nx);
        v.y = T(ny);
        v.z = T(bdx);
        v.w = T(bdy);
        bullets[size_t(i) * BC + w] = v;
    }
    w += int(keep && fits);
    dropped += int(keep && !fits);
}

template <typename T, int S, int PMAX>
__global__ __launch_bounds__(BLOCK) void astro_step_kernel(AstroParams p, AstroState st, TickDriver drv,
                                                           float *__restrict__ reward,
                                                           uint8_t *__restrict__ done_out,
                                                           unsigned long long *stats,
                                                           int auto_reset) {
    using V = typename Store<T>::V;
    const int N = st.n_env;
    const int i = blockIdx.x * BLOCK + threadIdx.x;
    const bool active = i < N;
    uint32_t n_bin = 0, n_bout = 0, n_pl = 0, n_drop = 0;
    bool f_reset = false, f_coll = false, f_tout = false;
#ifdef ASTRO_STAMPS
    unsigned long long stamp_[NSTAMP] = {};
#endif
    STAMP(0);

    if (active) {
        const size_t NN = size_t(N);
        const size_t BC = size_t(p.b_cap);   // bullets: [N][b_cap] rows
        V *ships = reinterpret_cast<V *>(st.ships);
        T *ships_b = reinterpret_cast<T *>(st.ships_b);
        V *planets = reinterpret_cast<V *>(st.planets);
        V *bullets = reinterpret_cast<V *>(st.bullets);

        // ---- round 1 of loads: header, ships, control (independent)
        const int4 h = reinterpret_cast<const int4 *>(st.hdr)[i];
        double sx[S], sy[S], sdx[S], sdy[S], sb[S];
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const V v = ships[size_t(s) * NN + i];
            sx[s] = double(v.x);
            sy[s] = double(v.y);
            sdx[s] = double(v.z);
            sdy[s] = double(v.w);
            sb[s] = double(ships_b[size_t(s) * NN + i]);
        }
        int ctl[S];   // (one tick per launch: the host loops astro_rollout's ticks)
        if (S == 2 && drv.policy == ASTRO_POLICY_CONTROL) {
            const uint16_t c2 = reinterpret_cast<const uint16_t *>(drv.control)[i];
            ctl[0] = int(int8_t(c2 & 0xff));
            ctl[S - 1] = int(int8_t(c2 >> 8));
        } else {
#pragma unroll
            for (int s = 0; s < S; ++s) ctl[s] = tick_control<S>(drv, i, s, NN, 0);
        }
        const int tick = int(uint32_t(h.x) & TICK_MASK);
        const bool key_valid = (uint32_t(h.z) & KEY_VALID) != 0;
        const bool undrawn = (uint32_t(h.z) & UNDRAWN) != 0;
        uint32_t pend_seed = uint32_t(h.z) & SEED_MASK;
        int np = h.y & 0xff;
        int flags = (h.y >> 8) & 0xff;
        const int nb = int(uint32_t(h.y) >> 16);
        np = np < 1 ? 1 : (np > PMAX ? PMAX : np);
        const bool live = tick < p.timeout_tick;
        const bool t0 = tick == 0;
        STAMP(1);

        // ---- round 2: planets (every slot: padding is masked below, so
        //      these loads do not wait for the header), the fire word, the
        //      first bullet chunk
        double px[PMAX], py[PMAX], pdx[PMAX], pdy[PMAX];
#pragma unroll
        for (int j = 0; j < PMAX; ++j) {
            const int jj = j < p.p_pad ? j : 0;
            const V v = planets[size_t(jj) * NN + i];
            px[j] = double(v.x);
            py[j] = double(v.y);
            pdx[j] = double(v.z);
            pdy[j] = double(v.w);
        }
        const uint32_t fire_word = p.fire_bits[(live ? tick : 0) >> 5];
        // key[397] of the next game's seed, fetched once per game, off the reset path
        uint32_t pend_key = uint32_t(h.w);
        if (!key_valid && !undrawn && p.key_table) pend_key = p.key_table[pend_seed & SEED_MASK];
        // stream cursor, for check_pending: loaded branch-free, see the quad kernel
        const bool want_c = undrawn || (!key_valid && p.key_table && p.planets_only);
        uintptr_t c_stream = reinterpret_cast<uintptr_t>(st.stream), c_hdr = reinterpret_cast<uintptr_t>(st.hdr);
        asm volatile("" : "+v"(c_stream), "+v"(c_hdr));
        const uint4 c_pend = load_u4_global(want_c ? c_stream : c_hdr, size_t(i));
        V buf[BCHUNK];
#pragma unroll
        for (int u = 0; u < BCHUNK; ++u) {
            const int k = u < nb ? u : 0;
            buf[u] = bullets[size_t(i) * BC + k];
        }
        n_pl = uint32_t(np);
        if (drv.policy == ASTRO_POLICY_BOTS) {   // ScriptBot ships decide on the old state
#pragma unroll
            for (int s = 0; s < S; ++s) {
                const int o = S - 1 - s;
                if (ship_bot(drv, s) == ASTRO_BOT_SCRIPT)
                    ctl[s] = script_control<S, PMAX>(drv, p.solo != 0, t0, np, px, py, pdx, pdy, sx[s], sy[s],
                                                     sdx[s], sdy[s], sb[s], sx[o], sy[o], sdx[o], sdy[o]);
            }
        }

        // ---- ship acceleration (core.py:234-239): thrust along direction(b)
        //      + gravity; floored //2 and %2 of the control code
        float ds[S], dc[S];
        double ax[S], ay[S], dbear[S];
#pragma unroll
        for (int s = 0; s < S; ++s) {
            np_sincosf(float(sb[s]), ds[s], dc[s]);
            double gx, gy;
            if (t0) {
                float fx, fy;
                field<float, PMAX>(px, py, np, sx[s], sy[s], p.gm, fx, fy);
                gx = double(fx);
                gy = double(fy);
            } else {
                field<double, PMAX>(px, py, np, sx[s], sy[s], p.gm, gx, gy);
            }
            const double thr = p.thrust * double(ctl[s] & 1);
            ax[s] = thr * double(ds[s]) + gx;
            ay[s] = thr * double(dc[s]) + gy;
            dbear[s] = p.db * double((ctl[s] >> 1) - 1);
        }

        STAMP(2);
        // ---- collisions on the old state (core.py:241-253): ships vs
        //      ships/planets here, ships/planets vs bullets in the bullet pass
        bool hit[S];
        {
            const Guard gsp(p.r2_sp), gss(p.r2_ss);
            bool amb = false;
#pragma unroll
            for (int s = 0; s < S; ++s) {
                bool hs = false;
#pragma unroll
                for (int j = 0; j < PMAX; ++j)
                    hs |= near32(float(sx[s]), float(sy[s]), j < np ? float(px[j]) : -FAR_POS,
                                 j < np ? float(py[j]) : -FAR_POS, gsp, amb);
                hit[s] = hs;
            }
            bool hh = false;
            if (S == 2) hh = near32(float(sx[0]), float(sy[0]), float(sx[S - 1]), float(sy[S - 1]), gss, amb);
            amb |= t0;
            if (__any(amb)) {   // the exact tests, for the ambiguous lanes (never tick 0, see near32_t0)
#pragma unroll
                for (int s = 0; s < S; ++s) {
                    bool hs = false;
#pragma unroll
                    for (int j = 0; j < PMAX; ++j) hs |= (j < np) & closer_exact(sx[s], sy[s], px[j], py[j], gsp, t0);
                    hit[s] = amb ? hs : hit[s];
                }
                if (S == 2) hh = amb ? closer_exact(sx[0], sy[0], sx[S - 1], sy[S - 1], gss, t0) : hh;
            }
            hit[0] = hit[0] || hh;
            hit[S - 1] = hit[S - 1] || hh;
        }

        STAMP(3);
        // ---- bullets
        int w = 0, dropped = 0;
        if (t0)
            bullet_pass<float, T, S, PMAX>(p, bullets, BC, i, nb, np, px, py, sx, sy, buf, hit, w, dropped, true);
        else
            bullet_pass<double, T, S, PMAX>(p, bullets, BC, i, nb, np, px, py, sx, sy, buf, hit, w, dropped, false);
        n_bin = uint32_t(nb);
        STAMP(4);

        const bool collided = S == 2 ? (hit[0] || hit[S - 1]) : hit[0];
        const bool timeout = !collided && !live;
        const uint8_t done = collided ? 1 : (timeout ? 2 : 0);

        // rewards (core.py:253-260)
        float rw[S];
#pragma unroll
        for (int s = 0; s < S; ++s)
            rw[s] = collided ? (hit[s] ? -1.0f : 1.0f) : (timeout ? p.timeout_reward : 0.0f);
        if (S == 2) {
            reinterpret_cast<float2 *>(reward)[i] = make_float2(rw[0], rw[S - 1]);
        } else {
            reward[i] = rw[0];
        }
        done_out[i] = done;
        STAMP(5);

        if (!done) {
            // ---- fire from the OLD ship state, after the survivors (core.py:267-280)
            if ((fire_word >> (tick & 31)) & 1u) {
#pragma unroll
                for (int s = 0; s < S; ++s) {
                    if (t0)
                        spawn<float, T>(p, bullets, BC, i, sx[s], sy[s], sdx[s], sdy[s], ds[s], dc[s], w, dropped);
                    else
                        spawn<double, T>(p, bullets, BC, i, sx[s], sy[s], sdx[s], sdy[s], ds[s], dc[s], w, dropped);
                }
            }

            // ---- ships: semi-implicit Euler, wrap (core.py:283-288, 189-197)
#pragma unroll
            for (int s = 0; s < S; ++s) {
                const double ndx = sdx[s] + ax[s] * p.dt;
                const double ndy = sdy[s] + ay[s] * p.dt;
                V v;
                v.x = T(wrap_unit<double>(sx[s] + p.dt * ndx));
                v.y = T(wrap_unit<double>(sy[s] + p.dt * ndy));
                v.z = T(ndx);
                v.w = T(ndy);
                ships[size_t(s) * NN + i] = v;
                ships_b[size_t(s) * NN + i] = T(sb[s] + dbear[s]);
            }

            STAMP(6);
            // ---- planets: mutual gravity (core.py:289-294); float32 at tick 0
            //      (create's float32 positions) and for a lone planet (its
            //      arrays stay float32 for the whole game)
            const float dtf = float(p.dt);
            if (np == 1) {
                // a lone planet's own field: r = +0, so gm / max(1e-12, 0) * r
                // is a zero with the sign of gm, exactly
                const float g0 = p.gm < 0.0 ? -0.0f : 0.0f;
                const float ndx = float(pdx[0]) + g0 * dtf;
                const float ndy = float(pdy[0]) + g0 * dtf;
                V v;
                v.x = T(wrap_unit<float>(float(px[0]) + dtf * ndx));
                v.y = T(wrap_unit<float>(float(py[0]) + dtf * ndy));
                v.z = T(ndx);
                v.w = T(ndy);
                planets[i] = v;
            } else {
                double gx[PMAX], gy[PMAX];
                if (t0) {
                    float fx[PMAX], fy[PMAX];
                    planet_field<float, PMAX>(px, py, np, p.gm, fx, fy);
#pragma unroll
                    for (int j = 0; j < PMAX; ++j) {
                        gx[j] = double(fx[j] * dtf);   // float32 a * dt, then float64 add
                        gy[j] = double(fy[j] * dtf);
                    }
                } else {
                    planet_field<double, PMAX>(px, py, np, p.gm, gx, gy);
#pragma unroll
                    for (int j = 0; j < PMAX; ++j) {
                        gx[j] = gx[j] * p.dt;
                        gy[j] = gy[j] * p.dt;
                    }
                }
#pragma unroll
                for (int j = 0; j < PMAX; ++j) {
                    if (j < np) {
                        const double ndx = pdx[j] + gx[j];
                        const double ndy = pdy[j] + gy[j];
                        V v;
                        v.x = T(wrap_unit<double>(px[j] + p.dt * ndx));
                        v.y = T(wrap_unit<double>(py[j] + p.dt * ndy));
                        v.z = T(ndx);
                        v.w = T(ndy);
                        planets[size_t(j) * NN + i] = v;
                    }
                }
            }
            STAMP(7);
            if (dropped) flags |= 1;
            const uint32_t kv = check_pending(p, st, i, key_valid, undrawn, c_pend, pend_seed, pend_key);
            reinterpret_cast<int4 *>(st.hdr)[i] =
                make_int4(tick + 1, np | (flags << 8) | (w << 16), int(pend_seed | kv), int(pend_key));
            n_bout = uint32_t(w);
            n_drop = uint32_t(dropped);
            STAMP(8);
        } else {
            STAMP(9);
            f_coll = collided;
            f_tout = timeout;
            if (auto_reset) {
                const uint4 c = reinterpret_cast<const uint4 *>(st.stream)[i];
                const NextGame<S> ng = next_game<S>(p, pend_seed, pend_key, key_valid || p.key_table, undrawn, c,
                                                    stream_ring_of(st, i));
                restart_env<T, S, PMAX>(p, st, i, ng, 0, GlobalSink<T>{st});
                f_reset = true;
            }
            STAMP(10);
        }
    }
    STAMP(11);
#ifdef ASTRO_STAMPS
    if (stats && (threadIdx.x & 63) == 0) {
        unsigned long long *row = stats + size_t(blockIdx.x * (BLOCK / 64) + threadIdx.x / 64) * NSTAMP;
#pragma unroll
        for (int k = 0; k < NSTAMP; ++k) row[k] = stamp_[k];
    }
    return;
#endif

    // ---- statistics: one private slot per wave (contention-free no-return
    //      atomics; summed over slots by the host)
    if (stats) {
        const uint64_t m_reset = __ballot(f_reset), m_coll = __ballot(f_coll), m_tout = __ballot(f_tout);
        // per-lane counts are < 2^16 and, for b_cap <= 1023, so are their
        // wave sums: pack two counters per 32-bit reduction
        const bool packed = p.b_cap <= 1023;
        const uint32_t a = wave_sum32(packed ? (n_bin | (n_bout << 16)) : n_bin);
        const uint32_t b = wave_sum32(packed ? (n_pl | (n_drop << 16)) : n_bout);
        const uint32_t c = packed ? 0u : wave_sum32(n_pl | (n_drop << 16));
        if ((threadIdx.x & 63) == 0) {
            unsigned long long *slot = stats + size_t(blockIdx.x * (BLOCK / 64) + threadIdx.x / 64) * ASTRO_NSTATS;
            const uint64_t bin = packed ? (a & 0xffff) : a;
            const uint64_t bout = packed ? (a >> 16) : b;
            const uint64_t pl = packed ? (b & 0xffff) : (c & 0xffff);
            const uint64_t drop = packed ? (b >> 16) : (c >> 16);
            if (bin) atomicAdd(slot + ASTRO_STAT_BULLETS_IN, (unsigned long long)bin);
            if (bout) atomicAdd(slot + ASTRO_STAT_BULLETS_OUT, (unsigned long long)bout);
            if (m_reset) atomicAdd(slot + ASTRO_STAT_RESETS, (unsigned long long)__popcll(m_reset));
            if (m_coll) atomicAdd(slot + ASTRO_STAT_COLLISIONS, (unsigned long long)__popcll(m_coll));
            if (m_tout) atomicAdd(slot + ASTRO_STAT_TIMEOUTS, (unsigned long long)__popcll(m_tout));
            if (drop) atomicAdd(slot + ASTRO_STAT_OVERFLOWS, (unsigned long long)drop);
            if (pl) atomicAdd(slot + ASTRO_STAT_PLANETS, (unsigned long long)pl);
        }
    }
}

// ---------------------------------------------------------------------------
// The quad kernel: FOUR lanes per env (16 envs per wave).
//
// At 65,536 envs a lane-per-env launch is 1,024 waves = one per SIMD, and one
// wave alone issues a VALU op at best every 4 cycles with nothing to hide
// its waits (measured: 3.1k VALU ops + 17k cycles of waits per wave).  Here
// the same envs make 4,096 waves (4 per SIMD) and each lane does a quarter of
// its env: lane q owns planet slots q, q+4, .. and bullet slots q, q+4, ..;
// lanes 0..S-1 own the ships.  Positions are broadcast inside the quad with
// DPP quad_perm (no LDS, no memory), hit flags are OR-ed and surviving
// bullets compacted in order with one ballot per round.  Every float64 sum
// keeps the reference's sequential order, so results are bit-identical to
// the lane-per-env kernel.

// Lane groups of LPE = 4 (quad kernel) or 2 (pair kernel) lanes per env.
// Broadcast lane J of the caller's group with DPP quad_perm: (J,J,J,J) for
// quads, (J,J,J+2,J+2) for the two pairs of a quad.
template <int J, int LPE = 4>
__device__ __forceinline__ int quad_bcast_i(int v) {
    static_assert(LPE == 4 || LPE == 2, "groups of 4 or 2 lanes");
    constexpr int sel = LPE == 4 ? J * 0x55 : (J | (J << 2) | ((J + 2) << 4) | ((J + 2) << 6));
    return __builtin_amdgcn_mov_dpp(v, sel, 0xf, 0xf, false);
}
template <int J, int LPE = 4>
__device__ __forceinline__ float quad_bcast(float v) {
    return __int_as_float(quad_bcast_i<J, LPE>(__float_as_int(v)));
}
template <int J, int LPE = 4>
__device__ __forceinline__ double quad_bcast(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = quad_bcast_i<J, LPE>(int(b & 0xffffffffll));
    const int hi = quad_bcast_i<J, LPE>(int(b >> 32));
    return __longlong_as_double((long long)(uint32_t(lo)) | ((long long)hi << 32));
}

// broadcast slot m of every lane J of the group into out[LPE*m + J]
template <typename T, int PPL, int LPE>
__device__ __forceinline__ void bcast_slots(const T (&mine)[PPL], double (&out)[LPE * PPL]) {
#pragma unroll
    for (int m = 0; m < PPL; ++m) {
        out[LPE * m + 0] = double(quad_bcast<0, LPE>(mine[m]));
        out[LPE * m + 1] = double(quad_bcast<1, LPE>(mine[m]));
        if constexpr (LPE == 4) {
            out[LPE * m + 2] = double(quad_bcast<2, LPE>(mine[m]));
            out[LPE * m + 3] = double(quad_bcast<3, LPE>(mine[m]));
        }
    }
}

// a double from lane A/B/C/D of the caller's quad (DPP quad_perm(A,B,C,D):
// lane i of the quad reads lane (A,B,C,D)[i])
template <int A, int B, int C, int D>
__device__ __forceinline__ double quad_perm_d(double v) {
    constexpr int sel = A | (B << 2) | (C << 4) | (D << 6);
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp(int(b & 0xffffffffll), sel, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_mov_dpp(int(b >> 32), sel, 0xf, 0xf, false);
    return __longlong_as_double((long long)(uint32_t(lo)) | ((long long)hi << 32));
}

// a double from the other lane of the caller's pair (quad_perm(1,0,3,2))
__device__ __forceinline__ double pair_swap(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp(int(b & 0xffffffffll), 0xB1, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_mov_dpp(int(b >> 32), 0xB1, 0xf, 0xf, false);
    return __longlong_as_double((long long)(uint32_t(lo)) | ((long long)hi << 32));
}

// Within each 16-lane row of the wave (the reset pass's rows), by DPP:
// lane K of the row to the whole row (row_newbcast), and lane (u + R) mod 16
// to lane u (row_ror:16-R).  A DPP move instead of an LDS-routed ds_bpermute.
template <int K>
__device__ __forceinline__ int row_bcast_i(int v) {
    return __builtin_amdgcn_update_dpp(0, v, 0x150 + K, 0xf, 0xf, false);
}
template <int K>
__device__ __forceinline__ float row_bcast(float v) {
    return __int_as_float(row_bcast_i<K>(__float_as_int(v)));
}
template <int K>
__device__ __forceinline__ double row_bcast(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = row_bcast_i<K>(int(b & 0xffffffffll));
    const int hi = row_bcast_i<K>(int(b >> 32));
    return __longlong_as_double((long long)(uint32_t(lo)) | ((long long)hi << 32));
}
template <int R>
__device__ __forceinline__ int row_from_i(int v) {   // lane u of the row reads lane (u + R) mod 16
    static_assert(R > 0 && R < 16, "row rotation");
    return __builtin_amdgcn_update_dpp(0, v, 0x120 + (16 - R), 0xf, 0xf, false);
}
template <int R>
__device__ __forceinline__ float row_from(float v) {
    return __int_as_float(row_from_i<R>(__float_as_int(v)));
}

// OR of a per-lane flag over the lane's group (all group lanes must be active)
template <int LPE = 4>
__device__ __forceinline__ bool quad_any(bool f, int lane) {
    return ((__ballot(f) >> (lane & ~(LPE - 1))) & ((1ull << LPE) - 1)) != 0;
}

#ifndef ASTRO_QUAD_WAVES
#define ASTRO_QUAD_WAVES 4
#endif
// step waves per workgroup of the small-N (quad) helper instance: config
// 2's 256 waves spread over more CUs (four: 6.18 us, two: 5.52, one: 5.31
// with its helper, i.e. 128-thread workgroups; c3 wants eight, below)
#ifndef ASTRO_QW_SMALL
#define ASTRO_QW_SMALL 1
#endif
constexpr int QW_SMALL = ASTRO_QW_SMALL;
#ifndef ASTRO_QW_PAIR_HELP
#define ASTRO_QW_PAIR_HELP 8
#endif
// step waves per workgroup of the pair instance with helpers (c3: eight,
// 16-wave workgroups, 12.55 -> 12.13 us A/B; two: 13.12)
constexpr int QW_PAIR_HELP = ASTRO_QW_PAIR_HELP;
#ifndef ASTRO_QW_PAIR
#define ASTRO_QW_PAIR 4
#endif
constexpr int QW_PAIR = ASTRO_QW_PAIR;   // 4-slot pair instance without helpers (1M: 4 = 111, 8 = 114, 16 = 131 us)
#ifndef ASTRO_HELP_MAX_WAVES
#define ASTRO_HELP_MAX_WAVES 2048
#endif
// Waves per quad-kernel workgroup.  The waves of a workgroup share nothing
// (each has its own LDS rows and syncs only itself); four per workgroup make
// a quarter as many workgroups for the dispatcher (launch floor 2.0 -> 1.6
// us, tools/mb_launch.hip).
constexpr int QW = ASTRO_QUAD_WAVES;
constexpr int QBLOCK = 64 * QW;

// A wave's own LDS traffic in order: every lane's writes before any lane's
// later reads (LDS runs a wave's instructions in issue order; this keeps the
// compiler from reordering around it).  No s_barrier: waves never wait for
// each other.
__device__ __forceinline__ void wave_sync() {
    if constexpr (QW == 1) {
        __syncthreads();
    } else {
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
}
constexpr int QWIN = 1024;        // live bullets per window of the quad kernel's LDS index


// Inclusive prefix sum over the 64 lanes of a wave (all lanes active): DPP
// row shifts inside each row of 16, then the row totals.
__device__ __forceinline__ int wave_incl_scan(int v, int lane) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);   // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);   // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);   // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);   // row_shr:8
    const int r0 = __builtin_amdgcn_readlane(v, 15);
    const int r1 = __builtin_amdgcn_readlane(v, 31);
    const int r2 = __builtin_amdgcn_readlane(v, 47);
    const int row = lane >> 4;
    return v + (row > 0 ? r0 : 0) + (row > 1 ? r1 : 0) + (row > 2 ? r2 : 0);
}

// Bullet index word (LDS): env in the wave | slot << 5 | last-of-env << 21 |
// nplanets << 22 | tick-0 << 27
__device__ __forceinline__ int bw_env(uint32_t w) { return int(w & 31u); }
__device__ __forceinline__ int bw_slot(uint32_t w) { return int((w >> 5) & 0xffffu); }
__device__ __forceinline__ bool bw_last(uint32_t w) { return (w >> 21) & 1u; }
__device__ __forceinline__ int bw_np(uint32_t w) { return int((w >> 22) & 31u); }
__device__ __forceinline__ bool bw_t0(uint32_t w) { return (w >> 27) & 1u; }
__device__ __forceinline__ uint32_t bw_tag(int e, int np, bool t0) {
    return uint32_t(e) | (uint32_t(np) << 22) | (t0 ? 1u << 27 : 0u);
}

// Index window [w0, w0 + QWIN) of the wave's live bullets: the group of an
// env whose bullets are numbered off .. off + nb - 1 writes the words of
// those in the window, lane q a contiguous run of ceil(nb / LPE) slots (the
// word of slot k + 1 is the word of slot k plus 1 << 5: an add and an LDS
// store per slot; the last slot's flag is OR-ed in after the loop).
template <int LPE, int QWN = QWIN>
__device__ __forceinline__ void index_window(uint32_t *s_index, int w0, int off, int nb, int q, uint32_t tag) {
    const int h = (nb + LPE - 1) / LPE;
    const int k0 = max(q * h, w0 - off), k1 = min(min(nb, (q + 1) * h), w0 + QWN - off);
    uint32_t w = tag | (uint32_t(k0) << 5);
    uint32_t *dst = s_index + (off + k0 - w0);
    for (int k = k0; k < k1; ++k, w += 1u << 5) *dst++ = w;
    if (k1 == nb && k1 > k0) dst[-1] = w - (1u << 5) + (1u << 21);   // last of the env
}

// create()'s ship s (second: s == 1 of two) and planet values from the
// draws and the direction()s (core.py:93-121); shared by the reset pass and
// the pair helpers' pre-create so that both are the same arithmetic
template <typename T, int S>
__device__ __forceinline__ typename Store<T>::V create_ship(const AstroParams &p, const CreateDraws<S> &d, bool second,
                                                           float is, float ic, T &b_out) {
    const float u0 = float(d.u_out[0]) - 0.5f;
    const float u1 = float(d.u_out[1]) - 0.5f;
    const float o0 = p.outer_pos * (u0 > 0.0f ? 1.0f : (u0 < 0.0f ? -1.0f : 0.0f));
    const float o1 = p.outer_pos * (u1 > 0.0f ? 1.0f : (u1 < 0.0f ? -1.0f : 0.0f));
    const float i0 = p.inner_pos * is, i1 = p.inner_pos * ic;
    const bool outer_first = d.u_choice < 0.5;
    float sx, sy;
    if (d.n == 1) {
        sx = second ? -o0 : o0;
        sy = second ? -o1 : o1;
    } else {
        const bool outer = second ? !outer_first : outer_first;
        sx = outer ? o0 : i0;
        sy = outer ? o1 : i1;
    }
    b_out = T(6.2831855f * float(second ? d.u_bear[S - 1] : d.u_bear[0]));
    typename Store<T>::V v;
    v.x = T(sx);
    v.y = T(sy);
    v.z = T(0);
    v.w = T(0);
    return v;
}

// planet j of an n-planet game: position angle (sn, cs), velocity angle (vs, vc)
template <typename T>
__device__ __forceinline__ typename Store<T>::V create_planet(const AstroParams &p, int n, float sn, float cs,
                                                             float vs, float vc) {
    typename Store<T>::V v;
    if (n <= 1) {
        v.x = v.y = v.z = v.w = T(0);
    } else {
        const double amp = sqrt(p.gravity * p.planet_mass * double(n - 1) / 2.0);
        v.x = T(p.planet_orbit * sn);
        v.y = T(p.planet_orbit * cs);
        v.z = T(amp * double(vs));
        v.w = T(amp * double(vc));
    }
    return v;
}

// create() of one env spread over a row of 16 lanes, for PMAX <= 8: each
// lane evaluates ONE direction() -- planet u's position angle (u < PMAX),
// planet u - PMAX's velocity angle, or the inner ship slot's (u = 2 PMAX;
// with 8 planet slots every lane evaluates that one as a second) -- and the
// results move by shuffles; lane s < S writes ship s, lane j < n planet j
// (same arithmetic as create_env, bit for bit).  All lanes of the row must
// be active; `write` gates the stores.
template <typename T, int S, int PMAX, class Sink>
__device__ __forceinline__ int create_env_row(const AstroParams &p, const Sink &sink, int ie,
                                              const CreateDraws<S> &d, int u, int row0, bool write) {
    static_assert(2 * PMAX <= 16, "one planet angle per lane of a 16-lane row");
    constexpr bool INNER_LANE = 2 * PMAX + 1 <= 16;   // the inner ship angle on lane 2 PMAX
    using V = typename Store<T>::V;
    int n = d.n;
    const double stp = TWO_PI / double(n);
    const double base = TWO_PI * d.u_base;
    const double turn = double(d.reverse) * PI / 2.0;
    const int j = u < PMAX ? u : (u < 2 * PMAX ? u - PMAX : 0);
    const double orient = base + double(j) * stp;
    float ang = u < PMAX ? float(orient) : float(orient + turn);
    if (INNER_LANE) ang = u == 2 * PMAX ? float(TWO_PI * d.u_inner) : ang;
    float sn, cs;
    np_sincosf(ang, sn, cs);
    float is, ic;
    if constexpr (INNER_LANE) {
        is = row_bcast<INNER_LANE ? 2 * PMAX : 0>(sn);
        ic = row_bcast<INNER_LANE ? 2 * PMAX : 0>(cs);
    } else {
        np_sincosf(float(TWO_PI * d.u_inner), is, ic);
    }
    const float vs = row_from<PMAX>(sn), vc = row_from<PMAX>(cs);   // (lanes u < PMAX: lane PMAX + u's)

    // ships (core.py:93-109): lane u < S writes ship u
    T b;
    const V sv = create_ship<T, S>(p, d, S == 2 && u == 1, is, ic, b);
    if (write && u < S) sink.ship(u, ie, sv, b);
    // planets (core.py:111-121): lane j < n writes planet j
    if (write && u < PMAX) {
        const V v = create_planet<T>(p, n, sn, cs, vs, vc);
        if (u < n) sink.planet(u, 0, ie, v);
    }
    if (n > PMAX) n = PMAX;
    return n;
}

// One pass of the quad kernel's auto-reset: the next game (core.py:83,
// 86-135) of up to four finished envs at once, 16 lanes per env (row r of
// the wave serves the r-th lowest leader lane in `todo`).  create()'s draws
// are the first 12 + 2S outputs of RandomState(seed) when randint(1,
// max_planets + 1) accepts its first word: lane u of the row yields output
// u, its two init-key inputs coming from the row's lanes 0 (seed chain) and
// 1 (key[397] chain) through LDS, so the serial part is one chain step per
// output instead of two chains plus tempering; the float work of create()
// then runs spread over the row (ship u, planet u).  An env whose first
// randint word is rejected is flagged in s_serial for the quad's serial
// create, and so is one whose game ended at its first step (its seed still
// UNDRAWN).  The stream cursor is left alone: the next game's seed is drawn
// by the env's first step.  Returns the leaders not yet served.
template <typename T, int S, int PMAX, int LPE, bool PRE = false, class Sink = GlobalSink<T>>
__device__ __forceinline__ uint64_t wave_reset_pass(const AstroParams &p, const AstroState &st, uint64_t todo,
                                                    int lane, int i, uint32_t pend_seed, uint32_t pend_key,
                                                    bool have_key, bool undrawn, uint32_t (*s_chain)[2][13 + 2 * S],
                                                    int *s_serial, const Sink &sink_all STAMP_ARG,
                                                    const uint32_t (*pre)[2][13 + 2 * S] = nullptr) {
    constexpr int NW = 12 + 2 * S;   // outputs create() draws, randint accepting its first word
    int leader[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {   // uniform
        leader[r] = todo ? int(__builtin_ctzll(todo)) : -1;
        todo &= todo ? todo - 1 : 0;
    }
    const int row = lane >> 4, u = lane & 15, row0 = lane & ~15;
    const int L = row == 0 ? leader[0] : row == 1 ? leader[1] : row == 2 ? leader[2] : leader[3];
    const bool on = L >= 0;
    const int src = on ? L : 0;
    const int ie = __shfl(i, src, 64);
    const uint32_t seed = uint32_t(__shfl(int(pend_seed), src, 64));
    const uint32_t key = uint32_t(__shfl(int(pend_key), src, 64));
    const bool hk = __shfl(int(have_key), src, 64) != 0;
    const bool ud = __shfl(int(undrawn), src, 64) != 0;

    const int uw = u < NW ? u : 0;
    uint32_t a0, a1, b0;
    if constexpr (PRE) {   // the env's two chains, made ahead (a helper wave, HelpBox)
        const int le = src / LPE;
        a0 = pre[le][0][uw];
        a1 = pre[le][0][uw + 1];
        b0 = pre[le][1][uw];
    } else {
        // init-key chains: even lanes run key[0..] from the seed, odd lanes key[397..]
        const uint32_t k397 = hk ? key : mt_key_at(seed, 0, MT_PROLOGUE);
        const bool bchain = u & 1;
        const uint32_t koff = bchain ? 397u : 0u;
        uint32_t xs[NW + 1];
        xs[0] = bchain ? k397 : seed;
#pragma unroll
        for (int k = 0; k < NW; ++k) xs[k + 1] = mt_key_next(xs[k], koff + uint32_t(k + 1));
        if (u < 2) {
#pragma unroll
            for (int k = 0; k <= NW; ++k) s_chain[row][u][k] = xs[k];
        }
        wave_sync();
        a0 = s_chain[row][0][uw];
        a1 = s_chain[row][0][uw + 1];
        b0 = s_chain[row][1][uw];
        wave_sync();   // s_chain is free for the next pass
    }
    const uint32_t y = (a0 & 0x80000000u) | (a1 & 0x7fffffffu);
    const uint32_t w = mt_temper(b0 ^ (y >> 1) ^ ((a1 & 1u) ? 0x9908b0dfu : 0u));   // output u
    STAMP(16);

    // randint(1, max_planets + 1) on output 0
    const uint32_t rng = uint32_t(p.max_planets - 1);
    uint32_t mask = rng;
    mask |= mask >> 1;
    mask |= mask >> 2;
    mask |= mask >> 4;
    mask |= mask >> 8;
    mask |= mask >> 16;
    const uint32_t v = uint32_t(row_bcast_i<0>(int(w))) & mask;
    const bool fast = !ud && rng != 0 && v <= rng && (p.planets_only == 0 || int(v) + 1 == p.planets_only);
    // lane k of the row: R_k = rand() of outputs k, k + 1
    const uint32_t wn = uint32_t(row_from_i<1>(int(w)));
    const double R = rand53(w, wn);
    CreateDraws<S> d;
    d.n = 1 + int(v);
    const bool many = d.n > 1;
    d.u_out[0] = row_bcast<1>(R);
    d.u_out[1] = row_bcast<3>(R);
    d.u_inner = row_bcast<5>(R);
    // (every shuffle unconditional: its source lane must be active)
    const double r_choice = row_bcast<7>(R);
    const double r_base = row_bcast<9 + 2 * S>(R);
    const uint32_t w_rev = uint32_t(row_bcast_i<11 + 2 * S>(int(w)));
    d.u_choice = many ? r_choice : 1.0;
#pragma unroll
    for (int s = 0; s < S; ++s) d.u_bear[s] = many ? (s == 0 ? row_bcast<9>(R) : row_bcast<11>(R))
                                                   : (s == 0 ? r_choice : row_bcast<9>(R));
    d.u_base = many ? r_base : 0.0;
    d.reverse = many && (w_rev & 1u) == 0 ? -1 : 1;
    d.exhausted = false;   // NW outputs, far below the 227 the lazy generator covers
    STAMP(17);

    const Sink sink = sink_all.for_row(row);   // where row `row`'s game goes
    int n, cf = 0;
    if constexpr (2 * PMAX <= 16) {
        n = create_env_row<T, S, PMAX>(p, sink, ie, d, u, row0, on && fast);
    } else {
        if (on && fast) n = create_env<T, S, PMAX, 16, Sink>(p, sink, ie, d, cf, u);
    }
    STAMP(18);
    if (on && fast) {
        if (u == 0) {   // the stream record's game seed and the header, as restart_env
            sink.stream_seed(ie, seed);
            sink.header(ie, make_int4(0, n | (cf ? 2 << 8 : 0), int(UNDRAWN), 0));
        }
    }
    if (on && !fast && u == 0) s_serial[L / LPE] = 1;
    STAMP(19);
    return todo;
}

// Counters one tick of a quad-kernel wave adds to its stats row.
struct QuadCounts {
    uint32_t n_bin, n_bout, n_pl, n_drop;   // per lane
    uint32_t c_reset, c_coll, c_tout;       // per wave
    uint32_t c_serial;                      // per wave: resets by the serial create
};


// The value every lane of the wave holds, or 0 when they differ (wave-uniform,
// in an SGPR: a uniform planet count lets the sums drop their per-lane
// k < np selects, e.g. config 3's 3-planet games)
__device__ __forceinline__ int wave_uniform_count(int v) {
    const int v0 = __builtin_amdgcn_readfirstlane(v);
    return __builtin_amdgcn_readfirstlane(int(__all(v == v0))) ? v0 : 0;
}

// One tick of the quad kernel's wave (16 envs), tick kt of the launch.
// The surviving envs' planet update (core.py:289-294): gravity of all
// planets incl. self, in the reference's order; float32 at tick 0 / for a
// lone planet.  Lane q's planet slots q + LPE m -> out[m] (slots < np);
// every lane of a group calls it (DPP broadcasts).  The step wave runs it
// for its surviving envs, or -- with helper waves -- the helper runs it for
// every env during the step and stores the survivors' after the post.
template <typename T, int S, int PMAX, int LPE, int PPL>
__device__ __forceinline__ void planet_update(const AstroParams &p, const typename Store<T>::V (&pv)[PPL],
                                              const T (&mpx)[PPL], const T (&mpy)[PPL], int q, int np, bool t0,
                                              bool slot_last, typename Store<T>::V (&out)[PPL]) {
    using V = typename Store<T>::V;
    const int np_uni = wave_uniform_count(np);
    const float dtf = float(p.dt);
    double px[PMAX], py[PMAX];
    {   // the planets again from the quad (DPP) rather than 2*PMAX
        // doubles held live across the bullet pass
        T rx[PPL], ry[PPL];
#pragma unroll
        for (int m = 0; m < PPL; ++m) {
            rx[m] = mpx[m];
            ry[m] = mpy[m];
            asm volatile("" : "+v"(rx[m]), "+v"(ry[m]));
        }
        bcast_slots<T, PPL, LPE>(rx, px);
        bcast_slots<T, PPL, LPE>(ry, py);
    }
    // Pair kernel, 4 slots: the float64 planet-planet factors
    // gm / max(1e-12, d2) of the 6 distinct pairs, 3 per lane (d2 and
    // so the factor are the same bit for bit both ways round), the
    // partner's two by DPP; row i of lane q's planets i = q, q + 2 is
    // then F(i, j) for j = 0..3 (see symmetric_rows)
    double Fr[PPL][PMAX];
    if constexpr (LPE == 2 && PMAX == 4) {
        const bool l0 = q == 0;
        // F(i, j) on lane 0, F(i1, j1) on lane 1: operands selected
        // first, one division per lane
        // (both lanes' differences, then one selected: a select between the
        // array elements would index the arrays in memory)
        auto fac = [&](int i, int j, int i1, int j1) {
            const double dx0 = px[j] - px[i], dx1 = px[j1] - px[i1];
            const double dy0 = py[j] - py[i], dy1 = py[j1] - py[i1];
            const double ddx = l0 ? dx0 : dx1, ddy = l0 ? dy0 : dy1;
            return div_gravity(p.gm, max_floor(ddx * ddx + ddy * ddy));
        };
        // lane 0: A = F01, B = F03, C = F02; lane 1: A = F12, B = F23, C = F13
        // (B is only read for planet slot 3: skipped when no env has it)
        const double A = fac(0, 1, 1, 2);
        const double B = slot_last ? fac(0, 3, 2, 3) : 0.0;
        const double C = fac(0, 2, 1, 3);
        const double A2 = pair_swap(A), B2 = pair_swap(B);   // lane 0: F12, F23; lane 1: F01, F03
        const double z = p.gm;   // (self: any finite factor of gm's sign, see below)
        // planet q:     lane 0 [-, F01, F02, F03]   lane 1 [F10, -, F12, F13]
        // planet q + 2: lane 0 [F20, F21, -, F23]   lane 1 [F30, F31, F32, -]
        Fr[0][0] = l0 ? z : A2;
        Fr[0][1] = l0 ? A : z;
        Fr[0][2] = l0 ? C : A;
        Fr[0][3] = l0 ? B : C;
        Fr[1][0] = l0 ? C : B2;
        Fr[1][1] = l0 ? A2 : C;
        Fr[1][2] = l0 ? z : B;
        Fr[1][3] = l0 ? B2 : z;
    }
    // Quad kernel, 4 slots (config 2): lane q's planet is q; F(q, q + 1) and
    // F(q, q + 2) (mod 4) computed here from the neighbours' planets (DPP
    // rotations), F(q, q + 3) = F(q + 3, q) is lane q + 3's first: 2 divisions
    // per lane instead of field()'s 4 (self term included)
    if constexpr (LPE == 4 && PMAX == 4) {
        const double ox = double(mpx[0]), oy = double(mpy[0]);
        const double x1 = quad_perm_d<1, 2, 3, 0>(ox), y1 = quad_perm_d<1, 2, 3, 0>(oy);
        const double x2 = quad_perm_d<2, 3, 0, 1>(ox), y2 = quad_perm_d<2, 3, 0, 1>(oy);
        const double dx1 = x1 - ox, dy1 = y1 - oy, dx2 = x2 - ox, dy2 = y2 - oy;
        const double A = div_gravity(p.gm, max_floor(dx1 * dx1 + dy1 * dy1));   // F(q, q + 1)
        const double B = div_gravity(p.gm, max_floor(dx2 * dx2 + dy2 * dy2));   // F(q, q + 2)
        const double C = quad_perm_d<3, 0, 1, 2>(A);                              // F(q, q + 3)
#pragma unroll
        for (int k = 0; k < PMAX; ++k) {
            const int d = (k - q) & 3;   // (self, d == 0: gm, see below)
            Fr[0][k] = d == 1 ? A : (d == 2 ? B : (d == 3 ? C : p.gm));
        }
    }
    // Pair kernel, 8 slots (config 5): the 28 distinct pair factors, 14 per
    // lane instead of 32 (each own planet's 8 terms), exchanged by DPP.
    // Lane q owns planets q + 2m (m < 4): the 6 pairs among its own planets
    // it computes alone (Sf); the 16 pairs of an own planet with a partner
    // planet (Xf[m][j] = F(own m, partner planet j), planet j of the other
    // lane = 2j + 1 - q) are split: pair (a, b), a != b, computed by both
    // lanes at once -- lane 0 F(2a, 2b + 1), lane 1 F(2a + 1, 2b) -- gives
    // each lane Xf[a][b] and, from the other lane, Xf[b][a]; the 4 diagonal
    // pairs (2a, 2a + 1) two per lane, swapped likewise.
    if constexpr (LPE == 2 && PMAX == 8) {
        const bool l0 = q == 0;
        auto fac = [&](double ax, double ay, double bx, double by) {
            const double dx = bx - ax, dy = by - ay;   // (either sign: d2 is the same bit for bit)
            return div_gravity(p.gm, max_floor(dx * dx + dy * dy));
        };
        double ox[PPL], oy[PPL], tx[PPL], ty[PPL];   // own planets; the other lane's
#pragma unroll
        for (int m = 0; m < PPL; ++m) {
            ox[m] = double(mpx[m]);
            oy[m] = double(mpy[m]);
            tx[m] = l0 ? px[2 * m + 1] : px[2 * m];
            ty[m] = l0 ? py[2 * m + 1] : py[2 * m];
        }
        double Sf[PPL][PPL], Xf[PPL][PPL];
#pragma unroll
        for (int a = 0; a < PPL; ++a) {
            Sf[a][a] = p.gm;   // (self: gm, see below)
#pragma unroll
            for (int b = a + 1; b < PPL; ++b) {
                Sf[a][b] = Sf[b][a] = fac(ox[a], oy[a], ox[b], oy[b]);
                const double v = fac(ox[a], oy[a], tx[b], ty[b]);
                Xf[a][b] = v;
                Xf[b][a] = pair_swap(v);
            }
        }
#pragma unroll
        for (int d = 0; d < PPL / 2; ++d) {   // lane 0: pair (4d, 4d + 1), lane 1: (4d + 2, 4d + 3)
            const double v = fac(l0 ? ox[2 * d] : ox[2 * d + 1], l0 ? oy[2 * d] : oy[2 * d + 1],
                                 l0 ? tx[2 * d] : tx[2 * d + 1], l0 ? ty[2 * d] : ty[2 * d + 1]);
            const double w = pair_swap(v);
            Xf[2 * d][2 * d] = l0 ? v : w;
            Xf[2 * d + 1][2 * d + 1] = l0 ? w : v;
        }
#pragma unroll
        for (int m = 0; m < PPL; ++m) {
#pragma unroll
            for (int k = 0; k < PMAX; ++k) Fr[m][k] = (k & 1) == q ? Sf[m][k >> 1] : Xf[m][k >> 1];
        }
    }
#pragma unroll
    for (int m = 0; m < PPL; ++m) {
        const int j = q + LPE * m;
        if (j < np) {
            const double pxj = double(mpx[m]), pyj = double(mpy[m]);
            const double pdx = double(pv[m].z), pdy = double(pv[m].w);
            V v;
            if (np == 1) {
                // a lone planet's own field: r = +0, so gm / max(1e-12, 0) * r
                // is a zero with the sign of gm, exactly
                const float g0 = p.gm < 0.0 ? -0.0f : 0.0f;
                const float ndx = float(pdx) + g0 * dtf, ndy = float(pdy) + g0 * dtf;
                v.x = T(wrap_unit<float>(float(pxj) + dtf * ndx));
                v.y = T(wrap_unit<float>(float(pyj) + dtf * ndy));
                v.z = T(ndx);
                v.w = T(ndy);
            } else {
                double ndx, ndy;
                if (t0) {
                    float gx, gy;
                    field<float, PMAX>(px, py, np, pxj, pyj, p.gm, gx, gy);
                    ndx = pdx + double(gx * dtf);
                    ndy = pdy + double(gy * dtf);
                } else {
                    double gx, gy;
                    if constexpr ((LPE == 2 && (PMAX == 4 || PMAX == 8)) || (LPE == 4 && PMAX == 4)) {
                        // field<double> at planet j from the shared factors:
                        // term k = F(j, k) * (p_k - p_j) summed in k order.  The
                        // self term is the reference's gm / 1e-12 * (+0): a zero
                        // with gm's sign, which the table's self factor (gm
                        // itself) times p_j - p_j = +0 gives exactly
                        double ax = 0.0, ay = 0.0;
                        if (PMAX <= 4 && np_uni == PMAX - 1) {   // uniform: every env of the wave has PMAX - 1 planets
#pragma unroll
                            for (int k = 0; k < PMAX - 1; ++k) {
                                const double tx = Fr[m][k] * (px[k] - pxj);
                                const double ty = Fr[m][k] * (py[k] - pyj);
                                ax = k == 0 ? tx : ax + tx;
                                ay = k == 0 ? ty : ay + ty;
                            }
                        } else {
#pragma unroll
                            for (int k = 0; k < PMAX; ++k) {
                                const double tx = Fr[m][k] * (px[k] - pxj);
                                const double ty = Fr[m][k] * (py[k] - pyj);
                                if (k == 0) {
                                    ax = tx;
                                    ay = ty;
                                } else {
                                    ax = k < np ? ax + tx : ax;
                                    ay = k < np ? ay + ty : ay;
                                }
                            }
                        }
                        gx = ax;
                        gy = ay;
                    } else {
                        field<double, PMAX>(px, py, np, pxj, pyj, p.gm, gx, gy);
                    }
                    ndx = pdx + gx * p.dt;
                    ndy = pdy + gy * p.dt;
                }
                v.x = T(wrap_unit<double>(pxj + p.dt * ndx));
                v.y = T(wrap_unit<double>(pyj + p.dt * ndy));
                v.z = T(ndx);
                v.w = T(ndy);
            }
            out[m] = v;
        }
    }

}

// HELP: each step wave has a helper wave in its workgroup (waves QW..2QW-1)
// that creates its finished games' next ones.  The step wave posts its
// finished envs here as soon as it knows them -- before the surviving envs'
// update -- and goes on; the helper, asleep until then, runs the reset
// passes meanwhile, so a wave that has a finished game no longer ends a
// reset pass (~3.9k cycles) after its physics.
// An LDS word accessed as volatile through the LDS address space: ds_read /
// ds_write, ordered by lgkmcnt only.  (A volatile access through the plain
// generic pointer compiles to a flat load/store with sc0 sc1 and an
// s_waitcnt vmcnt(0): a wait for every global load and store the wave has
// in flight.)
typedef volatile __attribute__((address_space(3))) uint32_t lds_vu32;
__device__ __forceinline__ lds_vu32 *lds_word(const uint32_t &w) {
    return (lds_vu32 *)size_t(uint32_t(reinterpret_cast<uintptr_t>(&w)));   // a generic LDS address's low half is its offset
}

struct HelpBox {
    uint32_t flag;                 // set (1) by the step wave once `todo` is written
    uint32_t seen;                 // set (nonzero) by the helper once its header load has returned
    uint32_t pad[2];
    unsigned long long todo;       // leader lanes (q == 0) of the finished envs
};

// Post a step wave's finished envs (leader lanes `todo`) to its helper.
__device__ __forceinline__ void help_post(HelpBox &bx, uint64_t todo, int lane) {
#ifdef ASTRO_DEBUG_DROP_POST   // fault-injection build only: the helper's wait must expire and report
    (void)bx; (void)todo; (void)lane;
    return;
#endif
    if (lane == 0) bx.todo = todo;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the mask before the flag (LDS: in order per wave)
    if (lane == 0) *lds_word(bx.flag) = 1u;
}

// A bounded wait for an LDS word another wave of the workgroup sets: true
// once it is nonzero, false when the bound (2^22 s_sleep 1, ~0.1 s) expires.
// The bound only keeps a fault from hanging the device; an expired wait is
// reported through the state's error word (report_error), never ignored.
__device__ __forceinline__ bool wait_lds_word(const uint32_t &w) {
    for (uint32_t spin = 0; spin < (1u << 22); ++spin) {
        if (*lds_word(w) != 0u) return true;
        __builtin_amdgcn_s_sleep(1);
    }
    return *lds_word(w) != 0u;
}

// Set bits of the state's device error word (AstroState.errors, optional).
__device__ __forceinline__ void report_error(const AstroState &st, uint32_t bits, int lane) {
    if (st.errors && lane == 0) atomicOr(st.errors, bits);
}

// One lane's part of its env across the launch (quad/pair layout): the header
// (every lane of the env), its own ship (lanes q < S), its planet slots
// q + LPE m, and how far into the env's bullet row the launch has written.
template <typename T, int S, int PMAX, int LPE>
struct ResEnv {
    using V = typename Store<T>::V;
    int4 h;
    V sv;
    T sb;
    V pv[PMAX / LPE];
    int hw;   // slots [0, hw) of the env's LDS row were written by this launch (or loaded)
};

// A new game made by a reset pass into LDS instead of the state arrays: the
// resident rollout's (one per row of the pass, over the wave's body rows,
// which are free once the bullet pass is over), and a helper wave's early
// creates (games that end by a ship collision or the timeout, made before the
// step wave posts and stored after it).  Float32 state.
template <int S, int PMAX>
struct ResStage {
    float4 ship[S];
    float b[4];
    float4 planet[PMAX];
    int4 hdr;
    uint32_t seed;   // the stream record's current-game seed (stream[4 i + 3])
    uint32_t pad[3];
};

// Reset-pass sink: row r of the pass writes its env's new game into stage[r]
template <typename T, int S, int PMAX>
struct StageSink {
    using V = typename Store<T>::V;
    ResStage<S, PMAX> *stage;
    __device__ void ship(int s, int, const V &v, T b) const {
        stage->ship[s] = make_float4(v.x, v.y, v.z, v.w);
        stage->b[s] = b;
    }
    __device__ void planet(int j, int, int, const V &v) const { stage->planet[j] = make_float4(v.x, v.y, v.z, v.w); }
    __device__ void header(int, const int4 &h) const { stage->hdr = h; }
    __device__ void stream_seed(int, uint32_t seed) const { stage->seed = seed; }
    __device__ StageSink for_row(int r) const { return StageSink{stage + r}; }
};

// Serial-create sink (create_env with NPART = LPE, part = q): the lane's own
// ship and planet slots go straight into its registers
template <typename T, int S, int PMAX, int LPE>
struct RegSink {
    using V = typename Store<T>::V;
    ResEnv<T, S, PMAX, LPE> *r;
    __device__ void ship(int, int, const V &v, T b) const {
        r->sv = v;
        r->sb = b;
    }
    __device__ void planet(int, int m, int, const V &v) const { r->pv[m] = v; }
    __device__ void header(int, const int4 &h) const { r->h = h; }
};

// ---------------------------------------------------------------------------
// The dense bullet pass of the quad/pair kernels (core.py:241-251, 264-266,
// 295-300), in two parts so the first rounds' loads can fly during other
// work: bullets_begin (after the header) numbers the wave's live bullets --
// bullet k of env e is g = off_e + k, so the pass runs ceil(sum nb / 64)
// rounds instead of max over envs of ceil(nb / LPE) -- writes the first
// index window, clears the envs' LDS words and loads the first two rounds'
// bullets; bullets_rounds stages the envs' old bodies in LDS, collides,
// moves, culls and compacts every live bullet, and leaves per env the kept
// count (s_kept) and the ships the bullets hit (s_hit).
template <typename T>
struct BulletsIn {
    int total, off;
    uint32_t tag, bw0, bw1;
    typename Store<T>::V cur0, cur1;
};

// Where the dense pass finds the wave's bullet rows and, for its rare exact
// tests, the old bodies at full precision.  BulletsGlobal: the state's rows
// in HBM ([n_env][b_cap], env base + e); BulletsLds: the resident rollout's
// rows in LDS ([QENV][RES_BCAP] per wave, float32 state) with the old bodies
// from the pass's own float32 copies (exact: the state is float32).
template <typename T>
struct BulletsGlobal {
    using V = typename Store<T>::V;
    V *rows;
    const V *ships, *planets;
    size_t BC, NN;
    int base;
    __device__ V load(int e, int slot) const { return rows[size_t(base + e) * BC + slot]; }
    __device__ void store(int e, int slot, const V &v) const { st_out(&rows[size_t(base + e) * BC + slot], v); }
    __device__ double2 planet(int e, int j) const {
        const V v = planets[size_t(j) * NN + size_t(base + e)];
        return make_double2(double(v.x), double(v.y));
    }
    __device__ double2 ship(int e, int s) const {
        const V v = ships[size_t(s) * NN + size_t(base + e)];
        return make_double2(double(v.x), double(v.y));
    }
};

typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v2f __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) v4f lds_f4;
typedef __attribute__((address_space(3))) v2f lds_f2;
__device__ __forceinline__ lds_f4 *lds_ptr(const void *p) {   // a generic LDS address's low half is its offset
    return (lds_f4 *)size_t(uint32_t(reinterpret_cast<uintptr_t>(p)));
}

constexpr int RES_BCAP = 32;   // bullet slots per env the resident rollout keeps in LDS

template <int S, int NBOD2>
struct BulletsLds {
    using V = F4;
    lds_f4 *rows;     // [QENV][RES_BCAP]
    lds_f4 *body;     // [QENV][NBOD2]: (x, y) of ships then planets, float32 = the state's values
    __device__ V load(int e, int slot) const {
        const v4f v = rows[e * RES_BCAP + slot];
        return F4{v.x, v.y, v.z, v.w};
    }
    __device__ void store(int e, int slot, const V &v) const {
        v4f w;
        w.x = v.x;
        w.y = v.y;
        w.z = v.z;
        w.w = v.w;
        rows[e * RES_BCAP + slot] = w;
    }
    __device__ double2 planet(int e, int j) const {
        const v2f v = reinterpret_cast<lds_f2 *>(body + e * NBOD2)[S + j];
        return make_double2(double(v.x), double(v.y));
    }
    __device__ double2 ship(int e, int s) const {
        const v2f v = reinterpret_cast<lds_f2 *>(body + e * NBOD2)[s];
        return make_double2(double(v.x), double(v.y));
    }
};

// EAGER (default): the first two rounds' bullets are loaded here, to fly
// during the physics; otherwise (the helper-less one-tick instance of
// millions of envs, where occupancy hides the latency and the registers held
// across the physics cost a wave per SIMD) bullets_rounds loads them.
template <typename T, int LPE, int QWN = QWIN, bool EAGER = true, class BM>
__device__ __forceinline__ BulletsIn<T> bullets_begin(const BM &bm, int lane, int e, int q, int nb, int np, bool t0,
                                                      uint32_t *s_index, int *s_kept, int *s_hit, int *s_serial) {
    using V = typename Store<T>::V;
    BulletsIn<T> b;
    const int incl = wave_incl_scan(q == 0 ? nb : 0, lane);
    b.off = incl - nb;
    b.total = __builtin_amdgcn_readlane(incl, 63);
    b.tag = bw_tag(e, np, t0);
    if (q == 0) {
        s_kept[e] = 0;
        s_hit[e] = 0;
        s_serial[e] = 0;
    }
    if (b.total == 0) {   // uniform: no live bullet in the wave (config 2): no index, no loads
        b.bw0 = b.bw1 = 0u;
        b.cur0 = b.cur1 = V{};
        return b;
    }
    index_window<LPE, QWN>(s_index, 0, b.off, nb, q, b.tag);
    if constexpr (EAGER) {
        wave_sync();
        b.bw0 = lane < b.total ? s_index[lane] : 0u;
        b.bw1 = lane + 64 < min(b.total, QWN) ? s_index[lane + 64] : 0u;
        b.cur0 = bm.load(bw_env(b.bw0), bw_slot(b.bw0));
        b.cur1 = bm.load(bw_env(b.bw1), bw_slot(b.bw1));
    }
    return b;
}

// sxf/syf: both ships' old positions (float32); mpxf/mpyf: the lane's own
// planet slots q + LPE m (float32, slots past the env's planets parked at
// -FAR_POS).  Ends with the wave's LDS results readable (wave_sync).
template <typename T, int S, int PMAX, int LPE, int NRW = 2, int QWN = QWIN, bool EAGER = true, class BM>
__device__ __forceinline__ void bullets_rounds(const AstroParams &p, const BM &bm, const BulletsIn<T> &b,
                                               int lane, int e, int q, int nb, const float (&sxf)[S],
                                               const float (&syf)[S], const float (&mpxf)[PMAX / LPE],
                                               const float (&mpyf)[PMAX / LPE],
                                               float4 (*s_body)[(S + PMAX + 1) / 2], uint32_t *s_index,
                                               int *s_kept, int *s_hit, const Guard &gp, const Guard &gs STAMP_ARG) {
    using V = typename Store<T>::V;
    constexpr int PPL = PMAX / LPE;
    constexpr int NBOD2 = (S + PMAX + 1) / 2;
    const int total = b.total, off = b.off;
    const uint32_t tag = b.tag;
    uint32_t bw0 = b.bw0, bw1 = b.bw1;
    V cur0 = b.cur0, cur1 = b.cur1;
    if (total == 0) {   // uniform: nothing to do (bullets_begin left s_kept, s_hit cleared)
        wave_sync();
        return;
    }
    if constexpr (!EAGER) {   // the first two rounds' index words and bullets, now
        wave_sync();
        bw0 = lane < total ? s_index[lane] : 0u;
        bw1 = lane + 64 < min(total, QWN) ? s_index[lane + 64] : 0u;
        cur0 = bm.load(bw_env(bw0), bw_slot(bw0));
        cur1 = bm.load(bw_env(bw1), bw_slot(bw1));
    }
    // ---- old positions of the env's bodies for the bullet pass (LDS)
    {
        float2 *body = reinterpret_cast<float2 *>(&s_body[e][0]);
        // (the ships' values made opaque first: `q == 0 ? a[0] : a[1]` on an
        // array parameter becomes a[q], an array indexed in scratch memory)
        float x0 = sxf[0], y0 = syf[0], x1 = sxf[S - 1], y1 = syf[S - 1];
        asm volatile("" : "+v"(x0), "+v"(y0), "+v"(x1), "+v"(y1));
        if (q < S) body[q] = make_float2(q == 0 ? x0 : x1, q == 0 ? y0 : y1);
#pragma unroll
        for (int m = 0; m < PPL; ++m) body[S + q + LPE * m] = make_float2(mpxf[m], mpyf[m]);
    }
    wave_sync();
    STAMP(16);
    // lane g of a round takes live bullet r0 + g of the wave: collide with the
    // OLD bodies, move, cull, and compact in slot order within its env, in
    // place (a bullet is only ever written to a slot <= the one it was read
    // from, and every slot is read before any later round writes)
    {
        const uint64_t lanes_below = (1ull << lane) - 1;
        const double dt = p.dt;
        int kept_before = 0;   // kept bullets of the wave in earlier rounds
        int carry = 0;         // kept_before at the start of the env spanning into the next round
        for (int w0 = 0; w0 < total; w0 += QWN) {   // uniform; one window unless > QWN / 32 bullets/env
          const int wend = min(total, w0 + QWN);
          if (w0 > 0) {
              wave_sync();   // the previous window is read
              index_window<LPE, QWN>(s_index, w0, off, nb, q, tag);
              wave_sync();
              bw0 = w0 + lane < wend ? s_index[lane] : 0u;
              bw1 = w0 + 64 + lane < wend ? s_index[64 + lane] : 0u;
              cur0 = bm.load(bw_env(bw0), bw_slot(bw0));
              cur1 = bm.load(bw_env(bw1), bw_slot(bw1));
          }
          // one round: lane g takes live bullet r0 + g (index word bw, data cur)
          // NR rounds at once, lane g of round r taking live bullet r0 + 64 r + g
          // (index words bws[r], data curs[r]): their collision tests and moves
          // are independent, so they are evaluated side by side (the latency
          // chains of one round overlap the other's: a pair-kernel SIMD has
          // only two waves to switch between); the compaction then runs round
          // by round, in order
          auto rounds = [&](auto nr_tag, int r0, const uint32_t *bws, const V *curs) {
              constexpr int NR = decltype(nr_tag)::value;
              bool valid[NR], amb[NR], bh[NR], bt0[NR], hs[NR][S];
              int be[NR];
#pragma unroll
              for (int r = 0; r < NR; ++r) {
                  valid[r] = r0 + 64 * r + lane < total;
                  be[r] = bw_env(bws[r]);
                  bt0[r] = bw_t0(bws[r]);
                  float bx[2 * NBOD2], by[2 * NBOD2];
#pragma unroll
                  for (int u = 0; u < NBOD2; ++u) {
                      const float4 v = s_body[be[r]][u];
                      bx[2 * u] = v.x;
                      by[2 * u] = v.y;
                      bx[2 * u + 1] = v.z;
                      by[2 * u + 1] = v.w;
                  }
                  const float xf = valid[r] ? float(curs[r].x) : FAR_POS;
                  const float yf = valid[r] ? float(curs[r].y) : FAR_POS;
                  // float32 prefilter.  Planets only matter through the nearest
                  // one: below the band it is a certain hit, inside the band the
                  // exact tests run, above it no planet is hit.  Ships one by one
                  float pmin = __builtin_huge_valf();
#pragma unroll
                  for (int j = 0; j < PMAX; ++j) {
                      const float dx = xf - bx[S + j], dy = yf - by[S + j];
                      pmin = __builtin_fminf(pmin, dx * dx + dy * dy);
                  }
                  bh[r] = pmin < gp.lo;
                  bool am = (pmin >= gp.lo) & (pmin <= gp.hi);
#pragma unroll
                  for (int s = 0; s < S; ++s) hs[r][s] = near32(xf, yf, bx[s], by[s], gs, am);
                  amb[r] = am | (valid[r] & bt0[r]);
              }
              bool any_amb = false;
#pragma unroll
              for (int r = 0; r < NR; ++r) any_amb |= amb[r];
              if (__any(any_amb)) {   // rare: the exact tests; the old bodies are still in memory
#pragma unroll
                  for (int r = 0; r < NR; ++r) {
                      if (amb[r]) {
                          const int bnp = bw_np(bws[r]);
                          const double x = double(curs[r].x), y = double(curs[r].y);
                          bool bh64 = false;
#pragma unroll
                          for (int j = 0; j < PMAX; ++j) {
                              if (j < bnp) {
                                  const double2 pj = bm.planet(be[r], j);
                                  bh64 |= closer_exact(x, y, pj.x, pj.y, gp, bt0[r]);
                              }
                          }
#pragma unroll
                          for (int s = 0; s < S; ++s) {
                              const double2 sj = bm.ship(be[r], s);
                              hs[r][s] = closer_exact(x, y, sj.x, sj.y, gs, bt0[r]);
                          }
                          bh[r] = bh64;
                      }
                  }
              }
              bool any_hit = false;
#pragma unroll
              for (int r = 0; r < NR; ++r) {
                  bool ship_hit = false;
#pragma unroll
                  for (int s = 0; s < S; ++s) ship_hit |= hs[r][s];
                  bh[r] |= ship_hit;
                  any_hit |= ship_hit;
              }
              if (__any(any_hit)) {   // rare: record which ships of the env were hit
#pragma unroll
                  for (int r = 0; r < NR; ++r) {
                      const int hb = (hs[r][0] ? 1 : 0) | (S == 2 && hs[r][S - 1] ? 2 : 0);
                      if (hb) atomicOr(&s_hit[be[r]], hb);   // (an invalid lane never hits: it sits at FAR_POS)
                  }
              }
              // move without gravity and cull (core.py:295-300, 195)
              bool keep[NR];
              V out[NR];
              bool any_t0 = false;
#pragma unroll
              for (int r = 0; r < NR; ++r) {
                  // dx + 0 * dt in the state's own type: exact either way
                  const V &cur = curs[r];
                  const T ndx = cur.z + T(0), ndy = cur.w + T(0);
                  const double nx = double(cur.x) + dt * double(ndx), ny = double(cur.y) + dt * double(ndy);
                  keep[r] = (__builtin_fabs(nx) <= 1.0) || (__builtin_fabs(ny) <= 1.0);   // -1 <= v <= 1
                  out[r].x = T(nx);
                  out[r].y = T(ny);
                  out[r].z = ndx;
                  out[r].w = ndy;
                  any_t0 |= valid[r] & bt0[r];
              }
              if (__any(any_t0)) {   // tick-0 bullets exist only in hand-made states: float32
                  const float dtf = float(p.dt);
#pragma unroll
                  for (int r = 0; r < NR; ++r) {
                      if (valid[r] && bt0[r]) {
                          const V &cur = curs[r];
                          const float ndx = float(cur.z) + 0.0f, ndy = float(cur.w) + 0.0f;
                          const float nx = float(cur.x) + dtf * ndx, ny = float(cur.y) + dtf * ndy;
                          keep[r] = (-1.0f <= nx && nx <= 1.0f) || (-1.0f <= ny && ny <= 1.0f);
                          out[r].x = T(nx);
                          out[r].y = T(ny);
                          out[r].z = T(ndx);
                          out[r].w = T(ndy);
                      }
                  }
              }
              // compaction in slot order, round by round
#pragma unroll
              for (int r = 0; r < NR; ++r) {
                  const bool kp = keep[r] & valid[r] & !bh[r];
                  const uint64_t kb = __ballot(kp);
                  const int kg = kept_before + __popcll(kb & lanes_below);
                  const int first = lane - bw_slot(bws[r]);   // lane of the env's slot 0 (< 0: an earlier round)
                  const int k0 = first >= 0 ? kept_before + __popcll(kb & ((1ull << (first & 63)) - 1)) : carry;
                  const int pos = kg - k0;
                  if (kp) bm.store(be[r], pos, out[r]);
                  if (valid[r] && bw_last(bws[r])) s_kept[be[r]] = pos + int(kp);
                  carry = __builtin_amdgcn_readlane(k0, 63);
                  kept_before += __popcll(kb);
              }
          };
          // The first rounds straight-line: each round's data was loaded a
          // round or more ahead and no register rotation sits between a load
          // and its use, so the waits before a round cover its own load only,
          // never an earlier round's stores (a loop with rotating prefetch
          // registers waited vmcnt(0) -- every store -- at each round)
          uint32_t bws[3] = {bw0, bw1, 0u};
          V curs[3] = {cur0, cur1, cur0};
          const int nr = (wend - w0 + 63) / 64;   // uniform
          // two rounds side by side with 4 planet slots (NRW = 2: the launches
          // latency sets, with helper waves or K ticks); with 8 the registers
          // of two rounds spill (measured: c5 30.8 -> 34.3 us), and the
          // one-tick instances without helpers (millions of envs, HBM-bound)
          // keep the registers for occupancy instead (4 waves per SIMD with
          // no spills: c3 at 1M envs 127.5 -> 119.2 us,
          // profiles/round4/ab_1m_waves.jsonl): one at a time
          constexpr int NR2 = PMAX <= 4 ? (NRW < 2 ? NRW : 2) : 1;
          // NRW = 3 (4 slots): a wave with a third round runs all three side by
          // side (config 3's waves hold ~130 live bullets: half need a third)
          constexpr bool NR3 = NRW >= 3 && PMAX <= 4;
          if (nr >= 3) {
              bws[2] = w0 + 128 + lane < wend ? s_index[128 + lane] : 0u;
              curs[2] = bm.load(bw_env(bws[2]), bw_slot(bws[2]));
          }
          if (NR3 && nr >= 3) {
              rounds(std::integral_constant<int, NR3 ? 3 : 1>(), w0, bws, curs);
          } else if (nr >= 2) {
              rounds(std::integral_constant<int, NR2>(), w0, bws, curs);
              if (NR2 == 1) rounds(std::integral_constant<int, 1>(), w0 + 64, bws + 1, curs + 1);
          } else {
              rounds(std::integral_constant<int, 1>(), w0, bws, curs);
          }
          STAMP(17);
          if (!NR3 && nr >= 3) rounds(std::integral_constant<int, 1>(), w0 + 128, bws + 2, curs + 2);
          for (int r0 = w0 + 192; r0 < wend; r0 += 64) {   // uniform; rare
              const uint32_t bw = r0 + lane < wend ? s_index[r0 + lane - w0] : 0u;
              const V cur = bm.load(bw_env(bw), bw_slot(bw));
              rounds(std::integral_constant<int, 1>(), r0, &bw, &cur);
          }
        }
    }
    wave_sync();
}

template <typename T, int S, int PMAX, int LPE, bool OPAQUE = false, bool BOTS = false, bool HELP = false,
          int WPG = QW>
__device__ __forceinline__ QuadCounts quad_tick(const AstroParams &p, const AstroState &st, const TickDriver &drv,
                                                float *__restrict__ reward_all, uint8_t *__restrict__ done_all,
                                                bool stats, int auto_reset, int kt STAMP_ARG) {
    using V = typename Store<T>::V;
    constexpr int PPL = PMAX / LPE;   // planet slots per lane
    constexpr int QENV = 64 / LPE;    // envs per wave
    constexpr int NBOD2 = (S + PMAX + 1) / 2;
    // LDS, one set per wave of the workgroup
    __shared__ float4 s_body_all[WPG][QENV][NBOD2];       // float32 (x, y): ships, then planets (padding far)
    __shared__ uint32_t s_index_all[WPG][QWIN];           // a window of the wave's live bullets, see bw_*
    __shared__ int s_kept_all[WPG][QENV], s_hit_all[WPG][QENV], s_serial_all[WPG][QENV];
    __shared__ uint32_t s_chain_all[WPG][4][2][13 + 2 * S];   // init-key chains of a reset pass, see below
    __shared__ HelpBox s_box_all[HELP ? WPG : 1];
    __shared__ uint32_t s_pre_all[HELP ? WPG : 1][HELP ? QENV : 1][2][13 + 2 * S];   // a helper's chains, made ahead

    // (wave_sync syncs one wave whenever the build's QW > 1, whatever this instance's WPG)
    static_assert(!HELP || (QW > 1 && !OPAQUE), "helper waves: one-tick launches, wave-scoped LDS sync");
    // The helper waves check their step waves' pending seeds (check_pending's
    // draw, key gather, filter and redraw) and store header words 2-3 of the
    // survivors; the step waves only write words 0-1.  Quad instance only: its
    // step waves are the critical path (c2 5.36 -> 5.20 us A/B); in the pair
    // instance the helpers' resets are the tail (c3 12.19 -> 12.52 us)
    constexpr bool PENDING_ON_HELPER = HELP && LPE == 4;
    // the planet update on the helpers: pair instance only (the quad instance
    // of c2 lost with it there: 5.08 -> 5.33 us, ab_quad_planets_on_helper.jsonl)
    constexpr bool PLANETS_ON_HELPER = HELP && LPE == 2;
    const bool helper = HELP && int(threadIdx.x >> 6) >= WPG;
    // Helper wave WPG + h serves step wave (h + 1) mod WPG: a workgroup's waves
    // go round the 4 SIMDs in order, so a helper would otherwise share its
    // SIMD with its own step wave, and the two are each other's competition
    // at the launch's end (a late post: the step wave's stores and its
    // helper's reset pass).  c3 10.17 -> 10.08 us, c2 unchanged
    // (profiles/round6/ab_helper_simd.jsonl)
#ifndef ASTRO_HELPER_SHIFT
#define ASTRO_HELPER_SHIFT 1
#endif
    // Wave priorities (s_setprio), pair instance: step waves 2 until their
    // post, then 0; helpers 1.  After its post a step wave's work (fire, own
    // ship, header) ends nothing but itself, while the helpers' reset passes
    // end the launch: c3 10.13 -> 9.74 us (the digits of ASTRO_PRIO: step
    // wave before / after the post, helper before / after; 2011 kept, 1011
    // 9.78, 3021 9.74, 2012 9.98, 1000 10.13, 1001 10.21; the quad instance
    // of c2 lost with 1011, 4.09 -> 4.24; priorities from the wave's live
    // bullets, or for helpers with resets only, were even or slower:
    // profiles/round6/ab_wave_priority.jsonl)
#ifndef ASTRO_PRIO
#define ASTRO_PRIO 2011
#endif
    constexpr bool PRIO = HELP && LPE == 2 && ASTRO_PRIO != 0;
    constexpr int PRIO_SP = (ASTRO_PRIO / 1000) % 10, PRIO_SQ = (ASTRO_PRIO / 100) % 10;
    constexpr int PRIO_HP = (ASTRO_PRIO / 10) % 10, PRIO_HQ = ASTRO_PRIO % 10;
    const int wv = WPG == 1 ? 0
                            : (helper ? (int(threadIdx.x >> 6) - WPG + ASTRO_HELPER_SHIFT) % WPG
                                      : int(threadIdx.x >> 6));   // (a helper: its step wave's)
    float4 (*s_body)[NBOD2] = s_body_all[wv];
    uint32_t *s_index = s_index_all[wv];
    int *s_kept = s_kept_all[wv], *s_hit = s_hit_all[wv], *s_serial = s_serial_all[wv];
    uint32_t (*s_chain)[2][13 + 2 * S] = s_chain_all[wv];

    const int N = st.n_env;
    int lane = threadIdx.x & 63;
    if constexpr (OPAQUE) asm volatile("" : "+v"(lane));   // (see the rollout kernel)
    const int q = lane & (LPE - 1);
    const int e = lane / LPE;
    const int base = (blockIdx.x * WPG + wv) * QENV;
    const bool active = base + e < N;     // uniform over the quad
    const int i = active ? base + e : N - 1;   // spare quads of the last wave shadow env N-1, store nothing
    const size_t NN = size_t(N);
    if constexpr (HELP) {
        // LDS holds the previous launch's leftovers: clear the flag before
        // any step wave can post (every wave of the workgroup passes this
        // one barrier; a wave past the last env returns after it, with its
        // helper)
        HelpBox &bx = s_box_all[wv];
        if (helper && lane == 0) {
            bx.flag = 0;
            bx.seen = 0;
            bx.todo = 0;
        }
        __syncthreads();
        if (base >= N) return QuadCounts{};
        if constexpr (PRIO) {
            if (helper) __builtin_amdgcn_s_setprio(PRIO_HP);
            else __builtin_amdgcn_s_setprio(PRIO_SP);
        }
        if (helper) {
            HSTAMP_R(23);
            HSTAMP_T(24);
            // While its step wave steps, the helper makes the MT19937 init-key
            // chains of every env's pending game (the first 13 + 2S words from
            // the seed and from key[397]; 2 lanes per env, all envs at once):
            // a reset pass then starts from its draws.  A finished env's
            // header is never written by its step wave, so the helper reads
            // the same pending seed and key (the step wave's gather of a
            // first-step env's key repeated here).
            constexpr int NW = 12 + 2 * S;
            uint32_t (*pre)[2][13 + 2 * S] = s_pre_all[wv];
            const int4 hh = reinterpret_cast<const int4 *>(st.hdr)[i];
            // the step wave stores the survivors' new headers (tick + 1) at
            // its end: it waits for this word, so the header read here is the
            // launch's input whatever the memory system's timing (the store
            // depends on the loaded value: it waits for the load's return)
            if (lane == 0) *lds_word(bx.seen) = uint32_t(hh.x) | 1u;
            const uint32_t hseed = uint32_t(hh.z) & SEED_MASK;
            const bool kvalid = (uint32_t(hh.z) & KEY_VALID) != 0;
            const bool hud = (uint32_t(hh.z) & UNDRAWN) != 0;   // (a reset then takes the serial path)
            uint32_t hkey = uint32_t(hh.w);
            const bool hk = kvalid || p.key_table != nullptr;
            if (q == 1 && !kvalid && !hud) hkey = p.key_table ? p.key_table[hseed & SEED_MASK] : mt_key_at(hseed, 0, MT_PROLOGUE);
            // ... and (PENDING_ON_HELPER) the step wave's check of every env's
            // pending seed, as check_pending does it: the draw of a first-step
            // env's UNDRAWN seed, key[397] of a pending seed, and with
            // planets_only the seed's planet count (a failing seed is
            // replaced by the stream's next draw).  The
            // results -- header words 2-3 and the advanced stream cursor -- are
            // stored for the surviving envs after the post (a finished env's
            // reset starts from the unchecked pending seed and the cursor in
            // memory, as without helpers)
            uint32_t w2 = uint32_t(hh.z), w3 = uint32_t(hh.w);   // the survivors' header words 2-3
            bool drew = false;
            uint4 cnew = make_uint4(0u, 0u, 0u, 0u);
            if constexpr (PENDING_ON_HELPER) {
                if (q == 0 && active && (hud || (!kvalid && p.key_table))) {   // (rare: a game's first steps)
                    bool draw = hud;
                    if (!hud) {
                        const uint32_t k397 = p.key_table[hseed];
                        w3 = k397;
                        if (seed_passes(p, hseed, k397)) w2 = hseed | KEY_VALID;
                        else draw = true;   // (planets_only) the next candidate, checked next launch
                    }
                    if (draw) {
                        const uint4 c = reinterpret_cast<const uint4 *>(st.stream)[i];
                        MTStream g{c.x, c.y, c.z, stream_ring_of(st, i)};   // (its ring store is the same
                        w2 = g.next() & SEED_MASK;                           //  word whoever draws it)
                        w3 = 0u;
                        cnew = make_uint4(g.a, g.b, g.k, c.w);
                        drew = true;
                    }
                }
            }
            // ... and, pair instance, the planet update of every env of the
            // step wave (the survivors' stored after the post; the step wave
            // then skips it: c3 12.39 -> 11.92 us with eight step waves per
            // workgroup; the quad instance of config 2 keeps it, 5.45 vs 5.50)
            constexpr bool PLANETS = PLANETS_ON_HELPER;
            const size_t NN = size_t(N);
            V *planets = reinterpret_cast<V *>(st.planets);
            constexpr int PPL = PMAX / LPE;
            int np = hh.y & 0xff;
            np = np < 1 ? 1 : (np > PMAX ? PMAX : np);
            const bool t0 = (uint32_t(hh.x) & TICK_MASK) == 0;
            const bool slot_last = __builtin_amdgcn_readfirstlane(int(__any(np == PMAX))) != 0;
            V hpv[PPL], hout[PPL];
            T hpx[PPL], hpy[PPL];
            if constexpr (PLANETS) {
#pragma unroll
                for (int m = 0; m < PPL; ++m) {   // (8 slots: a slot past np aliased to slot 0, as the step wave reads)
                    const int j = q + LPE * m;
                    hpv[m] = planets[size_t(j < np ? j : 0) * NN + i];
                    hpx[m] = hpv[m].x;
                    hpy[m] = hpv[m].y;
                }
            }

            if (q < 2) {
                uint32_t x = q == 0 ? hseed : hkey;
                const uint32_t koff = q == 0 ? 0u : 397u;
#pragma unroll
                for (int k = 0; k <= NW; ++k) {
                    pre[e][q][k] = x;
                    x = mt_key_next(x, koff + uint32_t(k + 1));
                }
            }
            wave_sync();
            HSTAMP_T(25);
            if constexpr (PLANETS) planet_update<T, S, PMAX, LPE, PPL>(p, hpv, hpx, hpy, q, np, t0, slot_last, hout);
            HSTAMP_T(26);
            // until the step wave posts (bounded: it always posts; if the
            // bound expires the mask is not trusted -- no stores, no resets --
            // and the launch reports ASTRO_ERR_HELPER_WAIT)
            if (!wait_lds_word(bx.flag)) {
                report_error(st, ASTRO_ERR_HELPER_WAIT, lane);
                return QuadCounts{};
            }
            asm volatile("" ::: "memory");
            if constexpr (PRIO && PRIO_HQ != PRIO_HP) __builtin_amdgcn_s_setprio(PRIO_HQ);
            HSTAMP_R(20);
            HSTAMP_T(27);
            QuadCounts hc{};
            const uint64_t todo0 = bx.todo;
            if (PLANETS && active && !((todo0 >> (lane & ~(LPE - 1))) & 1ull)) {   // a surviving env: its new planets
#pragma unroll
                for (int m = 0; m < PPL; ++m) {
                    const int j = q + LPE * m;
                    if (j < np) st_out(&planets[size_t(j) * NN + i], hout[m]);
                }
            }
            if (PENDING_ON_HELPER && q == 0 && active && !((todo0 >> lane) & 1ull)) {   // a surviving env: its
                reinterpret_cast<int2 *>(st.hdr)[2 * i + 1] = make_int2(int(w2), int(w3));   // pending seed
                if (drew) reinterpret_cast<uint4 *>(st.stream)[i] = cnew;
            }
            HSTAMP_T(28);
            if (todo0) {   // uniform
                for (uint64_t todo = todo0; todo;)   // uniform
                    todo = wave_reset_pass<T, S, PMAX, LPE, true>(p, st, todo, lane, i, hseed, hkey, hk, hud, s_chain,
                                                                  s_serial, GlobalSink<T>{st} STAMP_PASS, pre);
                HSTAMP_T(29);
#ifdef ASTRO_STAMPS
                stamp_[32] = stamp_[16];
                stamp_[33] = stamp_[17];
                stamp_[34] = stamp_[18];
                stamp_[35] = stamp_[19];
#endif
                wave_sync();
                if (stats) hc.c_serial = __popcll(__ballot(active && q == 0 && s_serial[e]));
                if (active && s_serial[e]) {   // uniform over the quad; rare
                    const uint32_t kq = uint32_t(quad_bcast_i<1, LPE>(int(hkey)));   // (lane q == 1 has the key)
                    const uint4 c = reinterpret_cast<const uint4 *>(st.stream)[i];
                    const NextGame<S> ng = next_game<S>(p, hseed, kq, hk, hud, c, stream_ring_of(st, i));
                    restart_env<T, S, PMAX, LPE>(p, st, i, ng, q, GlobalSink<T>{st});
                }
            }
            HSTAMP_R(21);
            HSTAMP_T(30);
#ifdef ASTRO_STAMPS
            stamp_[22] = __popcll(todo0);
#endif
            return hc;
        }
    }
    const size_t BC = size_t(p.b_cap);
    V *ships = reinterpret_cast<V *>(st.ships);
    T *ships_b = reinterpret_cast<T *>(st.ships_b);
    V *planets = reinterpret_cast<V *>(st.planets);
    V *bullets = reinterpret_cast<V *>(st.bullets);
    uint32_t n_bin = 0, n_bout = 0, n_pl = 0, n_drop = 0;   // per lane, summed over the launch's ticks
    uint32_t c_reset = 0, c_coll = 0, c_tout = 0, c_serial = 0;           // per wave
    const int sq = q < S ? q : 0;
    float *__restrict__ reward = reward_all + size_t(kt) * NN * S;
    uint8_t *__restrict__ done_out = done_all + size_t(kt) * NN;
    bool f_reset = false, f_coll = false, f_tout = false;
    bool need_reset = false;   // leader lane (q == 0) of an env whose game ended, auto-reset on
    STAMP(0);

    // ---- loads, all independent of each other: header, own ship (lanes <
    //      S), control, own planet slots (read whether live or not; padding
    //      is masked below)
    const int4 h = reinterpret_cast<const int4 *>(st.hdr)[i];
    const V sv = ships[size_t(sq) * NN + i];
    const T sbv = ships_b[size_t(sq) * NN + i];
    int ctl = tick_control<S>(drv, i, sq, NN, kt);
    V pv[PPL];
    T mpx[PPL], mpy[PPL];
    // 4 planet slots: read with the header, every slot (padding is masked
    // below).  8 slots (config 5: 1-8 planets, 3.5 padded slots per env on
    // average): read after the header, a slot past the env's planets
    // aliased to slot 0 -- the line already read, no traffic -- one more
    // round trip, which three waves per SIMD hide (c5: 56 B less per env,
    // time unchanged in the A/B)
    constexpr bool PLANETS_AFTER_HDR = PMAX > 4;
    // With planets_only (config 3's 3-planet games) a filtered game never
    // has a planet in the slots past it: those alias slot 0 (the line just
    // read, no traffic; c3 reads 1 MB less per launch, 12.10 -> 12.03 us
    // A/B) -- a kernarg bound, so the loads still go out with the header's.
    // Pair instance with helpers only: the quad instance (c2) lost 2% to the
    // fallback below, the helper-less pair instance (1M, rollouts) spilled
    constexpr bool ALIAS = HELP && LPE == 2;
    const int p_live = ALIAS && p.planets_only ? p.planets_only : p.p_pad;
    if constexpr (!PLANETS_AFTER_HDR) {
#pragma unroll
        for (int m = 0; m < PPL; ++m) {
            const int j = q + LPE * m;
            pv[m] = planets[size_t(j < p_live ? j : 0) * NN + i];
        }
    }
    const int tick = int(uint32_t(h.x) & TICK_MASK);
    const bool key_valid = (uint32_t(h.z) & KEY_VALID) != 0;
    const bool undrawn = (uint32_t(h.z) & UNDRAWN) != 0;
    uint32_t pend_seed = uint32_t(h.z) & SEED_MASK;
    int np = h.y & 0xff;
    const int flags = (h.y >> 8) & 0xff;
    const int nb = active ? min(int(uint32_t(h.y) >> 16), p.b_cap) : 0;
    np = np < 1 ? 1 : (np > PMAX ? PMAX : np);
    if constexpr (PLANETS_AFTER_HDR) {
#pragma unroll
        for (int m = 0; m < PPL; ++m) {
            const int j = q + LPE * m;
            pv[m] = planets[size_t(j < np ? j : 0) * NN + i];
        }
    }
    else if (ALIAS && __builtin_amdgcn_readfirstlane(int(__any(np > p_live))) != 0) {   // uniform; only
#pragma unroll                                                                         // a loaded state
        for (int m = 0; m < PPL; ++m) {
            const int j = q + LPE * m;
            if (j >= p_live && j < np) pv[m] = planets[size_t(j) * NN + i];
        }
    }
#pragma unroll
    for (int m = 0; m < PPL; ++m) {
        mpx[m] = pv[m].x;
        mpy[m] = pv[m].y;
    }
    // does any env of the wave use the last planet slot?  (uniform; with
    // planets_only < PMAX, e.g. the 3-planet games of config 3, none does
    // and the float64 fields skip that slot's division)
    const bool slot_last = __builtin_amdgcn_readfirstlane(int(__any(np == PMAX))) != 0;
    const int np_uni = wave_uniform_count(np);   // (config 3's 3-planet games: 3)
    const bool live = tick < p.timeout_tick;
    const bool t0 = tick == 0;
    STAMP(1);
    const uint32_t fire_word = p.fire_bits[(live ? tick : 0) >> 5];
    uint32_t pend_key = uint32_t(h.w);
    n_pl += active && q == 0 ? uint32_t(np) : 0u;

    // ---- index the wave's live bullets densely (bullets_begin); their first
    //      two rounds load during the physics below
    const BulletsGlobal<T> bgl{bullets, ships, planets, BC, NN, base};
    // (the helper-less 4-slot pair instance of millions of envs: bullets
    // loaded in the pass, see bullets_begin; 1M envs 118.8 -> 118.1 us,
    // profiles/round5/ab_lazy_bullets_1m.jsonl)
    constexpr bool EAGER_BULLETS = HELP || OPAQUE || LPE != 2 || PMAX > 4;
    const BulletsIn<T> bin =
        bullets_begin<T, LPE, QWIN, EAGER_BULLETS>(bgl, lane, e, q, nb, np, t0, s_index, s_kept, s_hit, s_serial);
    const int total = bin.total;
    STAMP(19);
    // key[397] of the next game's seed (first step of a game): a random
    // gather into the 4 GiB key table, issued after every load the physics
    // waits for, so only its consumers (header store, reset) wait for it
    if (!PENDING_ON_HELPER && q == 0 && !key_valid && !undrawn && p.key_table)
        pend_key = p.key_table[pend_seed & SEED_MASK];
    // stream cursor, for check_pending (read there under this same condition
    // only).  Every lane loads, the others their own header again (the line
    // just read: no traffic).  A conditional load made the compiler merge
    // its value with the other lanes' zeros right after it, i.e. wait for it
    // -- and for every load before it, the key-table gather included -- at
    // the top of the wave (c3 13.10 -> 12.65 us, c2 6.74 -> 6.64 us, A/B)
    const bool want_c = !PENDING_ON_HELPER && q == 0 && (undrawn || (!key_valid && p.key_table && p.planets_only));
    uintptr_t c_stream = reinterpret_cast<uintptr_t>(st.stream), c_hdr = reinterpret_cast<uintptr_t>(st.hdr);
    asm volatile("" : "+s"(c_stream), "+s"(c_hdr));   // values, not a select between the fields' addresses
    const uint4 c_pend = load_u4_global(want_c ? c_stream : c_hdr, size_t(i));

    // ---- quad broadcasts: all planets, both ships
    double px[PMAX], py[PMAX], sx[S], sy[S];
    bcast_slots<T, PPL, LPE>(mpx, px);
    bcast_slots<T, PPL, LPE>(mpy, py);
    sx[0] = double(quad_bcast<0, LPE>(sv.x));
    sy[0] = double(quad_bcast<0, LPE>(sv.y));
    if (S == 2) {
        sx[S - 1] = double(quad_bcast<S - 1, LPE>(sv.x));
        sy[S - 1] = double(quad_bcast<S - 1, LPE>(sv.y));
    }

    // ---- own ship (lanes < S): direction, thrust + gravity (core.py:234-239)
    const double mx = double(sv.x), my = double(sv.y), mdx = double(sv.z), mdy = double(sv.w);
    const double mb = double(sbv);
    if constexpr (BOTS) {   // (the ScriptBot instance) ScriptBot ships decide on the old state
        if (drv.policy == ASTRO_POLICY_BOTS) {   // uniform
            double pdx[PMAX], pdy[PMAX];
            T mpdx[PPL], mpdy[PPL];
#pragma unroll
            for (int m = 0; m < PPL; ++m) {
                mpdx[m] = pv[m].z;
                mpdy[m] = pv[m].w;
            }
            bcast_slots<T, PPL, LPE>(mpdx, pdx);
            bcast_slots<T, PPL, LPE>(mpdy, pdy);
            const double d0x = double(quad_bcast<0, LPE>(sv.z)), d0y = double(quad_bcast<0, LPE>(sv.w));
            const double d1x = double(quad_bcast<S - 1, LPE>(sv.z)), d1y = double(quad_bcast<S - 1, LPE>(sv.w));
            const int oe = q == 0 ? S - 1 : 0;   // the other ship
            if (q < S && ship_bot(drv, q) == ASTRO_BOT_SCRIPT)
                ctl = script_control<S, PMAX>(drv, p.solo != 0, t0, np, px, py, pdx, pdy, mx, my, mdx, mdy, mb,
                                              sx[oe], sy[oe], oe == 0 ? d0x : d1x, oe == 0 ? d0y : d1y);
        }
    }
    float ds, dc;
    np_sincosf(float(mb), ds, dc);
    double ax = 0.0, ay = 0.0;
    // Quad kernel, 4 slots: the ships' float64 fields split over the quad --
    // lane q evaluates ship (q & 1)'s terms of planet slots q >> 1 and
    // (q >> 1) + 2, and the ship's lane adds them in slot order (2 divisions
    // per lane instead of 3-4 on the ship lanes alone)
    double sgx = 0.0, sgy = 0.0;
    if constexpr (LPE == 4 && PMAX == 4) {
        double s0x = sx[0], s0y = sy[0], s1x = sx[S - 1], s1y = sy[S - 1];
        double p0x = px[0], p0y = py[0], p1x = px[1], p1y = py[1], p2x = px[2], p2y = py[2], p3x = px[3], p3y = py[3];
        asm volatile("" : "+v"(s0x), "+v"(s0y), "+v"(s1x), "+v"(s1y));   // (selects, not an indexed array)
        asm volatile("" : "+v"(p0x), "+v"(p0y), "+v"(p1x), "+v"(p1y), "+v"(p2x), "+v"(p2y), "+v"(p3x), "+v"(p3y));
        const bool odd = (q & 1) != 0, hi = q >= 2;
        const double shx = odd ? s1x : s0x, shy = odd ? s1y : s0y;
        const double ax_ = hi ? p1x : p0x, ay_ = hi ? p1y : p0y;   // slot q >> 1
        const double bx_ = hi ? p3x : p2x, by_ = hi ? p3y : p2y;   // slot (q >> 1) + 2
        const double rax = ax_ - shx, ray = ay_ - shy, rbx = bx_ - shx, rby = by_ - shy;
        const double fa = div_gravity(p.gm, max_floor(rax * rax + ray * ray));
        const double fb = div_gravity(p.gm, max_floor(rbx * rbx + rby * rby));
        const double tax = fa * rax, tay = fa * ray, tbx = fb * rbx, tby = fb * rby;
        // the ship's lane (q < 2) holds slots 0 and 2; slots 1 and 3 from lane q + 2
        const double t1x = quad_perm_d<2, 3, 2, 3>(tax), t1y = quad_perm_d<2, 3, 2, 3>(tay);
        const double t3x = quad_perm_d<2, 3, 2, 3>(tbx), t3y = quad_perm_d<2, 3, 2, 3>(tby);
        sgx = tax;
        sgy = tay;
        sgx = 1 < np ? sgx + t1x : sgx;
        sgy = 1 < np ? sgy + t1y : sgy;
        sgx = 2 < np ? sgx + tbx : sgx;
        sgy = 2 < np ? sgy + tby : sgy;
        sgx = slot_last && 3 < np ? sgx + t3x : sgx;
        sgy = slot_last && 3 < np ? sgy + t3y : sgy;
    }
    if (q < S) {
        double gx, gy;
        if (t0) {
            float fx, fy;
            field<float, PMAX>(px, py, np, mx, my, p.gm, fx, fy);
            gx = double(fx);
            gy = double(fy);
        } else {
            if constexpr (LPE == 4 && PMAX == 4) {
                gx = sgx;
                gy = sgy;
            } else {
                field<double, PMAX>(px, py, np, mx, my, p.gm, gx, gy, slot_last, PMAX <= 4 ? np_uni : 0);
            }
        }
        const double thr = p.thrust * double(ctl & 1);
        ax = thr * double(ds) + gx;
        ay = thr * double(dc) + gy;
    }

    STAMP(2);
    // ---- ship collisions (core.py:241-253): lane q tests its planets and
    //      lane 0 the ship pair; quad-OR afterwards
    const Guard gsp(p.r2_sp), gss(p.r2_ss), gp(p.r2_p0), gs(p.r2_s0);
    float sxf[S], syf[S], mpxf[PPL], mpyf[PPL];   // float32 copies, padding parked far away
#pragma unroll
    for (int s = 0; s < S; ++s) {
        sxf[s] = float(sx[s]);
        syf[s] = float(sy[s]);
    }
#pragma unroll
    for (int m = 0; m < PPL; ++m) {
        mpxf[m] = q + LPE * m < np ? float(mpx[m]) : -FAR_POS;
        mpyf[m] = q + LPE * m < np ? float(mpy[m]) : -FAR_POS;
    }
    bool hsp[S];
    {
        bool amb = false;
#pragma unroll
        for (int s = 0; s < S; ++s) {
            bool hs = false;
#pragma unroll
            for (int m = 0; m < PPL; ++m) hs |= near32_t0(sxf[s], syf[s], mpxf[m], mpyf[m], gsp, amb, t0);
            hsp[s] = hs;
        }
        bool hh = false;
        if (S == 2 && q == 0) hh = near32_t0(sxf[0], syf[0], sxf[S - 1], syf[S - 1], gss, amb, t0);
        if (__any(amb)) {   // the exact tests, for the ambiguous lanes (never tick 0, see near32_t0)
#pragma unroll
            for (int s = 0; s < S; ++s) {
                bool hs = false;
#pragma unroll
                for (int m = 0; m < PPL; ++m)
                    hs |= (q + LPE * m < np) & closer_exact(sx[s], sy[s], double(mpx[m]), double(mpy[m]), gsp, t0);
                hsp[s] = amb ? hs : hsp[s];
            }
            if (S == 2 && q == 0) hh = amb ? closer_exact(sx[0], sy[0], sx[S - 1], sy[S - 1], gss, t0) : hh;
        }
#pragma unroll
        for (int s = 0; s < S; ++s) hsp[s] = hsp[s] || hh;
    }

    // (quad instance only: in the pair instance the extra live range spills)
    constexpr bool EARLY_POST = HELP && LPE == 4;
    if constexpr (EARLY_POST) {
        // a wave without live bullets (every wave of config 2) knows its
        // finished envs now -- a ship collision or the timeout -- so it
        // posts them before its bullet pass and output section, not after
        if (total == 0) {   // uniform
            bool fin = !live;
#pragma unroll
            for (int s = 0; s < S; ++s) fin |= quad_any<LPE>(hsp[s], lane);
            help_post(s_box_all[wv], __ballot(active && fin && auto_reset && q == 0), lane);
        }
    }

    STAMP(3);
    // ---- bullets (core.py:241-251, 264-266, 295-300): collide with the old
    //      bodies, move, cull, compact in place (bullets_rounds)
    bullets_rounds<T, S, PMAX, LPE, (HELP || OPAQUE) ? 2 : 1, QWIN, EAGER_BULLETS>(
        p, bgl, bin, lane, e, q, nb, sxf, syf, mpxf, mpyf, s_body, s_index, s_kept, s_hit, gp, gs STAMP_PASS);
    if constexpr (HELP) {   // the helper has its copy of the headers before any is rewritten (HelpBox.seen)
        if (!wait_lds_word(s_box_all[wv].seen)) report_error(st, ASTRO_ERR_HEADER_WAIT, lane);
    }
    const int wr_in = s_kept[e];
    const int hit_bits = s_hit[e];
    // the stores below recompute their addresses from an opaque copy of the
    // env index (holding the load addresses live across the bullet pass
    // costs registers the bullet pass needs)
    int is = i;
    asm volatile("" : "+v"(is));
    n_bin += active && q == 0 ? uint32_t(nb) : 0u;
    STAMP(4);

    if (active) {
        bool hit[S];
#pragma unroll
        for (int s = 0; s < S; ++s) hit[s] = quad_any<LPE>(hsp[s], lane) || ((hit_bits >> s) & 1);
        const bool collided = S == 2 ? (hit[0] || hit[S - 1]) : hit[0];
        const bool timeout = !collided && !live;
        const uint8_t done = collided ? 1 : (timeout ? 2 : 0);
        if (q < S) {   // rewards (core.py:253-260): lane s writes ship s's
            const bool mh = q == 0 ? hit[0] : hit[S - 1];
            reward[size_t(is) * S + q] = collided ? (mh ? -1.0f : 1.0f) : (timeout ? p.timeout_reward : 0.0f);
        }
        if (q == 0) done_out[is] = done;
        STAMP(5);
        if constexpr (HELP) {   // post the finished envs to the helper wave, then go on
            // (lane 0 is active in every wave that gets here: base < N)
            if (!EARLY_POST || total > 0)   // uniform (a wave without bullets posted before its bullet pass)
                help_post(s_box_all[wv], __ballot(done && auto_reset && q == 0), lane);
            if constexpr (PRIO && PRIO_SQ != PRIO_SP) __builtin_amdgcn_s_setprio(PRIO_SQ);
        }

        if (!done) {   // uniform over the quad
            // ---- fire: ship s's bullet appended after the survivors, in ship order
            int wr = wr_in;
            if ((fire_word >> (tick & 31)) & 1u) {
                bool keep = false;
                V out;
                if (q < S) {
                    const float os = p.spawn_off * ds, oc = p.spawn_off * dc;
                    const float vs = p.bullet_speed * ds, vc = p.bullet_speed * dc;
                    if (t0) {
                        const float dtf = float(p.dt);
                        const float bx = float(mx) + os, by = float(my) + oc;
                        const float bdx = (float(mdx) + vs) + 0.0f, bdy = (float(mdy) + vc) + 0.0f;
                        const float nx = bx + dtf * bdx, ny = by + dtf * bdy;
                        keep = (-1.0f <= nx && nx <= 1.0f) || (-1.0f <= ny && ny <= 1.0f);
                        out.x = T(nx);
                        out.y = T(ny);
                        out.z = T(bdx);
                        out.w = T(bdy);
                    } else {
                        const double bx = mx + double(os), by = my + double(oc);
                        const double bdx = (mdx + double(vs)) + 0.0, bdy = (mdy + double(vc)) + 0.0;
                        const double nx = bx + p.dt * bdx, ny = by + p.dt * bdy;
                        keep = (-1.0 <= nx && nx <= 1.0) || (-1.0 <= ny && ny <= 1.0);
                        out.x = T(nx);
                        out.y = T(ny);
                        out.z = T(bdx);
                        out.w = T(bdy);
                    }
                }
                const uint64_t nib = (__ballot(keep) >> (lane & ~(LPE - 1))) & ((1ull << LPE) - 1);
                const int pos = wr + __popcll(nib & ((1ull << q) - 1));
                if (keep && pos < p.b_cap) st_out(&bullets[size_t(is) * BC + pos], out);
                wr += __popcll(nib);
            }
            const int w = wr < p.b_cap ? wr : p.b_cap;
            const int dropped = wr - w;

            // ---- own ship: semi-implicit Euler + wrap (core.py:283-288)
            if (q < S) {
                const double ndx = mdx + ax * p.dt;
                const double ndy = mdy + ay * p.dt;
                V v;
                v.x = T(wrap_unit<double>(mx + p.dt * ndx));
                v.y = T(wrap_unit<double>(my + p.dt * ndy));
                v.z = T(ndx);
                v.w = T(ndy);
                st_out(&ships[size_t(q) * NN + is], v);
                st_out(&ships_b[size_t(q) * NN + is], T(mb + p.db * double((ctl >> 1) - 1)));
            }

            STAMP(6);
            // ---- own planets (core.py:289-294); the pair instance's helper waves do it
            if constexpr (!PLANETS_ON_HELPER) {
                V pout[PPL];
                planet_update<T, S, PMAX, LPE, PPL>(p, pv, mpx, mpy, q, np, t0, slot_last, pout);
#pragma unroll
                for (int m = 0; m < PPL; ++m) {
                    const int j = q + LPE * m;
                    if (j < np) st_out(&planets[size_t(j) * NN + is], pout[m]);
                }
            }

            STAMP(7);
            if (q == 0) {
                const int fl = flags | (dropped ? 1 : 0);
                if constexpr (PENDING_ON_HELPER) {   // words 2-3: the helper's
                    st_out(&reinterpret_cast<int2 *>(st.hdr)[2 * is], make_int2(tick + 1, np | (fl << 8) | (w << 16)));
                } else {
                    const uint32_t kv = check_pending(p, st, is, key_valid, undrawn, c_pend, pend_seed, pend_key);
                    st_out(&reinterpret_cast<int4 *>(st.hdr)[is],
                           make_int4(tick + 1, np | (fl << 8) | (w << 16), int(pend_seed | kv), int(pend_key)));
                }
                n_bout += uint32_t(w);
                n_drop += uint32_t(dropped);
            }
            STAMP(8);
        } else {
            STAMP(9);
            f_coll = q == 0 && collided;
            f_tout = q == 0 && timeout;
            need_reset = auto_reset && q == 0;
            f_reset = need_reset;
        }
    }

    // ---- auto-reset: the wave creates its finished envs' next games together,
    //      up to four per pass with 16 lanes each (wave_reset_pass); rejected
    //      randint words (max_planets not a power of two) take the serial path
    if constexpr (!HELP)
    for (uint64_t todo = __ballot(need_reset); todo;)   // uniform
        todo = wave_reset_pass<T, S, PMAX, LPE>(p, st, todo, lane, is, pend_seed, pend_key, key_valid || p.key_table,
                                           undrawn, s_chain, s_serial, GlobalSink<T>{st} STAMP_PASS);
    if (!HELP && auto_reset) {
        wave_sync();
        if (stats) c_serial += __popcll(__ballot(active && q == 0 && s_serial[e]));
        if (active && s_serial[e]) {   // uniform over the quad; rare
            const uint32_t kq = uint32_t(quad_bcast_i<0, LPE>(int(pend_key)));   // lane q == 0 fetched it
            const uint4 c = reinterpret_cast<const uint4 *>(st.stream)[is];
            const NextGame<S> ng = next_game<S>(p, pend_seed, kq, key_valid || p.key_table, undrawn, c,
                                                stream_ring_of(st, is));
            restart_env<T, S, PMAX, LPE>(p, st, is, ng, q, GlobalSink<T>{st});
        }
    }
    STAMP(10);
    if (stats) {
        c_reset += __popcll(__ballot(f_reset));
        c_coll += __popcll(__ballot(f_coll));
        c_tout += __popcll(__ballot(f_tout));
    }
#ifdef ASTRO_STAMPS
    {   // where the wave ran and what it carried: per-SIMD load attribution
        unsigned hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        const unsigned long long n_res = __popcll(__ballot(f_reset));
        const unsigned long long n_t0 = __popcll(__ballot(active && q == 0 && t0));
        stamp_[14] = (unsigned long long)hw | ((unsigned long long)xcc << 32);
        stamp_[15] = n_res | (n_t0 << 8) | ((unsigned long long)total << 16);
    }
#endif
    return QuadCounts{n_bin, n_bout, n_pl, n_drop, c_reset, c_coll, c_tout, c_serial};
}

// Add one tick's counters to the wave's private stats row (lane 0).  A
// lane's per-tick counts are < 2^16 and, for b_cap * (envs per wave) <
// 65,536, so are their sums over the wave's envs: two counters then share
// one wave sum.
__device__ __forceinline__ void flush_counts(unsigned long long *slot, const QuadCounts &c, bool packed) {
    const uint32_t a = wave_sum32(packed ? (c.n_bin | (c.n_bout << 16)) : c.n_bin);
    const uint32_t b = wave_sum32(packed ? (c.n_pl | (c.n_drop << 16)) : c.n_bout);
    const uint32_t x = packed ? 0u : wave_sum32(c.n_pl);
    const uint32_t y = packed ? 0u : wave_sum32(c.n_drop);
    if ((threadIdx.x & 63) == 0) {
        const uint64_t bin = packed ? (a & 0xffff) : a;
        const uint64_t bout = packed ? (a >> 16) : b;
        const uint64_t pl = packed ? (b & 0xffff) : x;
        const uint64_t drop = packed ? (b >> 16) : y;
        if (bin) atomicAdd(slot + ASTRO_STAT_BULLETS_IN, (unsigned long long)bin);
        if (bout) atomicAdd(slot + ASTRO_STAT_BULLETS_OUT, (unsigned long long)bout);
        if (c.c_reset) atomicAdd(slot + ASTRO_STAT_RESETS, (unsigned long long)c.c_reset);
        if (c.c_coll) atomicAdd(slot + ASTRO_STAT_COLLISIONS, (unsigned long long)c.c_coll);
        if (c.c_tout) atomicAdd(slot + ASTRO_STAT_TIMEOUTS, (unsigned long long)c.c_tout);
        if (drop) atomicAdd(slot + ASTRO_STAT_OVERFLOWS, (unsigned long long)drop);
        if (pl) atomicAdd(slot + ASTRO_STAT_PLANETS, (unsigned long long)pl);
        if (c.c_serial) atomicAdd(slot + ASTRO_STAT_SERIAL, (unsigned long long)c.c_serial);
    }
}

// astro_rollout's quad kernel takes its arguments as ONE struct, so the
// tick function can read them straight from the kernarg segment (scalar
// loads) instead of from a private copy.
struct QuadArgs {
    AstroParams p;
    AstroState st;
    TickDriver drv;
    float *reward;
    uint8_t *done;
    unsigned long long *stats;
    int auto_reset;
};
typedef const __attribute__((address_space(4))) QuadArgs *KernArgs;


// Waves per SIMD the one-tick instances without helpers are built for:
// 8 planet slots: 3 (141 VGPRs, no spills; at 4: 128 VGPRs, 41 spilled, c5
// 34.3 -> 31.1 us); 4 slots: 4 (127 VGPRs with one bullet round at a time,
// no spills; c3 at 1M envs 131.8 us at 3, 119.2 at 4,
// profiles/round4/ab_1m_waves.jsonl).
// The K-tick (rollout) instances: 4 planet slots at 3 waves per SIMD (168
// VGPRs; at 2 the 1M-env rollouts ran 110 vs 91 us per tick,
// profiles/round4/ab_packed_bullets_v1.jsonl), 8 slots and the ScriptBot
// instance at 2 (at 3 they spill 25 / 55 VGPRs).
// The 4-slot instances with helper waves share the bound: at 4 waves per
// SIMD the quad helper instance holds 109-111 VGPRs and the pair one 121-123,
// no scratch in either (-Rpass-analysis=kernel-resource-usage, round 5).
// (-DASTRO_P4_WAVES / _P8_WAVES / _M4_WAVES: occupancy A/B builds only)
#ifndef ASTRO_P8_WAVES
#define ASTRO_P8_WAVES 3
#endif
#ifndef ASTRO_P4_WAVES
#define ASTRO_P4_WAVES 4
#endif
#ifndef ASTRO_M4_WAVES
#define ASTRO_M4_WAVES 3
#endif
constexpr int P8_WAVES = ASTRO_P8_WAVES, P4_WAVES = ASTRO_P4_WAVES, M4_WAVES = ASTRO_M4_WAVES;

// STATS: the one-tick instances come in two builds, with the counters and
// without (a launch with a null stats pointer): compiled in but switched off
// at run time they still cost c3 0.6 us per launch, switched on 1.6 us of
// 12.1 (the per-lane counts, the wave sums and the row atomics at the
// slowest waves' ends; profiles/round5/ab_stats_flush.jsonl)
template <typename T, int S, int PMAX, bool MULTI, int LPE, bool BOTS = false, bool HELP = false,
          int WPG = QW, bool STATS = true>
__global__ __launch_bounds__(HELP ? 2 * (64 * WPG) : (64 * WPG), MULTI ? (BOTS || PMAX > 4 ? 2 : M4_WAVES) : (PMAX > 4 ? P8_WAVES : P4_WAVES)) void astro_step_quad_kernel(AstroParams p, AstroState st, TickDriver drv,
                                                                float *__restrict__ reward_all,
                                                                uint8_t *__restrict__ done_all,
                                                                unsigned long long *stats, int auto_reset) {
#ifdef ASTRO_STAMPS
    unsigned long long stamp_[NSTAMP] = {};
    quad_tick<T, S, PMAX, LPE, false, false, HELP, WPG>(p, st, drv, reward_all, done_all, STATS && stats != nullptr,
                                                       auto_reset, 0,
                                                   stamp_);
    STAMP(11);
    if (stats && (threadIdx.x & 63) == 0) {   // a helper wave: slots 20-22 of its step wave's row
        const bool hw = int(threadIdx.x) >= (64 * WPG);
        unsigned long long *row = stats + size_t(blockIdx.x * WPG + (threadIdx.x / 64) % WPG) * NSTAMP;
        // (constant indices only: a loop over a runtime range put the stamp
        // array in scratch, and its stores then sat in the same vmcnt queue
        // as the wave's first loads -- the header wait measured them too)
#pragma unroll
        for (int k = 0; k < NSTAMP; ++k)
            if (hw == (k >= 20)) row[k] = stamp_[k];
    }
    if constexpr (!MULTI && !HELP) {   // (astro_game_step's completion word, as below)
        if (drv.flag != nullptr && (threadIdx.x & 63) == 0)
            __hip_atomic_store(drv.flag, drv.flag_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
#else
    // ---- the launch's ticks: each wave steps its 16 envs on its own, no
    //      grid-wide barrier between ticks (envs never interact); the
    //      counters go to the wave's stats row after every tick, so nothing
    //      but the tick number lives across the loop
    // (HELP: waves WPG.. are the helpers of waves 0..WPG-1, same stats row)
    if (!HELP && int(blockIdx.x * WPG + threadIdx.x / 64) * (64 / LPE) >= st.n_env) return;   // a spare wave of the last block
    // (HELP: a spare wave returns inside quad_tick, after the workgroup's one
    // barrier)  A one-tick grid larger than the device holds at once runs in
    // rounds; the blocks of its last, partial round start last and end the
    // launch, so they run at a higher priority than the previous round's
    // stragglers (c5: 1.33 rounds, 28.15 -> 26.97 us; the last quarter of the
    // grid measured: profiles/round6/ab_late_round_priority.jsonl)
    if constexpr (!MULTI && !HELP) {
        if (drv.late_block > 0 && int(blockIdx.x) >= drv.late_block) __builtin_amdgcn_s_setprio(1);
    }
    const int n_ticks = MULTI ? drv.ticks : 1;   // (astro_step: a one-tick instance without the loop)
    for (int kt = 0; kt < n_ticks; ++kt) {
        QuadCounts c;
        if constexpr (MULTI) {
            // the arguments through an opaque copy of the kernarg pointer:
            // scalar loads re-issued each tick instead of hoisted out of the
            // loop and held across it (which spilled ~120 VGPRs)
            auto kp = __builtin_amdgcn_kernarg_segment_ptr();
            asm volatile("" : "+s"(kp));
            const QuadArgs &a = *(const QuadArgs *)(KernArgs(kp));
            c = quad_tick<T, S, PMAX, LPE, true, BOTS>(a.p, a.st, a.drv, a.reward, a.done, a.stats != nullptr,
                                                        a.auto_reset, kt);
        } else {
            c = quad_tick<T, S, PMAX, LPE, false, false, HELP, WPG>(p, st, drv, reward_all, done_all,
                                                               STATS && stats != nullptr, auto_reset, kt);
        }
        if (STATS && stats) {
            const int row = __builtin_amdgcn_readfirstlane(int(blockIdx.x * WPG + (threadIdx.x / 64) % WPG));
            if (row * (64 / LPE) < st.n_env)
                flush_counts(stats + size_t(row) * ASTRO_NSTATS, c, p.b_cap * (64 / LPE) < 65536);
        }
        // this tick's stores (other lanes' bullets included) before the
        // wave's next tick reads them: vmcnt(0), on this CU's own L1
        if (kt + 1 < n_ticks) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    }
    if constexpr (!MULTI && !HELP) {
        // a single game's tick (astro_game_step: one env, one wave): the
        // completion word after every store of the wave (a system-scope
        // release), which the host reads ahead of the stream's completion
        if (drv.flag != nullptr && (threadIdx.x & 63) == 0)
            __hip_atomic_store(drv.flag, drv.flag_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
#endif
}

// ---------------------------------------------------------------------------
// The resident rollout: astro_rollout's K ticks with the env state ON CHIP
// (core.play's tick loop, core.py:377-410, for open-loop or on-device
// controls).  A wave loads its envs once -- header, ships and planets into
// the registers of the env's lanes (the quad/pair layout of quad_tick), the
// live bullets into the wave's LDS rows -- steps them K ticks from there, and
// stores them once at the end.  No state crosses memory between ticks, so a
// tick is its arithmetic: no load round trip, no wait for the previous
// tick's stores.  What a tick still sends to memory: its reward and done
// (the launch's outputs), and, for the first steps of a game, the pending
// seed's key gather and its seed-stream draw (check_pending, global stream
// record and ring: rare, consumed at the end of the tick).  Finished games
// are re-created in the same tick (wave_reset_pass into an LDS stage the
// env's lanes then read; the serial create into the lanes' own registers).
// Float32 state with b_cap <= RES_BCAP only (the LDS rows); other rollouts
// run quad_tick's K-tick instance.  Results are those of K astro_step
// launches, bit for bit, on every state array (tests/test_gpu_parity.py
// test_rollout_equals_stepping): every slot the launch writes in LDS is
// stored back, and a slot it never wrote is left as it was.

constexpr int RES_QWIN = 256;   // live bullets per LDS index window (a wave holds up to 32 x 32)
constexpr int RES_WPG = 4;      // waves per workgroup; two workgroups per CU fit the LDS
// bullet rounds side by side in the resident rollout (bullets_rounds NRW):
// three when a wave has a third round (c3 100-tick rollouts 7.49 -> 7.12 us
// per tick; in the one-tick instance with helpers three spill 4 VGPRs and
// lose, 10.08 -> 10.30 us; profiles/round6/ab_three_rounds.jsonl)
#ifndef ASTRO_RES_NRW
#define ASTRO_RES_NRW 3
#endif
constexpr int RES_NRW = ASTRO_RES_NRW;

template <int LPE>
__device__ __forceinline__ int4 group_bcast0(const int4 &v) {   // lane 0 of the env's group to the group
    return make_int4(quad_bcast_i<0, LPE>(v.x), quad_bcast_i<0, LPE>(v.y), quad_bcast_i<0, LPE>(v.z),
                     quad_bcast_i<0, LPE>(v.w));
}

// One tick of a resident wave (quad_tick's physics, the state from R and the
// wave's LDS rows).  ctl: this lane's control for the tick.
template <typename T, int S, int PMAX, int LPE>
__device__ __forceinline__ void res_tick(const AstroParams &p, const AstroState &st, float *__restrict__ reward_all,
                                         uint8_t *__restrict__ done_all, int auto_reset, int kt, int ctl, int lane,
                                         int base, ResEnv<T, S, PMAX, LPE> &R, lds_f4 *rows,
                                         float4 (*s_body)[(S + PMAX + 1) / 2], uint32_t *s_index, int *s_kept,
                                         int *s_hit, int *s_serial, QuadCounts &cnt) {
    using V = typename Store<T>::V;
    static_assert(std::is_same<T, float>::value, "the resident rollout holds float32 state");
    constexpr int PPL = PMAX / LPE;
    constexpr int NBOD2 = (S + PMAX + 1) / 2;
    const int q = lane & (LPE - 1);
    const int e = lane / LPE;
    const int N = st.n_env;
    const size_t NN = size_t(N);
    const bool active = base + e < N;
    const int i = active ? base + e : N - 1;
    float *__restrict__ reward = reward_all + size_t(kt) * NN * S;
    uint8_t *__restrict__ done_out = done_all + size_t(kt) * NN;
    bool f_reset = false, f_coll = false, f_tout = false, need_reset = false;
#ifdef ASTRO_STAMPS
    unsigned long long stamp_[NSTAMP] = {};   // (the stamp build's sections; not recorded here)
#endif

    // ---- the state, from registers
    const int4 h = R.h;
    const V sv = R.sv;
    const T sbv = R.sb;
    V pv[PPL];
    T mpx[PPL], mpy[PPL];
#pragma unroll
    for (int m = 0; m < PPL; ++m) {
        pv[m] = R.pv[m];
        mpx[m] = pv[m].x;
        mpy[m] = pv[m].y;
    }
    const int tick = int(uint32_t(h.x) & TICK_MASK);
    const bool key_valid = (uint32_t(h.z) & KEY_VALID) != 0;
    const bool undrawn = (uint32_t(h.z) & UNDRAWN) != 0;
    uint32_t pend_seed = uint32_t(h.z) & SEED_MASK;
    int np = h.y & 0xff;
    const int flags = (h.y >> 8) & 0xff;
    const int nb = active ? min(int(uint32_t(h.y) >> 16), p.b_cap) : 0;
    np = np < 1 ? 1 : (np > PMAX ? PMAX : np);
    const bool slot_last = __builtin_amdgcn_readfirstlane(int(__any(np == PMAX))) != 0;
    const int np_uni = wave_uniform_count(np);
    const bool live = tick < p.timeout_tick;
    const bool t0 = tick == 0;
    const uint32_t fire_word = p.fire_bits[(live ? tick : 0) >> 5];
    uint32_t pend_key = uint32_t(h.w);
    cnt.n_pl += active && q == 0 ? uint32_t(np) : 0u;
    float rw_out = 0.0f;   // this tick's reward (lanes q < S) and done (q == 0), stored last
    uint8_t done_v = 0;

    // ---- the wave's live bullets numbered densely, first rounds read (LDS)
    const BulletsLds<S, NBOD2> bm{rows, lds_ptr(&s_body[0][0])};
    const BulletsIn<T> bin = bullets_begin<T, LPE, RES_QWIN>(bm, lane, e, q, nb, np, t0, s_index, s_kept, s_hit,
                                                             s_serial);
    // the pending seed's key gather and stream cursor (check_pending, a
    // game's first steps): issued now, consumed at the end of the tick
    if (q == 0 && !key_valid && !undrawn && p.key_table) pend_key = p.key_table[pend_seed & SEED_MASK];
    const bool want_c = q == 0 && (undrawn || (!key_valid && p.key_table && p.planets_only));
    uintptr_t c_stream = reinterpret_cast<uintptr_t>(st.stream), c_hdr = reinterpret_cast<uintptr_t>(st.hdr);
    asm volatile("" : "+s"(c_stream), "+s"(c_hdr));   // (as quad_tick: loaded branch-free)
    const uint4 c_pend = load_u4_global(want_c ? c_stream : c_hdr, size_t(i));

    // ---- broadcasts, own ship's direction, thrust + gravity (core.py:234-239)
    double px[PMAX], py[PMAX], sx[S], sy[S];
    bcast_slots<T, PPL, LPE>(mpx, px);
    bcast_slots<T, PPL, LPE>(mpy, py);
    sx[0] = double(quad_bcast<0, LPE>(sv.x));
    sy[0] = double(quad_bcast<0, LPE>(sv.y));
    if (S == 2) {
        sx[S - 1] = double(quad_bcast<S - 1, LPE>(sv.x));
        sy[S - 1] = double(quad_bcast<S - 1, LPE>(sv.y));
    }
    const double mx = double(sv.x), my = double(sv.y), mdx = double(sv.z), mdy = double(sv.w);
    const double mb = double(sbv);
    float ds, dc;
    np_sincosf(float(mb), ds, dc);
    double ax = 0.0, ay = 0.0;
    double sgx = 0.0, sgy = 0.0;
    if constexpr (LPE == 4 && PMAX == 4) {   // the ships' fields split over the quad (as quad_tick)
        double s0x = sx[0], s0y = sy[0], s1x = sx[S - 1], s1y = sy[S - 1];
        double p0x = px[0], p0y = py[0], p1x = px[1], p1y = py[1], p2x = px[2], p2y = py[2], p3x = px[3], p3y = py[3];
        asm volatile("" : "+v"(s0x), "+v"(s0y), "+v"(s1x), "+v"(s1y));
        asm volatile("" : "+v"(p0x), "+v"(p0y), "+v"(p1x), "+v"(p1y), "+v"(p2x), "+v"(p2y), "+v"(p3x), "+v"(p3y));
        const bool odd = (q & 1) != 0, hi = q >= 2;
        const double shx = odd ? s1x : s0x, shy = odd ? s1y : s0y;
        const double ax_ = hi ? p1x : p0x, ay_ = hi ? p1y : p0y;
        const double bx_ = hi ? p3x : p2x, by_ = hi ? p3y : p2y;
        const double rax = ax_ - shx, ray = ay_ - shy, rbx = bx_ - shx, rby = by_ - shy;
        const double fa = div_gravity(p.gm, max_floor(rax * rax + ray * ray));
        const double fb = div_gravity(p.gm, max_floor(rbx * rbx + rby * rby));
        const double tax = fa * rax, tay = fa * ray, tbx = fb * rbx, tby = fb * rby;
        const double t1x = quad_perm_d<2, 3, 2, 3>(tax), t1y = quad_perm_d<2, 3, 2, 3>(tay);
        const double t3x = quad_perm_d<2, 3, 2, 3>(tbx), t3y = quad_perm_d<2, 3, 2, 3>(tby);
        sgx = tax;
        sgy = tay;
        sgx = 1 < np ? sgx + t1x : sgx;
        sgy = 1 < np ? sgy + t1y : sgy;
        sgx = 2 < np ? sgx + tbx : sgx;
        sgy = 2 < np ? sgy + tby : sgy;
        sgx = slot_last && 3 < np ? sgx + t3x : sgx;
        sgy = slot_last && 3 < np ? sgy + t3y : sgy;
    }
    if (q < S) {
        double gx, gy;
        if (t0) {
            float fx, fy;
            field<float, PMAX>(px, py, np, mx, my, p.gm, fx, fy);
            gx = double(fx);
            gy = double(fy);
        } else if constexpr (LPE == 4 && PMAX == 4) {
            gx = sgx;
            gy = sgy;
        } else {
            field<double, PMAX>(px, py, np, mx, my, p.gm, gx, gy, slot_last, PMAX <= 4 ? np_uni : 0);
        }
        const double thr = p.thrust * double(ctl & 1);
        ax = thr * double(ds) + gx;
        ay = thr * double(dc) + gy;
    }

    // ---- ship collisions (core.py:241-253)
    const Guard gsp(p.r2_sp), gss(p.r2_ss), gp(p.r2_p0), gs(p.r2_s0);
    float sxf[S], syf[S], mpxf[PPL], mpyf[PPL];
#pragma unroll
    for (int s = 0; s < S; ++s) {
        sxf[s] = float(sx[s]);
        syf[s] = float(sy[s]);
    }
#pragma unroll
    for (int m = 0; m < PPL; ++m) {
        mpxf[m] = q + LPE * m < np ? float(mpx[m]) : -FAR_POS;
        mpyf[m] = q + LPE * m < np ? float(mpy[m]) : -FAR_POS;
    }
    bool hsp[S];
    {
        bool amb = false;
#pragma unroll
        for (int s = 0; s < S; ++s) {
            bool hs = false;
#pragma unroll
            for (int m = 0; m < PPL; ++m) hs |= near32_t0(sxf[s], syf[s], mpxf[m], mpyf[m], gsp, amb, t0);
            hsp[s] = hs;
        }
        bool hh = false;
        if (S == 2 && q == 0) hh = near32_t0(sxf[0], syf[0], sxf[S - 1], syf[S - 1], gss, amb, t0);
        if (__any(amb)) {
#pragma unroll
            for (int s = 0; s < S; ++s) {
                bool hs = false;
#pragma unroll
                for (int m = 0; m < PPL; ++m)
                    hs |= (q + LPE * m < np) & closer_exact(sx[s], sy[s], double(mpx[m]), double(mpy[m]), gsp, t0);
                hsp[s] = amb ? hs : hsp[s];
            }
            if (S == 2 && q == 0) hh = amb ? closer_exact(sx[0], sy[0], sx[S - 1], sy[S - 1], gss, t0) : hh;
        }
#pragma unroll
        for (int s = 0; s < S; ++s) hsp[s] = hsp[s] || hh;
    }

    // ---- bullets (core.py:241-251, 264-266, 295-300), in the LDS rows
    bullets_rounds<T, S, PMAX, LPE, RES_NRW, RES_QWIN>(p, bm, bin, lane, e, q, nb, sxf, syf, mpxf, mpyf, s_body,
                                                       s_index, s_kept, s_hit, gp, gs STAMP_PASS);
    const int wr_in = s_kept[e];
    const int hit_bits = s_hit[e];
    cnt.n_bin += active && q == 0 ? uint32_t(nb) : 0u;
    R.hw = max(R.hw, wr_in);   // (the pass compacted the row's first wr_in slots, finished game or not)

    if (active) {
        bool hit[S];
#pragma unroll
        for (int s = 0; s < S; ++s) hit[s] = quad_any<LPE>(hsp[s], lane) || ((hit_bits >> s) & 1);
        const bool collided = S == 2 ? (hit[0] || hit[S - 1]) : hit[0];
        const bool timeout = !collided && !live;
        const uint8_t done = collided ? 1 : (timeout ? 2 : 0);
        // rewards (core.py:253-260); stored at the end of the tick, after
        // the tick's last wait for its own loads (a store issued before a
        // wait for every memory op in flight would be waited for there)
        const bool mh = q == 0 ? hit[0] : hit[S - 1];
        rw_out = collided ? (mh ? -1.0f : 1.0f) : (timeout ? p.timeout_reward : 0.0f);
        done_v = done;

        if (!done) {   // uniform over the env's lanes
            // ---- fire: ship s's bullet after the survivors, in ship order (core.py:267-280)
            int wr = wr_in;
            if ((fire_word >> (tick & 31)) & 1u) {
                bool keep = false;
                V out;
                if (q < S) {
                    const float os = p.spawn_off * ds, oc = p.spawn_off * dc;
                    const float vs = p.bullet_speed * ds, vc = p.bullet_speed * dc;
                    if (t0) {
                        const float dtf = float(p.dt);
                        const float bx = float(mx) + os, by = float(my) + oc;
                        const float bdx = (float(mdx) + vs) + 0.0f, bdy = (float(mdy) + vc) + 0.0f;
                        const float nx = bx + dtf * bdx, ny = by + dtf * bdy;
                        keep = (-1.0f <= nx && nx <= 1.0f) || (-1.0f <= ny && ny <= 1.0f);
                        out.x = T(nx);
                        out.y = T(ny);
                        out.z = T(bdx);
                        out.w = T(bdy);
                    } else {
                        const double bx = mx + double(os), by = my + double(oc);
                        const double bdx = (mdx + double(vs)) + 0.0, bdy = (mdy + double(vc)) + 0.0;
                        const double nx = bx + p.dt * bdx, ny = by + p.dt * bdy;
                        keep = (-1.0 <= nx && nx <= 1.0) || (-1.0 <= ny && ny <= 1.0);
                        out.x = T(nx);
                        out.y = T(ny);
                        out.z = T(bdx);
                        out.w = T(bdy);
                    }
                }
                const uint64_t nib = (__ballot(keep) >> (lane & ~(LPE - 1))) & ((1ull << LPE) - 1);
                const int pos = wr + __popcll(nib & ((1ull << q) - 1));
                if (keep && pos < p.b_cap) bm.store(e, pos, out);
                wr += __popcll(nib);
            }
            const int w = wr < p.b_cap ? wr : p.b_cap;
            const int dropped = wr - w;
            R.hw = max(R.hw, w);

            // ---- own ship: semi-implicit Euler + wrap (core.py:283-288)
            if (q < S) {
                const double ndx = mdx + ax * p.dt;
                const double ndy = mdy + ay * p.dt;
                V v;
                v.x = T(wrap_unit<double>(mx + p.dt * ndx));
                v.y = T(wrap_unit<double>(my + p.dt * ndy));
                v.z = T(ndx);
                v.w = T(ndy);
                R.sv = v;
                R.sb = T(mb + p.db * double((ctl >> 1) - 1));
            }
            // ---- own planets (core.py:289-294)
            {
                V pout[PPL];
                planet_update<T, S, PMAX, LPE, PPL>(p, pv, mpx, mpy, q, np, t0, slot_last, pout);
#pragma unroll
                for (int m = 0; m < PPL; ++m)
                    if (q + LPE * m < np) R.pv[m] = pout[m];
            }
            // ---- header: the pending seed checked by lane 0 (check_pending), to every lane
            const int fl = flags | (dropped ? 1 : 0);
            uint32_t kv = 0;
            if (q == 0) kv = check_pending(p, st, i, key_valid, undrawn, c_pend, pend_seed, pend_key);
            const int w2 = quad_bcast_i<0, LPE>(int(pend_seed | kv)), w3 = quad_bcast_i<0, LPE>(int(pend_key));
            R.h = make_int4(tick + 1, np | (fl << 8) | (w << 16), w2, w3);
            if (q == 0) {
                cnt.n_bout += uint32_t(w);
                cnt.n_drop += uint32_t(dropped);
            }
        } else {
            f_coll = q == 0 && collided;
            f_tout = q == 0 && timeout;
            need_reset = auto_reset && q == 0;
            f_reset = need_reset;
        }
    }

    // ---- auto-reset: reset passes (four games at a time) into the LDS stage,
    //      each env's lanes then take their part of its new game
    ResStage<S, PMAX> *stage = reinterpret_cast<ResStage<S, PMAX> *>(&s_body[0][0]);
    static_assert(4 * sizeof(ResStage<S, PMAX>) <= sizeof(float4) * (64 / LPE) * NBOD2, "stage over the body rows");
    uint32_t(*s_chain)[2][13 + 2 * S] = reinterpret_cast<uint32_t(*)[2][13 + 2 * S]>(s_index);
    static_assert(4 * 2 * (13 + 2 * S) <= RES_QWIN, "the reset chains over the index window");
    const StageSink<T, S, PMAX> ssink{stage};
    for (uint64_t todo = __ballot(need_reset); todo;) {   // uniform
        const uint64_t before = todo;
        todo = wave_reset_pass<T, S, PMAX, LPE, false, StageSink<T, S, PMAX>>(
            p, st, todo, lane, i, pend_seed, pend_key, key_valid || p.key_table, undrawn, s_chain, s_serial,
            ssink STAMP_PASS);
        const uint64_t served = before & ~todo;
        wave_sync();
        const int ldr = lane & ~(LPE - 1);
        if (((served >> ldr) & 1ull) && !s_serial[e]) {   // uniform over the env's lanes
            const ResStage<S, PMAX> &g = stage[__popcll(served & ((1ull << ldr) - 1))];
            const int4 nh = g.hdr;
            if (q == 0) st.stream[4 * size_t(i) + 3] = g.seed;
            const int sq = q < S ? q : 0;
            const float4 shv = g.ship[sq];
            R.sv = V{shv.x, shv.y, shv.z, shv.w};
            R.sb = g.b[sq];
            const int n_new = nh.y & 0xff;
#pragma unroll
            for (int m = 0; m < PPL; ++m) {
                if (q + LPE * m < n_new) {
                    const float4 pl = g.planet[q + LPE * m];
                    R.pv[m] = V{pl.x, pl.y, pl.z, pl.w};
                }
            }
            R.h = nh;
        }
        wave_sync();   // the stage is free for the next pass
    }
    if (auto_reset) {
        wave_sync();
        cnt.c_serial += __popcll(__ballot(active && q == 0 && s_serial[e]));
        if (active && s_serial[e]) {   // uniform over the env's lanes; rare
            const uint32_t kq = uint32_t(quad_bcast_i<0, LPE>(int(pend_key)));
            const uint4 c = reinterpret_cast<const uint4 *>(st.stream)[i];
            const NextGame<S> ng = next_game<S>(p, pend_seed, kq, key_valid || p.key_table, undrawn, c,
                                                stream_ring_of(st, i));
            restart_env<T, S, PMAX, LPE, RegSink<T, S, PMAX, LPE>>(p, st, i, ng, q, RegSink<T, S, PMAX, LPE>{&R});
            R.h = group_bcast0<LPE>(R.h);   // (restart_env set the header on lane 0)
        }
    }
    cnt.c_reset += __popcll(__ballot(f_reset));
    cnt.c_coll += __popcll(__ballot(f_coll));
    cnt.c_tout += __popcll(__ballot(f_tout));
    if (active) {   // the tick's outputs
        if (q < S) reward[size_t(i) * S + q] = rw_out;
        if (q == 0) done_out[i] = done_v;
    }
}

// Controls of the resident rollout: RANDOM / NOTHING / a control array
// (the next tick's array entry loaded a tick ahead).  (ScriptBot policies
// stay on quad_tick's BOTS instance: a resident ScriptBot instance, decisions
// from the registers at each tick's start, ran 12.86-13.13 vs 12.48-12.77 us
// per c3 tick -- the ticks are bound by the bots' arithmetic, and two bullet
// rounds side by side spilled there; profiles/round6/ab_resident_bots.jsonl)
template <typename T, int S, int PMAX, int LPE>
__global__ __launch_bounds__(64 * RES_WPG, 2) void astro_rollout_res_kernel(AstroParams p, AstroState st,
                                                                           TickDriver drv,
                                                                           float *__restrict__ reward_all,
                                                                           uint8_t *__restrict__ done_all,
                                                                           unsigned long long *stats,
                                                                           int auto_reset) {
    using V = typename Store<T>::V;
    constexpr int PPL = PMAX / LPE;
    constexpr int QENV = 64 / LPE;
    constexpr int NBOD2 = (S + PMAX + 1) / 2;
    __shared__ float4 s_rows_all[RES_WPG][QENV * RES_BCAP];
    __shared__ float4 s_body_all[RES_WPG][QENV][NBOD2];
    __shared__ uint32_t s_index_all[RES_WPG][RES_QWIN];
    __shared__ int s_kept_all[RES_WPG][QENV], s_hit_all[RES_WPG][QENV], s_serial_all[RES_WPG][QENV];
    const int wv = int(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int q = lane & (LPE - 1);
    const int e = lane / LPE;
    const int N = st.n_env;
    const size_t NN = size_t(N);
    const int base = (blockIdx.x * RES_WPG + wv) * QENV;
    if (base >= N) return;   // a spare wave of the last block (waves never wait for each other)
    const bool active = base + e < N;
    const int i = active ? base + e : N - 1;
    const int sq = q < S ? q : 0;
    lds_f4 *rows = lds_ptr(&s_rows_all[wv][0]);

    // ---- load the wave's envs
    ResEnv<T, S, PMAX, LPE> R;
    R.h = reinterpret_cast<const int4 *>(st.hdr)[i];
    R.sv = reinterpret_cast<const V *>(st.ships)[size_t(sq) * NN + i];
    R.sb = reinterpret_cast<const T *>(st.ships_b)[size_t(sq) * NN + i];
#pragma unroll
    for (int m = 0; m < PPL; ++m) {
        const int j = q + LPE * m;
        R.pv[m] = reinterpret_cast<const V *>(st.planets)[size_t(j < p.p_pad ? j : 0) * NN + i];
    }
    const int nb0 = active ? min(int(uint32_t(R.h.y) >> 16), p.b_cap) : 0;
    R.hw = nb0;
    {   // the env's live bullets into its LDS row, lane q taking slots q, q + LPE, ...
        const V *brow = reinterpret_cast<const V *>(st.bullets) + size_t(i) * size_t(p.b_cap);
        for (int k0 = 0; k0 < nb0; k0 += 4 * LPE) {
            V v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int k = k0 + q + LPE * u;
                v[u] = brow[k < nb0 ? k : 0];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int k = k0 + q + LPE * u;
                if (k < nb0) {
                    v4f w;
                    w.x = v[u].x;
                    w.y = v[u].y;
                    w.z = v[u].z;
                    w.w = v[u].w;
                    rows[e * RES_BCAP + k] = w;
                }
            }
        }
    }
    wave_sync();

    // ---- the ticks (the arguments re-read from the kernarg segment each tick,
    //      as the K-tick quad_tick instance does: scalar loads, not SGPRs
    //      held across the loop)
    QuadCounts cnt{};
    const bool from_array = drv.policy == ASTRO_POLICY_CONTROL;
    int ctl_next = from_array ? int(drv.control[size_t(i) * S + sq]) : 0;
    const int n_ticks = drv.ticks;
    for (int kt = 0; kt < n_ticks; ++kt) {
        auto kp = __builtin_amdgcn_kernarg_segment_ptr();
        asm volatile("" : "+s"(kp));
        const QuadArgs &a = *(const QuadArgs *)(KernArgs(kp));
        int ctl;
        if (from_array) {   // uniform: this tick's entry (loaded a tick ago); the next one's issued
            ctl = ctl_next;  // (the last tick re-reads its own: no branch around the load)
            const int kn = kt + 1 < n_ticks ? kt + 1 : kt;
            ctl_next = int(a.drv.control[(size_t(kn) * NN + size_t(i)) * S + sq]);
        } else {
            ctl = tick_control<S>(a.drv, i, sq, NN, kt);
        }
        res_tick<T, S, PMAX, LPE>(a.p, a.st, a.reward, a.done, a.auto_reset, kt, ctl, lane, base, R, rows,
                                  s_body_all[wv], s_index_all[wv], s_kept_all[wv], s_hit_all[wv],
                                  s_serial_all[wv], cnt);
    }

    // ---- store the wave's envs: every slot the launch wrote (padding
    //      planet slots hold what was loaded: storing them changes nothing)
    if (active) {
        if (q == 0) reinterpret_cast<int4 *>(st.hdr)[i] = R.h;
        if (q < S) {
            reinterpret_cast<V *>(st.ships)[size_t(q) * NN + i] = R.sv;
            reinterpret_cast<T *>(st.ships_b)[size_t(q) * NN + i] = R.sb;
        }
#pragma unroll
        for (int m = 0; m < PPL; ++m) {
            const int j = q + LPE * m;
            if (j < p.p_pad) reinterpret_cast<V *>(st.planets)[size_t(j) * NN + i] = R.pv[m];
        }
        V *brow = reinterpret_cast<V *>(st.bullets) + size_t(i) * size_t(p.b_cap);
        for (int k = q; k < R.hw; k += LPE) {
            const v4f w = rows[e * RES_BCAP + k];
            brow[k] = V{w.x, w.y, w.z, w.w};
        }
    }
    if (stats) {   // the launch's counters (sums over K ticks: unpacked)
        const int row = __builtin_amdgcn_readfirstlane(int(blockIdx.x * RES_WPG + wv));
        flush_counts(stats + size_t(row) * ASTRO_NSTATS, cnt, false);
    }
}

// ---------------------------------------------------------------------------
// Observation features: rl.ValueNetwork.get_features + to_batch
// (rl.py:36-112), one lane per (env, row).  The bearing feature is
// util.norm_angle(b) / pi (util.py:125-132) in the precision numpy uses: float32
// for create()'s float32 ships (tick 0), float64 after; every value is then
// stored as float32, as the reference's float32 feature array does.

// ((b + pi) % (2 pi) - pi) / pi with numpy's floored remainder
// (npy_divmod: fmod, + divisor when the signs differ, +0 for a zero result)
template <typename C>
__device__ __forceinline__ C norm_angle_over_pi(C b) {
    return np_norm_angle<C>(b) / C(3.141592653589793);
}

// A block covers 256 consecutive (env, row) items: the per-env part (every
// ship's five features, with norm_angle's exact fmod) is computed once per
// env into LDS rather than once per row, and the block's 256 x D floats go out
// through LDS as coalesced 16-byte stores (a lane per item storing its own D
// floats wrote 4-byte words 60 bytes apart).
constexpr int FEAT_BLOCK = 256;

template <typename T, int S>
__global__ __launch_bounds__(FEAT_BLOCK) void astro_features_kernel(AstroParams p, AstroState st,
                                                                   float *__restrict__ out, int rows) {
    using V = typename Store<T>::V;
    constexpr int D = 1 + 5 * S + 4;
    constexpr int MAXE = FEAT_BLOCK + 1;   // envs a block can touch (rows >= 1)
    __shared__ float s_ship[MAXE][5 * S];
    __shared__ int s_cnt[MAXE][2];         // nplanets, nbullets
    __shared__ float4 s_out[FEAT_BLOCK * D / 4 + 1];
    const int N = st.n_env;
    const size_t NN = size_t(N);
    const int64_t total = int64_t(N) * rows;
    const int64_t b0 = int64_t(blockIdx.x) * FEAT_BLOCK;
    const int64_t b1 = min(total, b0 + FEAT_BLOCK);   // items [b0, b1)
    const int e0 = int(b0 / rows), ne = int((b1 - 1) / rows) - e0 + 1;
    const int t = threadIdx.x;

    // per env: counts and the ships' features (float32 for create()'s float32
    // ships at tick 0, float64 after, as numpy)
    for (int k = t; k < ne * S; k += FEAT_BLOCK) {
        const int le = k / S, s = k - le * S, i = e0 + le;
        const int4 h = reinterpret_cast<const int4 *>(st.hdr)[i];
        if (s == 0) {
            int np = h.y & 0xff;
            s_cnt[le][0] = np < 1 ? 1 : (np > p.p_pad ? p.p_pad : np);
            s_cnt[le][1] = min(int(uint32_t(h.y) >> 16), p.b_cap);
        }
        const bool t0 = (uint32_t(h.x) & TICK_MASK) == 0;
        const V v = reinterpret_cast<const V *>(st.ships)[size_t(s) * NN + i];
        const T b = reinterpret_cast<const T *>(st.ships_b)[size_t(s) * NN + i];
        float *f = s_ship[le] + 5 * s;
        f[0] = float(v.x);
        f[1] = float(v.y);
        f[2] = float(v.z);
        f[3] = float(v.w);
        f[4] = t0 ? norm_angle_over_pi<float>(float(b)) : float(norm_angle_over_pi<double>(double(b)));
    }
    __syncthreads();

    // per item: its row
    const int64_t idx = b0 + t;
    if (idx < b1) {
        const int i = int(idx / rows), r = int(idx - int64_t(i) * rows), le = i - e0;
        const int np = s_cnt[le][0], nb = s_cnt[le][1];
        float f[D];
        if (r >= np + nb) {
#pragma unroll
            for (int k = 0; k < D; ++k) f[k] = -1.0f;   // to_batch padding
        } else {
            f[0] = r < np ? 0.0f : 1.0f;
#pragma unroll
            for (int k = 0; k < 5 * S; ++k) f[1 + k] = s_ship[le][k];
            const V o = r < np ? reinterpret_cast<const V *>(st.planets)[size_t(r) * NN + i]
                               : reinterpret_cast<const V *>(st.bullets)[size_t(i) * size_t(p.b_cap) + (r - np)];
            f[1 + 5 * S] = float(o.x);
            f[2 + 5 * S] = float(o.y);
            f[3 + 5 * S] = float(o.z);
            f[4 + 5 * S] = float(o.w);
        }
        float *so = reinterpret_cast<float *>(s_out) + t * D;
#pragma unroll
        for (int k = 0; k < D; ++k) so[k] = f[k];
    }
    __syncthreads();

    // the block's items out: floats [b0 D, b1 D), 16 bytes per lane and store
    // where the block's base is 16-byte aligned (out is; b0 D floats is a
    // multiple of 4 when D or FEAT_BLOCK is), else word by word
    const int64_t nf = (b1 - b0) * D;
    float *dst = out + b0 * D;
    const float *src = reinterpret_cast<const float *>(s_out);
    if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
        const int64_t n4 = nf / 4;
        // (nontemporal: the tensor is written once and read by the caller
        // later; 27.6-28.0 -> 25.9-26.2 us for [65,536, 36, 15],
        // profiles/round6/ab_features_nt.txt)
        for (int64_t k = t; k < n4; k += FEAT_BLOCK) st_out(reinterpret_cast<float4 *>(dst) + k, s_out[k]);
        for (int64_t k = n4 * 4 + t; k < nf; k += FEAT_BLOCK) dst[k] = src[k];
    } else {
        for (int64_t k = t; k < nf; k += FEAT_BLOCK) dst[k] = src[k];
    }
}

template <typename T, int S, int PMAX>
__global__ __launch_bounds__(BLOCK) void astro_reset_kernel(AstroParams p, AstroState st,
                                                            const uint32_t *__restrict__ seeds,
                                                            const uint8_t *__restrict__ mask) {
    const int i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= st.n_env) return;
    if (mask && !mask[i]) return;
    const int4 h = reinterpret_cast<const int4 *>(st.hdr)[i];
    if (!seeds) {
        const uint32_t seed = uint32_t(h.z) & SEED_MASK;
        const bool undrawn = (uint32_t(h.z) & UNDRAWN) != 0;
        const uint32_t key = (uint32_t(h.z) & KEY_VALID) ? uint32_t(h.w) : undrawn ? 0u : key397_of(p, seed);
        const uint4 c = reinterpret_cast<const uint4 *>(st.stream)[i];
        restart_env<T, S, PMAX>(p, st, i, next_game<S>(p, seed, key, true, undrawn, c, stream_ring_of(st, i)), 0,
                                GlobalSink<T>{st});
        return;
    }
    // explicit seed: full chain now; the stream's pending game stays queued
    int cf = 0;
    const uint32_t seed = seeds[i];
    const int n = create_env<T, S, PMAX>(p, GlobalSink<T>{st}, i,
                                         create_draws<S>(create_words<S>(p, seed, key397_of(p, seed))), cf);
    reinterpret_cast<int4 *>(st.hdr)[i] =
        make_int4(int(uint32_t(h.x) & ~TICK_MASK), n | ((cf ? 2 : 0) << 8), h.z, h.w);
    if (st.stream) reinterpret_cast<uint32_t *>(st.stream)[4 * i + 3] = seed;
}

__global__ __launch_bounds__(BLOCK) void astro_stream_init_kernel(AstroState st,
                                                                  const uint32_t *__restrict__ seeds) {
    const int i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= st.n_env) return;
    const uint32_t s0 = seeds[i];
    MTStream g{s0, mt_key_at(s0, 0, MT_PROLOGUE), 0u, stream_ring_of(st, i)};
    const uint32_t first = g.next() & SEED_MASK;   // game 0's seed, pending
    reinterpret_cast<uint4 *>(st.stream)[i] = make_uint4(g.a, g.b, g.k, 0u);
    reinterpret_cast<int4 *>(st.hdr)[i] = make_int4(0, 1, int(first), 0);
}

// key[397] for seeds first .. first+count-1; four independent chains per
// lane so the ~50-cycle step latency overlaps
__global__ __launch_bounds__(256) void astro_keytable_kernel(uint32_t *__restrict__ table, uint32_t first,
                                                             uint32_t count) {
    const uint32_t lanes = gridDim.x * 256u;
    const uint32_t t = blockIdx.x * 256u + threadIdx.x;
    for (uint32_t base = t; base < count; base += 4u * lanes) {
        uint32_t v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = first + base + uint32_t(u) * lanes;
        for (uint32_t k = 1; k <= MT_PROLOGUE; ++k) {
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = mt_key_next(v[u], k);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t idx = base + uint32_t(u) * lanes;
            if (idx < count) table[first + idx] = v[u];
        }
    }
}

// ---------------------------------------------------------------------------
// host side

thread_local char g_err[512] = "";

int fail(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

bool aligned16(const void *ptr) { return (reinterpret_cast<uintptr_t>(ptr) & 15u) == 0; }

int check_state(const AstroState *s) {
    if (!s) return fail(-2, "state is NULL");
    if (s->n_env < 0) return fail(-3, "n_env < 0");
    if (s->n_env == 0) return 0;
    if (!s->ships || !s->ships_b || !s->planets || !s->bullets || !s->hdr)
        return fail(-4, "a state array is NULL");
    if (!aligned16(s->ships) || !aligned16(s->planets) || !aligned16(s->bullets))
        return fail(-5, "ships/planets/bullets must be 16-byte aligned");
    if ((reinterpret_cast<uintptr_t>(s->hdr) & 15u) != 0) return fail(-5, "hdr must be 16-byte aligned");
    if (s->state_f64 != 0 && s->state_f64 != 1) return fail(-6, "state_f64 must be 0 or 1");
    if (s->stream && !aligned16(s->stream)) return fail(-5, "stream must be 16-byte aligned");
    if (s->stream && (!s->stream_ring || (reinterpret_cast<uintptr_t>(s->stream_ring) & 3u)))
        return fail(-7, "the stream array needs its stream_ring ([n_env][624] uint32, 4-byte aligned)");
    if (reinterpret_cast<uintptr_t>(s->errors) & 3u) return fail(-8, "errors must be 4-byte aligned");
    return 0;
}

int check_params(const AstroParams *p) {
    if (!p) return fail(-10, "params is NULL");
    if (p->nships != 1 && p->nships != 2) return fail(-11, "nships must be 1 or 2");
    if (p->nships != (p->solo ? 1 : 2)) return fail(-12, "nships must be 1 iff solo");
    if (p->p_pad < 1 || p->p_pad > 16) return fail(-13, "p_pad must be in [1, 16]");
    if (p->max_planets < 1 || p->max_planets > p->p_pad)
        return fail(-14, "max_planets must be in [1, p_pad]");
    if (p->b_cap < 1 || p->b_cap > 65535) return fail(-15, "b_cap must be in [1, 65535]");
    if (p->timeout_tick < 0 || p->timeout_tick >= int(TICK_MASK)) return fail(-16, "timeout_tick out of [0, 2^22)");
    if (p->timeout_tick > 0 && !p->fire_bits) return fail(-17, "fire_bits is NULL");
    if (p->kernel < 0 || p->kernel > 3) return fail(-18, "kernel must be 0 (auto), 1 (lane), 2 (quad) or 3 (pair)");
    if (p->planets_only < 0 || p->planets_only > p->max_planets)
        return fail(-19, "planets_only must be in [0, max_planets]");
    if (p->planets_only && (p->max_planets & (p->max_planets - 1)))
        return fail(-19, "planets_only needs max_planets a power of two (one MT word decides the count)");
    return 0;
}

int check_policy(const AstroPolicy *q, int nships) {
    if (q->kind < ASTRO_POLICY_CONTROL || q->kind > ASTRO_POLICY_BOTS)
        return fail(-71, "policy kind must be CONTROL, NOTHING, RANDOM or BOTS");
    if (q->kind == ASTRO_POLICY_BOTS) {
        for (int s = 0; s < nships; ++s) {
            const int b = (q->bots >> (4 * s)) & 15;
            if (b != ASTRO_BOT_NOTHING && b != ASTRO_BOT_SCRIPT && b != ASTRO_BOT_RANDOM)
                return fail(-75, "bot of ship %d must be ASTRO_BOT_NOTHING, _SCRIPT or _RANDOM", s);
        }
    }
    return 0;
}

TickDriver driver_of(const AstroPolicy &q, int ticks) {
    TickDriver d{};
    d.policy = q.kind;
    d.ticks = ticks;
    d.seed = q.seed;
    d.tick0 = q.tick0;
    d.env_offset = q.env_offset;
    d.bots = q.bots;
    d.script_r2 = q.script_r2;
    d.script_threshold = q.script_threshold;
    d.ship_thrust = q.ship_thrust;
    d.ship_rspeed = q.ship_rspeed;
    d.bullet_speed = q.bullet_speed;
    d.ship_radius = q.ship_radius;
    return d;
}

int launched(const char *what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(-1000 - int(e), "%s launch failed: %s", what, hipGetErrorString(e));
    return 0;
}

// kernel choice: the quad kernel fills the chip with 4 waves per SIMD where a
// lane per env would leave it at <= 2 (fewer than 2 x 64 x 1024 envs); past
// that the lane-per-env kernel has the occupancy and fewer instructions
// AUTO: measured on MI355X (profiles/round1/kernel_choice.jsonl, bench.py's
// timed region).  PAIR (2 lanes per env) wins from 65,536 envs up to the
// largest size measured (1M: 8.6e9 vs 6.8e9 LANE, 6.6e9 QUAD; c5's 8 planet
// slots: 4.3e9 vs 3.8e9 QUAD, 2.5e9 LANE); below that QUAD's 4 lanes per env
// give the SIMDs more waves to hide latency with (16,384 envs: 8.7 us vs
// 10.2 PAIR); 16 planet slots spill both, LANE.
int pick_kernel(const AstroParams &p, int n_env) {
    if (p.p_pad > 8) return ASTRO_KERNEL_LANE;   // (QUAD/PAIR are built for up to 8 planet slots)
    if (p.kernel == ASTRO_KERNEL_LANE || p.kernel == ASTRO_KERNEL_QUAD || p.kernel == ASTRO_KERNEL_PAIR)
        return p.kernel;
    return n_env <= ASTRO_QUAD_MAX_ENVS ? ASTRO_KERNEL_QUAD : ASTRO_KERNEL_PAIR;
}

// The first block of a grid's last, partial round: blocks the device holds
// at once = blocks per CU at this kernel's occupancy x CUs (cached per
// kernel and device); 0 when the grid runs in one round or in whole rounds
__host__ inline int late_block_of(const void *fn, int block, int grid) {
    static std::mutex mu;
    static std::map<std::pair<const void *, int>, int> cache;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    int cap = 0;
    {
        std::lock_guard<std::mutex> lock(mu);
        const auto key = std::make_pair(fn, dev);
        const auto it = cache.find(key);
        if (it != cache.end()) {
            cap = it->second;
        } else {
            int per_cu = 0, cus = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, block, 0) != hipSuccess) per_cu = 0;
            if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 0;
            cap = per_cu * cus;
            cache[key] = cap;
        }
    }
    return cap > 0 && grid > cap && grid % cap != 0 ? (grid / cap) * cap : 0;
}

template <typename T, int S, int PM>
int launch_step(const AstroParams &p, const AstroState &s, const TickDriver &drv, float *r, uint8_t *d,
                uint64_t *stats, int ar, hipStream_t stream) {
    unsigned long long *st = reinterpret_cast<unsigned long long *>(stats);
#ifdef ASTRO_STAMPS   // (stamp rows go to `stats`; the one-tick launches stamped are the counter-free ones)
    const bool count = false;
#else
    const bool count = st != nullptr;
#endif
    const int kind = pick_kernel(p, s.n_env);
    if constexpr (PM <= 8)
    if (kind == ASTRO_KERNEL_QUAD || kind == ASTRO_KERNEL_PAIR) {   // all ticks in one launch
        const int lpe = kind == ASTRO_KERNEL_QUAD ? 4 : 2;
        const int grid = int((int64_t(s.n_env) * lpe + QBLOCK - 1) / QBLOCK);
        const bool one = drv.ticks == 1;
        if (drv.policy == ASTRO_POLICY_BOTS) {   // ScriptBot code lives in its own (pair) instance only
            const int g2 = int((int64_t(s.n_env) * 2 + QBLOCK - 1) / QBLOCK);
            hipLaunchKernelGGL((astro_step_quad_kernel<T, S, PM, true, 2, true>), dim3(g2), dim3(QBLOCK), 0, stream,
                               p, s, drv, r, d, st, ar);
            return launched("astro_step(pair, bots)");
        }
        // a one-tick launch of at most ASTRO_HELP_MAX_WAVES waves (two per
        // SIMD: c2, c3) gets helper waves for its resets (HelpBox)
        if (one && ar && int64_t(s.n_env) * lpe <= int64_t(64) * ASTRO_HELP_MAX_WAVES) {
            if (lpe == 4) {   // (small N: two step waves per workgroup spread the few waves over more CUs)
                const dim3 g(int((int64_t(s.n_env) * 4 + 64 * QW_SMALL - 1) / (64 * QW_SMALL))), b(2 * 64 * QW_SMALL);
                if (count)
                    hipLaunchKernelGGL((astro_step_quad_kernel<T, S, PM, false, 4, false, true, QW_SMALL, true>), g, b,
                                       0, stream, p, s, drv, r, d, st, ar);
                else
                    hipLaunchKernelGGL((astro_step_quad_kernel<T, S, PM, false, 4, false, true, QW_SMALL, false>), g,
                                       b, 0, stream, p, s, drv, r, d, st, ar);
            } else {   // (8 planet slots: four, a 16-wave workgroup would cap the 8-slot code at 128 VGPRs)
                constexpr int W = PM > 4 ? 4 : QW_PAIR_HELP;
                const dim3 g(int((int64_t(s.n_env) * 2 + 64 * W - 1) / (64 * W))), b(2 * 64 * W);
                if (count)
                    hipLaunchKernelGGL((astro_step_quad_kernel<T, S, PM, false, 2, false, true, W, true>), g, b, 0,
                                       stream, p, s, drv, r, d, st, ar);
                else
                    hipLaunchKernelGGL((astro_step_quad_kernel<T, S, PM, false, 2, false, true, W, false>), g, b, 0,
                                       stream, p, s, drv, r, d, st, ar);
            }
            return launched(lpe == 4 ? "astro_step(quad, helpers)" : "astro_step(pair, helpers)");
        }
#ifndef ASTRO_NO_RESIDENT   // (A/B builds only: every K-tick rollout on quad_tick's instance)
        if constexpr (std::is_same<T, float>::value) {
            // K ticks with the state on chip, while the grid is at most two
            // waves per SIMD (c3: 7.3 -> 7.0 us per tick; at 1M envs the
            // quad_tick instance's three waves per SIMD win: 93 vs 99 us,
            // profiles/round5/ab_lazy_bullets_1m.jsonl)
            if (!one && p.b_cap <= RES_BCAP && int64_t(s.n_env) * lpe <= int64_t(64) * ASTRO_HELP_MAX_WAVES) {
                const int gr = int((int64_t(s.n_env) * lpe + 64 * RES_WPG - 1) / (64 * RES_WPG));
                if (lpe == 4)
                    hipLaunchKernelGGL((astro_rollout_res_kernel<T, S, PM, 4>), dim3(gr), dim3(64 * RES_WPG), 0,
                                       stream, p, s, drv, r, d, st, ar);
                else
                    hipLaunchKernelGGL((astro_rollout_res_kernel<T, S, PM, 2>), dim3(gr), dim3(64 * RES_WPG), 0,
                                       stream, p, s, drv, r, d, st, ar);
                return launched(lpe == 4 ? "astro_rollout(quad, resident)" : "astro_rollout(pair, resident)");
            }
        }
#endif
        if (lpe == 4 && one) {
            if (count)
                hipLaunchKernelGGL((astro_step_quad_kernel<T, S, PM, false, 4, false, false, QW, true>), dim3(grid),
                                   dim3(QBLOCK), 0, stream, p, s, drv, r, d, st, ar);
            else
                hipLaunchKernelGGL((astro_step_quad_kernel<T, S, PM, false, 4, false, false, QW, false>), dim3(grid),
                                   dim3(QBLOCK), 0, stream, p, s, drv, r, d, st, ar);
        }
        else if (lpe == 4)
            hipLaunchKernelGGL((astro_step_quad_kernel<T, S, PM, true, 4>), dim3(grid), dim3(QBLOCK), 0, stream, p,
                               s, drv, r, d, st, ar);
        else if (one) {
            constexpr int W = PM > 4 ? QW : QW_PAIR;
            const dim3 g(int((int64_t(s.n_env) * 2 + 64 * W - 1) / (64 * W))), b(64 * W);
            TickDriver dl = drv;
            if (count) {
                dl.late_block = late_block_of(
                    reinterpret_cast<const void *>(&astro_step_quad_kernel<T, S, PM, false, 2, false, false, W, true>),
                    int(b.x), int(g.x));
                hipLaunchKernelGGL((astro_step_quad_kernel<T, S, PM, false, 2, false, false, W, true>), g, b, 0, stream,
                                   p, s, dl, r, d, st, ar);
            } else {
                dl.late_block = late_block_of(
                    reinterpret_cast<const void *>(&astro_step_quad_kernel<T, S, PM, false, 2, false, false, W, false>),
                    int(b.x), int(g.x));
                hipLaunchKernelGGL((astro_step_quad_kernel<T, S, PM, false, 2, false, false, W, false>), g, b, 0,
                                   stream, p, s, dl, r, d, st, ar);
            }
        }
        else
            hipLaunchKernelGGL((astro_step_quad_kernel<T, S, PM, true, 2>), dim3(grid), dim3(QBLOCK), 0, stream, p,
                               s, drv, r, d, st, ar);
        return launched(lpe == 4 ? "astro_step(quad)" : "astro_step(pair)");
    }
    const int grid = (s.n_env + BLOCK - 1) / BLOCK;
    const size_t N = size_t(s.n_env);
    for (int k = 0; k < drv.ticks; ++k) {   // the lane kernel: one launch per tick
        TickDriver one = drv;
        one.ticks = 1;
        one.tick0 = drv.tick0 + k;
        if (drv.control) one.control = drv.control + size_t(k) * N * size_t(S);
        hipLaunchKernelGGL((astro_step_kernel<T, S, PM>), dim3(grid), dim3(BLOCK), 0, stream, p, s, one,
                           r + size_t(k) * N * size_t(S), d + size_t(k) * N, st, ar);
        if (int rc = launched("astro_step")) return rc;
    }
    return 0;
}

template <typename T, int S, int PM>
int launch_reset(const AstroParams &p, const AstroState &s, const uint32_t *seeds, const uint8_t *mask,
                 hipStream_t stream) {
    const int grid = (s.n_env + BLOCK - 1) / BLOCK;
    hipLaunchKernelGGL((astro_reset_kernel<T, S, PM>), dim3(grid), dim3(BLOCK), 0, stream, p, s, seeds, mask);
    return launched("astro_reset");
}

// core.Bots.control for every env (astro_controls): one lane per env reads the
// state and runs each ship's bot, as the step kernels do at a tick's start
template <typename T, int S, int PMAX>
__global__ __launch_bounds__(BLOCK) void astro_controls_kernel(AstroParams p, AstroState st, TickDriver drv,
                                                               int8_t *__restrict__ out) {
    using V = typename Store<T>::V;
    const int i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= st.n_env) return;
    const size_t NN = size_t(st.n_env);
    const int4 h = reinterpret_cast<const int4 *>(st.hdr)[i];
    const int tick = int(uint32_t(h.x) & TICK_MASK);
    int np = h.y & 0xff;
    np = np < 1 ? 1 : (np > PMAX ? PMAX : np);
    double sx[S], sy[S], sdx[S], sdy[S], sb[S], px[PMAX], py[PMAX], pdx[PMAX], pdy[PMAX];
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const V v = reinterpret_cast<const V *>(st.ships)[size_t(s) * NN + i];
        sx[s] = double(v.x);
        sy[s] = double(v.y);
        sdx[s] = double(v.z);
        sdy[s] = double(v.w);
        sb[s] = double(reinterpret_cast<const T *>(st.ships_b)[size_t(s) * NN + i]);
    }
#pragma unroll
    for (int j = 0; j < PMAX; ++j) {
        const V v = reinterpret_cast<const V *>(st.planets)[size_t(j < p.p_pad ? j : 0) * NN + i];
        px[j] = double(v.x);
        py[j] = double(v.y);
        pdx[j] = double(v.z);
        pdy[j] = double(v.w);
    }
#pragma unroll
    for (int s = 0; s < S; ++s) {
        int c = tick_control<S>(drv, i, s, NN, 0);
        const int o = S - 1 - s;
        if (ship_bot(drv, s) == ASTRO_BOT_SCRIPT)
            c = script_control<S, PMAX>(drv, p.solo != 0, tick == 0, np, px, py, pdx, pdy, sx[s], sy[s], sdx[s],
                                        sdy[s], sb[s], sx[o], sy[o], sdx[o], sdy[o]);
        out[size_t(i) * S + s] = int8_t(c);
    }
}

// dispatch over (storage type, ships, planet register capacity)
template <template <typename, int, int> class L, typename... A>
int dispatch(const AstroParams &p, const AstroState &s, A... a) {
    const int pm = p.p_pad <= 4 ? 4 : (p.p_pad <= 8 ? 8 : 16);
#define ASTRO_CASE(T, S, PM) \
    if (std::is_same<T, double>::value == bool(s.state_f64) && p.nships == S && pm == PM) \
        return L<T, S, PM>::run(p, s, a...);
#ifdef ASTRO_ONLY_F32_S2   // A/B builds of the bench workloads only (tools/ab.py): a quarter of the compile time
    ASTRO_CASE(float, 2, 4) ASTRO_CASE(float, 2, 8)
#else
    ASTRO_CASE(float, 1, 4) ASTRO_CASE(float, 1, 8) ASTRO_CASE(float, 1, 16)
    ASTRO_CASE(float, 2, 4) ASTRO_CASE(float, 2, 8) ASTRO_CASE(float, 2, 16)
    ASTRO_CASE(double, 1, 4) ASTRO_CASE(double, 1, 8) ASTRO_CASE(double, 1, 16)
    ASTRO_CASE(double, 2, 4) ASTRO_CASE(double, 2, 8) ASTRO_CASE(double, 2, 16)
#endif
#undef ASTRO_CASE
    return fail(-20, "no kernel instance for this configuration");
}

template <typename T, int S, int PM>
struct FeatL {   // (no PMAX dependence: one instance per T, S)
    static int run(const AstroParams &p, const AstroState &s, float *out, int rows, hipStream_t st) {
        const int64_t lanes = int64_t(s.n_env) * rows;
        hipLaunchKernelGGL((astro_features_kernel<T, S>), dim3(unsigned((lanes + FEAT_BLOCK - 1) / FEAT_BLOCK)),
                           dim3(FEAT_BLOCK), 0, st, p, s,
                           out, rows);
        return launched("astro_features");
    }
};
template <typename T, int S, int PM>
struct StepL {
    static int run(const AstroParams &p, const AstroState &s, const TickDriver &drv, float *r, uint8_t *d,
                   uint64_t *stats, int ar, hipStream_t st) {
        return launch_step<T, S, PM>(p, s, drv, r, d, stats, ar, st);
    }
};
template <typename T, int S, int PM>
struct CtlL {
    static int run(const AstroParams &p, const AstroState &s, const TickDriver &drv, int8_t *out, hipStream_t st) {
        hipLaunchKernelGGL((astro_controls_kernel<T, S, PM>), dim3((s.n_env + BLOCK - 1) / BLOCK), dim3(BLOCK), 0,
                           st, p, s, drv, out);
        return launched("astro_controls");
    }
};
template <typename T, int S, int PM>
struct ResetL {
    static int run(const AstroParams &p, const AstroState &s, const uint32_t *seeds, const uint8_t *mask,
                   hipStream_t st) {
        return launch_reset<T, S, PM>(p, s, seeds, mask, st);
    }
};

}  // namespace

extern "C" {

int astro_abi_version(void) { return ASTRO_ABI_VERSION; }

const char *astro_last_error(void) { return g_err; }

static int step_checked(const AstroParams *p, const AstroState *s, const int8_t *control, float *reward,
                        uint8_t *done, uint64_t *stats, int32_t auto_reset, void *stream, uint32_t *flag,
                        uint32_t flag_seq) {
    int rc = check_params(p);
    if (rc) return rc;
    if ((rc = check_state(s))) return rc;
    if (s->n_env == 0) return 0;
    if (!control || !reward || !done) return fail(-30, "control/reward/done is NULL");
    if (auto_reset && !s->stream) return fail(-31, "auto_reset needs the stream array");
    if (p->nships == 2 && ((reinterpret_cast<uintptr_t>(control) & 1u) || (reinterpret_cast<uintptr_t>(reward) & 7u)))
        return fail(-32, "control must be 2-byte and reward 8-byte aligned");
    if (int64_t(s->n_env) * 4 > int64_t(0x7fffffff)) return fail(-34, "n_env too large");
    if (stats && (reinterpret_cast<uintptr_t>(stats) & 7u)) return fail(-33, "stats must be 8-byte aligned");
    TickDriver drv{};
    drv.control = control;
    drv.policy = ASTRO_POLICY_CONTROL;
    drv.ticks = 1;
    drv.flag = flag;
    drv.flag_seq = flag_seq;
    return dispatch<StepL>(*p, *s, drv, reward, done, stats, int(auto_reset), reinterpret_cast<hipStream_t>(stream));
}

int astro_step(const AstroParams *p, const AstroState *s, const int8_t *control, float *reward,
               uint8_t *done, uint64_t *stats, int32_t auto_reset, void *stream) {
    return step_checked(p, s, control, reward, done, stats, auto_reset, stream, nullptr, 0);
}

int astro_step_many(const AstroParams *p, const AstroState *s, const int8_t *control, int32_t k, float *reward,
                    uint8_t *done, uint64_t *stats, int32_t auto_reset, void *stream) {
    if (k < 0) return fail(-35, "k must be >= 0");
    if (k == 0) return 0;
    int rc = astro_step(p, s, control, reward, done, stats, auto_reset, stream);   // checks the arguments
    if (rc || s->n_env == 0) return rc;
    const size_t per = size_t(s->n_env) * size_t(p->nships);
    TickDriver drv{};
    drv.policy = ASTRO_POLICY_CONTROL;
    drv.ticks = 1;
    for (int32_t t = 1; t < k; ++t) {
        drv.control = control + size_t(t) * per;
        rc = dispatch<StepL>(*p, *s, drv, reward + size_t(t) * per, done + size_t(t) * size_t(s->n_env), stats,
                             int(auto_reset), reinterpret_cast<hipStream_t>(stream));
        if (rc) return rc;
    }
    return 0;
}

int astro_rollout(const AstroParams *p, const AstroState *s, const AstroPolicy *policy, int32_t ticks,
                  const int8_t *control, float *reward, uint8_t *done, uint64_t *stats, int32_t auto_reset,
                  void *stream) {
    int rc = check_params(p);
    if (rc) return rc;
    if ((rc = check_state(s))) return rc;
    if (!policy) return fail(-70, "policy is NULL");
    if ((rc = check_policy(policy, p->nships))) return rc;
    if (ticks < 1) return fail(-72, "ticks must be >= 1");
    if (s->n_env == 0) return 0;
    if (policy->kind == ASTRO_POLICY_CONTROL && !control) return fail(-73, "policy CONTROL needs control");
    if (!reward || !done) return fail(-30, "control/reward/done is NULL");
    if (auto_reset && !s->stream) return fail(-31, "auto_reset needs the stream array");
    if (p->nships == 2 && ((reinterpret_cast<uintptr_t>(control) & 1u) || (reinterpret_cast<uintptr_t>(reward) & 7u)))
        return fail(-32, "control must be 2-byte and reward 8-byte aligned");
    if (int64_t(s->n_env) * 4 > int64_t(0x7fffffff)) return fail(-34, "n_env too large");
    if (stats && (reinterpret_cast<uintptr_t>(stats) & 7u)) return fail(-33, "stats must be 8-byte aligned");
    TickDriver drv = driver_of(*policy, ticks);
    drv.control = control;
    return dispatch<StepL>(*p, *s, drv, reward, done, stats, int(auto_reset), reinterpret_cast<hipStream_t>(stream));
}

int astro_controls(const AstroParams *p, const AstroState *s, const AstroPolicy *policy, int8_t *control,
                   void *stream) {
    int rc = check_params(p);
    if (rc) return rc;
    if ((rc = check_state(s))) return rc;
    if (!policy) return fail(-70, "policy is NULL");
    if ((rc = check_policy(policy, p->nships))) return rc;
    if (policy->kind == ASTRO_POLICY_CONTROL) return fail(-71, "astro_controls: CONTROL is not a policy");
    if (s->n_env == 0) return 0;
    if (!control) return fail(-74, "control is NULL");
    return dispatch<CtlL>(*p, *s, driver_of(*policy, 1), control, reinterpret_cast<hipStream_t>(stream));
}

int astro_reset(const AstroParams *p, const AstroState *s, const uint32_t *seeds, const uint8_t *mask,
                void *stream) {
    int rc = check_params(p);
    if (rc) return rc;
    if ((rc = check_state(s))) return rc;
    if (s->n_env == 0) return 0;
    if (!seeds && !s->stream) return fail(-40, "reset without seeds needs the stream array");
    return dispatch<ResetL>(*p, *s, seeds, mask, reinterpret_cast<hipStream_t>(stream));
}

int astro_keytable_build(uint32_t *table, uint32_t first, uint32_t count, void *stream) {
    if (!table) return fail(-50, "table is NULL");
    if (uint64_t(first) + count > (uint64_t(1) << 30)) return fail(-51, "key table covers seeds < 2^30");
    if (count == 0) return 0;
    const uint32_t lanes_needed = (count + 3) / 4;
    const uint32_t grid = (lanes_needed + 255) / 256 < 65536u ? (lanes_needed + 255) / 256 : 65536u;
    hipLaunchKernelGGL(astro_keytable_kernel, dim3(grid), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                       table, first, count);
    return launched("astro_keytable_build");
}

int astro_stream_init(const AstroState *s, const uint32_t *stream_seeds, void *stream) {
    if (!s) return fail(-2, "state is NULL");
    if (s->n_env < 0) return fail(-3, "n_env < 0");
    if (s->n_env == 0) return 0;
    if (!s->stream || !stream_seeds) return fail(-41, "stream / stream_seeds is NULL");
    if (reinterpret_cast<uintptr_t>(s->stream) & 15u) return fail(-5, "stream must be 16-byte aligned");
    if (!s->stream_ring || (reinterpret_cast<uintptr_t>(s->stream_ring) & 3u))
        return fail(-7, "the stream array needs its stream_ring ([n_env][624] uint32, 4-byte aligned)");
    if (!s->hdr || (reinterpret_cast<uintptr_t>(s->hdr) & 15u)) return fail(-5, "hdr must be 16-byte aligned");
    const int grid = (s->n_env + BLOCK - 1) / BLOCK;
    hipLaunchKernelGGL(astro_stream_init_kernel, dim3(grid), dim3(BLOCK), 0,
                       reinterpret_cast<hipStream_t>(stream), *s, stream_seeds);
    return launched("astro_stream_init");
}

int astro_host_alloc(uint64_t bytes, void **host, void **device) {
    if (!host || !device) return fail(-80, "host/device is NULL");
    *host = *device = nullptr;
    if (bytes == 0) return fail(-81, "bytes must be > 0");
    void *h = nullptr;
    hipError_t e = hipHostMalloc(&h, size_t(bytes), hipHostMallocMapped | hipHostMallocCoherent);
    if (e != hipSuccess) return fail(-1000 - int(e), "hipHostMalloc(%llu) failed: %s", (unsigned long long)bytes,
                                     hipGetErrorString(e));
    void *d = nullptr;
    e = hipHostGetDevicePointer(&d, h, 0);
    if (e != hipSuccess) {
        (void)hipHostFree(h);
        return fail(-1000 - int(e), "hipHostGetDevicePointer failed: %s", hipGetErrorString(e));
    }
    *host = h;
    *device = d;
    return 0;
}

int astro_host_free(void *host) {
    if (!host) return 0;
    // (a single game's last launch may still be finishing after its
    // completion word: nothing is freed under a running kernel)
    (void)hipDeviceSynchronize();
    const hipError_t e = hipHostFree(host);
    return e == hipSuccess ? 0 : fail(-1000 - int(e), "hipHostFree failed: %s", hipGetErrorString(e));
}

int astro_dev_alloc(uint64_t bytes, int32_t kind, void **device) {
    if (!device) return fail(-82, "device is NULL");
    *device = nullptr;
    if (bytes == 0) return fail(-81, "bytes must be > 0");
    unsigned flags;
    switch (kind) {
    case ASTRO_MEM_DEFAULT: flags = hipDeviceMallocDefault; break;
    case ASTRO_MEM_FINEGRAINED: flags = hipDeviceMallocFinegrained; break;
    case ASTRO_MEM_UNCACHED: flags = hipDeviceMallocUncached; break;
    default: return fail(-83, "kind must be ASTRO_MEM_DEFAULT, _FINEGRAINED or _UNCACHED (got %d)", int(kind));
    }
    void *d = nullptr;
    hipError_t e = hipExtMallocWithFlags(&d, size_t(bytes), flags);
    if (e != hipSuccess) return fail(-1000 - int(e), "hipExtMallocWithFlags(%llu, %u) failed: %s",
                                     (unsigned long long)bytes, flags, hipGetErrorString(e));
    e = hipMemset(d, 0, size_t(bytes));
    if (e != hipSuccess) {
        (void)hipFree(d);
        return fail(-1000 - int(e), "hipMemset failed: %s", hipGetErrorString(e));
    }
    *device = d;
    return 0;
}

int astro_dev_free(void *device) {
    if (!device) return 0;
    const hipError_t e = hipFree(device);
    return e == hipSuccess ? 0 : fail(-1000 - int(e), "hipFree failed: %s", hipGetErrorString(e));
}

int astro_game_step(AstroGameTick *t) {
    if (!t) return fail(-91, "tick record is NULL");
    const int S = t->params.nships, np = t->nplanets, nb = t->nbullets;
    if (S != 1 && S != 2) return fail(-11, "nships must be 1 or 2");
    if (np < 1 || np > t->params.p_pad) return fail(-92, "nplanets must be in [1, p_pad]");
    if (nb < 0 || nb > t->params.b_cap) return fail(-93, "nbullets must be in [0, b_cap]");
    if (t->state.n_env != 1 || t->state.state_f64 != 1) return fail(-94, "the game arena is one float64 env");
    const double *in = t->in;
    // the input state into the arena, in the kernels' layout
    for (int s = 0; s < S; ++s) {
        double *v = t->ships + 4 * s;
        v[0] = in[2 * s];
        v[1] = in[2 * s + 1];
        v[2] = in[2 * S + 2 * s];
        v[3] = in[2 * S + 2 * s + 1];
        t->ships_b[s] = in[4 * S + s];
    }
    const double *pin = in + 5 * S;
    for (int j = 0; j < np; ++j) {
        double *v = t->planets + 4 * j;
        v[0] = pin[2 * j];
        v[1] = pin[2 * j + 1];
        v[2] = pin[2 * np + 2 * j];
        v[3] = pin[2 * np + 2 * j + 1];
    }
    const double *bin = pin + 4 * np;
    for (int k = 0; k < nb; ++k) {
        double *v = t->bullets + 4 * k;
        v[0] = bin[2 * k];
        v[1] = bin[2 * k + 1];
        v[2] = bin[2 * nb + 2 * k];
        v[3] = bin[2 * nb + 2 * k + 1];
    }
    const int tick = t->first_step ? 0 : 1;
    t->hdr[0] = int32_t((uint32_t(t->hdr[0]) & ~TICK_MASK) | uint32_t(tick));
    t->hdr[1] = np | (nb << 16);
    t->control[0] = int8_t(t->control0);
    if (S == 2) t->control[1] = int8_t(t->control1);
    t->fire[0] = uint32_t(t->fire_now ? 1 : 0) << tick;
    AstroParams p = t->params;
    p.timeout_tick = t->timeout_now ? tick : tick + 1;
    p.fire_bits = t->fire_dev;
    hipStream_t stream = reinterpret_cast<hipStream_t>(t->stream);
    // the completion word: only the one-wave quad/pair launch stores it (the
    // lane kernel and a helper instance never do: the stream's completion then)
    const bool use_flag = t->flag && t->flag_dev && pick_kernel(p, 1) != ASTRO_KERNEL_LANE;
    const uint32_t seq = ++t->seq;
    int rc = step_checked(&p, &t->state, t->control_dev, t->reward_dev, t->done_dev, nullptr, 0, stream,
                          use_flag ? t->flag_dev : nullptr, seq);
    if (rc) return rc;
    hipError_t e = hipErrorNotReady;
    if (use_flag) {
        // the word, with a look at the stream every 64 reads (a fault ends
        // the launch without it)
        const volatile uint32_t *fl = t->flag;
        for (uint32_t k = 1; *fl != seq; ++k) {
            if ((k & 63) == 0 && (e = hipStreamQuery(stream)) != hipErrorNotReady) {
                if (e != hipSuccess || *fl == seq) break;
                return fail(-95, "astro_game_step: the launch ended without its completion word");
            }
        }
        __atomic_thread_fence(__ATOMIC_ACQUIRE);
        if (e != hipErrorNotReady && e != hipSuccess)
            return fail(-1000 - int(e), "astro_game_step: %s", hipGetErrorString(e));
    } else {
        while ((e = hipStreamQuery(stream)) == hipErrorNotReady) {
        }
        if (e != hipSuccess) return fail(-1000 - int(e), "astro_game_step: %s", hipGetErrorString(e));
    }
    if (*t->errors) {
        const uint32_t bits = *t->errors;
        *t->errors = 0;
        return fail(-90, "astro_step reported device error 0x%x", bits);
    }
    t->done_out = *t->done;
    t->reward_out[0] = t->reward[0];
    t->reward_out[1] = S == 2 ? t->reward[1] : 0.0f;
    if (t->done_out) return 0;
    // the next state, packed (the planets' count is the input's)
    const int nb2 = int(uint32_t(t->hdr[1]) >> 16);
    t->out_nbullets = nb2;
    double *out = t->out;
    for (int s = 0; s < S; ++s) {
        const double *v = t->ships + 4 * s;
        out[2 * s] = v[0];
        out[2 * s + 1] = v[1];
        out[2 * S + 2 * s] = v[2];
        out[2 * S + 2 * s + 1] = v[3];
        out[4 * S + s] = t->ships_b[s];
    }
    double *pout = out + 5 * S;
    for (int j = 0; j < np; ++j) {
        const double *v = t->planets + 4 * j;
        pout[2 * j] = v[0];
        pout[2 * j + 1] = v[1];
        pout[2 * np + 2 * j] = v[2];
        pout[2 * np + 2 * j + 1] = v[3];
    }
    double *bout = pout + 4 * np;
    for (int k = 0; k < nb2; ++k) {
        const double *v = t->bullets + 4 * k;
        bout[2 * k] = v[0];
        bout[2 * k + 1] = v[1];
        bout[2 * nb2 + 2 * k] = v[2];
        bout[2 * nb2 + 2 * k + 1] = v[3];
    }
    return 0;
}

int astro_features(const AstroParams *p, const AstroState *s, float *out, int32_t rows, void *stream) {
    int rc = check_params(p);
    if (rc) return rc;
    if ((rc = check_state(s))) return rc;
    if (s->n_env == 0) return 0;
    if (!out || (reinterpret_cast<uintptr_t>(out) & 3u)) return fail(-60, "out is NULL or not 4-byte aligned");
    if (rows < 1) return fail(-61, "rows must be >= 1");
    if (int64_t(s->n_env) * rows > (int64_t(1) << 40)) return fail(-62, "n_env * rows too large");
    return dispatch<FeatL>(*p, *s, out, int(rows), reinterpret_cast<hipStream_t>(stream));
}

}  // extern "C"
