// Latency of one create() (core.py:86-135) as the step kernel runs it on a
// reset: one quad (4 lanes) per wave, one wave per SIMD, N creates in a row.
// Diagnostic only.  Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//         -fhip-fp32-correctly-rounded-divide-sqrt -I include tools/mb_create_latency.hip -o tools/mb_create_latency
#include "../astro_amd/csrc/astro_kernels.hip"

#include <cstdio>

namespace {

template <int NPART>
__global__ void k_create(AstroParams p, AstroState st, int reps, unsigned long long *cyc) {
    const int lane = threadIdx.x & 63;
    if (lane >= NPART) return;
    const int i = blockIdx.x;
    uint32_t seed = 1000u + uint32_t(i);
    const uint4 c = make_uint4(7u, 9u, 3u, 0u);
    unsigned long long t0 = __builtin_readcyclecounter();
    for (int k = 0; k < reps; ++k) {
        const NextGame<2> ng = next_game<2>(p, seed, seed * 2654435761u, true, c.x, c.y, c.z);
        restart_env<float, 2, 4, NPART>(p, st, i, seed, ng, lane);
        seed += uint32_t(ng.words.n) + 1u;
    }
    unsigned long long t1 = __builtin_readcyclecounter();
    if (lane == 0) cyc[i] = (t1 - t0) / reps;
}

// one env's auto-reset pass as the quad kernel runs it (1 wave per SIMD)
__global__ void k_pass(AstroParams p, AstroState st, int reps, unsigned long long *cyc) {
    __shared__ uint32_t s_chain[4][2][13 + 2 * 2];
    __shared__ int s_serial[16];
    const int lane = threadIdx.x & 63;
    const int i = blockIdx.x;
    const uint32_t seed0 = 1000u + uint32_t(i);
    unsigned long long t0 = __builtin_readcyclecounter();
    for (int k = 0; k < reps; ++k) {
        const uint32_t seed = seed0 + 7919u * uint32_t(k);
        uint64_t todo = 1;   // lane 0 = the leader of env i's quad
        while (todo)
            todo = wave_reset_pass<float, 2, 4>(p, st, todo, lane, i, seed, seed * 2654435761u, true, s_chain,
                                                s_serial);
    }
    unsigned long long t1 = __builtin_readcyclecounter();
    if (lane == 0) cyc[i] = (t1 - t0) / reps;
}

__global__ void k_cdraws(AstroParams p, double *out, int reps, unsigned long long *cyc) {
    if (threadIdx.x != 0) return;
    uint32_t seed = 1000u + blockIdx.x;
    double acc = 0.0;
    unsigned long long t0 = __builtin_readcyclecounter();
    for (int k = 0; k < reps; ++k) {
        const CreateDraws<2> d = create_draws<2>(create_words<2>(p, seed, seed * 2654435761u));
        acc += d.u_out[0] + d.u_out[1] + d.u_inner + d.u_choice + d.u_bear[0] + d.u_bear[1] + d.u_base + d.reverse;
        seed += uint32_t(d.n) + 1u;
    }
    unsigned long long t1 = __builtin_readcyclecounter();
    out[blockIdx.x] = acc;
    cyc[blockIdx.x] = (t1 - t0) / reps;
}

__global__ void k_draws(uint32_t *out, int reps, unsigned long long *cyc) {
    if (threadIdx.x != 0) return;
    MTLazy g;
    g.seed_from(7u + blockIdx.x, 99u * blockIdx.x);
    uint32_t acc = 0;
    unsigned long long t0 = __builtin_readcyclecounter();
    for (int k = 0; k < reps; ++k) acc ^= g.next();
    unsigned long long t1 = __builtin_readcyclecounter();
    out[blockIdx.x] = acc;
    cyc[blockIdx.x] = (t1 - t0) / reps;
}

__global__ void k_sincos(float *out, int reps, unsigned long long *cyc) {
    if (threadIdx.x != 0) return;
    float x = 0.001f * float(blockIdx.x), acc = 0.0f;
    unsigned long long t0 = __builtin_readcyclecounter();
    for (int k = 0; k < reps; ++k) {
        float s, c;
        np_sincosf(x, s, c);
        x = s + c;
        acc += s;
    }
    unsigned long long t1 = __builtin_readcyclecounter();
    out[blockIdx.x] = acc;
    cyc[blockIdx.x] = (t1 - t0) / reps;
}

double mean(const unsigned long long *h, int n) {
    double s = 0;
    for (int i = 0; i < n; ++i) s += double(h[i]);
    return s / n;
}

}  // namespace

int main() {
    const int waves = 1024;
    unsigned long long *cyc, h[1024];
    hipMalloc(&cyc, waves * 8);
    uint32_t *u;
    hipMalloc(&u, waves * 4);
    float *ships, *sb, *planets, *bullets;
    int *hdr;
    uint32_t *stream;
    hipMalloc(&ships, size_t(waves) * 2 * 16);
    hipMalloc(&sb, size_t(waves) * 2 * 4);
    hipMalloc(&planets, size_t(waves) * 4 * 16);
    hipMalloc(&bullets, size_t(waves) * 16);
    hipMalloc(&hdr, size_t(waves) * 16);
    hipMalloc(&stream, size_t(waves) * 16);
    AstroState st{ships, sb, planets, bullets, hdr, stream, waves, 0};
    AstroParams p{};
    p.gm = 0.05; p.dt = 0.02; p.gravity = 0.05; p.planet_mass = 1.0;
    p.outer_pos = 0.9f; p.inner_pos = 0.2f; p.planet_orbit = 0.5f;
    p.nships = 2; p.max_planets = 4; p.p_pad = 4; p.b_cap = 1;
    auto show = [&](const char *name) {
        hipDeviceSynchronize();
        hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
        printf("%-34s %8.0f cycles\n", name, mean(h, waves));
    };
    hipLaunchKernelGGL(k_draws, waves, 64, 0, 0, u, 64, cyc);
    show("one MT word (dependent)");
    hipLaunchKernelGGL(k_sincos, waves, 64, 0, 0, (float *)u, 64, cyc);
    show("one np_sincosf (dependent)");
    hipLaunchKernelGGL(k_pass, waves, 64, 0, 0, p, st, 16, cyc);
    show("wave reset pass, 1 env");
    hipLaunchKernelGGL(k_cdraws, waves, 64, 0, 0, p, (double *)ships, 16, cyc);
    show("create's words+draws, vector");
    hipLaunchKernelGGL(k_create<1>, waves, 64, 0, 0, p, st, 16, cyc);
    show("next game + create, 1 lane");
    hipLaunchKernelGGL(k_create<4>, waves, 64, 0, 0, p, st, 16, cyc);
    show("next game + create, quad");
    return 0;
}
