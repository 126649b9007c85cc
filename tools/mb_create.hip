// Micro-benchmark of create()'s ingredients, one lane per env (diagnostic).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I include
//        tools/mb_create.hip -o tools/mb_create
#include "../astro_amd/csrc/astro_kernels.hip"

#include <cstdio>
#include <vector>

namespace {

__global__ void k_chain(uint32_t *out, int n, int steps) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= n) return;
    uint32_t v = 12345u + uint32_t(i);
    for (int k = 1; k <= steps; ++k) v = mt_key_next(v, uint32_t(k));
    out[i] = v;
}

__global__ void k_chain24(uint32_t *out, int n, int steps) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= n) return;
    uint32_t v = 12345u + uint32_t(i);
    for (int k = 1; k <= steps; ++k) {
        const uint32_t x = v ^ (v >> 30);
        // 1812433253 = 0x6C078965 = 0x6C07 << 16 | 0x8965 ; 24-bit multiplies
        const uint32_t lo = __umul24(x & 0xffff, 0x8965u);
        const uint32_t mid = __umul24(x >> 16, 0x8965u) + __umul24(x & 0xffff, 0x6C07u);
        v = lo + (mid << 16) + uint32_t(k);
    }
    out[i] = v;
}

__global__ void k_draws(uint32_t *out, int n, int draws) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= n) return;
    MTLazy g;
    g.seed_from(7u + uint32_t(i), 99u * uint32_t(i));
    uint32_t acc = 0;
    for (int k = 0; k < draws; ++k) acc ^= g.next();
    out[i] = acc;
}

__global__ void k_sincos(float *out, int n, int reps) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= n) return;
    float x = 0.001f * float(i), acc = 0.0f;
    for (int k = 0; k < reps; ++k) {
        float s, c;
        np_sincosf(x, s, c);
        x = s + c;   // dependent chain
        acc += s;
    }
    out[i] = acc;
}

template <typename T, int S, int PMAX>
__global__ void k_create(AstroParams p, AstroState st, int reps) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= st.n_env) return;
    uint32_t seed = 1000u + uint32_t(i);
    for (int k = 0; k < reps; ++k) {
        int cf;
        const int n = create_env<T, S, PMAX>(p, st, i, seed, seed * 2654435761u, cf);
        seed += uint32_t(n);
    }
}

float time_ms(hipEvent_t a, hipEvent_t b) {
    float ms;
    hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b);
    return ms;
}

}  // namespace

int main() {
    const int n = 65536;
    uint32_t *u;
    float *f;
    hipMalloc(&u, n * 4);
    hipMalloc(&f, n * 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int grid = n / 64;
    auto run = [&](const char *name, auto launch) {
        launch();
        hipDeviceSynchronize();
        hipEventRecord(a);
        launch();
        hipEventRecord(b);
        printf("%-28s %9.2f us\n", name, time_ms(a, b) * 1e3);
    };
    run("chain 397 (mul_lo)", [&] { hipLaunchKernelGGL(k_chain, grid, 64, 0, 0, u, n, 397); });
    run("chain 3970 (mul_lo)", [&] { hipLaunchKernelGGL(k_chain, grid, 64, 0, 0, u, n, 3970); });
    run("chain 397 (mul_u24)", [&] { hipLaunchKernelGGL(k_chain24, grid, 64, 0, 0, u, n, 397); });
    run("chain 3970 (mul_u24)", [&] { hipLaunchKernelGGL(k_chain24, grid, 64, 0, 0, u, n, 3970); });
    run("16 MT draws", [&] { hipLaunchKernelGGL(k_draws, grid, 64, 0, 0, u, n, 16); });
    run("160 MT draws", [&] { hipLaunchKernelGGL(k_draws, grid, 64, 0, 0, u, n, 160); });
    run("9 sincos (chained)", [&] { hipLaunchKernelGGL(k_sincos, grid, 64, 0, 0, f, n, 9); });
    run("90 sincos (chained)", [&] { hipLaunchKernelGGL(k_sincos, grid, 64, 0, 0, f, n, 90); });

    // full create into real state arrays
    float *ships, *sb, *planets, *bullets;
    int *hdr;
    uint32_t *stream;
    hipMalloc(&ships, size_t(n) * 2 * 16);
    hipMalloc(&sb, size_t(n) * 2 * 4);
    hipMalloc(&planets, size_t(n) * 4 * 16);
    hipMalloc(&bullets, size_t(n) * 16);
    hipMalloc(&hdr, size_t(n) * 16);
    hipMalloc(&stream, size_t(n) * 16);
    AstroState st{ships, sb, planets, bullets, hdr, stream, n, 0};
    AstroParams p{};
    p.gm = 0.05; p.dt = 0.02; p.gravity = 0.05; p.planet_mass = 1.0;
    p.outer_pos = 0.9f; p.inner_pos = 0.2f; p.planet_orbit = 0.5f;
    p.nships = 2; p.max_planets = 4; p.p_pad = 4; p.b_cap = 1;
    run("create x1", [&] { hipLaunchKernelGGL((k_create<float, 2, 4>), grid, 64, 0, 0, p, st, 1); });
    run("create x10", [&] { hipLaunchKernelGGL((k_create<float, 2, 4>), grid, 64, 0, 0, p, st, 10); });
    hipDeviceSynchronize();
    return 0;
}
