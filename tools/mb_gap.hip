// The time between back-to-back launches of a c3-shaped kernel (stamps,
// profiles/round4/stamps_c3_b2b.json: the step launch's waves span 7.5 us
// of an 11.0 us period; 2.5-3.6 us pass between one launch's last wave and
// the next one's first).  What sets that gap: c3's grid (256 workgroups of
// 1,024 threads), each wave busy for a while, then storing 1-4 KB (the
// step wave's state write-back at its end) or storing it at its start, with
// or without c3's ~86 KB of LDS per workgroup.  Per-launch period of 100
// launches in one hipGraph, best of 5 replays.
//   hipcc --offload-arch=gfx950 -O3 tools/mb_gap.hip -o tools/mb_gap
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); std::exit(1); } } while (0)

constexpr int BLOCKS = 256, THREADS = 1024, WAVES = BLOCKS * THREADS / 64;

// a 16-byte store with cache-policy bits POL: 0 plain, 1 nt, 2 sc1 (device
// scope), 3 sc0 sc1 (system scope), 4 nt sc1
template <int POL>
__device__ __forceinline__ void st16(float4 *p, float4 v) {
    typedef float v4f __attribute__((ext_vector_type(4)));
    const v4f w = {v.x, v.y, v.z, v.w};
    if constexpr (POL == 0) asm volatile("global_store_dwordx4 %0, %1, off" ::"v"(p), "v"(w) : "memory");
    if constexpr (POL == 1) asm volatile("global_store_dwordx4 %0, %1, off nt" ::"v"(p), "v"(w) : "memory");
    if constexpr (POL == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(w) : "memory");
    if constexpr (POL == 3) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(w) : "memory");
    if constexpr (POL == 4) asm volatile("global_store_dwordx4 %0, %1, off nt sc1" ::"v"(p), "v"(w) : "memory");
}

// mode 0: busy, then store; mode 1: store, then busy; mode 2: busy only
template <int POL>
__global__ __launch_bounds__(THREADS) void k_gap(float4 *buf, int ticks, int nst, int mode, int lds_touch) {
    extern __shared__ float4 lds[];
    const int lane = threadIdx.x & 63;
    const int w = blockIdx.x * (THREADS / 64) + threadIdx.x / 64;
    const float4 v = make_float4(float(w), 1.f, 2.f, 3.f);
    if (lds_touch) lds[threadIdx.x] = v;   // (the allocation is what matters; one store so it is kept)
    if (mode == 1)
        for (int k = 0; k < nst; ++k) st16<POL>(&buf[(size_t(k) * WAVES + w) * 64 + lane], v);
    // busy: a dependent float chain (no memory traffic: polling the clock
    // would put requests beside the stores)
    float a = v.x;
#pragma unroll 1
    for (int k = 0; k < ticks; ++k) a = __builtin_fmaf(a, 1.0000001f, 1e-7f);
    if (a == -1.f) buf[1] = v;
    if (mode == 0)
        for (int k = 0; k < nst; ++k) st16<POL>(&buf[(size_t(k) * WAVES + w) * 64 + lane], v);
    if (lds_touch && lds[(threadIdx.x + 64) % THREADS].x == -1.f) buf[0] = v;
}

template <int POL>
static float period(hipStream_t s, float4 *buf, int ticks, int nst, int mode, int lds_bytes) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int k = 0; k < 100; ++k)
        k_gap<POL><<<BLOCKS, THREADS, lds_bytes, s>>>(buf, ticks, nst, mode, lds_bytes > 0);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        CK(hipEventRecord(a, s));
        CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        best = ms * 10.f < best ? ms * 10.f : best;   // us per launch
    }
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    return best;
}

int main() {
    hipStream_t s;
    CK(hipStreamCreate(&s));
    const int MAXST = 4;   // up to 4 x 1 KB per wave: 16 MB over the 4,096 waves
    float4 *buf;
    CK(hipMalloc(&buf, sizeof(float4) * size_t(MAXST) * WAVES * 64));
    CK(hipMemset(buf, 0, sizeof(float4) * size_t(MAXST) * WAVES * 64));
    CK(hipFuncSetAttribute((const void *)k_gap<0>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024));
    const int spin = 300;   // iterations of the dependent chain (the busy-only line says how long)
    struct C { const char *name; int ticks, nst, mode, lds; } cs[] = {
        {"empty", 0, 0, 2, 0},
        {"busy", spin, 0, 2, 0},
        {"busy_lds86k", spin, 0, 2, 86 * 1024},
        {"busy_store_end_4MB", spin, 1, 0, 0},
        {"busy_store_end_16MB", spin, 4, 0, 0},
        {"busy_store_start_16MB", spin, 4, 1, 0},
        {"busy_store_end_16MB_lds86k", spin, 4, 0, 86 * 1024},
    };
    std::printf("{\"grid\": [%d, %d], \"waves\": %d", BLOCKS, THREADS, WAVES);
    for (auto &c : cs) std::printf(", \"%s_us\": %.3f", c.name, period<0>(s, buf, c.ticks, c.nst, c.mode, c.lds));
    // the 16 MB stored at the end under each cache policy
    std::printf(", \"store_end_16MB_nt_us\": %.3f", period<1>(s, buf, spin, 4, 0, 0));
    std::printf(", \"store_end_16MB_sc1_us\": %.3f", period<2>(s, buf, spin, 4, 0, 0));
    std::printf(", \"store_end_16MB_sc0sc1_us\": %.3f", period<3>(s, buf, spin, 4, 0, 0));
    std::printf(", \"store_end_16MB_nt_sc1_us\": %.3f", period<4>(s, buf, spin, 4, 0, 0));
    std::printf(", \"store_start_16MB_sc1_us\": %.3f", period<2>(s, buf, spin, 4, 1, 0));
    std::printf("}\n");
    CK(hipFree(buf));
    return 0;
}
