// Kernel-end write-back microbenchmark: does the data a launch leaves dirty
// in L2 cost time after its last wave ends?  2,048 one-wave... four-wave
// workgroups (the pair kernel's c3 grid) each spin ~5 us of VALU, then
// write (or read) W bytes spread over the grid -- at the end of the wave
// ("late") or before the spin ("early") -- with plain or nontemporal
// stores.  Per-launch time, back to back in a hipGraph of 100 launches.
//   hipcc --offload-arch=gfx950 -O3 tools/mb_flush.hip -o tools/mb_flush
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); std::exit(1); } } while (0)

__device__ __forceinline__ double spin(int iters) {
    double a = threadIdx.x, b = 1.0000001, c = 0.5, d = 0.25;
    for (int k = 0; k < iters; ++k) {
        a = __builtin_fma(a, b, 1e-9);
        c = __builtin_fma(c, b, 1e-9);
        d = __builtin_fma(d, b, 1e-9);
        b = __builtin_fma(b, 1.0, 1e-12);
    }
    return a + c + d;
}

// mode: 0 = no memory, 1 = late plain stores, 2 = late nontemporal stores,
// 3 = early plain stores, 4 = late loads, 5..8 = late stores with cache
// policy sc0 sc1 / sc1 / sc0 / sc0 sc1 nt (write-through variants), 9 / 10 =
// early plain stores + buffer_wbl2 by every wave / the first wave of each block
__global__ __launch_bounds__(256) void k_flush(float4 *buf, int n4, int per_lane, int iters, int mode, double *sink) {
    const int lanes = gridDim.x * blockDim.x;
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    float4 v = make_float4(float(g), 1.0f, 2.0f, 3.0f);
    if (mode == 3 || mode == 9 || mode == 10)
        for (int k = 0; k < per_lane; ++k) {
            const int j = g + k * lanes;
            if (j < n4) buf[j] = v;
        }
    // 9: every wave writes its L2's dirty lines back right after its stores;
    // 10: the first wave of each workgroup only
    if (mode == 9 || (mode == 10 && threadIdx.x < 64)) asm volatile("buffer_wbl2 sc1" ::: "memory");
    const double s = spin(iters);
    v.y = float(s);
    float acc = 0.0f;
    for (int k = 0; k < per_lane; ++k) {
        const int j = g + k * lanes;
        if (j >= n4) break;
        if (mode == 1) buf[j] = v;
        if (mode == 2) {
            typedef float f4v __attribute__((ext_vector_type(4)));
            const f4v e = {v.x, v.y, v.z, v.w};
            __builtin_nontemporal_store(e, reinterpret_cast<f4v *>(&buf[j]));
        }
        if (mode == 4) acc += buf[j].x;
        if (mode >= 5 && mode <= 8) {
            typedef float f4v __attribute__((ext_vector_type(4)));
            const f4v e = {v.x, v.y, v.z, v.w};
            float4 *ptr = &buf[j];
            if (mode == 5) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(ptr), "v"(e) : "memory");
            if (mode == 6) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(ptr), "v"(e) : "memory");
            if (mode == 7) asm volatile("global_store_dwordx4 %0, %1, off sc0" ::"v"(ptr), "v"(e) : "memory");
            if (mode == 8) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" ::"v"(ptr), "v"(e) : "memory");
        }
    }
    if (acc == 12345.0f || s == 12345.0) sink[blockIdx.x] = s + acc;
}

template <typename F>
static float time_graph(hipStream_t s, F launch, int per_graph, int reps) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int k = 0; k < per_graph; ++k) launch();
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));   // warm
    CK(hipStreamSynchronize(s));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a, s));
    for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    return ms * 1e3f / float(per_graph * reps);   // us per launch
}

int main() {
    hipStream_t s;
    CK(hipStreamCreate(&s));
    const size_t max_bytes = 48u << 20;
    float4 *buf;
    double *sink;
    CK(hipMalloc(&buf, max_bytes));
    CK(hipMalloc(&sink, 1 << 20));
    CK(hipMemset(buf, 0, max_bytes));
    const int blocks = 512, threads = 256;
    const char *names[] = {"none", "late_store", "late_nt_store", "early_store", "late_load",
                           "late_sc0sc1", "late_sc1", "late_sc0", "late_sc0sc1nt", "early_store_wbl2_all",
                           "early_store_wbl2_wg"};
    for (int iters : {0, 300}) {
        for (size_t mb : {0, 6, 12, 24}) {
            const int n4 = int((mb << 20) / 16);
            const int per_lane = (n4 + blocks * threads - 1) / (blocks * threads);
            std::printf("{\"spin_iters\": %d, \"MB\": %zu", iters, mb);
            for (int mode = 0; mode < 11; ++mode) {
                if (mb == 0 && mode > 0) break;
                const float t = time_graph(
                    s, [&] { k_flush<<<blocks, threads, 0, s>>>(buf, n4, per_lane, iters, mode, sink); }, 100, 10);
                std::printf(", \"%s_us\": %.3f", names[mode], t);
            }
            std::printf("}\n");
        }
    }
    CK(hipFree(buf));
    CK(hipFree(sink));
    return 0;
}
