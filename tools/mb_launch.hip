// Launch-floor microbenchmark: per-launch time of stub kernels on the step
// kernel's grid shapes, back to back in one hipGraph (100 launches per
// graph, as bench.py replays).  Answers: how much of a 15 us astro_step
// launch is dispatch + drain of 4,096 one-wave workgroups, and does a grid
// of fewer, larger workgroups dispatch faster.
//   hipcc --offload-arch=gfx950 -O3 tools/mb_launch.hip -o tools/mb_launch
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); std::exit(1); } } while (0)

__global__ void k_empty(int *sink) {
    if (sink && threadIdx.x == 1024) sink[0] = 1;   // never true
}

// each lane moves `per_lane` float4s (read + write, in place)
__global__ void k_copy(float4 *buf, int n4, int per_lane) {
    const int lanes = gridDim.x * blockDim.x;
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    for (int k = 0; k < per_lane; ++k) {
        const int j = g + k * lanes;
        if (j < n4) {
            float4 v = buf[j];
            v.x += 1.0f;
            buf[j] = v;
        }
    }
}

// VALU spin: `iters` dependent-free f64 fma chains of 4 (issue-bound)
__global__ void k_spin(double *out, int iters) {
    double a = threadIdx.x, b = 1.0000001, c = 0.5, d = 0.25;
    for (int k = 0; k < iters; ++k) {
        a = __builtin_fma(a, b, 1e-9);
        c = __builtin_fma(c, b, 1e-9);
        d = __builtin_fma(d, b, 1e-9);
        b = __builtin_fma(b, 1.0, 1e-12);
    }
    if (a + c + d == 12345.0) out[blockIdx.x] = a;
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
    const size_t bytes = 24u << 20;   // ~ one c3 launch's state
    float4 *buf;
    double *out;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&out, 1 << 20));
    CK(hipMemset(buf, 0, bytes));
    const int n4 = int(bytes / 16);
    struct G { int blocks, threads; } grids[] = {{4096, 64}, {2048, 128}, {1024, 256}, {512, 512}, {256, 1024}};
    for (auto g : grids) {
        const float t_empty = time_graph(s, [&] { k_empty<<<g.blocks, g.threads, 0, s>>>(nullptr); }, 100, 20);
        const int per_lane = (n4 + g.blocks * g.threads - 1) / (g.blocks * g.threads);
        const float t_copy = time_graph(s, [&] { k_copy<<<g.blocks, g.threads, 0, s>>>(buf, n4, per_lane); }, 100, 20);
        const float t_spin = time_graph(s, [&] { k_spin<<<g.blocks, g.threads, 0, s>>>(out, 500); }, 100, 20);
        std::printf("{\"blocks\": %d, \"threads\": %d, \"empty_us\": %.3f, \"copy24MB_us\": %.3f, "
                    "\"copy_GBps\": %.0f, \"spin500_us\": %.3f}\n",
                    g.blocks, g.threads, t_empty, t_copy, 2.0 * bytes / (t_copy * 1e-6) / 1e9, t_spin);
    }
    CK(hipFree(buf));
    CK(hipFree(out));
    return 0;
}
