// Host cost of a kernel launch on this stack: N launches of an empty kernel
// from a C loop, host time per call -- small vs ~400-byte kernel arguments
// (astro_step passes AstroParams + AstroState + TickDriver by value), with
// and without hipGetLastError after each, and hipEventRecord / Query costs.
//   hipcc --offload-arch=gfx950 -O3 tools/mb_hostlaunch.hip -o tools/mb_hostlaunch
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); std::exit(1); } } while (0)

struct Big { double v[50]; };   // 400 bytes

__global__ void k_small(int *o) { if (o && threadIdx.x == 1023) o[0] = 1; }
__global__ void k_big(Big b, int *o) { if (o && threadIdx.x == 1023) o[0] = int(b.v[3]); }

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    hipStream_t s;
    CK(hipStreamCreate(&s));
    Big b{};
    const int N = 2000;
    for (int rep = 0; rep < 3; ++rep) {
        for (int mode = 0; mode < 4; ++mode) {   // 0 small, 1 big, 2 big + hipGetLastError, 3 big, 1024-thread grid of 512 blocks
            CK(hipStreamSynchronize(s));
            const double t0 = now_us();
            for (int i = 0; i < N; ++i) {
                if (mode == 0) hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, s, nullptr);
                else if (mode == 3) hipLaunchKernelGGL(k_big, dim3(512), dim3(1024), 0, s, b, nullptr);
                else hipLaunchKernelGGL(k_big, dim3(1), dim3(64), 0, s, b, nullptr);
                if (mode == 2) (void)hipGetLastError();
            }
            const double t1 = now_us();
            CK(hipStreamSynchronize(s));
            const double t2 = now_us();
            std::printf("{\"rep\": %d, \"mode\": \"%s\", \"host_us_per_launch\": %.2f, \"until_done_us_per_launch\": %.2f}\n",
                        rep, mode == 0 ? "small_args" : mode == 1 ? "400B_args" : mode == 2 ? "400B_args+getlasterror" : "400B_args_512x1024",
                        (t1 - t0) / N, (t2 - t0) / N);
        }
        hipEvent_t e;
        CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        double t0 = now_us();
        for (int i = 0; i < N; ++i) CK(hipEventRecord(e, s));
        double t1 = now_us();
        CK(hipStreamSynchronize(s));
        double t2 = now_us();
        for (int i = 0; i < N; ++i) (void)hipEventQuery(e);
        double t3 = now_us();
        // a launch + record + busy-poll round trip (the single-game tick's skeleton)
        double t4 = now_us();
        for (int i = 0; i < 500; ++i) {
            hipLaunchKernelGGL(k_big, dim3(1), dim3(64), 0, s, b, nullptr);
            CK(hipEventRecord(e, s));
            while (hipEventQuery(e) == hipErrorNotReady) {}
        }
        double t5 = now_us();
        std::printf("{\"rep\": %d, \"event_record_us\": %.2f, \"event_query_us\": %.2f, \"launch_record_poll_roundtrip_us\": %.2f}\n",
                    rep, (t1 - t0) / N, (t3 - t2) / N, (t5 - t4) / 500);
        CK(hipEventDestroy(e));
    }
    return 0;
}
