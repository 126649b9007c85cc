// What c3's header wait is: on c3's grid (2,048
// waves of 32 envs, 8 per workgroup, plus as many idle helper waves), each
// wave loads its 512-B header block, then `extra` more bytes of other arrays
// at once (the state a step wave reads with its header: ships, bearings,
// planets, controls, first bullet rounds), and records with s_memrealtime
// (a read of the real-time counter, 100 MHz) when it started, when the
// header arrived and when everything arrived.  If the header's arrival
// grows with the bytes every wave requests beside it, the wait is the
// launch's opening read burst queueing, not the header's own latency.
//   hipcc --offload-arch=gfx950 -O3 tools/mb_hdr_burst.hip -o tools/mb_hdr_burst
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); std::exit(1); } } while (0)

constexpr int WAVES = 2048, WPG = 8, LANES = 64;
constexpr int MAXV = 8;   // up to 8 extra 16-B loads per lane = 8 KB per wave

__device__ __forceinline__ unsigned long long rt() {
    unsigned long long t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

// Each wave: its header load, then NV KB of other loads at once; the wave
// waits for the header alone first (vmcnt = the extra loads still allowed in
// flight: loads return in order), then for everything.
template <int NV>
__global__ __launch_bounds__(2 * 64 * WPG) void k_hdr_first_wait(const int4 *hdr, const float4 *state,
                                                                 unsigned long long *out, float *sink) {
    const int wv = threadIdx.x / 64;
    if (wv >= WPG) return;
    const int lane = threadIdx.x & 63;
    const int w = blockIdx.x * WPG + wv;
    const unsigned long long t0 = rt();
    const int4 h = hdr[w * 32 + lane / 2];
    float4 v[NV > 0 ? NV : 1];
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = state[(size_t(k) * WAVES + w) * LANES + lane];
    // loads return in order per wave: vmcnt(NV) = the header is in
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NV) : "memory");
    int hx = h.x ^ h.y ^ h.z ^ h.w;
    asm volatile("" : "+v"(hx));
    const unsigned long long t1 = rt();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long t2 = rt();
    float acc = float(hx);
#pragma unroll
    for (int k = 0; k < NV; ++k) acc += v[k].x + v[k].y + v[k].z + v[k].w;
    if (acc == 1234.5f) sink[w] = acc;
    if (lane == 0) {
        out[3 * w + 0] = t0;
        out[3 * w + 1] = t1;
        out[3 * w + 2] = t2;
    }
}

template <int NV>
static void run(const int4 *hdr, const float4 *state, unsigned long long *out, float *sink, hipStream_t s) {
    std::vector<unsigned long long> h(3 * WAVES);
    // warm: a few launches, then the measured one
    for (int r = 0; r < 4; ++r)
        k_hdr_first_wait<NV><<<WAVES / WPG, 2 * 64 * WPG, 0, s>>>(hdr, state, out, sink);
    CK(hipStreamSynchronize(s));
    std::vector<double> hw, all;
    for (int rep = 0; rep < 5; ++rep) {
        k_hdr_first_wait<NV><<<WAVES / WPG, 2 * 64 * WPG, 0, s>>>(hdr, state, out, sink);
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(h.data(), out, sizeof(unsigned long long) * 3 * WAVES, hipMemcpyDeviceToHost));
        unsigned long long first = ~0ull;
        for (int w = 0; w < WAVES; ++w) first = std::min(first, h[3 * w]);
        for (int w = 0; w < WAVES; ++w) {
            hw.push_back((h[3 * w + 1] - h[3 * w]) * 0.01);   // 100 MHz ticks -> us
            all.push_back((h[3 * w + 2] - first) * 0.01);
        }
    }
    std::sort(hw.begin(), hw.end());
    std::sort(all.begin(), all.end());
    auto mean = [](const std::vector<double> &v) { double a = 0; for (double x : v) a += x; return a / v.size(); };
    std::printf("{\"extra_bytes_per_wave\": %d, \"hdr_wait_us_mean\": %.3f, \"hdr_wait_us_p95\": %.3f, "
                "\"all_loads_in_us_after_first_wave_start_p50\": %.3f, \"p100\": %.3f}\n",
                NV * 1024, mean(hw), hw[size_t(0.95 * hw.size())], all[all.size() / 2], all.back());
}

int main() {
    hipStream_t s;
    CK(hipStreamCreate(&s));
    int4 *hdr;
    float4 *state;
    unsigned long long *out;
    float *sink;
    CK(hipMalloc(&hdr, sizeof(int4) * WAVES * 32));
    CK(hipMalloc(&state, sizeof(float4) * size_t(MAXV) * WAVES * LANES));
    CK(hipMalloc(&out, sizeof(unsigned long long) * 3 * WAVES));
    CK(hipMalloc(&sink, sizeof(float) * WAVES));
    CK(hipMemset(hdr, 0, sizeof(int4) * WAVES * 32));
    CK(hipMemset(state, 0, sizeof(float4) * size_t(MAXV) * WAVES * LANES));
    run<0>(hdr, state, out, sink, s);
    run<2>(hdr, state, out, sink, s);
    run<4>(hdr, state, out, sink, s);
    run<8>(hdr, state, out, sink, s);
    CK(hipFree(hdr));
    CK(hipFree(state));
    CK(hipFree(out));
    CK(hipFree(sink));
    return 0;
}
