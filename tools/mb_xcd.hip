// Does data a launch leaves in an XCD's L2 serve the next launch?  And does
// workgroup b land on the same XCD launch after launch?
//   1. placement: 16 launches of a 256-workgroup grid record HW_REG_XCC_ID
//      per workgroup: is block b's XCD the same every launch (eager and
//      graph-replayed), i.e. (xcc - b) mod 8 constant?
//   2. reuse: launch W writes 16 KiB per workgroup (plain stores), launch R
//      reads segment (b + shift) mod G -- shift 0 (the block that wrote it,
//      same XCD if placement is stable), 8 (another block of the same XCD
//      under round-robin), 1 (another XCD) -- and stamps one dependent load's
//      latency per wave (s_memtime around load + use); "cold" reads a buffer
//      no kernel touched since a 512 MiB sweep.
//   hipcc --offload-arch=gfx950 -O3 tools/mb_xcd.hip -o tools/mb_xcd
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); std::exit(1); } } while (0)

constexpr int G = 256, T = 256, SEG = 16384 / 16;   // workgroups, threads, float4 per segment

__global__ __launch_bounds__(T) void k_id(unsigned *out, int launch) {
    if (threadIdx.x == 0) {
        unsigned x;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
        out[launch * G + blockIdx.x] = x & 7u;
    }
}

__global__ __launch_bounds__(T) void k_write(float4 *buf, float v) {
    float4 *seg = buf + size_t(blockIdx.x) * SEG;
    for (int k = threadIdx.x; k < SEG; k += T) seg[k] = make_float4(v, v + 1, v + 2, float(k));
}

// one dependent load per wave, timed; the rest of the segment read normally
__global__ __launch_bounds__(T) void k_read(const float4 *buf, int shift, unsigned long long *lat, float *sink) {
    const int sb = (blockIdx.x + shift) % G;
    const float4 *seg = buf + size_t(sb) * SEG;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    unsigned long long t0, t1;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    float4 v = seg[w * 64 + lane];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    float a = v.x;
    asm volatile("" : "+v"(a));
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    if (lane == 0) lat[blockIdx.x * (T / 64) + w] = t1 - t0;
    float acc = a;
    for (int k = threadIdx.x + T; k < SEG; k += T) acc += seg[k].y;
    if (acc == 1234.5f) sink[blockIdx.x] = acc;
}

__global__ void k_sweep(float4 *big, size_t n4) {
    for (size_t k = size_t(blockIdx.x) * blockDim.x + threadIdx.x; k < n4; k += size_t(gridDim.x) * blockDim.x)
        big[k] = make_float4(1, 2, 3, 4);
}

int main() {
    unsigned *ids;
    CK(hipMalloc(&ids, 64 * G * sizeof(unsigned)));
    // 1. placement, eager then graph-replayed
    for (int l = 0; l < 16; ++l) hipLaunchKernelGGL(k_id, dim3(G), dim3(T), 0, 0, ids, l);
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipGraph_t gr;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int l = 16; l < 32; ++l) hipLaunchKernelGGL(k_id, dim3(G), dim3(T), 0, s, ids, l);
    CK(hipStreamEndCapture(s, &gr));
    CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    CK(hipDeviceSynchronize());
    std::vector<unsigned> h(64 * G);
    CK(hipMemcpy(h.data(), ids, 32 * G * sizeof(unsigned), hipMemcpyDeviceToHost));
    for (int l = 0; l < 32; ++l) {
        int rot = int((h[l * G] + 8) % 8), rr = 1;
        for (int b = 0; b < G; ++b) rr &= int(int((h[l * G + b] - b + 8 * 64) % 8) == rot);
        std::printf("{\"test\": \"placement\", \"launch\": %d, \"graph\": %d, \"xcc_of_block0\": %d, \"round_robin\": %d, "
                    "\"first8\": [%u,%u,%u,%u,%u,%u,%u,%u]}\n", l, l >= 16, rot, rr, h[l * G + 0], h[l * G + 1],
                    h[l * G + 2], h[l * G + 3], h[l * G + 4], h[l * G + 5], h[l * G + 6], h[l * G + 7]);
    }
    // 2. reuse across a launch boundary
    float4 *buf, *big, *cold;
    float *sink;
    unsigned long long *lat;
    const size_t big4 = (512ull << 20) / 16;
    CK(hipMalloc(&buf, size_t(G) * SEG * 16));
    CK(hipMalloc(&cold, size_t(G) * SEG * 16));
    CK(hipMalloc(&big, big4 * 16));
    CK(hipMalloc(&sink, G * 4));
    CK(hipMalloc(&lat, G * (T / 64) * 8));
    CK(hipMemset(cold, 0, size_t(G) * SEG * 16));
    std::vector<unsigned long long> hl(G * (T / 64));
    const char *names[] = {"same_block", "same_xcd_other_block", "other_xcd", "cold"};
    const int shifts[] = {0, 8, 1, 0};
    for (int rep = 0; rep < 3; ++rep) {
        for (int c = 0; c < 4; ++c) {
            hipLaunchKernelGGL(k_sweep, dim3(1024), dim3(256), 0, 0, big, big4);   // flush L2 / Infinity Cache
            if (c < 3) hipLaunchKernelGGL(k_write, dim3(G), dim3(T), 0, 0, buf, float(rep));
            hipLaunchKernelGGL(k_read, dim3(G), dim3(T), 0, 0, c < 3 ? buf : cold, shifts[c], lat, sink);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(hl.data(), lat, hl.size() * 8, hipMemcpyDeviceToHost));
            double m = 0;
            unsigned long long mx = 0;
            for (auto x : hl) { m += double(x); mx = x > mx ? x : mx; }
            std::printf("{\"test\": \"reuse\", \"rep\": %d, \"case\": \"%s\", \"load_cycles_mean\": %.0f, \"max\": %llu}\n",
                        rep, names[c], m / hl.size(), mx);
        }
    }
    return 0;
}
