// Partial-line read microbenchmark: when a wave reads only the first B bytes
// of each 128-B line (B = 128, 64, 32, 16), what does the L2 fetch from
// memory -- whole 128-B lines, or 64-/32-B requests -- and how fast is it?
// Decides whether a layout that leaves the unused part of a line unread
// (an env's short bullet row, planet slots past its planet count) saves
// memory-side bytes on gfx950.  1 GiB buffer (past the Infinity Cache),
// 16 B per lane, grid-stride; each variant is its own kernel so
// rocprofv3 --pmc TCC_EA0_RDREQ_{32B,64B,128B}_sum splits by kernel.
//   hipcc --offload-arch=gfx950 -O3 tools/mb_sector.hip -o tools/mb_sector
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); std::exit(1); } } while (0)

typedef float f4v __attribute__((ext_vector_type(4)));

// read the first B bytes of every 128-B line; NT: nontemporal loads
template <int B, bool NT>
__global__ __launch_bounds__(256) void k_read(const f4v *__restrict__ buf, long lines, float *sink) {
    constexpr int LPL = B / 16;   // lanes per line
    const long lanes = long(gridDim.x) * blockDim.x;
    const long g = long(blockIdx.x) * blockDim.x + threadIdx.x;
    f4v acc = {0, 0, 0, 0};
    for (long k = g; k < lines * LPL; k += lanes) {
        const long line = k / LPL, c = k % LPL;
        const f4v *p = buf + line * 8 + c;
        f4v v;
        if (NT) v = __builtin_nontemporal_load(p);
        else v = *p;
        acc += v;
    }
    if (acc.x + acc.y + acc.z + acc.w == 1234.5f) sink[g] = acc.x;
}

template <int B, bool NT>
float run(const f4v *buf, long lines, float *sink, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int grid = 256 * 16;
    hipLaunchKernelGGL((k_read<B, NT>), dim3(grid), dim3(256), 0, 0, buf, lines, sink);   // warm
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k_read<B, NT>), dim3(grid), dim3(256), 0, 0, buf, lines, sink);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main() {
    const long bytes = 1l << 30, lines = bytes / 128;
    f4v *buf;
    float *sink;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&sink, 256 * 16 * 256 * sizeof(float)));
    CK(hipMemset(buf, 0, bytes));
    const int reps = 10;
    struct R { const char *name; int b; float ms; } rs[] = {
        {"128B", 128, run<128, false>(buf, lines, sink, reps)},
        {"64B", 64, run<64, false>(buf, lines, sink, reps)},
        {"32B", 32, run<32, false>(buf, lines, sink, reps)},
        {"16B", 16, run<16, false>(buf, lines, sink, reps)},
        {"64B_nt", 64, run<64, true>(buf, lines, sink, reps)},
        {"32B_nt", 32, run<32, true>(buf, lines, sink, reps)},
    };
    for (const R &r : rs) {
        const double used = double(lines) * r.b, full = double(bytes);
        std::printf("{\"variant\": \"%s\", \"ms\": %.4f, \"used_GBps\": %.1f, \"line_GBps\": %.1f}\n", r.name, r.ms,
                    used / (r.ms * 1e-3) / 1e9, full / (r.ms * 1e-3) / 1e9);
    }
    CK(hipFree(buf));
    CK(hipFree(sink));
    return 0;
}
