// gather_probe.hip — what one random small read costs on MI355X (design probe for the
// sorted-slot dedup). Reads are independent random accesses into a table
// far larger than the Infinity Cache; each lane keeps 4 in flight and XORs what it read.
//   slot32 : a 32-B aligned slot (two 16-B loads)
//   slot64 : a 64-B aligned slot (four 16-B loads)
//   rec26  : 26 bytes at a random byte offset (the aligned 16-B chunks covering them, 2-3 loads)
//   line128: a 128-B aligned line (eight 16-B loads)
//   seq32  : 32-B slots read in order (the streaming reference)
// Build: hipcc -O3 --offload-arch=gfx950 tools/gather_probe.hip -o tools/bin/gather_probe
// Run:   tools/bin/gather_probe [table_MiB] [reads_M]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}

__device__ __forceinline__ uint32_t fold(uint4 v) { return v.x ^ v.y ^ v.z ^ v.w; }

template <int MODE>
__global__ __launch_bounds__(256) void k_probe(const uint8_t *__restrict__ T, uint64_t tbytes, uint64_t nreads,
                                               uint32_t *__restrict__ out) {
    const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const uint64_t nthr = (uint64_t)gridDim.x * blockDim.x;
    uint32_t acc = 0;
    for (uint64_t r0 = tid * 4; r0 < nreads; r0 += nthr * 4) {
        uint4 v[4][8];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint64_t h = mix(r0 + u + 0x9e3779b97f4a7c15ull);
            if (MODE == 0) {  // slot32
                const uint64_t o = (h % (tbytes / 32)) * 32;
                const uint4 *p = reinterpret_cast<const uint4 *>(T + o);
                v[u][0] = p[0]; v[u][1] = p[1];
            } else if (MODE == 1) {  // slot64
                const uint64_t o = (h % (tbytes / 64)) * 64;
                const uint4 *p = reinterpret_cast<const uint4 *>(T + o);
                v[u][0] = p[0]; v[u][1] = p[1]; v[u][2] = p[2]; v[u][3] = p[3];
            } else if (MODE == 2) {  // rec26
                const uint64_t o = h % (tbytes - 64);
                const uint64_t a = o & ~15ull;
                const uint4 *p = reinterpret_cast<const uint4 *>(T + a);
                v[u][0] = p[0]; v[u][1] = p[1];
                v[u][2] = (o - a) + 26 > 32 ? p[2] : make_uint4(0, 0, 0, 0);
            } else if (MODE == 3) {  // line128
                const uint64_t o = (h % (tbytes / 128)) * 128;
                const uint4 *p = reinterpret_cast<const uint4 *>(T + o);
#pragma unroll
                for (int k = 0; k < 8; ++k) v[u][k] = p[k];
            } else {  // seq32
                const uint64_t o = ((r0 + u) % (tbytes / 32)) * 32;
                const uint4 *p = reinterpret_cast<const uint4 *>(T + o);
                v[u][0] = p[0]; v[u][1] = p[1];
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int nk = MODE == 0 || MODE == 4 ? 2 : (MODE == 1 ? 4 : (MODE == 2 ? 3 : 8));
#pragma unroll
            for (int k = 0; k < 8; ++k)
                if (k < nk) acc ^= fold(v[u][k]);
        }
    }
    out[tid] = acc;
}

template <int MODE>
static float run(const uint8_t *T, uint64_t tb, uint64_t nreads, uint32_t *out, int grid) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL(k_probe<MODE>, dim3(grid), dim3(256), 0, 0, T, tb, nreads, out);  // warm-up
    CK(hipEventRecord(a));
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k_probe<MODE>, dim3(grid), dim3(256), 0, 0, T, tb, nreads, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / 3;
}

int main(int argc, char **argv) {
    const uint64_t tmib = argc > 1 ? strtoull(argv[1], 0, 10) : 2048;
    const uint64_t nreads = (argc > 2 ? strtoull(argv[2], 0, 10) : 64) << 20;
    const uint64_t tb = tmib << 20;
    uint8_t *T;
    uint32_t *out;
    const int grid = 256 * 16;
    CK(hipMalloc(&T, tb));
    CK(hipMalloc(&out, (size_t)grid * 256 * 4));
    CK(hipMemset(T, 0x5a, tb));
    CK(hipDeviceSynchronize());
    const char *names[5] = {"slot32", "slot64", "rec26", "line128", "seq32"};
    float ms[5];
    ms[0] = run<0>(T, tb, nreads, out, grid);
    ms[1] = run<1>(T, tb, nreads, out, grid);
    ms[2] = run<2>(T, tb, nreads, out, grid);
    ms[3] = run<3>(T, tb, nreads, out, grid);
    ms[4] = run<4>(T, tb, nreads, out, grid);
    CK(hipDeviceSynchronize());
    for (int m = 0; m < 5; ++m)
        printf("%-8s table %lu MiB, %lu M reads: %.3f ms, %.2f G reads/s, %.1f ns/read/CU-equiv, %.2f TB/s at 128 B/read\n",
               names[m], (unsigned long)tmib, (unsigned long)(nreads >> 20), ms[m], nreads / (ms[m] * 1e6),
               ms[m] * 1e6 / nreads * 256, nreads * 128.0 / (ms[m] * 1e9));
    CK(hipFree(T));
    CK(hipFree(out));
    return 0;
}
