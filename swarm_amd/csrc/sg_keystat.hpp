// sg_keystat.hpp — per-block partials of the sort keys' statistics (KeyStatD: OR, AND and
// the tag range of every key), shared by the passes that read or write the keys anyway (the
// prefix scan, the re-key, X1's matched-record gather).
#pragma once
#include "sg_internal.hpp"

namespace sg {

struct KeyStatAcc {
    uint64_t o = 0, a = ~0ull;
    uint32_t tmin = 255u, tmax = 0u;
    __device__ __forceinline__ void add(uint64_t k) {
        o |= k;
        a &= k;
        const uint32_t t = (uint32_t)(k & 0xffu);
        tmin = min(tmin, t);
        tmax = max(tmax, t);
    }
};
// Block-wide reduce (256 threads) into part[blockIdx.x]; s: 4 x KeyStatD of LDS.
__device__ __forceinline__ void kstat_flush(KeyStatAcc acc, KeyStatD *s, KeyStatD *part) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        acc.o |= (uint64_t)__shfl_xor((long long)acc.o, off, 64);
        acc.a &= (uint64_t)__shfl_xor((long long)acc.a, off, 64);
        acc.tmin = min(acc.tmin, (uint32_t)__shfl_xor((int)acc.tmin, off, 64));
        acc.tmax = max(acc.tmax, (uint32_t)__shfl_xor((int)acc.tmax, off, 64));
    }
    const int wid = threadIdx.x >> 6;
    if (lane_id() == 0) s[wid] = KeyStatD{acc.o, acc.a, acc.tmin, acc.tmax};
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 4; ++w) {
            acc.o |= s[w].o;
            acc.a &= s[w].a;
            acc.tmin = min(acc.tmin, s[w].tmin);
            acc.tmax = max(acc.tmax, s[w].tmax);
        }
        part[blockIdx.x] = KeyStatD{acc.o, acc.a, acc.tmin, acc.tmax};
    }
}

}  // namespace sg
