// sg_prims.hpp — device-wide primitives (templated on a functor), reduce-then-scan:
//   select2 : order-preserving compaction of up to two predicates at once (the k-th
//             A-index pairs with the k-th B-index, used for group start/end lists).
//             k_sel_count evaluates the predicate ONCE, keeps its two ballots per wave-row
//             as bit masks and reduces the tile counts; k_tile_scan; k_sel_apply turns the
//             masks into output positions (no second predicate evaluation).
//   scan64  : exclusive scan of a per-item u64 value (byte offsets of records):
//             k_scan64_count -> k_tile_scan -> k_scan64_apply.
#pragma once
#include "sg_common.hpp"

namespace sg {

constexpr int SEL_BLOCK = 256;
constexpr int SEL_ROWS = 16;
constexpr int SEL_TILE = SEL_BLOCK * SEL_ROWS;
constexpr int SEL_MASKS = SEL_ROWS * (SEL_BLOCK / 64);  // u64 ballots per tile and predicate

// Pred: __device__ uint32_t operator()(uint32_t i) const -> bit0 select-A, bit1 select-B.
// Items are striped (row j, thread t -> i = base + j*256 + t) so loads coalesce.
// tot[tile] = (countA << 31) | countB.
template <class Pred>
__global__ __launch_bounds__(SEL_BLOCK) void k_sel_count(Pred pred, uint32_t n, uint64_t *__restrict__ mA,
                                                         uint64_t *__restrict__ mB, uint64_t *__restrict__ tot) {
    __shared__ uint64_t s_red[SEL_BLOCK / 64];
    const int t = threadIdx.x, lane = lane_id(), wid = t >> 6;
    const uint32_t base = blockIdx.x * SEL_TILE;
    uint64_t cnt = 0;
    // every row's predicate first, then the ballots and mask stores: a store between two
    // rows kept the next row's (possibly aliasing) loads behind it (one latency per row)
    // (full tiles without the per-row bounds branch, so the rows' loads can issue together)
    uint32_t p[SEL_ROWS];
    if (base + SEL_TILE <= n) {
#pragma unroll
        for (int j = 0; j < SEL_ROWS; ++j) p[j] = pred(base + j * SEL_BLOCK + t);
    } else {
#pragma unroll
        for (int j = 0; j < SEL_ROWS; ++j) {
            const uint32_t i = base + j * SEL_BLOCK + t;
            p[j] = (i < n) ? pred(i) : 0u;
        }
    }
#pragma unroll
    for (int j = 0; j < SEL_ROWS; ++j) {
        const uint64_t ma = __ballot(p[j] & 1u), mb = __ballot(p[j] & 2u);
        if (lane == 0) {
            mA[(uint64_t)blockIdx.x * SEL_MASKS + j * 4 + wid] = ma;
            mB[(uint64_t)blockIdx.x * SEL_MASKS + j * 4 + wid] = mb;
        }
        cnt += ((uint64_t)__popcll(ma) << 31) | (uint64_t)__popcll(mb);
    }
    if (lane == 0) s_red[wid] = cnt;
    __syncthreads();
    if (t == 0) tot[blockIdx.x] = s_red[0] + s_red[1] + s_red[2] + s_red[3];
}

__global__ __launch_bounds__(SEL_BLOCK) void k_sel_apply(uint32_t n, const uint64_t *__restrict__ mA,
                                                         const uint64_t *__restrict__ mB,
                                                         const uint64_t *__restrict__ pre, uint32_t *__restrict__ outA,
                                                         uint32_t *__restrict__ outB);  // sg_runtime.hip

constexpr int SCAN_BLOCK = 256;
constexpr int SCAN_ITEMS = 8;
constexpr int SCAN_TILE = SCAN_BLOCK * SCAN_ITEMS;

// Fn: __device__ uint64_t operator()(uint32_t i) const. out[i] = sum_{j<i} fn(j).
template <class Fn>
__global__ __launch_bounds__(SCAN_BLOCK) void k_scan64_count(Fn fn, uint32_t n, uint64_t *__restrict__ tot) {
    __shared__ uint64_t s_red[SCAN_BLOCK / 64];
    const uint32_t base = blockIdx.x * SCAN_TILE;
    uint64_t sum = 0;
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j) {
        const uint32_t i = base + j * SCAN_BLOCK + threadIdx.x;
        if (i < n) sum += fn(i);
    }
    sum = wave_sum(sum);
    if (lane_id() == 0) s_red[threadIdx.x >> 6] = sum;
    __syncthreads();
    if (threadIdx.x == 0) tot[blockIdx.x] = s_red[0] + s_red[1] + s_red[2] + s_red[3];
}

template <class Fn>
__global__ __launch_bounds__(SCAN_BLOCK) void k_scan64_apply(Fn fn, uint32_t n, const uint64_t *__restrict__ pre,
                                                             uint64_t *__restrict__ out) {
    __shared__ uint64_t s_red[SCAN_BLOCK / 64];
    const int t = threadIdx.x;
    const uint32_t i0 = blockIdx.x * SCAN_TILE + t * SCAN_ITEMS;
    uint64_t v[SCAN_ITEMS];
    uint64_t sum = 0;
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j) {
        v[j] = (i0 + j < n) ? fn(i0 + j) : 0ull;
        sum += v[j];
    }
    uint64_t total;
    const uint64_t excl = block_excl_scan<SCAN_BLOCK>(sum, &total, s_red);
    uint64_t run = pre[blockIdx.x] + excl;
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j) {
        if (i0 + j < n) out[i0 + j] = run;
        run += v[j];
    }
}

}  // namespace sg
