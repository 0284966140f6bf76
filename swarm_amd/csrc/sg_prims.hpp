// sg_prims.hpp — device-wide single-pass primitives (templated on a functor), built on
// the decoupled look-back of sg_common.hpp:
//   k_select2 : order-preserving compaction of up to two predicates at once (the k-th
//               A-index pairs with the k-th B-index, used for group start/end lists)
//   k_scan64  : exclusive scan of a per-item u64 value (byte offsets of records)
#pragma once
#include "sg_common.hpp"

namespace sg {

constexpr int SEL_BLOCK = 256;
constexpr int SEL_ROWS = 16;
constexpr int SEL_TILE = SEL_BLOCK * SEL_ROWS;

// Pred: __device__ uint32_t operator()(uint32_t i) const -> bit0 select-A, bit1 select-B.
// Items are striped (row j, thread t -> i = base + j*256 + t) so loads coalesce; output
// order is index order. counter[1], counter[2] receive the A and B totals.
template <class Pred>
__global__ __launch_bounds__(SEL_BLOCK) void k_select2(Pred pred, uint32_t n, uint32_t *outA,
                                                       uint32_t *outB, uint64_t *status,
                                                       uint32_t *counter, uint32_t ntiles) {
    __shared__ uint32_t s_ca[SEL_ROWS * 4], s_cb[SEL_ROWS * 4];
    __shared__ uint64_t s_prefix;
    __shared__ uint32_t s_tile;
    const uint32_t tile = take_ticket(counter, &s_tile);
    const int t = threadIdx.x, lane = lane_id(), wid = t >> 6;
    const uint64_t lt = (1ull << lane) - 1ull;
    const uint32_t base = tile * SEL_TILE;
    uint32_t pa = 0, pb = 0;
    uint8_t ra[SEL_ROWS], rb[SEL_ROWS];
#pragma unroll
    for (int j = 0; j < SEL_ROWS; ++j) {
        const uint32_t i = base + j * SEL_BLOCK + t;
        const uint32_t p = (i < n) ? pred(i) : 0u;
        const uint64_t ma = __ballot(p & 1u), mb = __ballot(p & 2u);
        ra[j] = (uint8_t)__popcll(ma & lt);
        rb[j] = (uint8_t)__popcll(mb & lt);
        pa |= (p & 1u) << j;
        pb |= ((p >> 1) & 1u) << j;
        if (lane == 0) {
            s_ca[j * 4 + wid] = (uint32_t)__popcll(ma);
            s_cb[j * 4 + wid] = (uint32_t)__popcll(mb);
        }
    }
    __syncthreads();
    if (t < 64) {
        const uint32_t a = s_ca[t], b = s_cb[t];
        const uint32_t ia = wave_incl_scan(a), ib = wave_incl_scan(b);
        const uint32_t ta = __shfl(ia, 63, 64), tb = __shfl(ib, 63, 64);
        s_ca[t] = ia - a;
        s_cb[t] = ib - b;
        const uint64_t total = ((uint64_t)ta << 31) | tb;
        uint64_t prefix = 0;
        if (tile == 0) {
            if (t == 0) lb_store(status, LB_FLAG_INC, total);
        } else {
            if (t == 0) lb_store(status + tile, LB_FLAG_AGG, total);
            prefix = wave_lookback(status, tile);
            if (t == 0) lb_store(status + tile, LB_FLAG_INC, prefix + total);
        }
        if (t == 0) {
            s_prefix = prefix;
            if (tile == ntiles - 1) {
                counter[1] = (uint32_t)((prefix + total) >> 31);
                counter[2] = (uint32_t)((prefix + total) & 0x7fffffffu);
            }
        }
    }
    __syncthreads();
    const uint32_t preA = (uint32_t)(s_prefix >> 31), preB = (uint32_t)(s_prefix & 0x7fffffffu);
#pragma unroll
    for (int j = 0; j < SEL_ROWS; ++j) {
        const uint32_t i = base + j * SEL_BLOCK + t;
        if ((pa >> j) & 1u) outA[preA + s_ca[j * 4 + wid] + ra[j]] = i;
        if (outB && ((pb >> j) & 1u)) outB[preB + s_cb[j * 4 + wid] + rb[j]] = i;
    }
}

constexpr int SCAN_BLOCK = 256;
constexpr int SCAN_ITEMS = 8;
constexpr int SCAN_TILE = SCAN_BLOCK * SCAN_ITEMS;

// Fn: __device__ uint64_t operator()(uint32_t i) const. out[i] = sum_{j<i} fn(j);
// counter[1..2] = total (lo, hi).
template <class Fn>
__global__ __launch_bounds__(SCAN_BLOCK) void k_scan64(Fn fn, uint32_t n, uint64_t *out,
                                                       uint64_t *status, uint32_t *counter,
                                                       uint32_t ntiles) {
    __shared__ uint64_t s_red[SCAN_BLOCK / 64];
    __shared__ uint64_t s_prefix;
    __shared__ uint32_t s_tile;
    const uint32_t tile = take_ticket(counter, &s_tile);
    const int t = threadIdx.x;
    const uint32_t i0 = tile * SCAN_TILE + t * SCAN_ITEMS;
    uint64_t v[SCAN_ITEMS];
    uint64_t sum = 0;
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j) {
        v[j] = (i0 + j < n) ? fn(i0 + j) : 0ull;
        sum += v[j];
    }
    uint64_t total;
    const uint64_t excl = block_excl_scan<SCAN_BLOCK>(sum, &total, s_red);
    if (t < 64) {
        uint64_t prefix = 0;
        if (tile == 0) {
            if (t == 0) lb_store(status, LB_FLAG_INC, total);
        } else {
            if (t == 0) lb_store(status + tile, LB_FLAG_AGG, total);
            prefix = wave_lookback(status, tile);
            if (t == 0) lb_store(status + tile, LB_FLAG_INC, prefix + total);
        }
        if (t == 0) {
            s_prefix = prefix;
            if (tile == ntiles - 1) {
                const uint64_t tot = prefix + total;
                counter[1] = (uint32_t)tot;
                counter[2] = (uint32_t)(tot >> 32);
            }
        }
    }
    __syncthreads();
    uint64_t run = s_prefix + excl;
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j) {
        if (i0 + j < n) out[i0 + j] = run;
        run += v[j];
    }
}

}  // namespace sg
