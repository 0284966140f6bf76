// sg_lines.hip — A3 module-output parsing: split a line-delimited buffer in HBM into its
// non-empty records in ONE pass (decoupled look-back), emitting per record its start,
// its end and its 8-byte prefix key for the sort.
//
// Record starts and ends are purely local predicates with one byte of look-behind:
//   start at p : byte[p] != '\n' && (p == 0 || byte[p-1] == '\n')
//   end   at q : byte[q] == '\n' && q > 0 && byte[q-1] != '\n'   (plus q = n for an
//                unterminated last record: bytes >= n read as '\n')
// so the k-th start pairs with the k-th end and empty records vanish without any
// carried state. Each thread owns 64 contiguous bytes (four 16-B loads, coalesced per
// wave), builds a 64-bit newline mask with SWAR, and the block scans the packed
// (starts:31 | ends:31) counts. Algorithmic bytes: n read + 16 B written per record.
#include "sg_internal.hpp"

#include <stdlib.h>

namespace sg {

constexpr int LN_BLOCK = 256;

__device__ __forceinline__ uint32_t nl_mask4(uint32_t x) {
    uint32_t y = x ^ 0x0a0a0a0au;
    uint32_t r = ~(((y & 0x7f7f7f7fu) + 0x7f7f7f7fu) | y | 0x7f7f7f7fu);  // 0x80 where byte == '\n'
    return ((r >> 7) & 1u) | ((r >> 14) & 2u) | ((r >> 21) & 4u) | ((r >> 28) & 8u);
}

// BPT bytes per thread (32 or 64): the tile is LN_BLOCK * BPT bytes. Larger tiles halve
// the look-back chain and put more loads in flight per thread.
template <int BPT>
__global__ __launch_bounds__(LN_BLOCK) void k_lines(const uint8_t *__restrict__ buf, uint64_t n,
                                                    uint2 *__restrict__ spans,
                                                    uint64_t *__restrict__ keys, uint32_t cap,
                                                    uint64_t *status, uint32_t *counter,
                                                    uint32_t ntiles) {
    constexpr int TILE = LN_BLOCK * BPT;
    constexpr int NW = BPT / 4;
    __shared__ __attribute__((aligned(16))) uint8_t s_b[TILE + 16];
    __shared__ uint64_t s_red[LN_BLOCK / 64];
    __shared__ uint64_t s_prefix;
    __shared__ uint32_t s_tile;
    const uint32_t tile = take_ticket(counter, &s_tile);
    const uint32_t t = threadIdx.x;
    const uint64_t base = (uint64_t)tile * TILE;
    const uint64_t my0 = base + (uint64_t)t * BPT;

    uint32_t w[NW];
    if (base + TILE + 8 <= n) {
        const uint4 *p = reinterpret_cast<const uint4 *>(buf + my0);
#pragma unroll
        for (int j = 0; j < NW / 4; ++j) {
            const uint4 a = p[j];
            w[4 * j] = a.x; w[4 * j + 1] = a.y; w[4 * j + 2] = a.z; w[4 * j + 3] = a.w;
        }
        if (t < 8) s_b[TILE + t] = buf[base + TILE + t];
    } else {
#pragma unroll
        for (int j = 0; j < NW; ++j) {
            uint32_t x = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint64_t pos = my0 + 4 * j + k;
                const uint32_t byte = (pos < n) ? buf[pos] : 0x0au;
                x |= byte << (8 * k);
            }
            w[j] = x;
        }
        if (t < 8) {
            const uint64_t pos = base + TILE + t;
            s_b[TILE + t] = (pos < n) ? buf[pos] : (uint8_t)0x0a;
        }
    }
#pragma unroll
    for (int j = 0; j < NW / 4; ++j)
        reinterpret_cast<uint4 *>(s_b)[(NW / 4) * t + j] = make_uint4(w[4 * j], w[4 * j + 1], w[4 * j + 2], w[4 * j + 3]);

    uint64_t m = 0;
#pragma unroll
    for (int j = 0; j < NW; ++j) m |= (uint64_t)nl_mask4(w[j]) << (4 * j);
    __syncthreads();
    uint64_t cin;
    if (t > 0) cin = (s_b[t * BPT - 1] == 0x0a);
    else cin = (base == 0) ? 1u : (buf[base - 1] == 0x0a);
    const uint64_t prevnl = (m << 1) | cin;
    const uint64_t sm = ~m & prevnl & (BPT == 64 ? ~0ull : 0xffffffffull);
    const uint64_t em = m & ~prevnl;
    const uint64_t packed = ((uint64_t)__popcll(sm) << 31) | (uint64_t)__popcll(em);

    uint64_t total;
    const uint64_t excl = block_excl_scan<LN_BLOCK>(packed, &total, s_red);
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
            if (tile == ntiles - 1) counter[1] = (uint32_t)((prefix + total) >> 31);
        }
    }
    __syncthreads();
    const uint64_t pre = s_prefix + excl;
    uint32_t si = (uint32_t)(pre >> 31);
    uint32_t ei = (uint32_t)(pre & 0x7fffffffu);

    uint64_t bits = sm;
    while (bits) {
        const int b = __ffsll((long long)bits) - 1;
        bits &= bits - 1;
        if (si < cap) {
            spans[si].x = (uint32_t)(my0 + b);
            if (keys) {
                const int q = t * BPT + b;
                uint32_t rem = 8;
                uint64_t k = 0;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const uint32_t c = s_b[q + j];
                    if (c == 0x0a && rem == 8) rem = j;
                    if (j < 7 && (uint32_t)j < rem) k |= (uint64_t)c << (56 - 8 * j);
                }
                keys[si] = k | rem;
            }
        }
        ++si;
    }
    bits = em;
    while (bits) {
        const int b = __ffsll((long long)bits) - 1;
        bits &= bits - 1;
        if (ei < cap) spans[ei].y = (uint32_t)(my0 + b);
        ++ei;
    }
}

static int lines_bpt() {
    static int v = [] {
        const char *e = getenv("SG_LINES_BPT");
        return (e && atoi(e) == 32) ? 32 : 64;
    }();
    return v;
}

int run_lines(sg_ctx *c, const uint8_t *d_buf, uint64_t n, const SlotSet &ss, Lines *out, bool want_keys) {
    if (n > MAX_BYTES) { set_error("buffer of %llu bytes exceeds the 4 GiB per-call limit", (unsigned long long)n); return SG_E_TOO_LARGE; }
    if (((uintptr_t)d_buf & 15) != 0) { set_error("run_lines: device buffer not 16-byte aligned"); return SG_E_INVAL; }
    const int bpt = lines_bpt();
    const uint32_t tile_bytes = LN_BLOCK * bpt;
    const uint32_t ntiles = (uint32_t)(n / tile_bytes + 1);
    uint64_t *status;
    SG_TRY(slot(c, ss.lb, (size_t)ntiles + 2, &status));
    uint32_t *counter = reinterpret_cast<uint32_t *>(status + ntiles);
    uint64_t want = n / 16 + 4096;
    if (c->slot_cap[ss.starts] / 8 > want) want = c->slot_cap[ss.starts] / 8 - 64;
    for (int attempt = 0; attempt < 2; ++attempt) {
        uint32_t cap = (uint32_t)want;
        SG_TRY(slot(c, ss.starts, cap, &out->spans));
        out->keys = nullptr;
        if (want_keys) SG_TRY(slot(c, ss.keys, cap, &out->keys));
        SG_HIP(hipMemsetAsync(status, 0, ((size_t)ntiles + 2) * 8, c->stream));
        if (bpt == 32)
            SG_LAUNCH(c, "lines", k_lines<32>, ntiles, LN_BLOCK, 0, d_buf, n, out->spans, out->keys, cap, status,
                      counter, ntiles);
        else
            SG_LAUNCH(c, "lines", k_lines<64>, ntiles, LN_BLOCK, 0, d_buf, n, out->spans, out->keys, cap, status,
                      counter, ntiles);
        uint32_t R = 0;
        SG_TRY(ctx_readback(c, &R, counter + 1, 4));
        out->n_rec = R;
        out->tile_prefix = status;
        out->tile_bytes = tile_bytes;
        out->n_tiles = ntiles;
        prof_bytes(c, "lines", (double)n + (want_keys ? 16.0 : 8.0) * R);  // text read once + (start, end[, key0])
        if (R <= cap) return SG_OK;
        want = (uint64_t)R + 4096;
    }
    set_error("run_lines: capacity retry failed");
    return SG_E_NOMEM;
}

}  // namespace sg
