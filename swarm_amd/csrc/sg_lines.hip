// sg_lines.hip — A3 module-output parsing: split a line-delimited buffer in HBM into its
// non-empty records, emitting per record its (start, end) span and its 8-byte prefix key
// for the sort.
//
// Record starts and ends are purely local predicates with one byte of look-behind:
//   start at p : byte[p] != '\n' && (p == 0 || byte[p-1] == '\n')
//   end   at q : byte[q] == '\n' && q > 0 && byte[q-1] != '\n'   (plus q = n for an
//                unterminated last record: bytes >= n read as '\n')
// so the k-th start pairs with the k-th end and empty records vanish without any
// carried state. Each thread owns 64 contiguous bytes (four 16-B loads, coalesced per
// wave) and builds a 64-bit newline mask with SWAR. Reduce-then-scan: k_lines_count
// reduces the packed (starts:31 | ends:31) counts per 16 KiB tile, k_tile_scan turns them
// into tile prefixes, k_lines re-reads the tile and writes the records. Algorithmic bytes:
// 2 n read + 16 B written per record.
#include "sg_internal.hpp"
#include "sg_route.hpp"

#include <stdlib.h>
#include <string.h>

namespace sg {

constexpr int LN_BLOCK = 256;
constexpr int LN_BPT = 64;
constexpr int LN_TILE = LN_BLOCK * LN_BPT;
constexpr int LN_NW = LN_BPT / 4;
constexpr uint32_t LN_CAP = 768;  // records per tile assembled in LDS (~21 B or more per record on average)

__device__ __forceinline__ uint32_t nl_mask4(uint32_t x) {
    uint32_t y = x ^ 0x0a0a0a0au;
    uint32_t r = ~(((y & 0x7f7f7f7fu) + 0x7f7f7f7fu) | y | 0x7f7f7f7fu);  // 0x80 where byte == '\n'
    return ((r >> 7) & 1u) | ((r >> 14) & 2u) | ((r >> 21) & 4u) | ((r >> 28) & 8u);
}

// This thread's 64 bytes (bytes >= n read as '\n') and the byte before them.
__device__ __forceinline__ void load64(const uint8_t *__restrict__ buf, uint64_t n, uint64_t base, uint64_t my0,
                                       uint32_t (&w)[LN_NW], uint32_t *prev) {
    if (base + LN_TILE + 8 <= n) {
        const uint4 *p = reinterpret_cast<const uint4 *>(buf + my0);
#pragma unroll
        for (int j = 0; j < LN_NW / 4; ++j) {
            const uint4 a = p[j];
            w[4 * j] = a.x; w[4 * j + 1] = a.y; w[4 * j + 2] = a.z; w[4 * j + 3] = a.w;
        }
    } else {
#pragma unroll
        for (int j = 0; j < LN_NW; ++j) {
            uint32_t x = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint64_t pos = my0 + 4 * j + k;
                const uint32_t byte = (pos < n) ? buf[pos] : 0x0au;
                x |= byte << (8 * k);
            }
            w[j] = x;
        }
    }
    *prev = (my0 == 0) ? 0x0au : ((my0 - 1 < n) ? buf[my0 - 1] : 0x0au);
}

__device__ __forceinline__ void masks(const uint32_t (&w)[LN_NW], uint32_t prev, uint64_t *sm, uint64_t *em) {
    uint64_t m = 0;
#pragma unroll
    for (int j = 0; j < LN_NW; ++j) m |= (uint64_t)nl_mask4(w[j]) << (4 * j);
    const uint64_t prevnl = (m << 1) | (prev == 0x0au ? 1ull : 0ull);
    *sm = ~m & prevnl;
    *em = m & ~prevnl;
}

__global__ __launch_bounds__(LN_BLOCK) void k_lines_count(const uint8_t *__restrict__ buf, uint64_t n,
                                                          uint64_t *__restrict__ tot) {
    __shared__ uint64_t s_red[LN_BLOCK / 64];
    const uint64_t base = (uint64_t)blockIdx.x * LN_TILE;
    const uint64_t my0 = base + (uint64_t)threadIdx.x * LN_BPT;
    uint32_t w[LN_NW], prev;
    load64(buf, n, base, my0, w, &prev);
    uint64_t sm, em;
    masks(w, prev, &sm, &em);
    uint64_t v = ((uint64_t)__popcll(sm) << 31) | (uint64_t)__popcll(em);
    v = wave_sum(v);
    if (lane_id() == 0) s_red[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) tot[blockIdx.x] = s_red[0] + s_red[1] + s_red[2] + s_red[3];
}

// ROUTE (the piece partition's pass 1, k_lines_route): each record's part (sg_route.hpp) from
// its key0, taken from the staged tile bytes as the keys are, instead of a second pass that
// reads every record's head again (k_range_bytes); the splitters' key0s in LDS.
struct LinesRoute {
    const uint64_t *split_w = nullptr;
    const uint32_t *split_len = nullptr;
    uint32_t ns = 0;
    uint8_t *parts = nullptr;
};

template <bool ROUTE>
__device__ __forceinline__ void lines_body(const uint8_t *__restrict__ buf, uint64_t n, const uint64_t *__restrict__ pre,
                                           uint2 *__restrict__ spans, uint64_t *__restrict__ keys, const LinesRoute &rt) {
    __shared__ __attribute__((aligned(16))) uint8_t s_b[LN_TILE + 16];  // then the tile's span ends
    __shared__ uint64_t s_red[LN_BLOCK / 64];
    __shared__ uint32_t s_x[ROUTE ? 1 : LN_CAP];  // the tile's span starts
    __shared__ uint64_t s_kk[ROUTE ? 1 : LN_CAP];  // and their keys
    __shared__ uint64_t s_k0[ROUTE ? 256 : 1];
    const uint32_t t = threadIdx.x;
    const uint64_t base = (uint64_t)blockIdx.x * LN_TILE;
    const uint64_t my0 = base + (uint64_t)t * LN_BPT;
    if constexpr (ROUTE) {
        for (uint32_t q = t; q < rt.ns; q += LN_BLOCK) s_k0[q] = split_key0(rt.split_w, rt.split_len, q);
    }
    uint32_t w[LN_NW], prev;
    load64(buf, n, base, my0, w, &prev);
    const bool stage = ROUTE || keys;
    if (stage) {
#pragma unroll
        for (int j = 0; j < LN_NW / 4; ++j)
            reinterpret_cast<uint4 *>(s_b)[(LN_NW / 4) * t + j] = make_uint4(w[4 * j], w[4 * j + 1], w[4 * j + 2], w[4 * j + 3]);
        if (t < 8) {
            const uint64_t pos = base + LN_TILE + t;
            s_b[LN_TILE + t] = (pos < n) ? buf[pos] : (uint8_t)0x0a;
        }
    }
    uint64_t sm, em;
    masks(w, prev, &sm, &em);
    const uint64_t packed = ((uint64_t)__popcll(sm) << 31) | (uint64_t)__popcll(em);
    uint64_t total;
    const uint64_t excl = block_excl_scan<LN_BLOCK>(packed, &total, s_red);  // includes barriers
    const uint64_t tpre = pre[blockIdx.x];
    const uint64_t p0 = tpre + excl;
    uint32_t si = (uint32_t)(p0 >> 31);
    uint32_t ei = (uint32_t)(p0 & 0x7fffffffu);
    // The tile's spans and keys are assembled in LDS and leave as whole 8-B stores in record order
    // (each record's start and end used to be two 4-B stores from two lane loops, its end
    // often from the next lane or block). S0/E0: the tile's first start and end index; a
    // record started in the previous tile (E0 < S0) has its end written directly.
    const uint32_t S0 = (uint32_t)(tpre >> 31), E0 = (uint32_t)(tpre & 0x7fffffffu);
    const uint32_t ns = (uint32_t)(total >> 31), ne = (uint32_t)(total & 0x7fffffffu);
    // block-uniform; dense tiles and the routing parse (its LDS is one block per CU short,
    // and its part bytes dominate its stores) store directly
    const bool staged = !ROUTE && ns <= LN_CAP;

    uint64_t bits = sm;
    while (bits) {
        const int b = __ffsll((long long)bits) - 1;
        bits &= bits - 1;
        if (staged) s_x[si - S0] = (uint32_t)(my0 + b);
        else spans[si].x = (uint32_t)(my0 + b);
        if (stage) {
            // bytes [q, q+8) from three aligned dwords; tag = first '\n' in them (SWAR: the
            // lowest flagged byte is exact), key = the bytes before it (<= 7), big-endian
            const uint32_t q = t * LN_BPT + b;
            const uint32_t *w32 = reinterpret_cast<const uint32_t *>(s_b) + (q >> 2);
            const uint32_t w0 = w32[0], w1 = w32[1], w2 = w32[2];
            const uint64_t v = (uint64_t)__builtin_amdgcn_alignbyte(w1, w0, q & 3u) |
                               ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, q & 3u) << 32);
            const uint64_t y = v ^ 0x0a0a0a0a0a0a0a0aull;
            const uint64_t z = (y - 0x0101010101010101ull) & ~y & 0x8080808080808080ull;
            const uint32_t rem = z ? (uint32_t)(__builtin_ctzll(z) >> 3) : 8u;
            const uint32_t take = rem < 7u ? rem : 7u;
            const uint64_t m = (1ull << (8u * take)) - 1ull;
            const uint64_t k0 = (__builtin_bswap64(v & m) & ~0xffull) | rem;
            if (keys && staged) s_kk[si - S0] = k0;
            else if (keys) keys[si] = k0;
            if constexpr (ROUTE)
                rt.parts[si] = (uint8_t)route_record(buf, n, (uint32_t)(my0 + b), ~0u, k0, s_k0, rt.ns, rt.split_w,
                                                     rt.split_len);
        }
        ++si;
    }
    if (!staged) {
        bits = em;
        while (bits) {
            const int b = __ffsll((long long)bits) - 1;
            bits &= bits - 1;
            spans[ei].y = (uint32_t)(my0 + b);
            ++ei;
        }
        return;
    }
    __syncthreads();  // s_b (the tile's bytes) is read by the start loop's keys: free after this
    uint32_t *s_y = reinterpret_cast<uint32_t *>(s_b);
    bits = em;
    while (bits) {
        const int b = __ffsll((long long)bits) - 1;
        bits &= bits - 1;
        if (ei >= S0) s_y[ei - S0] = (uint32_t)(my0 + b);
        else spans[ei].y = (uint32_t)(my0 + b);  // the record the previous tile started
        ++ei;
    }
    __syncthreads();
    const uint32_t ended = E0 + ne - S0;  // records [0, ended) of this tile's starts end in it
    for (uint32_t i = t; i < ns; i += LN_BLOCK) {
        if (i < ended) spans[S0 + i] = make_uint2(s_x[i], s_y[i]);
        else spans[S0 + i].x = s_x[i];  // ends in the next tile (which writes .y)
        if (keys) keys[S0 + i] = s_kk[i];
    }
}

__global__ __launch_bounds__(LN_BLOCK) void k_lines(const uint8_t *__restrict__ buf, uint64_t n,
                                                    const uint64_t *__restrict__ pre, uint2 *__restrict__ spans,
                                                    uint64_t *__restrict__ keys) {
    lines_body<false>(buf, n, pre, spans, keys, LinesRoute{});
}

__global__ __launch_bounds__(LN_BLOCK) void k_lines_route(const uint8_t *__restrict__ buf, uint64_t n,
                                                          const uint64_t *__restrict__ pre, uint2 *__restrict__ spans,
                                                          const LinesRoute rt) {
    lines_body<true>(buf, n, pre, spans, nullptr, rt);
}

// Two buffers parsed with ONE host sync for both record counts (the dedup's prior and
// current scan): both count passes and tile scans are queued, both totals come back
// together, then both apply passes.
int run_lines2(sg_ctx *c, const uint8_t *a, uint64_t na, const SlotSet &sa, Lines *la, const uint8_t *b, uint64_t nb,
               const SlotSet &sb, Lines *lb) {
    const uint8_t *bufs[2] = {a, b};
    const uint64_t ns[2] = {na, nb};
    const SlotSet *ss[2] = {&sa, &sb};
    Lines *outs[2] = {la, lb};
    uint64_t *totals[2], *pres[2];
    uint32_t nts[2];
    for (int k = 0; k < 2; ++k) {
        if (ns[k] > MAX_BYTES) { set_error("buffer of %llu bytes exceeds the 4 GiB per-call limit", (unsigned long long)ns[k]); return SG_E_TOO_LARGE; }
        if (((uintptr_t)bufs[k] & 15) != 0) { set_error("run_lines: device buffer not 16-byte aligned"); return SG_E_INVAL; }
        const uint32_t ntiles = (uint32_t)(ns[k] / LN_TILE + 1);
        uint64_t *tp;
        SG_TRY(slot(c, ss[k]->lb, 2 * (size_t)ntiles + 4, &tp));
        uint64_t *tot = tp;
        pres[k] = tp + ntiles;
        totals[k] = tp + 2 * (size_t)ntiles;
        nts[k] = ntiles;
        // both totals side by side in the first buffer's slot (its spare words): one copy back
        if (k == 1) totals[1] = totals[0] + 1;
        SG_LAUNCH(c, "lines.count", k_lines_count, ntiles, LN_BLOCK, 0, bufs[k], ns[k], tot);
        SG_TRY(tile_scan(c, tot, ntiles, pres[k], totals[k]));
        prof_bytes(c, "lines.count", (double)ns[k]);
    }
    uint8_t *pin = (uint8_t *)c->pinned;
    SG_HIP(hipMemcpyAsync(pin, totals[0], 16, hipMemcpyDeviceToHost, c->stream));
    SG_HIP(hipStreamSynchronize(c->stream));
    for (int k = 0; k < 2; ++k) {
        uint64_t tv;
        memcpy(&tv, pin + 8 * k, 8);
        const uint32_t R = (uint32_t)(tv >> 31);
        if (R != (uint32_t)(tv & 0x7fffffffu)) { set_error("run_lines: start/end count mismatch"); return SG_E_HIP; }
        Lines *out = outs[k];
        SG_TRY(slot(c, ss[k]->starts, (size_t)R + 1, &out->spans));
        SG_TRY(slot(c, ss[k]->keys, (size_t)R + 1, &out->keys));
        SG_LAUNCH(c, "lines", k_lines, nts[k], LN_BLOCK, 0, bufs[k], ns[k], pres[k], out->spans, out->keys);
        out->n_rec = R;
        out->tile_excl = pres[k];
        out->tile_bytes = LN_TILE;
        out->n_tiles = nts[k];
        prof_bytes(c, "lines", (double)ns[k] + 16.0 * R);
    }
    return SG_OK;
}

int run_lines(sg_ctx *c, const uint8_t *d_buf, uint64_t n, const SlotSet &ss, Lines *out, bool want_keys, bool apply) {
    if (n > MAX_BYTES) { set_error("buffer of %llu bytes exceeds the 4 GiB per-call limit", (unsigned long long)n); return SG_E_TOO_LARGE; }
    if (((uintptr_t)d_buf & 15) != 0) { set_error("run_lines: device buffer not 16-byte aligned"); return SG_E_INVAL; }
    const uint32_t ntiles = (uint32_t)(n / LN_TILE + 1);
    uint64_t *tp;  // tot[ntiles] | pre[ntiles] | total
    SG_TRY(slot(c, ss.lb, 2 * (size_t)ntiles + 4, &tp));
    uint64_t *tot = tp, *pre = tp + ntiles, *total = tp + 2 * (size_t)ntiles;
    SG_LAUNCH(c, "lines.count", k_lines_count, ntiles, LN_BLOCK, 0, d_buf, n, tot);
    SG_TRY(tile_scan(c, tot, ntiles, pre, total));
    uint64_t tv = 0;
    SG_TRY(ctx_readback(c, &tv, total, 8));
    const uint32_t R = (uint32_t)(tv >> 31);
    if (R != (uint32_t)(tv & 0x7fffffffu)) { set_error("run_lines: start/end count mismatch"); return SG_E_HIP; }
    SG_TRY(slot(c, ss.starts, (size_t)R + 1, &out->spans));
    out->keys = nullptr;
    if (want_keys) SG_TRY(slot(c, ss.keys, (size_t)R + 1, &out->keys));
    if (apply) SG_LAUNCH(c, "lines", k_lines, ntiles, LN_BLOCK, 0, d_buf, n, pre, out->spans, out->keys);
    out->n_rec = R;
    out->tile_excl = pre;
    out->tile_bytes = LN_TILE;
    out->n_tiles = ntiles;
    // text read twice (count + apply) + (start, end[, key0]) per record
    if (apply) prof_bytes(c, "lines", (double)n + (want_keys ? 16.0 : 8.0) * R);
    prof_bytes(c, "lines.count", (double)n);
    return SG_OK;
}

// The piece partition's parse in two halves: lines_count_scan queues the count pass and its
// tile scan (tp: tot | pre | total, 2 * lines_tiles(n) + 4 words; the packed record count at
// tp[2 * nt], read back by the caller with the other pieces'), lines_route_apply the
// apply pass with routing (spans and one part byte per record).
uint32_t lines_tiles(uint64_t n) { return (uint32_t)(n / LN_TILE + 1); }

int lines_count_scan(sg_ctx *c, const uint8_t *d_buf, uint64_t n, uint64_t *tp) {
    if (n > MAX_BYTES) { set_error("buffer of %llu bytes exceeds the 4 GiB per-call limit", (unsigned long long)n); return SG_E_TOO_LARGE; }
    if (((uintptr_t)d_buf & 15) != 0) { set_error("run_lines: device buffer not 16-byte aligned"); return SG_E_INVAL; }
    const uint32_t nt = lines_tiles(n);
    SG_LAUNCH(c, "lines.count", k_lines_count, nt, LN_BLOCK, 0, d_buf, n, tp);
    SG_TRY(tile_scan(c, tp, nt, tp + nt, tp + 2 * (size_t)nt));
    prof_bytes(c, "lines.count", (double)n);
    return SG_OK;
}

int lines_route_apply(sg_ctx *c, const uint8_t *d_buf, uint64_t n, const uint64_t *tp, uint32_t R, uint2 *spans,
                      const uint64_t *split_w, const uint32_t *split_len, uint32_t ns, uint8_t *parts) {
    const uint32_t nt = lines_tiles(n);
    const LinesRoute rt{split_w, split_len, ns, parts};
    SG_LAUNCH(c, "lines", k_lines_route, nt, LN_BLOCK, 0, d_buf, n, tp + nt, spans, rt);
    // text read once more + (start, end) and a part byte per record
    prof_bytes(c, "lines", (double)n + 9.0 * R);
    return SG_OK;
}

}  // namespace sg

