// sg_emit.hpp — "emit": order-preserving select + byte-offset scan + record copy, as a
// reduce-then-scan pair (k_emit_count -> k_tile_scan -> k_emit_<use>).
//
// Item i (0 <= i < n) names a record of `src` by (start, len) and whether it is kept. Kept
// records are written to `dst` in item order, each '\n'-terminated; optionally the j-th
// kept record's output span (o, o + len) and a per-item u64 payload (the sort key) are
// written at j. Used for: materialising the sorted records (gather through a permutation),
// compacting the unique records out of the sorted buffer, the new-record output, and
// serialising partitions / match output.
//
// Tile = 4 waves x 4 rounds x 64 items. The apply pass scans each wave's 256 items' packed
// (count:32 | bytes:32) values and adds the tile prefix. The copy then goes round by round:
// the kept records of one round are one contiguous output span, assembled in a per-wave LDS
// window and written with 16-byte stores. A record whose aligned source span is <= 64 B is
// loaded by its own lane (four 16-B loads, the wave's loads all in flight together) and
// placed with dword stores built by funnel shifts; longer records are copied by 16-lane
// groups with coalesced word loads. Spans wider than the window go straight to HBM.
//
// Limits: fewer than 2^32 kept records and 2^32 output bytes per launch (checked by callers).
#pragma once
#include "sg_common.hpp"

namespace sg {

constexpr int EM_BLOCK = 256;
constexpr int EM_ROUNDS = 4;
constexpr uint32_t EM_TILE = EM_BLOCK * EM_ROUNDS;
// Per-wave LDS output window: a round's 64 records are assembled there when their span fits
// (else written straight from registers). Short-record inputs use the small window, which
// leaves room for 5 blocks per CU instead of 4 (C2 unique emit 253 -> 239 us); long records
// (httpx lines, ~100 B) need the large one (X1: 395 us with it, 495 with the small one).
constexpr uint32_t EM_WIN = 6144;
constexpr uint32_t EM_WIN_S = 3072;
constexpr uint64_t EM_ONE = 1ull << 32;

// Per-lane copy of a short record (aligned source span <= 64 B) whose 16-byte source
// chunks are already in registers: bytes [sh, sh+len) of c[] go to d[0..len), then '\n'.
template <class Ptr>
__device__ __forceinline__ void put_short(Ptr d, const uint4 (&c)[4], uint32_t sh, uint32_t len) {
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
        const uint32_t w4[4] = {c[k].x, c[k].y, c[k].z, c[k].w};
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) {
#pragma unroll
            for (uint32_t b = 0; b < 4; ++b) {
                const uint32_t p = 16 * k + 4 * q + b;
                if (p >= sh && p < sh + len) d[p - sh] = (uint8_t)(w4[q] >> (8 * b));
            }
        }
    }
    d[len] = 0x0a;
}

// LDS-window form of put_short. The 64-byte source window c[] is first normalised so the
// record starts at byte 0 (a dword barrel shift by sh>>2 done with mask blends, then a
// byte funnel shift by sh&3), masked (bytes >= len zero, '\n' at len), then re-aligned to
// the destination dword grid (funnel shift by 4 - (d&3)). Whole destination dwords are
// ds_write_b32; only the first and last partial dwords (shared with the neighbouring
// records) are written bytewise. No extra memory traffic beyond the chunk loads.
__device__ __forceinline__ void put_short_win(uint8_t *win, uint32_t d, const uint4 (&c)[4], uint32_t sh,
                                              uint32_t len) {
    const uint32_t dw[18] = {c[0].x, c[0].y, c[0].z, c[0].w, c[1].x, c[1].y, c[1].z, c[1].w,
                             c[2].x, c[2].y, c[2].z, c[2].w, c[3].x, c[3].y, c[3].z, c[3].w, 0u, 0u};
    const uint32_t t = sh >> 2, e = sh & 3u;
    const uint32_t m2 = (t & 2u) ? ~0u : 0u, m1 = (t & 1u) ? ~0u : 0u;
    uint32_t s1[16], s2[15], rec[14];
#pragma unroll
    for (int o = 0; o < 16; ++o) s1[o] = dw[o] ^ ((dw[o] ^ dw[o + 2]) & m2);
#pragma unroll
    for (int o = 0; o < 15; ++o) s2[o] = s1[o] ^ ((s1[o] ^ s1[o + 1]) & m1);
    // record bytes [4o, 4o+4) for o < 13 (len + 1 <= 50 bytes), masked
#pragma unroll
    for (int o = 0; o < 14; ++o) {
        uint32_t x = (o < 13) ? __builtin_amdgcn_alignbyte(s2[o + 1], s2[o], e) : 0u;
        const uint32_t b0 = 4u * o;
        if (b0 + 4u > len) {
            if (b0 <= len) {
                const uint32_t k = len - b0;
                x = (x & ((1u << (8u * k)) - 1u)) | (0x0au << (8u * k));
            } else {
                x = 0u;
            }
        }
        rec[o] = x;
    }
    // destination: bytes [d, d + len + 1); dword j of the grid starting at D = d - f
    const uint32_t f = d & 3u, D = d - f, end = f + len + 1u;  // end: bytes used from D
    const uint32_t mf = f ? ~0u : 0u;
#pragma unroll
    for (int j = 0; j < 14; ++j) {
        const uint32_t lo = (j > 0) ? rec[j - 1] : 0u;
        // f == 0: rec[j]; else bytes (4-f..3) of rec[j-1] then (0..f-1) of rec[j]
        const uint32_t sh_v = __builtin_amdgcn_alignbyte(rec[j], lo, (4u - f) & 3u);
        const uint32_t v = (rec[j] & ~mf) | (sh_v & mf);
        const uint32_t b0 = 4u * j;
        if (b0 >= end) continue;
        if (b0 >= f && b0 + 4u <= end) {
            *reinterpret_cast<uint32_t *>(win + D + b0) = v;
        } else {
#pragma unroll
            for (uint32_t b = 0; b < 4; ++b)
                if (b0 + b >= f && b0 + b < end) win[D + b0 + b] = (uint8_t)(v >> (8 * b));
        }
    }
}

// One 64-byte window of a medium record: bytes [sh, sh + len) of the window c[] (len <=
// 64 - sh) written at base + d, then '\n' when nl. Same normalise / mask / funnel scheme as
// put_short_win, for up to 64 bytes (17 destination dwords); base is an LDS window or HBM.
__device__ __forceinline__ void put_win64(uint8_t *base, uint32_t d, const uint4 (&c)[4], uint32_t sh, uint32_t len,
                                          bool nl) {
    const uint32_t dw[20] = {c[0].x, c[0].y, c[0].z, c[0].w, c[1].x, c[1].y, c[1].z, c[1].w,
                             c[2].x, c[2].y, c[2].z, c[2].w, c[3].x, c[3].y, c[3].z, c[3].w, 0u, 0u, 0u, 0u};
    const uint32_t t = sh >> 2, e = sh & 3u;
    const uint32_t m2 = (t & 2u) ? ~0u : 0u, m1 = (t & 1u) ? ~0u : 0u;
    uint32_t s1[18], s2[17], rec[17];
#pragma unroll
    for (int o = 0; o < 18; ++o) s1[o] = dw[o] ^ ((dw[o] ^ dw[o + 2]) & m2);
#pragma unroll
    for (int o = 0; o < 17; ++o) s2[o] = s1[o] ^ ((s1[o] ^ s1[o + 1]) & m1);
#pragma unroll
    for (int o = 0; o < 17; ++o) {
        uint32_t x = (o < 16) ? __builtin_amdgcn_alignbyte(s2[o + 1], s2[o], e) : 0u;
        const uint32_t b0 = 4u * o;
        if (b0 + 4u > len) {
            if (b0 <= len) {
                const uint32_t k = len - b0;
                x = (x & ((1u << (8u * k)) - 1u)) | (nl ? (0x0au << (8u * k)) : 0u);
            } else {
                x = 0u;
            }
        }
        rec[o] = x;
    }
    const uint32_t f = d & 3u, D = d - f, end = f + len + (nl ? 1u : 0u);
    const uint32_t mf = f ? ~0u : 0u;
#pragma unroll
    for (int j = 0; j < 18; ++j) {
        const uint32_t b0 = 4u * j;
        if (b0 >= end) break;
        const uint32_t cur = (j < 17) ? rec[j] : 0u;
        const uint32_t lo = (j > 0) ? rec[j - 1] : 0u;
        const uint32_t sh_v = __builtin_amdgcn_alignbyte(cur, lo, (4u - f) & 3u);
        const uint32_t v = (cur & ~mf) | (sh_v & mf);
        if (b0 >= f && b0 + 4u <= end) {
            *reinterpret_cast<uint32_t *>(base + D + b0) = v;
        } else {
#pragma unroll
            for (uint32_t b = 0; b < 4; ++b)
                if (b0 + b >= f && b0 + b < end) base[D + b0 + b] = (uint8_t)(v >> (8 * b));
        }
    }
}

// put_win64 for a global destination with fewer store instructions: the record's whole
// destination dwords leave as 16-, 8- and 4-byte stores (dword-aligned vectors), its partial
// first and last dwords as byte + 16-bit + byte stores. A lane-per-record copy issues every
// store instruction any lane of the wave needs: 18 dword and 8 byte stores per window before.
typedef uint32_t sg_u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t sg_u32x2_a4 __attribute__((ext_vector_type(2), aligned(4)));

__device__ __forceinline__ void put_win64_v(uint8_t *base, uint32_t d, const uint4 (&c)[4], uint32_t sh, uint32_t len,
                                            bool nl) {
    const uint32_t dw[20] = {c[0].x, c[0].y, c[0].z, c[0].w, c[1].x, c[1].y, c[1].z, c[1].w,
                             c[2].x, c[2].y, c[2].z, c[2].w, c[3].x, c[3].y, c[3].z, c[3].w, 0u, 0u, 0u, 0u};
    const uint32_t t = sh >> 2, e = sh & 3u;
    const uint32_t m2 = (t & 2u) ? ~0u : 0u, m1 = (t & 1u) ? ~0u : 0u;
    uint32_t s1[18], s2[17], rec[17];
#pragma unroll
    for (int o = 0; o < 18; ++o) s1[o] = dw[o] ^ ((dw[o] ^ dw[o + 2]) & m2);
#pragma unroll
    for (int o = 0; o < 17; ++o) s2[o] = s1[o] ^ ((s1[o] ^ s1[o + 1]) & m1);
#pragma unroll
    for (int o = 0; o < 17; ++o) {
        uint32_t x = (o < 16) ? __builtin_amdgcn_alignbyte(s2[o + 1], s2[o], e) : 0u;
        const uint32_t b0 = 4u * o;
        if (b0 + 4u > len) {
            if (b0 <= len) {
                const uint32_t k = len - b0;
                x = (x & ((1u << (8u * k)) - 1u)) | (nl ? (0x0au << (8u * k)) : 0u);
            } else {
                x = 0u;
            }
        }
        rec[o] = x;
    }
    const uint32_t f = d & 3u, D = d - f, end = f + len + (nl ? 1u : 0u);
    const uint32_t mf = f ? ~0u : 0u;
    // destination dword j (bytes [4j, 4j + 4) from D)
    uint32_t v[18];
#pragma unroll
    for (int j = 0; j < 18; ++j) {
        const uint32_t cur = (j < 17) ? rec[j] : 0u;
        const uint32_t lo = (j > 0) ? rec[j - 1] : 0u;
        const uint32_t sh_v = __builtin_amdgcn_alignbyte(cur, lo, (4u - f) & 3u);
        v[j] = (cur & ~mf) | (sh_v & mf);
    }
    if (end == 0u) return;
    uint8_t *B = base + D;
    const uint32_t je = end >> 2;           // dwords [0, je) end inside the record
    const uint32_t jf = f ? 1u : 0u;       // the first whole dword
    // partial edges: dword 0 when f > 0, dword je when end is not a multiple of 4
    if (f) put_edge(B, v[0], f, je == 0u ? end : 4u);
    if ((end & 3u) && je >= jf) {
        uint32_t vt = 0;
#pragma unroll
        for (int j = 1; j < 18; ++j) vt = (je == (uint32_t)j) ? v[j] : vt;
        if (je == 0u) vt = v[0];
        if (!(f && je == 0u)) put_edge(B + 4u * je, vt, 0u, end & 3u);
    }
    // whole dwords [jf, je): u[k] = v[jf + k]
    const uint32_t ni = je > jf ? je - jf : 0u;
    uint32_t u[17];
#pragma unroll
    for (int k = 0; k < 17; ++k) u[k] = f ? v[k + 1] : v[k];
    uint8_t *A = B + 4u * jf;
#pragma unroll
    for (int g = 0; g < 4; ++g)
        if (4u * g + 4u <= ni)
            *reinterpret_cast<sg_u32x4_a4 *>(A + 16u * g) = sg_u32x4_a4{u[4 * g], u[4 * g + 1], u[4 * g + 2], u[4 * g + 3]};
    const uint32_t r0 = ni & ~3u, rem = ni & 3u;
    auto sel = [&](uint32_t i) -> uint32_t {  // u[i], i in {0, 1, 2, 4, 5, 6, ..., 16}
        uint32_t x = 0;
#pragma unroll
        for (int k = 0; k < 17; ++k) x = (i == (uint32_t)k) ? u[k] : x;
        return x;
    };
    if (rem >= 2u) *reinterpret_cast<sg_u32x2_a4 *>(A + 4u * r0) = sg_u32x2_a4{sel(r0), sel(r0 + 1u)};
    if (rem & 1u) {
        const uint32_t i = r0 + (rem & 2u);
        *reinterpret_cast<uint32_t *>(A + 4u * i) = sel(i);
    }
}

// A medium record (longer than the short path, <= EM_MED bytes) copied by its own lane in
// 64-byte windows: each window's four 16-B loads are issued together, and all lanes of the
// wave copy their records at once (the 16-lane group path copies one record per group at a
// time: a load latency per record).
constexpr uint32_t EM_MED = 1024;

// The record's chunk_key(src, s, s + len, 0) from its first 64-byte window's loads c (record
// start at byte sh <= 15 of the window).
__device__ __forceinline__ uint64_t win_key0(const uint4 (&c)[4], uint32_t sh, uint32_t len) {
    // bytes [sh, sh + 8) of the window: dwords sh / 4 .. sh / 4 + 2 (sh <= 15)
    const uint32_t dw[6] = {c[0].x, c[0].y, c[0].z, c[0].w, c[1].x, c[1].y};
    const uint32_t a = sh >> 2, e = sh & 3u;
    uint32_t w0 = dw[0], w1 = dw[1], w2 = dw[2];
#pragma unroll
    for (uint32_t t = 1; t < 4; ++t)
        if (a == t) { w0 = dw[t]; w1 = dw[t + 1]; w2 = dw[t + 2]; }
    const uint32_t lo = __builtin_amdgcn_alignbyte(w1, w0, e), hi = __builtin_amdgcn_alignbyte(w2, w1, e);
    uint64_t v = (uint64_t)lo | ((uint64_t)hi << 32);
    const uint32_t take = len < 7u ? len : 7u;
    v &= (1ull << (8u * take)) - 1ull;
    return len ? ((__builtin_bswap64(v) & ~0xffull) | (uint64_t)(len < 8u ? len : 8u)) : 0ull;
}

// key0 (optional): the record's chunk_key(src, s, s + len, 0), taken from the first window's
// loads instead of loading its first bytes again.
template <bool KEY = false, bool VEC = false>
__device__ __forceinline__ void put_medium(const uint8_t *src, uint8_t *base, uint32_t d, uint32_t s, uint32_t len,
                                           uint64_t *key0 = nullptr) {
    const uint32_t q0 = s & ~15u, sh = s - q0;
    uint32_t done = 0;
    for (uint32_t wo = 0;; wo += 64u) {
        const uint32_t ws = wo ? 0u : sh;
        const uint32_t wl = min(64u - ws, len - done);
        uint4 c[4];
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k)
            c[k] = (16u * k < ws + wl) ? *reinterpret_cast<const uint4 *>(src + q0 + wo + 16u * k) : make_uint4(0u, 0u, 0u, 0u);
        if (KEY && wo == 0) *key0 = win_key0(c, sh, len);
        const bool nl = done + wl == len;
        if (VEC) put_win64_v(base, d + done, c, ws, wl, nl);
        else put_win64(base, d + done, c, ws, wl, nl);
        done += wl;
        if (nl) break;
    }
}

// Copy the records of one round into out[o0..oend) (base = o0 & ~15): lane-owned record
// (f, s, len, dst offset d from base). Short records: the lane loads its aligned 16-byte
// chunks (all loads of the wave in flight together) and places the bytes. Longer records:
// compacted into s_src/s_len/s_dst and copied by 16-lane groups with coalesced word loads.
// Assembled in the wave's LDS window when the span fits, then written with 16-byte stores.
// TWO: records come from two sources, src (start bit 31 clear) and src2 (bit 31 set).
template <uint32_t WIN = EM_WIN, bool TWO = false>
__device__ __forceinline__ void wave_copy_round(const uint8_t *__restrict__ src0, const uint8_t *__restrict__ src2,
                                                uint8_t *__restrict__ out,
                                                uint8_t *win, uint32_t *s_src, uint32_t *s_len, uint32_t *s_dst,
                                                bool f, uint32_t s_in, uint32_t len, uint32_t d, uint64_t o0,
                                                uint64_t oend, uint64_t base) {
    const uint32_t lane = lane_id();
    const uint64_t span = oend - base;
    const bool in_lds = span <= WIN;
    const uint8_t *src = (TWO && (s_in >> 31)) ? src2 : src0;
    const uint32_t s = TWO ? (s_in & 0x7fffffffu) : s_in;
    const uint32_t q0 = s & ~15u, sh = s - q0;
    const bool shortr = f && (sh + len <= 64u) && (len < 50u);
    uint4 c[4];
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
        c[k] = make_uint4(0u, 0u, 0u, 0u);
        if (shortr && 16u * k < sh + len) c[k] = *reinterpret_cast<const uint4 *>(src + q0 + 16u * k);
    }
    const bool medr = f && !shortr && len <= EM_MED;
    const bool longr = f && !shortr && !medr;
    const uint64_t ml = __ballot(longr);
    if (longr) {
        const uint32_t cidx = (uint32_t)__popcll(ml & ((1ull << lane) - 1ull));
        s_src[cidx] = s_in;
        s_len[cidx] = len;
        s_dst[cidx] = d;
    }
    if (shortr) {
        if (in_lds) put_short_win(win, d, c, sh, len);
        else put_short(out + base + d, c, sh, len);
    }
    if (medr) {
        if (in_lds) put_medium(src, win, d, s, len);
        else put_medium<false, true>(src, out + base, d, s, len);
    }
    if (ml) {
        __builtin_amdgcn_wave_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const uint32_t cnt = (uint32_t)__popcll(ml);
        const uint32_t g = lane >> 4, gl = lane & 15;
        for (uint32_t j = g; j < cnt; j += 4) {
            const uint32_t sjr = s_src[j], lj = s_len[j];
            const uint8_t *sbj = (TWO && (sjr >> 31)) ? src2 : src0;
            const uint32_t sj = TWO ? (sjr & 0x7fffffffu) : sjr;
            const uint32_t ej = sj + lj;
            const uint32_t a0 = sj & ~3u;
            uint8_t *dd = (in_lds ? win : out + base) + s_dst[j];
            for (uint32_t a = a0 + 4 * gl; a < ej; a += 64) {
                const uint32_t x = *reinterpret_cast<const uint32_t *>(sbj + a);
#pragma unroll
                for (uint32_t b = 0; b < 4; ++b) {
                    const uint32_t p = a + b;
                    if (p >= sj && p < ej) dd[p - sj] = (uint8_t)(x >> (8 * b));
                }
            }
            if (gl == 0) dd[lj] = 0x0a;
        }
    }
    if (!in_lds) return;
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const uint32_t nch = (uint32_t)((span + 15) / 16);
    for (uint32_t ch = lane; ch < nch; ch += 64) {
        const uint64_t ga = base + 16ull * ch;
        if (ga >= o0 && ga + 16 <= oend)
            *reinterpret_cast<uint4 *>(out + ga) = *reinterpret_cast<const uint4 *>(win + 16 * ch);
    }
    // the partial first and last 16-B chunks (shared with the neighbouring rounds' outputs):
    // one byte per lane, lanes 0-15 the first chunk, 16-31 the last — one store instruction
    // instead of a 16-iteration byte loop per chunk (round 3: 70 % of the emit's store
    // instructions were those loops' masked byte stores)
    if (lane < 32u) {
        const uint32_t ch = (lane < 16u) ? 0u : nch - 1u;
        const uint64_t ga = base + 16ull * ch;
        const uint64_t ad = ga + (lane & 15u);
        const bool partial = ga < o0 || ga + 16 > oend;
        if (partial && ad >= o0 && ad < oend) out[ad] = win[16 * ch + (lane & 15u)];
    }
}

// Reduce-then-scan form (3 launches, no inter-block waits):
//   k_emit_count<Item>: item i -> cache[i] = (start, len) or (0, EM_DROP); per-tile packed
//                       (count << 32 | bytes) aggregate -> tot[tile]
//   k_tile_scan:        exclusive tile prefixes + grand total
//   k_emit_apply:       per tile: re-scan the cached items, add the tile prefix, write
//                       out_spans / kout and copy the records
// The cache makes the apply pass a sequential read even when the item is a gather
// (PermItem: spans[V[i]]).
constexpr uint32_t EM_DROP = 0xffffffffu;

template <class Item>
__global__ __launch_bounds__(EM_BLOCK) void k_emit_count(Item item, uint32_t n, uint2 *__restrict__ cache,
                                                         uint64_t *__restrict__ tot) {
    __shared__ uint64_t s_red[EM_BLOCK / 64];
    const uint32_t base = blockIdx.x * EM_TILE;
    uint64_t sum = 0;
    // every round's item first, then the stores: a cache store between two item loads kept
    // the next round's (possibly aliasing) loads behind it, one latency per round
    uint32_t s[EM_ROUNDS], l[EM_ROUNDS];
    bool f[EM_ROUNDS];
#pragma unroll
    for (int r = 0; r < EM_ROUNDS; ++r) {
        const uint32_t i = base + r * EM_BLOCK + threadIdx.x;
        s[r] = 0;
        l[r] = 0;
        f[r] = (i < n) && item(i, &s[r], &l[r]);
    }
#pragma unroll
    for (int r = 0; r < EM_ROUNDS; ++r) {
        const uint32_t i = base + r * EM_BLOCK + threadIdx.x;
        if (i < n) {
            cache[i] = make_uint2(s[r], f[r] ? l[r] : EM_DROP);
            sum += f[r] ? (EM_ONE | (uint64_t)(l[r] + 1u)) : 0ull;
        }
    }
    sum = wave_sum(sum);
    if (lane_id() == 0) s_red[threadIdx.x >> 6] = sum;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t t = 0;
#pragma unroll
        for (int w = 0; w < EM_BLOCK / 64; ++w) t += s_red[w];
        tot[blockIdx.x] = t;
    }
}

// SPARSE (selections that drop items: unique compaction, new records): the wave's kept
// items are first packed in LDS in output order, then copied 64 per round, so a round is
// not spent on a 64-item slice that keeps only a few records.
template <bool SPARSE, uint32_t WIN = EM_WIN, bool TWO = false>
__device__ __forceinline__ void emit_apply_body(const uint2 *__restrict__ cache, uint32_t n,
                                                const uint64_t *__restrict__ pre,
                                                const uint8_t *__restrict__ src, const uint8_t *__restrict__ src2,
                                                uint8_t *__restrict__ dst,
                                                uint2 *__restrict__ out_spans,
                                                const uint64_t *__restrict__ kin, uint64_t *__restrict__ kout) {
    __shared__ __attribute__((aligned(16))) uint8_t s_win[4][WIN];
    __shared__ uint32_t s_src[4][64], s_len[4][64], s_dst[4][64];
    __shared__ uint64_t s_wt[4];
    constexpr int CK = SPARSE ? EM_ROUNDS * 64 : 1;
    __shared__ uint32_t s_cst[4][CK], s_cln[4][CK], s_co[4][CK];
    const uint32_t tile = blockIdx.x;
    const uint32_t wid = threadIdx.x >> 6, lane = lane_id();
    const uint32_t wbase = tile * EM_TILE + wid * 256u;
    uint32_t st[EM_ROUNDS], ln[EM_ROUNDS];
    uint64_t loc[EM_ROUNDS];
    uint64_t run = 0;
    uint32_t fmask = 0;
    // the rounds' cache entries loaded together (clamped index, no bounds branch: a branch
    // per round kept each load behind the previous round's wait)
    uint2 cvr[EM_ROUNDS];
#pragma unroll
    for (int r = 0; r < EM_ROUNDS; ++r) {
        const uint32_t i = wbase + r * 64u + lane;
        cvr[r] = cache[i < n ? i : n - 1u];
    }
#pragma unroll
    for (int r = 0; r < EM_ROUNDS; ++r) {
        const uint32_t i = wbase + r * 64u + lane;
        const uint2 cv = (i < n) ? cvr[r] : make_uint2(0u, EM_DROP);
        const bool f = cv.y != EM_DROP;
        st[r] = cv.x;
        ln[r] = f ? cv.y : 0u;
        const uint64_t v = f ? (EM_ONE | (uint64_t)(cv.y + 1u)) : 0ull;
        const uint64_t inc = wave_incl_scan(v);
        loc[r] = run + inc - v;
        run += __shfl(inc, 63, 64);
        fmask |= (f ? 1u : 0u) << r;
    }
    if (lane == 0) s_wt[wid] = run;
    __syncthreads();
    uint64_t woff = 0;
#pragma unroll
    for (uint32_t w = 0; w < 4; ++w) woff += (w < wid) ? s_wt[w] : 0ull;
    const uint64_t wpre = pre[tile] + woff;
    if constexpr (SPARSE) {
#pragma unroll
        for (int r = 0; r < EM_ROUNDS; ++r) {
            if (!((fmask >> r) & 1u)) continue;
            const uint64_t gp = wpre + loc[r];
            const uint32_t j = (uint32_t)(gp >> 32);
            const uint32_t o = (uint32_t)gp;
            if (out_spans) out_spans[j] = make_uint2(o, o + ln[r]);
            if (kout) kout[j] = kin[wbase + r * 64u + lane];
            const uint32_t e = (uint32_t)(loc[r] >> 32);  // kept rank within the wave
            s_cst[wid][e] = st[r];
            s_cln[wid][e] = ln[r];
            s_co[wid][e] = o;
        }
        const uint32_t kept = (uint32_t)(run >> 32);
        __builtin_amdgcn_wave_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        for (uint32_t k0 = 0; k0 < kept; k0 += 64u) {
            const uint32_t q = k0 + lane;
            const bool f = q < kept;
            const uint32_t s = f ? s_cst[wid][q] : 0u, l = f ? s_cln[wid][q] : 0u, o = f ? s_co[wid][q] : 0u;
            const uint32_t last = (kept - k0 >= 64u) ? 63u : kept - k0 - 1u;
            const uint64_t o0 = (uint32_t)__shfl((int)o, 0, 64);
            const uint64_t oend = (uint32_t)__shfl((int)(o + l + 1u), (int)last, 64);
            const uint64_t base = o0 & ~15ull;
            wave_copy_round<WIN, TWO>(src, src2, dst, s_win[wid], s_src[wid], s_len[wid], s_dst[wid], f, s, l,
                                      (uint32_t)(o - base), o0, oend, base);
            __builtin_amdgcn_wave_barrier();
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
        return;
    }
#pragma unroll
    for (int r = 0; r < EM_ROUNDS; ++r) {
        const bool f = (fmask >> r) & 1u;
        const uint64_t m = __ballot(f);
        if (!m) continue;
        const uint64_t gp = wpre + loc[r];
        const uint32_t j = (uint32_t)(gp >> 32);
        const uint64_t o = (uint32_t)gp;
        if (f) {
            if (out_spans) out_spans[j] = make_uint2((uint32_t)o, (uint32_t)o + ln[r]);
            if (kout) kout[j] = kin[wbase + r * 64u + lane];
        }
        const uint32_t first = (uint32_t)(__ffsll((long long)m) - 1);
        const uint32_t last = 63u - (uint32_t)__clzll((long long)m);
        const uint64_t o0 = __shfl(o, (int)first, 64);
        const uint64_t oend = __shfl(o + ln[r] + 1u, (int)last, 64);
        const uint64_t base = o0 & ~15ull;
        wave_copy_round<WIN, TWO>(src, src2, dst, s_win[wid], s_src[wid], s_len[wid], s_dst[wid], f, st[r], ln[r],
                        (uint32_t)(o - base), o0, oend, base);
        __builtin_amdgcn_wave_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
}

#ifndef SG_EMIT_DEVICE_ONLY  // (a translation unit that only needs the copy helpers)
// One symbol per use, so rocprofv3 kernel stats and PMC passes attribute each separately.
#define SG_EMIT_APPLY(NAME, SPARSE, WIN)                                                            \
    __global__ __launch_bounds__(EM_BLOCK) void NAME(                                               \
        const uint2 *__restrict__ cache, uint32_t n, const uint64_t *__restrict__ pre,              \
        const uint8_t *__restrict__ src, uint8_t *__restrict__ dst, uint2 *__restrict__ out_spans,  \
        const uint64_t *__restrict__ kin, uint64_t *__restrict__ kout) {                            \
        emit_apply_body<SPARSE, WIN>(cache, n, pre, src, nullptr, dst, out_spans, kin, kout);       \
    }
SG_EMIT_APPLY(k_emit_uniq, true, EM_WIN)
SG_EMIT_APPLY(k_emit_uniq_s, true, EM_WIN_S)
SG_EMIT_APPLY(k_emit_fresh, true, EM_WIN)
SG_EMIT_APPLY(k_emit_apply, false, EM_WIN)
#undef SG_EMIT_APPLY
#endif

// ------------------------------------------------------------------ common items
// Sorted position i -> input record V[i] (V null: record i).
struct PermItem {
    const uint32_t *V;
    const uint2 *spans;
    __device__ bool operator()(uint32_t i, uint32_t *s, uint32_t *l) const {
        const uint2 sp = spans[V ? V[i] : i];
        *s = sp.x;
        *l = sp.y - sp.x;
        return true;
    }
};

// Record i by its span, kept where flag[i] == want.
struct FlagItem {
    const uint2 *spans;
    const uint8_t *flag;
    uint8_t want;
    __device__ bool operator()(uint32_t i, uint32_t *s, uint32_t *l) const {
        if (flag[i] != want) return false;
        const uint2 sp = spans[i];
        *s = sp.x;
        *l = sp.y - sp.x;
        return true;
    }
};

}  // namespace sg
