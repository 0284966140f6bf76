// sg_bucket.hip — A7 sort -u + A8 new-record diff as a two-level bucket sample sort whose
// splitters are records of the prior scan (the previous sort -u output, already in byte order).
//
// The radix pipeline (sg_dedup.hip) sorts (key0, id) pairs in 7 LSD passes and then gathers
// every record at random to materialise the sorted order (~2.9x HBM over-fetch). Here record
// BYTES move, in coalesced 64-B-aligned runs, twice, and every final bucket is small enough
// to be sorted, deduplicated and diffed entirely in LDS:
//
//   pick     splitter j = the first prior record starting at or after byte j*W (W = prior
//            bytes / NB): byte-window quantiles of a sorted buffer need no record count, so
//            nothing waits for the host. Prior slice f = the prior records in
//            [splitter f, splitter f+1): exactly the prior records of cur bucket f.
//   L1 pass  every 48-KiB tile of the current buffer: records -> one of NB1 coarse buckets
//            (every NB2-th splitter; key0 binary search in LDS, byte compare against the
//            splitter record on key0 ties). count pass -> per-(bucket, tile) run sizes padded
//            to 64 B -> column scan -> apply pass assembles the tile's runs in LDS and writes
//            them with aligned 16-B stores ('\n' padding = empty lines, which parsing drops).
//   L2 pass  the same inside each coarse bucket, into its NB2 final buckets.
//   sort     one block per final bucket (NB = NB1*NB2, ~15 KB of records each): load the
//            bucket and its prior slice into LDS, parse both, bitonic sort of (key0, span) with
//            LDS byte compares on key0 ties, adjacent-equal dedup, membership of each unique
//            record in the slice by binary search, then the unique and new records written
//            in order (16-B stores) into the bucket's slot.
//   compact  the slots concatenated in bucket order (unaligned shift copy): the outputs.
//
// One host sync per call (the final sizes and the error word). Anything the LDS bounds do
// not cover — a record longer than the tile overhang, a bucket or slice over its LDS budget,
// a prior that is not strictly increasing — sets the error word and the caller runs the
// radix pipeline instead, so the result is exact for every input.
#include "sg_internal.hpp"

#include <math.h>
#include <stdlib.h>
#include <string.h>

namespace sg {

enum : uint32_t { BK_F_LONG = 1u, BK_F_CUR_CAP = 2u, BK_F_PRIOR_CAP = 4u, BK_F_UNSORTED = 8u };

// ------------------------------------------------------------------ L1/L2 pass geometry
constexpr int BP_THREADS = 1024;
constexpr uint32_t BP_SEG = 48;                      // bytes per thread
constexpr uint32_t BP_TILE = BP_THREADS * BP_SEG;    // 48 KiB
constexpr uint32_t BP_OVH = 2048;                    // longest record that may cross a tile end
constexpr uint32_t BP_PAD = 64;                      // run alignment ('\n' padding)
constexpr uint32_t BP_MAXB = 256;                    // buckets per level
constexpr uint32_t BP_IB = 16;                       // LDS offset of the tile's first byte
constexpr uint32_t BP_STAGE = BP_TILE + BP_OVH;
constexpr uint32_t BP_OUTCAP = BP_STAGE + BP_PAD * BP_MAXB;

// ------------------------------------------------------------------ final bucket geometry
constexpr int BS_THREADS = 512;
constexpr uint32_t BS_CCAP = 32768;   // cur bucket bytes (64 B per thread)
constexpr uint32_t BS_PCAP = 16384;   // prior slice bytes incl. 16-B alignment slack (32 B per thread)
constexpr uint32_t BS_NP = 640;       // prior records

constexpr uint32_t BK_SPFX = 32;      // splitter prefix bytes cached for LDS compares

__device__ __forceinline__ uint32_t ld4(const uint8_t *s, uint32_t p) {
    const uint32_t *w = reinterpret_cast<const uint32_t *>(s + (p & ~3u));
    return __builtin_amdgcn_alignbyte(w[1], w[0], p & 3u);
}

// key0 of the record starting at LDS byte q (bytes up to q + 12 readable): bytes [q, q+7)
// big-endian << 8 | tag = min(len, 8), the record ending at its first '\n'.
__device__ __forceinline__ uint64_t lds_key0(const uint8_t *s, uint32_t q) {
    const uint32_t *w32 = reinterpret_cast<const uint32_t *>(s + (q & ~3u));
    const uint32_t w0 = w32[0], w1 = w32[1], w2 = w32[2];
    const uint64_t v = (uint64_t)__builtin_amdgcn_alignbyte(w1, w0, q & 3u) |
                       ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, q & 3u) << 32);
    const uint64_t y = v ^ 0x0a0a0a0a0a0a0a0aull;
    const uint64_t z = (y - 0x0101010101010101ull) & ~y & 0x8080808080808080ull;
    const uint32_t rem = z ? (uint32_t)(__builtin_ctzll(z) >> 3) : 8u;
    const uint32_t take = rem < 7u ? rem : 7u;
    const uint64_t m = (1ull << (8u * take)) - 1ull;
    return (__builtin_bswap64(v & m) & ~0xffull) | rem;
}

// memcmp-then-length of two LDS records from byte `off`, 4 bytes per step.
__device__ __forceinline__ int lds_cmp(const uint8_t *ba, uint32_t sa, uint32_t la, const uint8_t *bb, uint32_t sb,
                                       uint32_t lb, uint32_t off) {
    const uint32_t m = la < lb ? la : lb;
    for (uint32_t o = off; o < m; o += 4) {
        uint32_t x = ld4(ba, sa + o), y = ld4(bb, sb + o);
        const uint32_t r = m - o;
        if (r < 4u) {
            const uint32_t mk = (1u << (8u * r)) - 1u;
            x &= mk;
            y &= mk;
        }
        if (x != y) return __builtin_bswap32(x) < __builtin_bswap32(y) ? -1 : 1;
    }
    return la < lb ? -1 : (la > lb ? 1 : 0);
}

// An LDS record against a global one (splitter records), bytewise from `off`.
__device__ __noinline__ int lds_glob_cmp(const uint8_t *s, uint32_t q, uint32_t len, const uint8_t *P, uint2 sp,
                                         uint32_t off) {
    const uint32_t lb = sp.y - sp.x;
    const uint32_t m = len < lb ? len : lb;
    for (uint32_t o = off; o < m; ++o) {
        const uint32_t x = s[q + o], y = P[sp.x + o];
        if (x != y) return x < y ? -1 : 1;
    }
    return len < lb ? -1 : (len > lb ? 1 : 0);
}

__device__ __forceinline__ uint32_t nl_mask4b(uint32_t x) {
    const uint32_t y = x ^ 0x0a0a0a0au;
    const uint32_t r = ~(((y & 0x7f7f7f7fu) + 0x7f7f7f7fu) | y | 0x7f7f7f7fu);
    return ((r >> 7) & 1u) | ((r >> 14) & 2u) | ((r >> 21) & 4u) | ((r >> 28) & 8u);
}

// Newline mask of NW dwords at LDS s + p (p 4-aligned).
template <int NW>
__device__ __forceinline__ uint64_t lds_nl_mask(const uint8_t *s, uint32_t p) {
    const uint32_t *w = reinterpret_cast<const uint32_t *>(s + p);
    uint64_t m = 0;
#pragma unroll
    for (int j = 0; j < NW; ++j) m |= (uint64_t)nl_mask4b(w[j]) << (4 * j);
    return m;
}

// First '\n' at or after LDS byte q (the region is '\n'-terminated by construction).
__device__ __forceinline__ uint32_t lds_find_nl(const uint8_t *s, uint32_t q) {
    uint32_t a = q & ~3u;
    uint32_t m = nl_mask4b(*reinterpret_cast<const uint32_t *>(s + a)) & (0xfu << (q - a));
    while (!m) {
        a += 4;
        m = nl_mask4b(*reinterpret_cast<const uint32_t *>(s + a));
    }
    return a + (uint32_t)__builtin_ctz(m);
}

// ------------------------------------------------------------------ splitters
// One wave per splitter j in 0..NB: span[j] = (start, end) of the first prior record starting
// at or after byte j*W (np when none), key[j] its key0 (~0 when none). span[0] = 0, span[NB] = np.
__global__ __launch_bounds__(256) void k_bk_pick(const uint8_t *__restrict__ P, uint64_t np, uint64_t W, uint32_t NB,
                                                 uint64_t *__restrict__ key, uint2 *__restrict__ span,
                                                 uint8_t *__restrict__ pfx) {
    const uint32_t j = blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t lane = lane_id();
    if (j > NB) return;
    if (j == 0 || j == NB) {
        if (lane == 0) {
            key[j] = j == 0 ? 0ull : ~0ull;
            span[j] = j == 0 ? make_uint2(0u, 0u) : make_uint2((uint32_t)np, (uint32_t)np);
        }
        return;
    }
    uint64_t p = np;
    for (uint64_t base = (uint64_t)j * W; base < np; base += 64) {
        const uint64_t q = base + lane;
        const bool st = q < np && P[q] != 0x0a && (q == 0 || P[q - 1] == 0x0a);
        const uint64_t m = __ballot(st);
        if (m) { p = base + (uint64_t)(__ffsll((long long)m) - 1); break; }
    }
    if (p >= np) {
        if (lane == 0) { key[j] = ~0ull; span[j] = make_uint2((uint32_t)np, (uint32_t)np); }
        return;
    }
    uint64_t e = np;
    for (uint64_t base = p; base < np; base += 64) {
        const uint64_t q = base + lane;
        const uint64_t m = __ballot(q < np && P[q] == 0x0a);
        if (m) { e = base + (uint64_t)(__ffsll((long long)m) - 1); break; }
    }
    if (lane < BK_SPFX) pfx[(size_t)j * BK_SPFX + lane] = p + lane < e ? P[p + lane] : 0;
    if (lane == 0) {
        const uint32_t len = (uint32_t)(e - p);
        const uint32_t take = len < 7u ? len : 7u;
        uint64_t v = 0;
        for (uint32_t i = 0; i < take; ++i) v |= (uint64_t)P[p + i] << (56 - 8 * i);
        key[j] = v | (len < 8u ? len : 8u);
        span[j] = make_uint2((uint32_t)p, (uint32_t)e);
    }
}

// ------------------------------------------------------------------ L1 / L2 passes
struct BPArgs {
    const uint8_t *src;       // L1: the current buffer; L2: the L1 output
    uint64_t n;               // L1: bytes of src
    uint32_t NT1, NB1, NB2;
    const uint64_t *base1;    // [NB1 + 1] coarse bucket offsets in the L1 output
    const uint64_t *tot1;     // [NB1] coarse bucket bytes
    const uint32_t *ts;       // [NB1 + 1] first L2 tile of each coarse bucket; ts[NB1] = L2 tiles
    const uint64_t *skey;     // final splitters: key0 [NB + 1]
    const uint2 *sspan;       //   and (start, end) in P
    const uint8_t *spfx;      //   and their first BK_SPFX bytes (zero-padded)
    const uint8_t *P;         // prior buffer
    uint32_t *cnt;            // L1: [NB1][NT1] run bytes; L2: [tile][NB2]
    const uint64_t *base2;    // [NB] final bucket offsets in the L2 output
    uint8_t *out;             // the level's output buffer
    uint32_t *flags;
    unsigned long long *dbg;  // phase timers (SG_BK_DEBUG; null: off): [kernel][phase]
    uint32_t *recs;           // per tile: BP_MAXREC record entries (count pass -> apply pass)
    uint32_t *nrec;           // per tile: records in the list
};

struct BPTile {
    uint64_t begin, end, rend;  // tile [begin, end) in src; its region ends at rend
    bool prev_nl;               // the byte before `begin` is a record boundary
    uint32_t tile, parent;      // L1: tile index; L2: global L2 tile index and coarse bucket
    uint32_t first, stride, ns, nbk;  // splitter table: entry i = final splitter first + i*stride
};

template <int LEVEL>
__device__ __forceinline__ bool bp_tile(const BPArgs &a, BPTile *t) {
    if (LEVEL == 1) {
        t->tile = blockIdx.x;
        t->begin = (uint64_t)blockIdx.x * BP_TILE;
        t->rend = a.n;
        t->end = t->begin + BP_TILE < a.n ? t->begin + BP_TILE : a.n;
        t->prev_nl = blockIdx.x == 0 || a.src[t->begin - 1] == 0x0a;
        t->parent = 0;
        t->first = a.NB2;
        t->stride = a.NB2;
        t->ns = a.NB1 - 1;
        t->nbk = a.NB1;
        return t->begin < a.n;
    } else {
        const uint32_t t2 = blockIdx.x;
        if (t2 >= a.ts[a.NB1]) return false;
        uint32_t lo = 0, hi = a.NB1;  // last p with ts[p] <= t2
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (a.ts[mid] <= t2) lo = mid; else hi = mid;
        }
        const uint32_t p = lo;
        const uint64_t r0 = a.base1[p];
        t->tile = t2;
        t->parent = p;
        t->begin = r0 + (uint64_t)(t2 - a.ts[p]) * BP_TILE;
        t->rend = r0 + a.tot1[p];
        t->end = t->begin + BP_TILE < t->rend ? t->begin + BP_TILE : t->rend;
        t->prev_nl = true;  // tiles start at a record start or inside '\n' padding
        if (t->begin > r0) t->prev_nl = a.src[t->begin - 1] == 0x0a;
        t->first = p * a.NB2 + 1;
        t->stride = 1;
        t->ns = a.NB2 - 1;
        t->nbk = a.NB2;
        return true;
    }
}

// Stage [begin, min(end + OVH, rend)) at s_in + BP_IB, the boundary byte before it, and 32
// bytes of '\n' after it. Returns the staged length.
__device__ __forceinline__ uint32_t bp_stage(const BPArgs &a, const BPTile &t, uint8_t *s_in) {
    const uint64_t se = t.end + BP_OVH < t.rend ? t.end + BP_OVH : t.rend;
    const uint32_t sn = (uint32_t)(se - t.begin);
    const uint32_t nfull = sn / 16;
    const uint4 *g = reinterpret_cast<const uint4 *>(a.src + t.begin);
    for (uint32_t c = threadIdx.x; c < nfull; c += BP_THREADS)
        reinterpret_cast<uint4 *>(s_in + BP_IB)[c] = g[c];
    for (uint32_t q = nfull * 16 + threadIdx.x; q < sn; q += BP_THREADS) s_in[BP_IB + q] = a.src[t.begin + q];
    if (threadIdx.x < 32) s_in[BP_IB + sn + threadIdx.x] = 0x0a;
    if (threadIdx.x == 0) s_in[BP_IB - 1] = t.prev_nl ? 0x0a : 0x00;
    return sn;
}

// Splitter table in LDS: key0, length and the first BK_SPFX bytes of every table splitter.
struct BPTab {
    uint64_t key[BP_MAXB];
    uint32_t len[BP_MAXB];
    __attribute__((aligned(16))) uint8_t pfx[BP_MAXB][BK_SPFX];
};

// Record (LDS s + q, len) against table splitter i from byte `off`: the cached prefix decides
// unless both share all BK_SPFX bytes (then the prior's bytes in HBM).
__device__ __forceinline__ int bp_tab_cmp(const uint8_t *s, uint32_t q, uint32_t len, const BPTab &tb, uint32_t i,
                                          const BPArgs &a, const BPTile &t, uint32_t off) {
    const uint32_t sl = tb.len[i];
    const uint32_t m = len < sl ? len : sl;
    const uint32_t mc = m < BK_SPFX ? m : BK_SPFX;
    for (uint32_t o = off; o < mc; ++o) {
        const uint32_t x = s[q + o], y = tb.pfx[i][o];
        if (x != y) return x < y ? -1 : 1;
    }
    if (m <= BK_SPFX) return len < sl ? -1 : (len > sl ? 1 : 0);
    return lds_glob_cmp(s, q, len, a.P, a.sspan[t.first + i * t.stride], BK_SPFX);
}

// Coarse/fine bucket of the record at LDS s_in + q (length len, key0 k): number of table
// splitters <= record.
__device__ __forceinline__ uint32_t bp_classify(const BPTab &tb, uint64_t k, const uint8_t *s_in, uint32_t q,
                                                uint32_t len, const BPArgs &a, const BPTile &t) {
    const uint64_t *s_tab = tb.key;
    uint32_t lb = 0, ub = 0;
#pragma unroll
    for (uint32_t st = 128; st; st >>= 1) {
        if (s_tab[lb + st - 1] < k) lb += st;
        if (s_tab[ub + st - 1] <= k) ub += st;
    }
    if (ub == lb || (k & 0xffu) < 8u) return ub;
    // splitters [lb, ub) share the record's first 7 bytes; they are in byte order, so the
    // number of them <= the record is a binary search by byte compare
    uint32_t lo = lb, hi = ub;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (bp_tab_cmp(s_in, q, len, tb, mid, a, t, 7) >= 0) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// Record starts of this thread's 48-B segment of the tile (bit b: a record starts at s0 + b)
// and the segment's newline mask.
__device__ __forceinline__ uint64_t bp_starts(const BPTile &t, const uint8_t *s_in, uint64_t *nlm) {
    const uint32_t s0 = threadIdx.x * BP_SEG;
    const uint32_t tl = (uint32_t)(t.end - t.begin);
    *nlm = 0;
    if (s0 >= tl) return 0;
    const uint64_t m = lds_nl_mask<BP_SEG / 4>(s_in + BP_IB, s0);
    const uint32_t prev = s_in[BP_IB + s0 - 1];
    uint64_t sm = ~m & ((m << 1) | (prev == 0x0a ? 1ull : 0ull)) & ((1ull << BP_SEG) - 1ull);
    if (tl - s0 < BP_SEG) sm &= (1ull << (tl - s0)) - 1ull;
    *nlm = m;
    return sm;
}

// Record entry of the per-tile list written by the count pass: start in the tile (16 bits) |
// bucket (8) | length (8; 255 = at least 255, re-measured by the apply pass).
constexpr uint32_t BP_MAXREC = 6144;   // records per tile (average >= 8 B)

__device__ __forceinline__ void bp_load_table(const BPArgs &a, const BPTile &t, BPTab &tb) {
    for (uint32_t i = threadIdx.x; i < BP_MAXB; i += BP_THREADS) {
        const bool ok = i < t.ns;
        tb.key[i] = ok ? a.skey[t.first + i * t.stride] : ~0ull;
        if (ok) {
            const uint2 sp = a.sspan[t.first + i * t.stride];
            tb.len[i] = sp.y - sp.x;
        }
    }
    for (uint32_t c = threadIdx.x; c < t.ns * (BK_SPFX / 16); c += BP_THREADS) {
        const uint32_t i = c / (BK_SPFX / 16), h = c % (BK_SPFX / 16);
        reinterpret_cast<uint4 *>(tb.pfx[i])[h] =
            reinterpret_cast<const uint4 *>(a.spfx + (size_t)(t.first + i * t.stride) * BK_SPFX)[h];
    }
}

// Count pass: every record of the tile classified once; padded run bytes per (bucket, tile)
// into the count matrix and the record list (start, bucket, length) for the apply pass.
template <int LEVEL>
__global__ __launch_bounds__(BP_THREADS) void k_bp_count(BPArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t s_in[BP_IB + BP_STAGE + 48];
    __shared__ BPTab s_tb;
    __shared__ uint32_t s_hist[BP_MAXB];
    __shared__ uint32_t s_red[BP_THREADS / 64];
    BPTile t;
    if (!bp_tile<LEVEL>(a, &t)) return;
    uint64_t t0 = a.dbg ? (uint64_t)wall_clock64() : 0ull, t1 = 0, t2 = 0;
    for (uint32_t i = threadIdx.x; i < BP_MAXB; i += BP_THREADS) s_hist[i] = 0;
    bp_load_table(a, t, s_tb);
    const uint32_t sn = bp_stage(a, t, s_in);
    __syncthreads();
    if (a.dbg) t1 = wall_clock64();
    uint64_t m;
    uint64_t sm = bp_starts(t, s_in, &m);
    uint32_t nrec;
    uint32_t k = block_excl_scan<BP_THREADS>((uint32_t)__popcll(sm), &nrec, s_red);
    if (nrec > BP_MAXREC) {
        if (threadIdx.x == 0) atomicOr(a.flags, BK_F_LONG);
        sm = 0;
    }
    uint32_t *rec = a.recs + (size_t)t.tile * BP_MAXREC;
    const uint32_t s0 = threadIdx.x * BP_SEG;
    while (sm) {
        const uint32_t b = (uint32_t)__builtin_ctzll(sm);
        sm &= sm - 1;
        const uint32_t q = s0 + b;
        const uint64_t after = m >> b;  // '\n' positions from q on inside the segment
        const uint32_t e = after ? q + (uint32_t)__builtin_ctzll(after) : lds_find_nl(s_in + BP_IB, s0 + BP_SEG);
        const uint32_t len = e - q;
        if (e >= sn && t.begin + sn < t.rend) {  // longer than the overhang: the radix pipeline
            atomicOr(a.flags, BK_F_LONG);
            rec[k++] = ~0u;  // skipped by the apply pass
            continue;
        }
        const uint32_t bk = bp_classify(s_tb, lds_key0(s_in + BP_IB, q), s_in + BP_IB, q, len, a, t);
        atomicAdd(&s_hist[bk], len + 1);
        rec[k++] = (q << 16) | (bk << 8) | (len < 255u ? len : 255u);
    }
    if (threadIdx.x == 0) a.nrec[t.tile] = nrec <= BP_MAXREC ? nrec : 0u;
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < t.nbk; b += BP_THREADS) {
        const uint32_t v = (s_hist[b] + BP_PAD - 1) & ~(BP_PAD - 1);
        if (LEVEL == 1) a.cnt[(size_t)b * a.NT1 + t.tile] = v;
        else a.cnt[(size_t)t.tile * a.NB2 + b] = v;
    }
    if (a.dbg && threadIdx.x == 0) {
        t2 = wall_clock64();
        unsigned long long *d = a.dbg + 8 + 8 * (2 * (LEVEL - 1));
        atomicAdd(&d[0], t1 - t0);
        atomicAdd(&d[1], t2 - t1);
        atomicAdd(&d[7], 1ull);
    }
}

// dst[d, d+n) = src[s, s+n) in LDS: head bytes to a 4-B boundary, then aligned dword stores of
// unaligned source words.
__device__ __forceinline__ void lds_copy(uint8_t *dst, uint32_t d, const uint8_t *src, uint32_t s, uint32_t n) {
    uint32_t i = 0;
    for (; i < n && ((d + i) & 3u); ++i) dst[d + i] = src[s + i];
    for (; i + 4 <= n; i += 4) *reinterpret_cast<uint32_t *>(dst + d + i) = ld4(src, s + i);
    for (; i < n; ++i) dst[d + i] = src[s + i];
}

// Apply pass: the tile's records (from the count pass's list) grouped into runs in LDS
// ('\n'-padded to 64 B), each run written with aligned 16-B stores at its place.
template <int LEVEL>
__global__ __launch_bounds__(BP_THREADS) void k_bp_apply(BPArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t s_in[BP_IB + BP_STAGE + 48];
    __shared__ __attribute__((aligned(16))) uint8_t s_out[BP_OUTCAP];
    __shared__ uint64_t s_dst[BP_MAXB];
    __shared__ uint32_t s_hist[BP_MAXB];
    __shared__ uint32_t s_cur[BP_MAXB];
    __shared__ uint32_t s_off[BP_MAXB + 1];
    __shared__ uint32_t s_red[BP_THREADS / 64];
    BPTile t;
    if (!bp_tile<LEVEL>(a, &t)) return;
    uint64_t tp[5] = {a.dbg ? (uint64_t)wall_clock64() : 0ull, 0, 0, 0, 0};
    for (uint32_t i = threadIdx.x; i < BP_MAXB; i += BP_THREADS) {
        s_hist[i] = 0;
        if (i < t.nbk) {
            if (LEVEL == 1) s_dst[i] = a.base1[i] + a.cnt[(size_t)i * a.NT1 + t.tile];
            else s_dst[i] = a.base2[t.parent * a.NB2 + i] + a.cnt[(size_t)t.tile * a.NB2 + i];
        }
    }
    const uint32_t nrec = a.nrec[t.tile];
    const uint32_t *rec = a.recs + (size_t)t.tile * BP_MAXREC;
    constexpr int RPT = (BP_MAXREC + BP_THREADS - 1) / BP_THREADS;
    uint32_t my[RPT];
#pragma unroll
    for (int r = 0; r < RPT; ++r) {
        const uint32_t k = threadIdx.x + r * BP_THREADS;
        my[r] = k < nrec ? rec[k] : 0u;
    }
    bp_stage(a, t, s_in);
    __syncthreads();
    if (a.dbg) tp[1] = wall_clock64();
    // lengths >= 255 re-measured; run sizes per bucket
#pragma unroll
    for (int r = 0; r < RPT; ++r) {
        const uint32_t k = threadIdx.x + r * BP_THREADS;
        if (k >= nrec || my[r] == ~0u) continue;
        uint32_t len = my[r] & 0xffu;
        const uint32_t q = my[r] >> 16;
        if (len == 255u) len = lds_find_nl(s_in + BP_IB, q) - q;
        atomicAdd(&s_hist[(my[r] >> 8) & 0xffu], len + 1);
    }
    __syncthreads();
    if (a.dbg) tp[2] = wall_clock64();
    const uint32_t hv = threadIdx.x < t.nbk ? s_hist[threadIdx.x] : 0u;
    const uint32_t pv = (hv + BP_PAD - 1) & ~(BP_PAD - 1);
    uint32_t total;
    const uint32_t ex = block_excl_scan<BP_THREADS>(pv, &total, s_red);
    if (threadIdx.x < t.nbk) { s_off[threadIdx.x] = ex; s_cur[threadIdx.x] = ex; }
    if (threadIdx.x == 0) s_off[t.nbk] = total;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < RPT; ++r) {
        const uint32_t k = threadIdx.x + r * BP_THREADS;
        if (k >= nrec || my[r] == ~0u) continue;
        const uint32_t q = my[r] >> 16, b = (my[r] >> 8) & 0xffu;
        uint32_t len = my[r] & 0xffu;
        if (len == 255u) len = lds_find_nl(s_in + BP_IB, q) - q;
        const uint32_t pos = atomicAdd(&s_cur[b], len + 1);
        lds_copy(s_out, pos, s_in + BP_IB, q, len);
        s_out[pos + len] = 0x0a;
    }
    // '\n' padding of each run
    if (threadIdx.x < t.nbk)
        for (uint32_t p = ex + hv; p < ex + pv; ++p) s_out[p] = 0x0a;
    __syncthreads();
    if (a.dbg) tp[3] = wall_clock64();
    const uint32_t nck = total / 16;
    for (uint32_t c = threadIdx.x; c < nck; c += BP_THREADS) {
        const uint32_t o = c * 16;
        uint32_t lo = 0, hi = t.nbk;  // last run with s_off <= o
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (s_off[mid] <= o) lo = mid; else hi = mid;
        }
        *reinterpret_cast<uint4 *>(a.out + s_dst[lo] + (o - s_off[lo])) = reinterpret_cast<const uint4 *>(s_out)[c];
    }
    if (a.dbg) {
        __syncthreads();
        if (threadIdx.x == 0) {
            tp[4] = wall_clock64();
            unsigned long long *d = a.dbg + 8 + 8 * (2 * (LEVEL - 1) + 1);
            for (int q = 0; q < 4; ++q) atomicAdd(&d[q], tp[q + 1] - tp[q]);
            atomicAdd(&d[7], 1ull);
        }
    }
}

// Column scan of the L1 counts: exclusive prefix over tiles per coarse bucket, in place; the
// bucket's total into tot1.
__global__ __launch_bounds__(256) void k_bp_cscan1(uint32_t *__restrict__ cnt, uint32_t NT1, uint64_t *__restrict__ tot1) {
    __shared__ uint32_t s_red[4];
    uint32_t *row = cnt + (size_t)blockIdx.x * NT1;
    uint32_t carry = 0;
    for (uint32_t b = 0; b < NT1; b += 256 * 4) {
        const uint32_t i0 = b + threadIdx.x * 4;
        uint32_t v[4], sum = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) { v[j] = (i0 + j < NT1) ? row[i0 + j] : 0u; sum += v[j]; }
        uint32_t tot;
        const uint32_t ex = block_excl_scan<256>(sum, &tot, s_red);
        uint32_t run = carry + ex;
#pragma unroll
        for (int j = 0; j < 4; ++j) { if (i0 + j < NT1) row[i0 + j] = run; run += v[j]; }
        carry += tot;
    }
    if (threadIdx.x == 0) tot1[blockIdx.x] = carry;
}

// Coarse bucket offsets and the L2 tile map (one block).
__global__ __launch_bounds__(256) void k_bp_base1(const uint64_t *__restrict__ tot1, uint32_t NB1,
                                                  uint64_t *__restrict__ base1, uint32_t *__restrict__ ts) {
    __shared__ uint64_t s_red[4];
    const uint32_t t = threadIdx.x;
    const uint64_t v = t < NB1 ? tot1[t] : 0ull;
    const uint64_t nt = (v + BP_TILE - 1) / BP_TILE;
    const uint64_t packed = (nt << 40) | v;  // bytes < 2^40, tiles < 2^24
    uint64_t total;
    const uint64_t ex = block_excl_scan<256>(packed, &total, s_red);
    if (t < NB1) { base1[t] = ex & ((1ull << 40) - 1); ts[t] = (uint32_t)(ex >> 40); }
    if (t == 0) { base1[NB1] = total & ((1ull << 40) - 1); ts[NB1] = (uint32_t)(total >> 40); }
}

// Per coarse bucket, per fine bucket: exclusive prefix of the L2 run sizes over the coarse
// bucket's tiles, in place; totals into tot2[p * NB2 + j].
__global__ __launch_bounds__(256) void k_bp_cscan2(uint32_t *__restrict__ cnt, const uint32_t *__restrict__ ts,
                                                   uint32_t NB2, uint64_t *__restrict__ tot2) {
    const uint32_t p = blockIdx.x, j = threadIdx.x;
    if (j >= NB2) return;
    const uint32_t t0 = ts[p], t1 = ts[p + 1];
    uint32_t run = 0;
    uint32_t t = t0;
    for (; t + 8 <= t1; t += 8) {
        uint32_t v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = cnt[(size_t)(t + u) * NB2 + j];
#pragma unroll
        for (int u = 0; u < 8; ++u) { cnt[(size_t)(t + u) * NB2 + j] = run; run += v[u]; }
    }
    for (; t < t1; ++t) {
        const uint32_t v = cnt[(size_t)t * NB2 + j];
        cnt[(size_t)t * NB2 + j] = run;
        run += v;
    }
    tot2[(size_t)p * NB2 + j] = run;
}

// ------------------------------------------------------------------ final buckets
struct BSArgs {
    const uint8_t *L2;
    const uint64_t *base2, *tot2;  // bucket f: L2[base2[f], base2[f] + tot2[f])
    const uint8_t *P;
    uint64_t np;
    const uint2 *sspan;            // prior slice f = [sspan[f].x, sspan[f+1].x)
    uint32_t NB;
    uint8_t *US, *FS;              // per-bucket slots (same offsets as the L2 output)
    uint64_t *uq, *fq;             // per bucket: records << 32 | bytes
    uint64_t *ncur;                // per bucket: prior records << 32 | cur records
    uint32_t *flags;
    const uint8_t *spfx;           // splitter prefixes (BK_SPFX bytes each)
    unsigned long long *dbg;       // phase timers (null: off)
};

// Parse a '\n'-separated LDS region (bytes past its end read as '\n'; the byte before it is a
// boundary) into record starts s_st[k] and ends s_en[k]; BPT bytes per thread. Returns the
// record count (block-uniform).
template <uint32_t BPT>
__device__ __forceinline__ uint32_t bs_parse(const uint8_t *s, uint32_t limit, uint32_t *s_st, uint32_t *s_en,
                                             uint32_t cap, uint64_t *s_red) {
    const uint32_t s0 = threadIdx.x * BPT;
    // bytes at or past `limit` read as '\n' (no LDS fill needed beyond a small tail)
    uint64_t m = ~0ull;
    if (s0 < limit) {
        m = lds_nl_mask<BPT / 4>(s, s0);
        if (limit - s0 < BPT) m |= ~0ull << (limit - s0);
    }
    const uint32_t prev = (s0 && s0 - 1 < limit) ? s[s0 - 1] : 0x0au;
    const uint64_t full = BPT == 64 ? ~0ull : ((1ull << BPT) - 1ull);
    const uint64_t prevnl = ((m << 1) | (prev == 0x0a ? 1ull : 0ull)) & full;
    const uint64_t sm = ~m & prevnl & full;
    // an end at position q: '\n' at q and a non-'\n' before it; the segment's last record may
    // end in a later segment, which counts that end
    const uint64_t em = m & ~prevnl & full;
    const uint64_t packed = ((uint64_t)__popcll(sm) << 32) | (uint64_t)__popcll(em);
    uint64_t total;
    const uint64_t ex = block_excl_scan<BS_THREADS>(packed, &total, s_red);
    const uint32_t nrec = (uint32_t)(total >> 32);
    if (nrec > cap) return nrec;
    uint32_t si = (uint32_t)(ex >> 32), ei = (uint32_t)ex;
    uint64_t bits = sm;
    while (bits) {
        const uint32_t b = (uint32_t)__builtin_ctzll(bits);
        bits &= bits - 1;
        s_st[si++] = s0 + b;
    }
    bits = em;
    while (bits) {
        const uint32_t b = (uint32_t)__builtin_ctzll(bits);
        bits &= bits - 1;
        s_en[ei++] = s0 + b;
    }
    return nrec;
}

__device__ __forceinline__ int bs_item_cmp(const uint8_t *s, uint64_t ka, uint32_t ma, uint64_t kb, uint32_t mb) {
    if (ka != kb) return ka < kb ? -1 : 1;
    if ((ka & 0xffu) < 8u) return 0;
    return lds_cmp(s, ma & 0xffffu, ma >> 16, s, mb & 0xffffu, mb >> 16, 7);
}

// Phase timers of k_bk_sort (SG_BK_DEBUG=1): wall-clock ticks (100 MHz) per phase, summed
// over blocks by thread 0 of each block.
constexpr int BS_NPH = 6;
constexpr uint32_t BS_NE = 1280;      // cur records per bucket
constexpr int BS_PT = (BS_NE + BS_THREADS - 1) / BS_THREADS;

// Sort inside a bucket without a comparison network. The prior slice is a sorted sample of
// the bucket's own key distribution (the previous scan of the same targets), so each cur
// record's insertion point in the slice (a binary search by key0, bytes on ties) is both its
// membership test for the diff and a sub-bucket: records are placed by insertion point
// (counting sort), then ranked exactly among the few records sharing it by full compares
// (ties by record index: the lowest index of equal records is the first copy).
__device__ __forceinline__ int bs_rec_cmp(const uint8_t *sa, uint64_t ka, uint32_t ma, const uint8_t *sb, uint64_t kb,
                                          uint32_t mb) {
    if (ka != kb) return ka < kb ? -1 : 1;
    if ((ka & 0xffu) < 8u) return 0;
    return lds_cmp(sa, ma & 0xffffu, ma >> 16, sb, mb & 0xffffu, mb >> 16, 7);
}

__global__ __launch_bounds__(BS_THREADS) void k_bk_sort(BSArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t s_cb[BS_CCAP + 64];
    __shared__ __attribute__((aligned(16))) uint8_t s_pb[BS_PCAP + 64];
    // union: parse (starts | ends), then items (key0 | meta | members | per-gap counts, offsets)
    __shared__ __attribute__((aligned(16))) uint8_t s_u[14 * BS_NE + 8 * (BS_NP + 2)];
    __shared__ uint64_t s_pkey[BS_NP];
    __shared__ uint32_t s_pmeta[BS_NP];
    __shared__ uint64_t s_red[BS_THREADS / 64];
    __shared__ __attribute__((aligned(16))) uint8_t s_nx[BK_SPFX];  // next splitter record's prefix
    uint32_t *s_st = reinterpret_cast<uint32_t *>(s_u);
    uint32_t *s_en = s_st + BS_NE;
    uint64_t *s_k0 = reinterpret_cast<uint64_t *>(s_u);                   // [BS_NE]
    uint32_t *s_m = reinterpret_cast<uint32_t *>(s_u + 8 * BS_NE);         // [BS_NE]
    uint16_t *s_mem = reinterpret_cast<uint16_t *>(s_u + 12 * BS_NE);      // [BS_NE]
    uint32_t *s_sc = reinterpret_cast<uint32_t *>(s_u + 14 * BS_NE);       // [BS_NP + 2]
    uint32_t *s_so = s_sc + BS_NP + 2;                                     // [BS_NP + 2]
    uint8_t *s_fl = reinterpret_cast<uint8_t *>(s_u + 12 * BS_NE);         // sorted flags (over members)
    const uint32_t f = blockIdx.x, tid = threadIdx.x;
    uint64_t t_ph[BS_NPH + 1];
    const bool dbg = a.dbg != nullptr;
    if (dbg) t_ph[0] = wall_clock64();
    const uint64_t cb0 = a.base2[f];
    const uint32_t clen = (uint32_t)a.tot2[f];
    const uint64_t pb0 = a.sspan[f].x, pb1 = a.sspan[f + 1].x;
    const uint64_t pa0 = pb0 & ~15ull;
    const bool has_next = f + 1 < a.NB && pb1 < a.np;
    if (a.tot2[f] > BS_CCAP || pb1 - pa0 >= BS_PCAP) {
        if (tid == 0) {
            atomicOr(a.flags, a.tot2[f] > BS_CCAP ? BK_F_CUR_CAP : BK_F_PRIOR_CAP);
            a.uq[f] = 0; a.fq[f] = 0; a.ncur[f] = 0;
        }
        return;
    }
    // ---- stage the bucket, its prior slice and the next splitter's prefix
    {
        const uint4 *g = reinterpret_cast<const uint4 *>(a.L2 + cb0);
        for (uint32_t c = tid; c < clen / 16; c += BS_THREADS) reinterpret_cast<uint4 *>(s_cb)[c] = g[c];
        if (tid < 16) reinterpret_cast<uint32_t *>(s_cb + clen)[tid] = 0x0a0a0a0au;  // over-read tail
        const uint32_t plen = (uint32_t)(pb1 - pa0);
        const uint4 *gp = reinterpret_cast<const uint4 *>(a.P + pa0);
        for (uint32_t c = tid; c < plen / 16; c += BS_THREADS) reinterpret_cast<uint4 *>(s_pb)[c] = gp[c];
        for (uint32_t q = (plen & ~15u) + tid; q < plen; q += BS_THREADS) s_pb[q] = a.P[pa0 + q];
        if (tid < BK_SPFX / 16 && has_next)
            reinterpret_cast<uint4 *>(s_nx)[tid] = reinterpret_cast<const uint4 *>(a.spfx + (size_t)(f + 1) * BK_SPFX)[tid];
        __syncthreads();
        // bytes before the slice (the previous record's tail) and after it read as '\n'
        for (uint32_t q = tid; q < (uint32_t)(pb0 - pa0); q += BS_THREADS) s_pb[q] = 0x0a;
        if (tid < 64) s_pb[plen + tid] = 0x0a;
        __syncthreads();
    }
    if (dbg) t_ph[1] = wall_clock64();
    // ---- parse both
    uint32_t *s_pen = reinterpret_cast<uint32_t *>(s_pkey);
    const uint32_t nc = bs_parse<BS_CCAP / BS_THREADS>(s_cb, clen, s_st, s_en, BS_NE, s_red);
    const uint32_t npr = bs_parse<BS_PCAP / BS_THREADS>(s_pb, (uint32_t)(pb1 - pa0), s_pmeta, s_pen, BS_NP, s_red);
    if (nc > BS_NE || npr > BS_NP) {
        if (tid == 0) {
            atomicOr(a.flags, nc > BS_NE ? BK_F_CUR_CAP : BK_F_PRIOR_CAP);
            a.uq[f] = 0; a.fq[f] = 0; a.ncur[f] = 0;
        }
        return;
    }
    __syncthreads();
    // ---- items into registers, prior keys into LDS
    uint64_t k0[BS_PT];
    uint32_t mm[BS_PT];
#pragma unroll
    for (int r = 0; r < BS_PT; ++r) {
        const uint32_t k = tid + r * BS_THREADS;
        mm[r] = 0;
        k0[r] = ~0ull;
        if (k < nc) {
            const uint32_t st = s_st[k], en = s_en[k];
            mm[r] = st | ((en - st) << 16);
            k0[r] = lds_key0(s_cb, st);
        }
    }
    {
        uint64_t pk[2] = {0, 0};
        uint32_t pm[2] = {0, 0};
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const uint32_t k = tid + r * BS_THREADS;
            if (k < npr) {
                const uint32_t st = s_pmeta[k], en = s_pen[k];
                pm[r] = st | ((en - st) << 16);
                pk[r] = lds_key0(s_pb, st);
            }
        }
        __syncthreads();  // parse arrays dead
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const uint32_t k = tid + r * BS_THREADS;
            if (k < npr) { s_pkey[k] = pk[r]; s_pmeta[k] = pm[r]; }
        }
    }
    for (uint32_t i = tid; i < BS_NP + 2; i += BS_THREADS) s_sc[i] = 0;
#pragma unroll
    for (int r = 0; r < BS_PT; ++r) {
        const uint32_t k = tid + r * BS_THREADS;
        if (k < nc) { s_k0[k] = k0[r]; s_m[k] = mm[r]; }
    }
    __syncthreads();
    // ---- insertion point in the prior slice (lower bound) and membership
    uint32_t gap[BS_PT], slot[BS_PT], inp = 0;
#pragma unroll
    for (int r = 0; r < BS_PT; ++r) {
        const uint32_t k = tid + r * BS_THREADS;
        gap[r] = 0;
        if (k >= nc) continue;
        uint32_t lo = 0, hi = npr;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (bs_rec_cmp(s_pb, s_pkey[mid], s_pmeta[mid], s_cb, k0[r], mm[r]) < 0) lo = mid + 1; else hi = mid;
        }
        gap[r] = lo;
        if (lo < npr && bs_rec_cmp(s_pb, s_pkey[lo], s_pmeta[lo], s_cb, k0[r], mm[r]) == 0) inp |= 1u << r;
        slot[r] = atomicAdd(&s_sc[lo], 1u);
    }
    __syncthreads();
    {
        // exclusive scan of the gap counts (npr + 1 <= BS_NP + 1 bins, 2 per thread)
        const uint32_t i0 = 2 * tid;
        const uint32_t v0 = i0 <= npr ? s_sc[i0] : 0u, v1 = i0 + 1 <= npr ? s_sc[i0 + 1] : 0u;
        uint32_t tot;
        const uint32_t ex = block_excl_scan<BS_THREADS>(v0 + v1, &tot, reinterpret_cast<uint32_t *>(s_red));
        if (i0 <= npr) s_so[i0] = ex;
        if (i0 + 1 <= npr) s_so[i0 + 1] = ex + v0;
        if (tid == 0) s_so[npr + 1] = tot;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < BS_PT; ++r) {
        const uint32_t k = tid + r * BS_THREADS;
        if (k < nc) s_mem[s_so[gap[r]] + slot[r]] = (uint16_t)k;
    }
    __syncthreads();
    if (dbg) t_ph[2] = wall_clock64();
    // ---- the prior slice must be strictly increasing, and below the next splitter record
    for (uint32_t k = tid + 1; k < npr; k += BS_THREADS) {
        if (bs_rec_cmp(s_pb, s_pkey[k - 1], s_pmeta[k - 1], s_pb, s_pkey[k], s_pmeta[k]) >= 0)
            atomicOr(a.flags, BK_F_UNSORTED);
    }
    if (tid < 64 && npr && has_next) {  // wave 0: last slice record vs the next splitter
        const uint32_t ml = s_pmeta[npr - 1];
        const uint32_t la = ml >> 16, sa = ml & 0xffffu;
        const uint2 sp = a.sspan[f + 1];
        const uint32_t lb = sp.y - sp.x;
        const uint32_t m = la < lb ? la : lb;
        const uint32_t mc = m < BK_SPFX ? m : BK_SPFX;
        const uint32_t o = tid;
        const bool diff = o < mc && s_pb[sa + o] != s_nx[o];
        const uint64_t dm = __ballot(diff);
        int c;
        if (dm) {
            const uint32_t fo = (uint32_t)__ffsll((long long)dm) - 1;
            c = s_pb[sa + fo] < s_nx[fo] ? -1 : 1;
        } else {
            c = m <= BK_SPFX ? (la < lb ? -1 : (la > lb ? 1 : 0)) : 2;
        }
        if (c == 2 && tid == 0) c = lds_glob_cmp(s_pb, sa, la, a.P, sp, BK_SPFX);
        if (tid == 0 && c >= 0) atomicOr(a.flags, BK_F_UNSORTED);
    }
    // ---- exact rank among the records sharing the insertion point
    uint32_t pos[BS_PT], dup = 0;
#pragma unroll
    for (int r = 0; r < BS_PT; ++r) {
        const uint32_t k = tid + r * BS_THREADS;
        pos[r] = 0;
        if (k >= nc) continue;
        const uint32_t m0 = s_so[gap[r]], m1 = s_so[gap[r] + 1];
        uint32_t rank = 0;
        bool d = false;
        for (uint32_t j = m0; j < m1; ++j) {
            const uint32_t o = s_mem[j];
            if (o == k) continue;
            const int c = bs_rec_cmp(s_cb, k0[r], mm[r], s_cb, s_k0[o], s_m[o]);
            if (c > 0 || (c == 0 && o < k)) ++rank;
            if (c == 0 && o < k) d = true;
        }
        pos[r] = m0 + rank;
        if (d) dup |= 1u << r;
    }
    __syncthreads();  // item arrays and members dead: the sorted order takes their place
#pragma unroll
    for (int r = 0; r < BS_PT; ++r) {
        if (tid + r * BS_THREADS >= nc) continue;
        s_m[pos[r]] = mm[r];
        s_fl[pos[r]] = ((dup >> r) & 1u) ? 1u : (((inp >> r) & 1u) ? 0u : 2u);  // 1 duplicate, 2 new
    }
    __syncthreads();
    if (dbg) t_ph[3] = wall_clock64();
    if (dbg) t_ph[4] = t_ph[3];
    // ---- output: offsets over contiguous positions; records assembled in LDS (the prior
    // slice area) and streamed out with 16-B stores; unique first, then new
    uint32_t UB = 0, UC = 0, FB = 0, FC = 0;
    {
        constexpr int OT = (BS_NE + BS_THREADS - 1) / BS_THREADS;
        uint32_t lu[OT], fr[OT];
        uint64_t packed = 0;
#pragma unroll
        for (int r = 0; r < OT; ++r) {
            const uint32_t i = tid * OT + r;
            const uint32_t fl = i < nc ? s_fl[i] : 1u;
            lu[r] = fl != 1u ? (s_m[i] >> 16) + 1 : 0u;
            fr[r] = fl == 2u;
            packed += lu[r] ? ((1ull << 52) | ((uint64_t)lu[r] << 32)) : 0ull;
            packed += fr[r] ? ((1ull << 20) | lu[r]) : 0ull;
        }
        uint64_t tot;
        const uint64_t ex = block_excl_scan<BS_THREADS>(packed, &tot, s_red);
        UB = (uint32_t)(tot >> 32) & 0xfffffu;
        UC = (uint32_t)(tot >> 52);
        FB = (uint32_t)tot & 0xfffffu;
        FC = (uint32_t)(tot >> 20) & 0xfffu;
#pragma unroll
        for (int w = 0; w < 2; ++w) {
            const uint32_t bytes = w ? FB : UB;
            uint8_t *dst = (w ? a.FS : a.US) + cb0;
            for (uint32_t wb = 0; wb < bytes; wb += BS_PCAP) {  // LDS windows of BS_PCAP bytes
                uint32_t o = w ? (uint32_t)ex & 0xfffffu : (uint32_t)(ex >> 32) & 0xfffffu;
#pragma unroll
                for (int r = 0; r < OT; ++r) {
                    const uint32_t i = tid * OT + r;
                    if (!lu[r] || (w && !fr[r])) continue;
                    const uint32_t mt = s_m[i], st = mt & 0xffffu, len = mt >> 16;
                    if (bytes <= BS_PCAP) {
                        lds_copy(s_pb, o, s_cb, st, len);
                        s_pb[o + len] = 0x0a;
                    } else {
                        for (uint32_t b = 0; b <= len; ++b) {
                            const uint32_t p = o + b;
                            if (p >= wb && p < wb + BS_PCAP) s_pb[p - wb] = b == len ? 0x0a : s_cb[st + b];
                        }
                    }
                    o += len + 1;
                }
                __syncthreads();
                const uint32_t wn = bytes - wb < BS_PCAP ? bytes - wb : BS_PCAP;
                for (uint32_t c = tid; c < (wn + 15) / 16; c += BS_THREADS)
                    *reinterpret_cast<uint4 *>(dst + wb + 16 * c) = reinterpret_cast<const uint4 *>(s_pb)[c];
                __syncthreads();
            }
        }
    }
    if (tid == 0) {
        a.uq[f] = ((uint64_t)UC << 32) | UB;
        a.fq[f] = ((uint64_t)FC << 32) | FB;
        a.ncur[f] = ((uint64_t)npr << 32) | nc;
        if (dbg) {
            t_ph[5] = wall_clock64();
            for (int q = 0; q < 5; ++q) atomicAdd(&a.dbg[q], (unsigned long long)(t_ph[q + 1] - t_ph[q]));
            atomicAdd(&a.dbg[5], 1ull);
        }
    }
}

// One block: exclusive scans of the per-bucket unique / new sizes, the cur record total.
// info[0] = unique (records << 32 | bytes), info[1] = new, info[2] = prior << 32 | cur records,
// info[3] = error word.
__global__ __launch_bounds__(1024) void k_bk_offs(const uint64_t *__restrict__ uq, const uint64_t *__restrict__ fq,
                                                  const uint64_t *__restrict__ ncur, uint32_t NB,
                                                  uint64_t *__restrict__ uo, uint64_t *__restrict__ fo,
                                                  const uint32_t *__restrict__ flags, uint64_t *__restrict__ info) {
    __shared__ uint64_t s_red[16];
    uint64_t cu = 0, cf = 0, cn = 0;
    for (uint32_t b0 = 0; b0 < NB; b0 += 1024 * 4) {
        const uint32_t i0 = b0 + threadIdx.x * 4;
        uint64_t vu[4], vf[4], su = 0, sf = 0, sn = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const bool ok = i0 + j < NB;
            vu[j] = ok ? uq[i0 + j] : 0ull;
            vf[j] = ok ? fq[i0 + j] : 0ull;
            su += vu[j];
            sf += vf[j];
            sn += ok ? ncur[i0 + j] : 0u;
        }
        uint64_t tu, tf, tn;
        const uint64_t eu = block_excl_scan<1024>(su, &tu, s_red);
        const uint64_t ef = block_excl_scan<1024>(sf, &tf, s_red);
        block_excl_scan<1024>(sn, &tn, s_red);
        uint64_t ru = cu + eu, rf = cf + ef;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (i0 + j < NB) { uo[i0 + j] = ru; fo[i0 + j] = rf; }
            ru += vu[j];
            rf += vf[j];
        }
        cu += tu;
        cf += tf;
        cn += tn;
    }
    if (threadIdx.x == 0) { info[0] = cu; info[1] = cf; info[2] = cn; info[3] = *flags; }
}

// 16 bytes starting at byte k (0..15) of the 32 bytes a || b.
__device__ __forceinline__ uint4 shift16(uint4 a, uint4 b, uint32_t k) {
    const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    const uint32_t q = k >> 2, r = k & 3u;
    uint32_t s[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const uint32_t x0 = w[i], x1 = w[i + 1], x2 = w[i + 2], x3 = (i + 3 < 8) ? w[i + 3] : 0u;
        s[i] = q == 0 ? x0 : (q == 1 ? x1 : (q == 2 ? x2 : x3));
    }
    return make_uint4(__builtin_amdgcn_alignbyte(s[1], s[0], r), __builtin_amdgcn_alignbyte(s[2], s[1], r),
                      __builtin_amdgcn_alignbyte(s[3], s[2], r), __builtin_amdgcn_alignbyte(s[4], s[3], r));
}

// Concatenate the per-bucket slots: block (f, y) copies bucket f's unique (y = 0) or new (y = 1)
// bytes from its 64-B-aligned slot to its offset in the output (interior: aligned 16-B stores
// of shifted source chunks; the two partial edges: byte stores).
__global__ __launch_bounds__(256) void k_bk_compact(const uint8_t *__restrict__ US, const uint8_t *__restrict__ FS,
                                                    const uint64_t *__restrict__ base2, const uint64_t *__restrict__ uq,
                                                    const uint64_t *__restrict__ fq, const uint64_t *__restrict__ uo,
                                                    const uint64_t *__restrict__ fo, uint8_t *__restrict__ OU,
                                                    uint8_t *__restrict__ OF) {
    const uint32_t f = blockIdx.x, y = blockIdx.y;
    const uint8_t *src = (y ? FS : US) + base2[f];
    const uint32_t len = (uint32_t)(y ? fq[f] : uq[f]);
    const uint64_t D = (uint32_t)(y ? fo[f] : uo[f]);
    uint8_t *dst = y ? OF : OU;
    if (!len) return;
    const uint64_t h0 = ((D + 15) & ~15ull) < D + len ? ((D + 15) & ~15ull) : D + len;
    const uint64_t h1 = ((D + len) & ~15ull) > h0 ? ((D + len) & ~15ull) : h0;
    for (uint64_t p = D + threadIdx.x; p < h0; p += 256) dst[p] = src[p - D];
    for (uint64_t p = h1 + threadIdx.x; p < D + len; p += 256) dst[p] = src[p - D];
    const uint32_t k = (uint32_t)((h0 - D) & 15u);
    const uint32_t base = (uint32_t)(h0 - D) & ~15u;  // source chunk of the first interior byte
    const uint32_t nck = (uint32_t)((h1 - h0) / 16);
    const uint4 *s4 = reinterpret_cast<const uint4 *>(src + base);
    for (uint32_t c = threadIdx.x; c < nck; c += 256)
        *reinterpret_cast<uint4 *>(dst + h0 + 16ull * c) = shift16(s4[c], s4[c + 1], k);
}

// ------------------------------------------------------------------ host
static uint64_t env_u64(const char *name, uint64_t dflt) {
    const char *v = getenv(name);
    return (v && *v) ? strtoull(v, nullptr, 10) : dflt;
}

int bucket_dedup_diff(sg_ctx *c, const uint8_t *d_cur, uint64_t n_cur, const uint8_t *d_prior, uint64_t n_prior,
                      sg_dev_result *res, bool *used) {
    *used = false;
    if (!env_u64("SG_BUCKET", 0)) return SG_OK;  // opt-in: slower than the radix pipeline so far
    if (!d_prior || n_prior == 0 || n_cur < env_u64("SG_BUCKET_MIN", 8ull << 20)) return SG_OK;
    if (((uintptr_t)d_cur & 15) || ((uintptr_t)d_prior & 15)) return SG_OK;
    const uint64_t target = env_u64("SG_BUCKET_TARGET", 15000);
    const uint64_t want = (n_cur + target - 1) / (target ? target : 1);
    uint32_t NB1 = (uint32_t)ceil(sqrt((double)want));
    NB1 = NB1 < 2 ? 2 : (NB1 > BP_MAXB ? BP_MAXB : NB1);
    uint32_t NB2 = (uint32_t)((want + NB1 - 1) / NB1);
    NB2 = NB2 < 1 ? 1 : (NB2 > BP_MAXB ? BP_MAXB : NB2);
    const uint32_t NB = NB1 * NB2;
    const uint64_t W = (n_prior + NB - 1) / NB;
    if (W < 64) return SG_OK;  // prior too small to split this finely
    const uint32_t NT1 = (uint32_t)((n_cur + BP_TILE - 1) / BP_TILE);
    const uint64_t l1_cap = n_cur + (uint64_t)BP_PAD * NT1 * NB1 + 64;
    const uint32_t NT2max = (uint32_t)(l1_cap / BP_TILE + NB1 + 1);
    const uint64_t l2_cap = l1_cap + (uint64_t)BP_PAD * NT2max * NB2 + 64;
    if (l2_cap >= (1ull << 40)) return SG_OK;

    uint64_t *skey, *tot1, *base1, *tot2, *base2, *uq, *fq, *uo, *fo, *info;
    uint2 *sspan;
    uint32_t *cnt1, *cnt2, *ts, *flags;
    uint64_t *ncur;
    uint8_t *L1, *L2, *US, *FS, *OU, *OF;
    SG_TRY(slot(c, S_BK_SKEY, (size_t)NB + 2, &skey));
    SG_TRY(slot(c, S_BK_SSPAN, (size_t)NB + 2, &sspan));
    uint8_t *spfx;
    SG_TRY(slot(c, S_BK_SPFX, ((size_t)NB + 2) * BK_SPFX, &spfx));
    unsigned long long *dbg = nullptr;
    const bool debug = env_u64("SG_BK_DEBUG", 0) != 0;
    if (debug) {
        SG_TRY(slot(c, S_BK_DBG, 48, &dbg));
        SG_HIP(hipMemsetAsync(dbg, 0, 48 * 8, c->stream));
    }
    SG_TRY(slot(c, S_BK_CNT1, (size_t)NB1 * NT1 + 16, &cnt1));
    SG_TRY(slot(c, S_BK_CNT2, (size_t)NT2max * NB2 + 16, &cnt2));
    SG_TRY(slot(c, S_BK_SMALL, 4 * (size_t)BP_MAXB + 64, &tot1));
    base1 = tot1 + BP_MAXB + 8;
    ts = reinterpret_cast<uint32_t *>(base1 + BP_MAXB + 8);
    info = base1 + 2 * BP_MAXB + 16;
    flags = reinterpret_cast<uint32_t *>(info + 8);
    SG_TRY(slot(c, S_BK_TOT2, 2 * (size_t)NB + 16, &tot2));
    base2 = tot2 + NB + 8;
    SG_TRY(slot(c, S_BK_Q, 4 * (size_t)NB + 32, &uq));
    fq = uq + NB + 8;
    uo = fq + NB + 8;
    fo = uo + NB + 8;
    SG_TRY(slot(c, S_BK_NCUR, (size_t)NB + 8, &ncur));
    uint32_t *recs, *nrecs;
    const uint32_t NTmax = NT1 > NT2max ? NT1 : NT2max;
    SG_TRY(slot(c, S_BK_RECS, (size_t)NTmax * BP_MAXREC, &recs));
    SG_TRY(slot(c, S_BK_NREC, (size_t)NTmax + 8, &nrecs));
    SG_TRY(slot(c, S_BK_L1, l1_cap + 64, &L1));
    SG_TRY(slot(c, S_BK_L2, l2_cap + 64, &L2));
    SG_TRY(slot(c, S_BK_US, l2_cap + 64, &US));
    SG_TRY(slot(c, S_BK_FS, l2_cap + 64, &FS));
    SG_TRY(slot(c, S_OUT_UNIQ, n_cur + 64, &OU));
    SG_TRY(slot(c, S_OUT_FRESH, n_cur + 64, &OF));
    SG_HIP(hipMemsetAsync(flags, 0, 4, c->stream));

    SG_LAUNCH(c, "bk_pick", k_bk_pick, (NB + 1 + 3) / 4, 256, 0, d_prior, n_prior, W, NB, skey, sspan, spfx);
    BPArgs a{};
    a.src = d_cur;
    a.n = n_cur;
    a.NT1 = NT1;
    a.NB1 = NB1;
    a.NB2 = NB2;
    a.base1 = base1;
    a.tot1 = tot1;
    a.ts = ts;
    a.skey = skey;
    a.sspan = sspan;
    a.spfx = spfx;
    a.P = d_prior;
    a.cnt = cnt1;
    a.base2 = base2;
    a.out = L1;
    a.flags = flags;
    a.dbg = dbg;
    a.recs = recs;
    a.nrec = nrecs;
    // model: the tile read (+ overhang), run sizes written
    SG_LAUNCH_B(c, "bk_l1_count", (double)n_cur + 4.0 * NB1 * NT1, k_bp_count<1>, NT1, BP_THREADS, 0, a);
    SG_LAUNCH(c, "bk_cscan1", k_bp_cscan1, NB1, 256, 0, cnt1, NT1, tot1);
    SG_LAUNCH(c, "bk_base1", k_bp_base1, 1, 256, 0, tot1, NB1, base1, ts);
    SG_LAUNCH_B(c, "bk_l1_apply", 2.0 * (double)n_cur, k_bp_apply<1>, NT1, BP_THREADS, 0, a);
    BPArgs b2 = a;
    b2.src = L1;
    b2.cnt = cnt2;
    b2.out = L2;
    SG_LAUNCH_B(c, "bk_l2_count", (double)n_cur, k_bp_count<2>, NT2max, BP_THREADS, 0, b2);
    SG_LAUNCH(c, "bk_cscan2", k_bp_cscan2, NB1, 256, 0, cnt2, ts, NB2, tot2);
    uint64_t *l2_total = info + 4;
    SG_TRY(tile_scan(c, tot2, NB, base2, l2_total));
    SG_LAUNCH_B(c, "bk_l2_apply", 2.0 * (double)n_cur, k_bp_apply<2>, NT2max, BP_THREADS, 0, b2);
    BSArgs s{};
    s.L2 = L2;
    s.base2 = base2;
    s.tot2 = tot2;
    s.P = d_prior;
    s.np = n_prior;
    s.sspan = sspan;
    s.NB = NB;
    s.US = US;
    s.FS = FS;
    s.uq = uq;
    s.fq = fq;
    s.ncur = ncur;
    s.flags = flags;
    s.spfx = spfx;
    s.dbg = dbg;
    SG_LAUNCH(c, "bk_sort", k_bk_sort, NB, BS_THREADS, 0, s);
    SG_LAUNCH(c, "bk_offs", k_bk_offs, 1, 1024, 0, uq, fq, ncur, NB, uo, fo, flags, info);
    uint64_t h[5];
    SG_TRY(ctx_readback(c, h, info, sizeof(h)));
    c->last_flags = (uint32_t)h[3];
    if (debug) {
        unsigned long long d[48];
        SG_TRY(ctx_readback(c, d, dbg, sizeof(d)));
        for (int kk = 0; kk < 4; ++kk) {
            const unsigned long long *e = d + 8 + 8 * kk;
            const double nt = e[7] ? (double)e[7] : 1.0;
            fprintf(stderr, "[bk_%s_%s] tiles=%llu us/tile: %.2f %.2f %.2f %.2f\n", kk < 2 ? "l1" : "l2",
                    (kk & 1) ? "apply(stage,classify,place,write)" : "count(stage,classify)", e[7], e[0] / nt / 100.0,
                    e[1] / nt / 100.0, e[2] / nt / 100.0, e[3] / nt / 100.0);
        }
        const double nb = d[5] ? (double)d[5] : 1.0;
        fprintf(stderr, "[bk_sort] NB=%u NB1=%u NB2=%u blocks=%llu us/block: stage %.2f parse+place %.2f rank %.2f "
                "diff %.2f out %.2f\n", NB, NB1, NB2, d[5], d[0] / nb / 100.0, d[1] / nb / 100.0, d[2] / nb / 100.0,
                d[3] / nb / 100.0, d[4] / nb / 100.0);
    }
    if (h[3]) return SG_OK;  // outside the LDS bounds or an unsorted prior: the radix pipeline
    const uint64_t ub = (uint32_t)h[0], fb = (uint32_t)h[1];
    // model: the bucket and its slice read, the unique and new records written
    if (c->profile) prof_bytes(c, "bk_sort", (double)h[4] + (double)n_prior + (double)ub + (double)fb);
    dim3 cg(NB, 2);
    SG_LAUNCH_B(c, "bk_compact", 2.0 * (double)(ub + fb), k_bk_compact, cg, 256, 0, US, FS, base2, uq, fq, uo, fo, OU, OF);
    res->uniq = OU;
    res->uniq_bytes = ub;
    res->uniq_records = h[0] >> 32;
    res->fresh = OF;
    res->fresh_bytes = fb;
    res->fresh_records = h[1] >> 32;
    res->in_records = (uint32_t)h[2];
    res->prior_records = h[2] >> 32;
    *used = true;
    return SG_OK;
}

}  // namespace sg
