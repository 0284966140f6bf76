// sg_dedup.hip — A7 sort -u dedup and A8 new-record diff on HBM-resident text.
//
// Pipeline (one stream), per buffer:
//   lines    -> (start, end, key0) per record; key0 = bytes [0,7) + tag min(len, 8)
//   sort     -> LSD radix sort of (key0, rec id)
//   big      -> equal-key0 groups of > 64 records sharing 7 bytes are split further by
//               radix rounds on the next 7-byte chunk (stable by chunk, then by group),
//               until every unresolved segment has <= 64 records; segment heads -> brk
//   emit     -> the records in that order, materialised ONCE into a contiguous sorted
//               buffer S (fused length scan + gather + copy, sg_emit.hpp); every later
//               step reads S sequentially instead of gathering records from the input
//   adjacent -> dup[i] = record i equals record i-1 (same segment, bytes from S);
//               bad[i] = same segment but different bytes (segment not yet ordered)
//   run sort -> each segment holding a bad position is ranked in registers (16-lane
//               groups up to 16 records, half or whole waves up to 64) by its 7-byte chunk
//               keys at offsets 7..34 and a byte compare beyond; spans permuted in place
//   emit     -> the records with dup == 0: the sort -u output, contiguous, + spans/key0
//   diff     -> per 1024 unique records, the prior's key range found by a 64-ary wave
//               search, its keys staged in LDS; membership by binary search over key0,
//               then wide compares (binary search over runs of equal key0)
//   emit     -> the records absent from the prior: the new-record output
// The result is exact for any input (NULs, CR, 0xff, long shared prefixes, duplicates of
// any multiplicity): ordering is decided by bytes, never by a hash.
#include "sg_internal.hpp"
#include "sg_keystat.hpp"
#include "sg_prims_host.hpp"
#include "sg_emit.hpp"
#include "sg_switches.hpp"

#include <stdlib.h>
#include <cmath>
#include <string.h>

namespace sg {

const SlotSet CUR_SLOTS = {S_STARTS, S_ENDS, S_KEYS, S_KEYS2, S_VALS, S_VALS2, S_UNIQ, S_LB};
const SlotSet PRIOR_SLOTS = {S_P_STARTS, S_P_ENDS, S_P_KEYS, S_P_KEYS2, S_P_VALS, S_P_VALS2, S_P_UNIQ, S_P_FLAG};

constexpr uint32_t WAVE_GROUP = 64;
// all-segments mode when the context's last sort -u kept less than this fraction of records
constexpr float SEG_ALL_UNIQ = 0.4f;

// ------------------------------------------------------------------ launch helpers
// Queue one emit (no host sync): count pass, tile scan, apply pass. *total_out: device u64,
// (records << 32 | bytes). `bytes_model`: algorithmic bytes credited to the apply launch
// (DESIGN.md §4).
typedef void (*EmitApplyFn)(const uint2 *, uint32_t, const uint64_t *, const uint8_t *, uint8_t *, uint2 *,
                            const uint64_t *, uint64_t *);

// dst_shift (< 16): the output starts dst_shift bytes past the 16-B aligned `dst` (byte
// offsets and out_spans include it; the total does not).
template <class Item>
static int run_emit(sg_ctx *c, EmitApplyFn kern, const char *name, const char *cname, int status_slot, Item item, uint32_t n,
                    const uint8_t *src, uint8_t *dst, uint2 *out_spans, const uint64_t *kin, uint64_t *kout,
                    uint64_t **total_out, double bytes_model, uint32_t dst_shift = 0) {
    const uint32_t ntiles = (n + EM_TILE - 1) / EM_TILE;
    uint64_t *tp;  // tot[ntiles] | pre[ntiles] | total
    SG_TRY(slot(c, status_slot, 2 * (size_t)ntiles + 4, &tp));
    uint64_t *tot = tp, *pre = tp + ntiles, *total = tp + 2 * (size_t)ntiles;
    *total_out = total;
    if (ntiles == 0) {
        SG_HIP(hipMemsetAsync(total, 0, 8, c->stream));
        return SG_OK;
    }
    uint2 *cache;
    SG_TRY(slot(c, S_ECACHE, (size_t)n + 1, &cache));
    SG_LAUNCH(c, cname, k_emit_count<Item>, ntiles, EM_BLOCK, 0, item, n, cache, tot);
    SG_TRY(tile_scan(c, tot, ntiles, pre, total, dst_shift));
    SG_LAUNCH_B(c, name, bytes_model, kern, ntiles, EM_BLOCK, 0, cache, n, pre, src, dst, out_spans, kin,
                kout);
    return SG_OK;
}

static inline uint32_t grid_for(uint64_t n, uint32_t block, uint32_t cap = 0x7fffffffu) {
    uint64_t g = (n + block - 1) / block;
    if (g == 0) g = 1;
    return (uint32_t)(g < cap ? g : cap);
}

// ------------------------------------------------------------------ key width
// The sort key of a record ("key0") is its first kw bytes from the common prefix `base`,
// big-endian in the top bits, with tag = min(remaining bytes, kw + 1) in bits 7..0 (kw = 7:
// the full-width key of sg_lines; kw = 5/6: narrowed when those bytes already spread the
// records, so fewer radix passes run). Equal keys with tag kw + 1 need bytes from base + kw.
// Kernels take both as one word: bk = base | kw << 16.
__host__ __device__ __forceinline__ uint32_t make_bk(uint32_t base, uint32_t kw) { return base | (kw << 16); }
__device__ __forceinline__ uint32_t bk_off(uint32_t bk) { return (bk & 0xffffu) + (bk >> 16); }
__device__ __forceinline__ uint32_t bk_full(uint32_t bk) { return (bk >> 16) + 1u; }
// key0 (kw = 7) -> the kw-byte key: bytes kw..6 cleared, the tag clamped to kw + 1 (as the
// sort's first pass narrows; idempotent, so narrowed keys pass through unchanged).
__device__ __forceinline__ uint64_t key_narrow(uint64_t k, uint32_t kw) {
    if (kw >= 7u) return k;
    const uint64_t t = k & 0xffu;
    return (k & (~0ull << (64u - 8u * kw))) | (t < kw + 1u ? t : (uint64_t)(kw + 1u));
}

// ------------------------------------------------------------------ predicates / functors
struct FlagPred {
    const uint8_t *f;
    __device__ uint32_t operator()(uint32_t i) const { return f[i] ? 1u : 0u; }
};

// Over the final order of a refinement round: sub-segments by (group, chunk key). brk at
// every sub-segment head; A/B = bounds of tag-8 sub-segments of more than WAVE_GROUP rows.
struct RoundGroupPred {
    const uint64_t *FK;     // chunk key (or its packed form), final order
    const uint32_t *G;      // group index, final order
    const uint32_t *P;      // global position, final order
    uint8_t *brk;
    uint32_t n;
    uint64_t tagmask;       // the tag's bits: 0xff, or 0xf in a packed key
    __device__ uint32_t operator()(uint32_t i) const {
        const uint64_t k = FK[i];
        const uint32_t g = G[i];
        const bool head = (i == 0) || FK[i - 1] != k || G[i - 1] != g;
        brk[P[i]] = head ? 1 : 0;
        if ((k & tagmask) != 8u) return 0u;
        const bool tail = (i + 1 == n) || FK[i + 1] != k || G[i + 1] != g;
        const bool bh = head && (i + WAVE_GROUP < n) && FK[i + WAVE_GROUP] == k && G[i + WAVE_GROUP] == g;
        const bool bt = tail && (i >= WAVE_GROUP) && FK[i - WAVE_GROUP] == k && G[i - WAVE_GROUP] == g;
        return (bh ? 1u : 0u) | (bt ? 2u : 0u);
    }
};

struct GroupSizeFn {
    const uint32_t *GS, *GE;
    __device__ uint64_t operator()(uint32_t g) const { return (uint64_t)(GE[g] - GS[g] + 1u); }
};

__device__ __forceinline__ int key_cmp_full(const uint8_t *buf, const uint2 *spans,
                                            uint64_t ka, uint32_t ra, uint64_t kb, uint32_t rb, uint32_t bk) {
    if (ka != kb) return ka < kb ? -1 : 1;
    if ((ka & 0xffu) < bk_full(bk)) return 0;
    return rec_cmp_w(buf, spans[ra].x, spans[ra].y, buf, spans[rb].x, spans[rb].y, bk_off(bk));
}

// ------------------------------------------------------------------ refinement rounds
// Sorted-order records are ids into `spans` (u32) or the spans themselves (uint2).
__device__ __forceinline__ uint2 span_of(const uint2 *spans, uint32_t v) { return spans[v]; }
__device__ __forceinline__ uint2 span_of(const uint2 *, uint2 v) { return v; }

// Expand big groups into member rows: row j -> group index, global position, and the
// record's chunk key at `off`. One wave per 1024 consecutive rows: the group of its first
// row by binary search, then each lane walks its rows forward (groups hold > 64 rows, so a
// lane's group index only advances), instead of a binary search per row.
constexpr uint32_t EXP_ROWS = 1024;
template <typename VT>
__global__ __launch_bounds__(256) void k_expand(const uint8_t *__restrict__ buf,
                                                const uint2 *__restrict__ spans,
                                                const uint32_t *__restrict__ GS,
                                                const uint64_t *__restrict__ goff, uint32_t B,
                                                const VT *__restrict__ V, uint32_t M,
                                                uint32_t off, uint64_t *RK, uint32_t *RG,
                                                uint32_t *RP) {
    const uint32_t j0 = (blockIdx.x * 4u + (threadIdx.x >> 6)) * EXP_ROWS;
    if (j0 >= M) return;
    uint32_t g = 0, hi = B;  // last k with goff[k] <= j0
    while (hi - g > 1) {
        const uint32_t mid = (g + hi) >> 1;
        if (goff[mid] <= j0) g = mid; else hi = mid;
    }
    const uint32_t je = min(M, j0 + EXP_ROWS);
    for (uint32_t j = j0 + lane_id(); j < je; j += 64) {
        while (g + 1 < B && goff[g + 1] <= j) ++g;
        const uint32_t pos = GS[g] + (j - (uint32_t)goff[g]);
        const uint2 sp = span_of(spans, V[pos]);
        RK[j] = chunk_key(buf, sp.x, sp.y, off);
        RG[j] = g;
        RP[j] = pos;
    }
}

__global__ void k_gid_keys(const uint32_t *__restrict__ RG, const uint32_t *__restrict__ perm,
                           uint64_t *GK, uint32_t M) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < M) GK[i] = RG[perm[i]];
}

// Final order of a round: T[i] = record now at final index i; FK its chunk key.
template <typename VT>
__global__ void k_round_gather(const uint8_t *__restrict__ buf, const uint2 *__restrict__ spans, const VT *__restrict__ V,
                               const uint32_t *__restrict__ RP, const uint32_t *__restrict__ perm,
                               uint32_t M, uint32_t off, VT *T, uint64_t *FK) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= M) return;
    const VT r = V[RP[perm[i]]];
    T[i] = r;
    if (!FK) return;  // the sorted packed keys serve as the final keys
    const uint2 sp = span_of(spans, r);
    FK[i] = chunk_key(buf, sp.x, sp.y, off);
}

template <typename VT>
__global__ void k_round_scatter(const VT *__restrict__ T, const uint32_t *__restrict__ RP,
                                uint32_t M, VT *V) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < M) V[RP[i]] = T[i];
}

__global__ void k_pos_of(const uint32_t *__restrict__ idx, const uint32_t *__restrict__ RP, uint32_t n,
                         uint32_t *out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = RP[idx[i]];
}

// ------------------------------------------------------------------ segment sort (spans in S)
// A segment is a maximal run [a, b] with brk[a] = 1 and brk[a+1..b] = 0: its records share
// their first 7 bytes (equal key0; inside big groups, the refined chunks too) but are not
// yet in byte order. A segment holding two different records ("bad") has <= 64 members:
// bigger groups went through the refinement rounds. Sorting permutes the segment's spans
// into S (and recomputes dup); the bytes in S stay where they are, and the unique emit
// gathers through the permuted spans (still inside the same few cache lines).
constexpr uint32_t SEG_SMALL = 16;

// Memcmp-then-length of record a of `ba` and record b of `bb` from byte `off`, 8 bytes per
// step.
__device__ __forceinline__ int rec_cmp8_2(const uint8_t *ba, uint32_t sa, uint32_t la, const uint8_t *bb,
                                          uint32_t sb, uint32_t lb, uint32_t off) {
    const uint32_t m = la < lb ? la : lb;
    for (uint32_t o = off; o < m; o += 8) {
        const uint32_t t = (m - o) < 8u ? (m - o) : 8u;
        const uint64_t x = load_le(ba, sa + o, t), y = load_le(bb, sb + o, t);
        if (x != y) return __builtin_bswap64(x) < __builtin_bswap64(y) ? -1 : 1;
    }
    return la < lb ? -1 : (la > lb ? 1 : 0);
}

// The same for two records of one buffer.
__device__ __forceinline__ int rec_cmp8(const uint8_t *buf, uint32_t sa, uint32_t la, uint32_t sb, uint32_t lb,
                                        uint32_t off) {
    return rec_cmp8_2(buf, sa, la, buf, sb, lb, off);
}

// The adjacent pass with the group marking folded in (no count/scan/apply select for the
// group marks).
// KEYS: group starts come from the keys (brk[i] = K[i] != K[i-1] is written here) and groups
// of more than WAVE_GROUP records with a full tag are appended as (GS, GE) pairs for the
// refinement rounds (rare: wave-aggregated atomics, unordered — the refinement rounds place
// each group's rows by their positions); otherwise brk is given (after refinement:
// sub-segment heads) and read.
// DUP: dup[i] = record i equals record i-1 inside its segment; where it differs, the
// segment's head is marked in segbad (the segment needs sorting; SegPred lists it).
// cnt[2] = big groups (zeroed by the caller).
// Bit j (0..15) = byte j of the 16-B word is nonzero.
__device__ __forceinline__ uint32_t swar_nonzero16(uint4 w) {
    const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
    uint32_t m = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t t = (((ww[q] & 0x7f7f7f7fu) + 0x7f7f7f7fu) | ww[q]) & 0x80808080u;
        m |= (((t >> 7) & 1u) | ((t >> 14) & 2u) | ((t >> 21) & 4u) | ((t >> 28) & 8u)) << (4 * q);
    }
    return m;
}

struct AdjLists {
    uint32_t *hs, *hb, *gs, *ge, *cnt;
    uint32_t cap_s, cap_b, cap_g;
};

// ZD (with !DUP, the all-segments mode): no byte compares at all. A segment whose key0 holds
// its records whole (tag below full) is a run of one record repeated (dup = not its head);
// every other segment of two or more records is marked bad at its head, so the segment sorts
// rank all of its members and set their dup flags (singletons: dup = 0).
template <bool KEYS, bool DUP, bool ZD = false>
__global__ __launch_bounds__(256) void k_adjacent2(const uint8_t *__restrict__ S, const uint2 *__restrict__ SS,
                                                   const uint64_t *__restrict__ K, uint8_t *__restrict__ brk, uint32_t n,
                                                   uint8_t *__restrict__ dup, uint8_t *__restrict__ segbad, AdjLists L,
                                                   uint32_t base) {
    const uint32_t i0 = blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = i0 < n;  // no early return: the appends below are wave-wide
    const uint32_t i = live ? i0 : n - 1;
    const uint32_t ip = i > 0 ? i - 1 : 0;
    const uint64_t ki = K[i];
    uint2 x = make_uint2(0u, 0u), y = make_uint2(0u, 0u);
    bool head;
    if constexpr (KEYS) {
        const uint64_t kp = K[ip];
        if constexpr (DUP) { x = SS[ip]; y = SS[i]; }
        head = (i == 0) || kp != ki;
        if (live) brk[i] = head ? 1 : 0;
        // a group of > WAVE_GROUP records sharing a full-tag key (rare): its last position by
        // galloping then bisecting over the sorted keys
        const bool big = live && head && (ki & 0xffu) == bk_full(base) && i + WAVE_GROUP < n && K[i + WAVE_GROUP] == ki;
        uint32_t last = 0;
        if (big) {
            uint32_t lo = i + WAVE_GROUP, step = WAVE_GROUP;  // K[lo] == ki
            while (lo + step < n && K[lo + step] == ki) { lo += step; step <<= 1; }
            uint32_t hi = min(n, lo + step);  // K[hi] != ki (or hi == n)
            while (hi - lo > 1) {
                const uint32_t mid = lo + (hi - lo) / 2;
                if (K[mid] == ki) lo = mid; else hi = mid;
            }
            last = lo;
        }
        // (start, end) pairs: one append per wave for both lists, same order
        const uint64_t m = __ballot(big);
        if (m) {
            const int lead = __ffsll((long long)m) - 1;
            uint32_t b = 0;
            if (lane_id() == lead) b = atomicAdd(&L.cnt[2], (uint32_t)__popcll(m));
            b = (uint32_t)__shfl((int)b, lead, 64);
            if (big) {
                const uint32_t q = b + (uint32_t)__popcll(m & ((1ull << lane_id()) - 1ull));
                if (q < L.cap_g) { L.gs[q] = i; L.ge[q] = last; }
            }
        }
    } else {
        const uint8_t bb = brk[i];
        if constexpr (DUP) { x = SS[ip]; y = SS[i]; }
        head = (i == 0) || bb;
    }
    if constexpr (!DUP) {
        if constexpr (ZD) {
            if (live) {
                const bool whole = (ki & 0xffu) < bk_full(base);
                if (head) {
                    bool multi;
                    if constexpr (KEYS) multi = i + 1 < n && K[i + 1] == ki;
                    else multi = i + 1 < n && !brk[i + 1];
                    if (multi && !whole) segbad[i] = 1;
                }
                dup[i] = (!head && whole) ? 1 : 0;
            }
        }
        return;
    }
    bool d = false;
    if (live && !head) {
        d = ((ki & 0xffu) < bk_full(base)) || rec_equal_w(S, x.x, x.y, S, y.x, y.y, bk_off(base));
        if (!d) {
            // i differs from i - 1 inside one segment: mark the segment's head (the last group
            // start at or before i - 1) bad
            uint32_t h = i - 1;
            bool found = true;
            if constexpr (KEYS) {
                // the run of ki ending at i - 1 starts in [i - 64, i - 1] unless it is a big
                // group (refinement rounds first, then this pass again): bisect the keys
                uint32_t lo = i >= WAVE_GROUP ? i - WAVE_GROUP : 0u;
                if (lo > 0 && K[lo] == ki) {
                    found = false;
                } else {
                    while (lo < h) {
                        const uint32_t mid = (lo + h) >> 1;
                        if (K[mid] == ki) h = mid; else lo = mid + 1;
                    }
                }
            } else {
                for (;;) {  // 16 brk bytes per aligned load instead of a dependent byte walk
                    const uint32_t a = h & ~15u;
                    const uint32_t m = swar_nonzero16(*reinterpret_cast<const uint4 *>(brk + a)) & ((2u << (h - a)) - 1u);
                    if (m) { h = a + 31u - (uint32_t)__clz(m); break; }
                    if (a == 0) { h = 0; break; }
                    h = a - 1;
                }
            }
            if (found) segbad[h] = 1;
        }
    }
    if (live) dup[i] = d ? 1 : 0;
}

// Heads of bad segments (segbad, marked by k_adjacent2): A = up to SEG_SMALL members, B = more
// (<= WAVE_GROUP). A bad head's segment is small iff a break (brk, or the end) lies in
// (i, i + SEG_SMALL]: two aligned 16-B loads of brk (the slot has 32 B of tail room).
struct SegPred {
    const uint8_t *brk, *segbad;
    uint32_t n;
    // Wave-cooperative (k_sel_count calls it with the wave's 64 lanes on 64 consecutive
    // positions): the row's brk bytes and the 16 after it as two ballots, each lane's window
    // a funnel shift of them — no per-lane 32-B window loads and SWAR reductions (those,
    // loaded for every position so the rows could issue together, were 100+ VALU ops per
    // position; behind a per-row branch, a latency chain). Lanes past n (a partial tile's
    // inactive lanes) lie past the end, which the boundary rule treats as a segment end.
    __device__ uint32_t operator()(uint32_t i) const {
        static_assert(SEG_SMALL == 16, "window of 16 positions");
        const uint32_t lane = lane_id(), r0 = i - lane;
        const uint32_t bad = segbad[i];
        const uint64_t lo = __ballot(brk[i] != 0);
        // every lane loads (lanes 16..63 repeat 0..15's bytes; past n a valid in-row byte)
        // so the load is unconditional and the row's loads issue together
        const uint32_t q = r0 + 64u + (lane & 15u);
        const uint32_t bq = brk[q < n ? q : i];
        const uint64_t hi = __ballot((lane < 16u) & ((q >= n) | (bq != 0u)));
        const uint32_t sft = lane + 1u;  // positions i+1 .. i+16
        uint32_t win = (uint32_t)((sft < 64u ? (lo >> sft) | (hi << (64u - sft)) : hi) & 0xffffu);
        const uint32_t rem = n - i - 1u;  // positions after i inside the input
        if (rem < 16u) win |= 0xffffu << rem;
        return bad ? (win ? 1u : 2u) : 0u;
    }
};

// Ranking inside a segment. Members share their first 7 bytes, so they are ordered by the
// 7-byte chunk keys at offsets 7, 14, 21, 28, 35 (chunk_key: big-endian bytes + tag, tag < 8
// ends the record) held in registers, and by a byte compare from offset 42 only when all
// five chunks tie with tag 8 (round 5: four chunks left C5's longer host:port records, 36-42
// bytes, to byte compares inside the rank loop for every duplicate pair: segment sorts
// 46.9 -> 39.6 ms per step with five; six were no better). dup = an equal member with a smaller index exists.
#ifndef SG_SEG_CH
#define SG_SEG_CH 5
#endif
constexpr int SEG_CH = SG_SEG_CH;

struct SegKeys {
    uint64_t c[SEG_CH];
};

// The SEG_CH chunk keys from one set of wide loads: the suffix's first 7 * SEG_CH bytes in at
// most four aligned 16-B loads (normalised), instead of scattered 8-B loads.
__device__ __forceinline__ SegKeys seg_keys(const uint8_t *S, uint2 x, uint32_t base) {
    SegKeys k;
    const uint32_t off = bk_off(base), len = x.y - x.x;
    const uint32_t rem = len > off ? len - off : 0u;
    uint4 c[4];
    load_chunks(S, x.x + off, rem < 7u * SEG_CH ? rem : 7u * SEG_CH, c);
    uint32_t r[13];
    normalize52(c, (x.x + off) & 15u, r);
#pragma unroll
    for (int q = 0; q < SEG_CH; ++q) {
        const uint32_t rq = rem > 7u * q ? rem - 7u * q : 0u;
        const uint32_t d = 7u * q, a = d >> 2, sh = d & 3u;
        const uint32_t lo = __builtin_amdgcn_alignbyte(r[a + 1], r[a], sh);
        const uint32_t hi = __builtin_amdgcn_alignbyte(r[a + 2], r[a + 1], sh);
        uint64_t v = (uint64_t)lo | ((uint64_t)hi << 32);
        const uint32_t take = rq < 7u ? rq : 7u;
        v &= (1ull << (8u * take)) - 1ull;
        k.c[q] = rq ? ((__builtin_bswap64(v) & ~0xffull) | (rq < 8u ? rq : 8u)) : 0ull;
    }
    return k;
}

// <0, 0, >0 for record a vs record b (spans xa, xb) given their chunk keys.
__device__ __forceinline__ int seg_cmp(const uint8_t *S, const SegKeys &a, uint2 xa, const SegKeys &b, uint2 xb,
                                       uint32_t base) {
#pragma unroll
    for (int q = 0; q < SEG_CH; ++q) {
        if (a.c[q] != b.c[q]) return a.c[q] < b.c[q] ? -1 : 1;
        if ((a.c[q] & 0xffu) < 8u) return 0;
    }
    return rec_cmp8(S, xa.x, xa.y - xa.x, xb.x, xb.y - xb.x, bk_off(base) + 7u * SEG_CH);
}

// Rank the k members a.. of one segment with the G lanes gbase.. of the wave (lane gl of
// the group = member gl): rank = members ordered before it (ties by index), dup = an
// equal member with a smaller index exists. Writes the member's span at its rank.
// Only two chunk keys per member travel between lanes: the group's first chunk where its
// members differ (chunks before it are equal for all of them: a host's records share their
// name), and the next; past those two the bytes are compared in the input (rare: the records
// still tie there). Equivalent to seg_cmp: equal leading chunks with a full tag decide nothing.
// The rank loop's byte compare past the chunk keys (members tying there: long records, X1's
// httpx lines): wide loads, 48 bytes per round trip (8-B steps before: X1 seg_small 0.128 ->
// 0.098 ms).
// WIDE only for long records: its code in the loop costs the short-record launches occupancy
// (C5 seg_wave 23.9 -> 27.9 ms with it).
#define SEG_BYTES_CMP(S_, x_, y_, o_)                                                              \
    (WIDE ? rec_cmp_w(S_, x_.x, x_.y, S_, y_.x, y_.y, o_) : rec_cmp8(S_, x_.x, x_.y - x_.x, y_.x, y_.y - y_.x, o_))
// The two chunk keys travel through LDS (s_w: this wave's SEG_WS entries): each rank step is
// one broadcast 16-B read instead of four 32-bit lane shuffles, and the other member's span,
// needed only for the rare byte compare, is read from SS then (two more shuffles per step
// before: C5 seg_wave + seg_small 39.4 ms per step).
constexpr uint32_t SEG_WS = 68;  // 64 members + a 16-B pad per 16-lane group (no bank conflicts)
__device__ __forceinline__ void seg_wave_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}
template <int G, bool WIDE>
__device__ __forceinline__ void seg_rank_group(const uint8_t *__restrict__ S, uint2 *__restrict__ SS,
                                               uint8_t *__restrict__ dup, uint32_t a, uint32_t k, uint32_t gl,
                                               uint32_t gbase, bool live, uint32_t base, uint4 *s_w) {
    const bool act = live && gl < k;
    const uint2 x = act ? SS[a + gl] : make_uint2(0u, 0u);
    const SegKeys mk = act ? seg_keys(S, x, base) : SegKeys{{0, 0, 0, 0}};
    // st: the first chunk that varies inside the group or ends its records (group-uniform)
    const uint64_t gmask = (G == 64) ? ~0ull : (((1ull << G) - 1ull) << gbase);
    uint32_t st = SEG_CH;
#pragma unroll
    for (int c = SEG_CH - 1; c >= 0; --c) {
        const uint64_t l = __shfl(mk.c[c], (int)gbase, 64);
        const bool dif = act && mk.c[c] != l;
        if ((__ballot(dif) & gmask) || (l & 0xffu) < 8u) st = (uint32_t)c;
    }
    auto pick = [&](uint32_t q) -> uint64_t {
        uint64_t v = 0;
#pragma unroll
        for (int c = 0; c < SEG_CH; ++c) v = (q == (uint32_t)c) ? mk.c[c] : v;
        return v;
    };
    const uint64_t m1 = pick(st), m2r = pick(st + 1);  // (past the last chunk: 0)
    // Branch-free order on (m1, m2): m2 counts only while m1 holds a full 7 bytes (a tag < 8
    // ends the record, so equal m1 then means equal records); `full`: equal keys leave the
    // order to the bytes past them (group-uniform given equal m1 and m2)
    const bool m1full = (m1 & 0xffu) >= 8u;
    const uint64_t m2 = m1full ? m2r : 0ull;
    const bool full = st >= SEG_CH || (m1full && (st + 1u >= SEG_CH || (m2 & 0xffu) >= 8u));
    const uint32_t boff = bk_off(base) + 7u * (st + 2u < SEG_CH ? st + 2u : SEG_CH);
    uint32_t rank = 0;
    bool d = false;
    const uint32_t kk = live ? k : 0u;
    // loop bound uniform across the wave (max over its groups)
    uint32_t kmax = kk;
#pragma unroll
    for (int o = G; o < 64; o <<= 1) kmax = max(kmax, (uint32_t)__shfl_xor((int)kmax, o, 64));
    uint4 *gw = s_w + gbase + (gbase >> 4);
    seg_wave_sync();  // the previous group's reads of s_w are done
    gw[gl] = make_uint4((uint32_t)m1, (uint32_t)(m1 >> 32), (uint32_t)m2, (uint32_t)(m2 >> 32));
    seg_wave_sync();
    // one member's comparison (j: its index in the group, ov: its keys from LDS)
    auto step = [&](uint32_t j, const uint4 ov) {
        const uint64_t o1 = (uint64_t)ov.x | ((uint64_t)ov.y << 32), o2 = (uint64_t)ov.z | ((uint64_t)ov.w << 32);
        // long records (WIDE) tie past the chunk keys often: their spans still travel by shuffle
        uint2 yw = make_uint2(0u, 0u);
        if constexpr (WIDE) {
            const int src = (int)(gbase + (j < kk ? j : 0u));
            yw = make_uint2((uint32_t)__shfl(x.x, src, 64), (uint32_t)__shfl(x.y, src, 64));
        }
#define SEG_Y (WIDE ? yw : SS[a + j])
        const bool valid = act && j < kk && j != gl;
        bool gt = (o1 < m1) || (o1 == m1 && o2 < m2);  // the other member orders first
        bool eq = o1 == m1 && o2 == m2;
        if (valid && eq && full) {  // rare on short records: the bytes decide
            const int c = SEG_BYTES_CMP(S, x, SEG_Y, boff);
            gt = c > 0;
            eq = c == 0;
        }
#undef SEG_Y
        const bool before = j < gl;
        rank += (valid && (gt || (eq && before))) ? 1u : 0u;
        d = d || (valid && eq && before);
    };
    uint4 nv = gw[0];
    for (uint32_t j = 0; j < kmax; ++j) {
        // the next member's keys read one step ahead (gw[j + 1] stays inside this wave's
        // SEG_WS entries; j >= kk: a stale entry, never used)
        const uint4 ov = nv;
        nv = gw[j + 1];
        step(j, ov);
    }
    if (act) {
        SS[a + rank] = x;
        dup[a + rank] = d ? 1 : 0;
    }
}

// 16 lanes per small segment (<= SEG_SMALL members).
template <bool WIDE>
__global__ __launch_bounds__(256) void k_seg_small(const uint8_t *__restrict__ S, uint2 *__restrict__ SS,
                                                   const uint8_t *__restrict__ brk, uint8_t *__restrict__ dup,
                                                   const uint32_t *__restrict__ heads, uint32_t nh, uint32_t n,
                                                   uint32_t base) {
    const uint32_t lane = lane_id(), gl = lane & 15u, gbase = lane & ~15u;
    const uint32_t q = blockIdx.x * 16u + (threadIdx.x >> 4);
    const bool live = q < nh;
    const uint32_t a = live ? heads[q] : 0u;
    const uint32_t pe = a + 1u + gl;
    const bool eb = !live || pe >= n || gl == 15u || brk[pe];
    const uint32_t me = (uint32_t)(__ballot(eb) >> gbase) & 0xffffu;
    const uint32_t k = 1u + (uint32_t)(__ffs((int)me) - 1);  // members: a .. a+k-1
    __shared__ uint4 s_w[4][SEG_WS];
    seg_rank_group<16, WIDE>(S, SS, dup, a, k, gl, gbase, live, base, s_w[threadIdx.x >> 6]);
}

// Larger segments (17..64 members), two heads per wave: two half-waves when both segments
// hold <= 32 members (the common case: a host's few ports x a few copies), else one
// segment after the other on the whole wave.
template <bool WIDE>
__global__ __launch_bounds__(256) void k_seg_wave(const uint8_t *__restrict__ S, uint2 *__restrict__ SS,
                                                  const uint8_t *__restrict__ brk, uint8_t *__restrict__ dup,
                                                  const uint32_t *__restrict__ heads, uint32_t nh, uint32_t n,
                                                  uint32_t *err, uint32_t base) {
    const uint32_t q0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 2u;
    const uint32_t lane = lane_id();
    if (q0 >= nh) return;
    uint32_t a[2], k[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const bool live = q0 + t < nh;
        a[t] = live ? heads[q0 + t] : 0u;
        const uint32_t pe = a[t] + 1u + lane;
        const uint64_t me = __ballot(!live || pe >= n || brk[pe]);
        if (!me) { if (lane == 0) atomicOr(err, 1u); return; }
        k[t] = live ? 1u + (uint32_t)(__ffsll((long long)me) - 1) : 0u;
    }
    __shared__ uint4 s_w[4][SEG_WS];
    uint4 *w = s_w[threadIdx.x >> 6];
    if (k[0] <= 32u && k[1] <= 32u) {
        const uint32_t t = lane >> 5;
        const uint32_t kt = t ? k[1] : k[0];
        seg_rank_group<32, WIDE>(S, SS, dup, t ? a[1] : a[0], kt, lane & 31u, lane & 32u, kt > 0, base, w);
    } else {
        seg_rank_group<64, WIDE>(S, SS, dup, a[0], k[0], lane, 0u, true, base, w);
        if (k[1]) seg_rank_group<64, WIDE>(S, SS, dup, a[1], k[1], lane, 0u, true, base, w);
    }
}

// Profiling only: members of the listed bad segments (their heads), for the byte model of
// the segment sorts (span in/out, the record bytes behind the chunk keys, dup flag).
__global__ __launch_bounds__(256) void k_seg_members(const uint8_t *__restrict__ brk, const uint32_t *__restrict__ heads,
                                                     uint32_t nh, uint32_t n, unsigned long long *__restrict__ out) {
    uint32_t sum = 0;
    for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < nh; q += gridDim.x * blockDim.x) {
        uint32_t j = heads[q] + 1;
        while (j < n && !brk[j] && j - heads[q] < 64u) ++j;
        sum += j - heads[q];
    }
    sum = wave_sum(sum);
    if (lane_id() == 0 && sum) atomicAdd(out, (unsigned long long)sum);
}

// ------------------------------------------------------------------ gathers / output
__global__ void k_gather_rl(const uint32_t *__restrict__ idx, const uint32_t *__restrict__ R,
                            const uint32_t *__restrict__ L, uint32_t n, uint32_t *R2, uint32_t *L2) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t q = idx[i];
    R2[i] = R[q];
    L2[i] = L[q];
}

__global__ __launch_bounds__(256) void k_gather_spans(const uint32_t *__restrict__ V, const uint2 *__restrict__ spans,
                                                      uint32_t n, uint2 *__restrict__ out) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) out[i] = spans[V[i]];
}

__global__ void k_mark(const uint32_t *__restrict__ idx, uint32_t n, uint8_t *flag) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) flag[idx[i]] = 1;
}

// Prior check: flag[0] = 1 if records are not strictly increasing.
__global__ void k_check_sorted(const uint8_t *__restrict__ buf, const uint2 *__restrict__ spans, const uint64_t *__restrict__ K,
                               uint32_t n, uint32_t *flag, uint32_t base) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x + 1;
    if (i >= n) return;
    if (key_cmp_full(buf, spans, K[i - 1], i - 1, K[i], i, base) >= 0) atomicOr(flag, 1u);
}

// ------------------------------------------------------------------ diff
// U (this scan's unique records) and P (the prior's) are both sorted and duplicate-free,
// and equal records have equal key0. So the work splits on key0 alone: tile t owns
// U[t*DF_TILE, (t+1)*DF_TILE) and the P records with keys in [U.K[i0], U.K[i1]), found by
// a wave-cooperative 64-ary lower_bound over P.K (4 dependent probes at 10M, no byte
// compares). A U record is present in P iff some P record with its key0 has its bytes: a
// tag < 8 key0 is the whole record; a tag-8 one is compared bytewise (from byte 7) with
// the equal-key P records (almost always exactly one).
struct RecSet {
    const uint8_t *buf;
    const uint2 *sp;
    const uint64_t *K;    // key0 per position
    uint32_t n;
};

constexpr uint32_t DF_TILE = 256;  // U records per block
constexpr uint32_t DF_PCAP = 512;  // P keys + spans staged in LDS per block
constexpr uint32_t DF_PER = DF_TILE / 256;

// One wave per boundary t: jb[t] = lower_bound(P.K, U.K[t * DF_TILE]) (P.n past the end).
__global__ __launch_bounds__(256) void k_diff_split(const uint64_t *__restrict__ UK, uint32_t nu,
                                                    const uint64_t *__restrict__ PK, uint32_t np, uint32_t nb,
                                                    uint32_t *__restrict__ jb, uint32_t kw) {
    const uint32_t t = blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t lane = lane_id();
    if (t >= nb) return;
    const uint64_t i = (uint64_t)t * DF_TILE;
    if (i >= nu) { if (lane == 0) jb[t] = np; return; }
    const uint64_t key = UK[i];
    uint32_t lo = 0, hi = np;  // answer in [lo, hi]
    while (hi > lo) {
        const uint32_t span = hi - lo;
        if (span <= 64) {
            const uint32_t p = lo + lane;
            const bool ge = (p >= hi) || key_narrow(PK[p], kw) >= key;
            const uint64_t m = __ballot(ge);
            lo = m ? lo + (uint32_t)(__ffsll((long long)m) - 1) : hi;  // span 64, all below: hi
            break;
        }
        const uint32_t p = lo + (uint32_t)(((uint64_t)span * (lane + 1)) / 65);
        const bool ge = key_narrow(PK[p], kw) >= key;
        const uint64_t m = __ballot(ge);
        if (!m) {
            lo = (uint32_t)__shfl((int)p, 63, 64) + 1;
        } else {
            const int f = __ffsll((long long)m) - 1;
            const uint32_t pf = (uint32_t)__shfl((int)p, f, 64);
            const uint32_t pp = (uint32_t)__shfl((int)p, f > 0 ? f - 1 : 0, 64);
            hi = pf;
            if (f > 0) lo = pp + 1;
        }
    }
    if (lane == 0) jb[t] = lo;
}

__device__ __forceinline__ void diff_tile_body(RecSet U, RecSet P, const uint32_t *__restrict__ jb,
                                               uint8_t *__restrict__ fresh, uint32_t base) {
    // the tile's P keys AND spans in LDS: after the key search the candidate's span is an
    // LDS read, so the byte compare waits one global round trip (U and P bytes together)
    // instead of two (P span, then bytes); U spans load with the U keys
    __shared__ uint64_t s_k[DF_PCAP];
    __shared__ uint2 s_sp[DF_PCAP];
    const uint32_t kw = base >> 16;  // the prior's keys are narrowed here, as they are read
    const uint32_t t = blockIdx.x;
    const uint32_t i0 = t * DF_TILE;
    const uint32_t j0 = jb[t], j1 = jb[t + 1];
    const uint32_t np = j1 - j0;
    const bool staged = np <= DF_PCAP;
    if (staged)
        for (uint32_t q = threadIdx.x; q < np; q += 256) {
            s_k[q] = key_narrow(P.K[j0 + q], kw);
            s_sp[q] = P.sp[j0 + q];
        }
    uint32_t idx[DF_PER], cand[DF_PER];
    uint64_t ku[DF_PER];
    uint2 us[DF_PER];
    bool need[DF_PER], pres[DF_PER];
#pragma unroll
    for (int k = 0; k < DF_PER; ++k) {
        idx[k] = i0 + threadIdx.x + 256u * k;
        ku[k] = idx[k] < U.n ? U.K[idx[k]] : 0ull;
        us[k] = idx[k] < U.n ? U.sp[idx[k]] : make_uint2(0u, 0u);
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < DF_PER; ++k) {
        // lower_bound of ku in P[j0, j1) (LDS when staged)
        uint32_t lo = 0, hi = np;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            const uint64_t v = staged ? s_k[mid] : key_narrow(P.K[j0 + mid], kw);
            if (v < ku[k]) lo = mid + 1; else hi = mid;
        }
        cand[k] = j0 + lo;
        const uint64_t kp = (lo < np) ? (staged ? s_k[lo] : key_narrow(P.K[j0 + lo], kw))
                                      : (j0 + lo < P.n ? key_narrow(P.K[j0 + lo], kw) : ~ku[k]);
        const bool eq = idx[k] < U.n && j0 + lo < P.n && kp == ku[k];
        pres[k] = eq && (ku[k] & 0xffu) < bk_full(base);
        need[k] = eq && !pres[k];
    }
    // tag-8 candidates: the P span (LDS when staged), then a wide compare (loads of all
    // items together)
    uint2 ps[DF_PER];
#pragma unroll
    for (int k = 0; k < DF_PER; ++k)
        ps[k] = need[k] ? (staged && cand[k] < j1 ? s_sp[cand[k] - j0] : P.sp[cand[k]]) : make_uint2(0u, 0u);
#pragma unroll
    for (int k = 0; k < DF_PER; ++k) {
        if (!need[k]) continue;
        if (rec_equal_w(U.buf, us[k].x, us[k].y, P.buf, ps[k].x, ps[k].y, bk_off(base))) { pres[k] = true; continue; }
        // other P records sharing this key0 (distinct records with the same first 7 bytes):
        // they are sorted by their remaining bytes, so binary-search the run [c+1, c_end)
        // by full compare instead of scanning it
        const uint32_t c0 = cand[k] + 1;
        uint32_t ce = c0;
        if (staged && c0 - j0 <= np) {
            uint32_t lo = c0 - j0, hi = np;  // upper bound of ku in the staged keys
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (s_k[mid] <= ku[k]) lo = mid + 1; else hi = mid;
            }
            ce = j0 + lo;
        }
        if (!staged || ce >= j1) {
            // the run reaches past the staged keys (key0 shared by many prior records, e.g. a
            // URL scheme): gallop, then bisect, for its end in P.K instead of walking it
            uint32_t step = 1, lo2 = ce, hi2 = P.n;  // [ce, lo2) all equal ku
            for (;;) {
                const uint32_t probe = lo2 + step - 1;
                if (probe >= P.n) break;
                if (key_narrow(P.K[probe], kw) != ku[k]) { hi2 = probe; break; }
                lo2 = probe + 1;
                step <<= 1;
            }
            while (lo2 < hi2) {  // first index in [lo2, hi2) whose key differs
                const uint32_t mid = (lo2 + hi2) >> 1;
                if (key_narrow(P.K[mid], kw) == ku[k]) lo2 = mid + 1; else hi2 = mid;
            }
            ce = lo2;
        }
        uint32_t lo = c0, hi = ce;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            const uint2 x = P.sp[mid];
            const int cmp = rec_cmp8_2(P.buf, x.x, x.y - x.x, U.buf, us[k].x, us[k].y - us[k].x, bk_off(base));
            if (cmp == 0) { pres[k] = true; break; }
            if (cmp < 0) lo = mid + 1; else hi = mid;
        }
    }
#pragma unroll
    for (int k = 0; k < DF_PER; ++k)
        if (idx[k] < U.n) fresh[idx[k]] = pres[k] ? 0 : 1;
}

__global__ __launch_bounds__(256) void k_diff_tile(RecSet U, RecSet P, const uint32_t *__restrict__ jb,
                                                   uint8_t *__restrict__ fresh, uint32_t base) {
    diff_tile_body(U, P, jb, fresh, base);
}


// ------------------------------------------------------------------ common prefix (URL-like data)
// L = the longest prefix every record of cur and prior shares (capped at 255). All order and
// equality questions are then decided from byte L on, and key0 is taken there: for URL lists
// (every record starts "https://") the first 7 bytes say nothing, and equal-key0 runs would
// span the whole buffer (binary searches over them in the diff, refinement rounds in the sort).
// Key statistics for the sort (sg_internal.hpp KeyStats, KeyStatD): OR and AND over every
// key (their XOR: the bits that vary) and the tag byte's range (the narrowed tag
// min(tag, kw + 1) varies iff its clamped ends differ). Each block writes its partial with
// plain stores; k_key_sample's first block combines them (512 blocks' atomics on one line
// serialised: +20 µs on C2's cur keys).

// The common prefix of one record (key k, span xs) with the reference record.
__device__ __forceinline__ uint32_t lcp_one(const uint8_t *buf, const uint2 *spans, uint32_t i, uint64_t k,
                                            const uint8_t *rbuf, const uint2 *rspans, uint64_t kr, uint32_t best) {
    // key0 = 7 bytes big-endian << 8 | min(len, 8): the first 7 bytes come from the keys
    const uint64_t x = (k ^ kr) >> 8;
    const uint32_t tk = (uint32_t)(k & 0xffu), tr = (uint32_t)(kr & 0xffu);
    if (x) return min((uint32_t)__builtin_clzll(x << 8) >> 3, min(tk, tr));
    if (tk < 8u || tr < 8u) return min(tk, tr);
    // both share their first 7 bytes (URL schemes): 8 bytes per step from byte 7
    const uint2 xs = spans[i], r = rspans[0];
    const uint32_t m = min(min(xs.y - xs.x, r.y - r.x), best);
    uint32_t l = 7;
    while (l < m) {
        const uint32_t t = (m - l) < 8u ? (m - l) : 8u;
        const uint64_t d = load_le(buf, xs.x + l, t) ^ load_le(rbuf, r.x + l, t);
        if (d) { l += (uint32_t)__builtin_ctzll(d) >> 3; break; }
        l += t;
    }
    return min(l, m);
}

// st (optional): the keys' KeyStatD partial per block, gathered in the same read (the cur
// keys, for the sort).
constexpr int LCP_U = 4;
// CHK (sg_dev_dedup_diff_spans_into): the scan also checks the handed-over parse of `buf` (nb
// bytes) before anything else indexes the bytes with it: records must tile the buffer in
// order (record 0 starts at 0, each starts right after its predecessor's '\n', is non-empty,
// and the last '\n' is the buffer's last byte), and the span_mix terms are summed (per-block
// partials in chk) for comparison with the producer's checksum; k_chk_sample checks the
// sampled records' bytes. The spans are read beside the keys (each lane also loads its
// predecessor's span: the same lines, from cache). rnb (any mode): bytes of the reference
// record's buffer when its span is not trusted (0: trusted); an out-of-place reference span
// turns every byte compare off (the call fails on the check anyway). Records out of place are
// counted into *cbad_out (one atomic per wave that saw one: none when the parse is intact).
constexpr uint32_t CHK_SAMPLE = 256;
struct SpanChkPart {
    uint64_t sum;
    uint32_t bad, pad;
};
template <bool CHK>
__global__ __launch_bounds__(256) void k_lcp(const uint8_t *__restrict__ buf, const uint2 *__restrict__ spans,
                                             const uint64_t *__restrict__ keys, uint32_t n,
                                             const uint8_t *__restrict__ rbuf, const uint2 *__restrict__ rspans,
                                             const uint64_t *__restrict__ rkeys, uint32_t *__restrict__ out,
                                             KeyStatD *__restrict__ st, uint64_t *__restrict__ keysL, uint32_t Ls,
                                             KeyStatD *__restrict__ stL, uint32_t rnb, SpanChkPart *__restrict__ chk,
                                             uint32_t nb, uint32_t *__restrict__ cbad_out) {
    __shared__ uint32_t s_min[4];
    __shared__ KeyStatD s_st[4];
    __shared__ SpanChkPart s_chk[4];
    const uint64_t kr = rkeys[0];
    uint32_t best = 255;
    KeyStatAcc acc, accL;
    uint64_t csum = 0;
    uint32_t cbad = 0;
    // grid-stride (at most 2048 blocks): at most one memory-side atomic per block and word;
    // LCP_U keys in flight per thread (one dependent load per trip left the loop latency-bound:
    // 1.6 TB/s on C2's cur keys)
    // Records sharing the reference's first 7 bytes (URL lists: every record) continue in the
    // bytes: their spans, then their bytes 7..14, are loaded for the LCP_U keys together (one
    // record after another, each was two dependent loads: 228 us on 10M URLs); lcp_one takes
    // the rare records that also tie there.
    const uint32_t stride = gridDim.x * blockDim.x * LCP_U;
    const uint2 r = rspans[0];
    const bool rok = rnb == 0u || (r.y > r.x && r.y < rnb);
    const uint32_t rlen = r.y - r.x, tr = (uint32_t)(kr & 0xffu);
    for (uint32_t i0 = blockIdx.x * blockDim.x * LCP_U + threadIdx.x; i0 < n; i0 += stride) {
        uint64_t k[LCP_U];
        uint2 cs[LCP_U];
        uint32_t py[LCP_U];
        bool okl[LCP_U];
#pragma unroll
        for (int u = 0; u < LCP_U; ++u) {
            const uint32_t i = i0 + u * blockDim.x;
            k[u] = i < n ? keys[i] : 0ull;
            if (CHK) {
                cs[u] = i < n ? spans[i] : make_uint2(0u, 0u);
                py[u] = (i < n && i > 0u) ? spans[i - 1u].y : 0xffffffffu;  // record 0 must start at 0
            }
        }
        if (CHK) {
#pragma unroll
            for (int u = 0; u < LCP_U; ++u) {
                const uint32_t i = i0 + u * blockDim.x;
                okl[u] = i < n && cs[u].y > cs[u].x && cs[u].y < nb;
                const bool tiled = cs[u].x == py[u] + 1u;
                const bool last = i + 1u != n || cs[u].y + 1u == nb;
                if (i < n) {
                    cbad += (okl[u] && tiled && last) ? 0u : 1u;
                    csum += span_mix(cs[u].y - cs[u].x, k[u]);
                }
            }
        }
        bool slow[LCP_U];
#pragma unroll
        for (int u = 0; u < LCP_U; ++u) {
            const uint32_t i = i0 + u * blockDim.x;
            const uint32_t tk = (uint32_t)(k[u] & 0xffu);
            // bytes are read through a span only when it (and the reference's) is in place
            const bool bytes_ok = rok && (!CHK || okl[u]);
            slow[u] = i < n && ((k[u] ^ kr) >> 8) == 0 && tk >= 8u && tr >= 8u && best > 7u && bytes_ok;
            if (i < n) {
                acc.add(k[u]);
                if (!slow[u] && bytes_ok) best = min(best, lcp_one(buf, spans, i, k[u], rbuf, rspans, kr, best));
            }
        }
        uint2 xs[LCP_U];
#pragma unroll
        for (int u = 0; u < LCP_U; ++u) xs[u] = slow[u] ? spans[i0 + u * blockDim.x] : make_uint2(0u, 0u);
        uint64_t d[LCP_U], raw[LCP_U];
        uint32_t m[LCP_U], tt[LCP_U];
#pragma unroll
        for (int u = 0; u < LCP_U; ++u) {
            m[u] = min(min(xs[u].y - xs[u].x, rlen), best);
            tt[u] = m[u] > 7u ? min(m[u] - 7u, 8u) : 0u;
            raw[u] = (slow[u] && tt[u]) ? load_le(buf, xs[u].x + 7u, tt[u]) : 0ull;
            d[u] = (slow[u] && tt[u]) ? (raw[u] ^ load_le(rbuf, r.x + 7u, tt[u])) : 0ull;
        }
#pragma unroll
        for (int u = 0; u < LCP_U; ++u) {
            if (!slow[u]) continue;
            uint32_t l;
            if (d[u]) l = 7u + ((uint32_t)__builtin_ctzll(d[u]) >> 3);
            else if (7u + tt[u] >= m[u]) l = m[u];
            else l = lcp_one(buf, spans, i0 + u * blockDim.x, k[u], rbuf, rspans, kr, best);
            best = min(best, min(l, m[u]));
        }
        // keysL (Ls >= 8, the last call's common prefix): the keys at Ls of the records that
        // tie the reference on key0 (their bytes are in cache). Every record is one of them
        // when the common prefix comes out at Ls again; otherwise the keys are rebuilt.
        if (keysL) {
#pragma unroll
            for (int u = 0; u < LCP_U; ++u) {
                if (!slow[u]) continue;
                // at Ls = 8 the key's bytes 8..14 are in hand (bytes 7..14 were just loaded)
                const uint32_t len = xs[u].y - xs[u].x, rem = len > Ls ? len - Ls : 0u;
                uint64_t kl;
                if (Ls == 8u && tt[u] == 8u) {
                    const uint32_t take = rem < 7u ? rem : 7u;
                    kl = rem ? ((__builtin_bswap64((raw[u] >> 8) & ((1ull << (8u * take)) - 1ull)) & ~0xffull) |
                                (uint64_t)(rem < 8u ? rem : 8u))
                             : 0ull;
                } else {
                    kl = chunk_key(buf, xs[u].x, xs[u].y, Ls);
                }
                keysL[i0 + u * blockDim.x] = kl;
                accL.add(kl);
            }
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) best = min(best, (uint32_t)__shfl_xor((int)best, o, 64));
    if (lane_id() == 0) s_min[threadIdx.x >> 6] = best;
    if (st) kstat_flush(acc, s_st, st);
    if (stL) {
        __syncthreads();  // s_st reused
        kstat_flush(accL, s_st, stL);
    }
    if (CHK) {
        if (__ballot(cbad != 0u)) {  // (rare: a damaged parse) one atomic per such wave
            const uint32_t wb = wave_sum(cbad);
            if (lane_id() == 0) atomicAdd(cbad_out, wb);
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) csum += (uint64_t)__shfl_xor((long long)csum, o, 64);
        if (lane_id() == 0) s_chk[threadIdx.x >> 6] = SpanChkPart{csum, 0u, 0u};
    }
    __syncthreads();
    if (CHK && threadIdx.x == 0)
        chk[blockIdx.x] = SpanChkPart{s_chk[0].sum + s_chk[1].sum + s_chk[2].sum + s_chk[3].sum, 0u, 0u};
    if (threadIdx.x == 0) {
        const uint32_t b = min(min(s_min[0], s_min[1]), min(s_min[2], s_min[3]));
        // skip the memory-side atomic when an earlier block already published as small a prefix
        if (b < 255u && b < __hip_atomic_load(out, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMin(out, b);
    }
}

// The handover check's per-block checksum partials summed into out[0..1], read back with the
// prefix scan's flags (out[2], the records out of place, is counted by the checking kernels).
__global__ __launch_bounds__(256) void k_chk_combine(const SpanChkPart *__restrict__ part, uint32_t np,
                                                     uint32_t *__restrict__ out) {
    __shared__ uint64_t s[4];
    uint64_t sum = 0;
    for (uint32_t b = threadIdx.x; b < np; b += 256u) sum += part[b].sum;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sum += (uint64_t)__shfl_xor((long long)sum, o, 64);
    if (lane_id() == 0) s[threadIdx.x >> 6] = sum;
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint64_t t = s[0] + s[1] + s[2] + s[3];
        out[0] = (uint32_t)t;
        out[1] = (uint32_t)(t >> 32);
    }
}

// The handover check's byte samples: every CHK_SAMPLE-th record, when its span lies inside the
// buffer, must end at a '\n' and carry the key of its own bytes (a delivery that left a region
// of the bytes stale or shifted while the parse arrived intact); out-of-place ones counted
// into *bad (one atomic per wave that saw one).
__global__ __launch_bounds__(256) void k_chk_sample(const uint8_t *__restrict__ buf, const uint2 *__restrict__ spans,
                                                    const uint64_t *__restrict__ keys, uint32_t n, uint32_t nb,
                                                    uint32_t *__restrict__ bad) {
    const uint32_t j = blockIdx.x * 256u + threadIdx.x, i = j * CHK_SAMPLE;
    uint32_t b = 0;
    if (i < n) {
        const uint2 x = spans[i];
        const uint64_t k = keys[i];
        if (x.y > x.x && x.y < nb) b = (buf[x.y] == 0x0a && chunk_key(buf, x.x, x.y, 0u) == k) ? 0u : 1u;
        else b = 1u;
    }
    if (__ballot(b != 0u)) {
        const uint32_t wb = wave_sum(b);
        if (lane_id() == 0) atomicAdd(bad, wb);
    }
}

// KeyStatD of keys already in place (the gathered cur records of the fused match step).
__global__ __launch_bounds__(256) void k_key_stats(const uint64_t *__restrict__ keys, uint32_t n, KeyStatD *__restrict__ st) {
    __shared__ KeyStatD s_st[4];
    KeyStatAcc acc;
    const uint32_t stride = gridDim.x * blockDim.x * LCP_U;
    for (uint32_t i0 = blockIdx.x * blockDim.x * LCP_U + threadIdx.x; i0 < n; i0 += stride) {
        uint64_t k[LCP_U];
#pragma unroll
        for (int u = 0; u < LCP_U; ++u) {
            const uint32_t i = i0 + u * blockDim.x;
            k[u] = i < n ? keys[i] : keys[i0];
        }
#pragma unroll
        for (int u = 0; u < LCP_U; ++u) acc.add(k[u]);
    }
    kstat_flush(acc, s_st, st);
}

// key0 (7 bytes + min(rem, 8)) -> the kw-byte key (kw bytes + min(rem, kw + 1)).
__global__ __launch_bounds__(256) void k_narrow_keys(uint64_t *__restrict__ keys, uint32_t n, uint32_t kw) {
    const uint64_t top = ~0ull << (64u - 8u * kw);
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint64_t k = keys[i];
        const uint64_t t = k & 0xffu;
        keys[i] = (k & top) | (t < kw + 1u ? t : (uint64_t)(kw + 1u));
    }
}

// st (optional): the new keys' KeyStatD, gathered as they are written.
__global__ __launch_bounds__(256) void k_rekey(const uint8_t *__restrict__ buf, const uint2 *__restrict__ spans, uint32_t n,
                                               uint32_t base, uint64_t *__restrict__ keys, KeyStatD *__restrict__ st) {
    __shared__ KeyStatD s_st[4];
    KeyStatAcc acc;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint2 x = spans[i];
        const uint64_t k = chunk_key(buf, x.x, x.y, base);
        keys[i] = k;
        acc.add(k);
    }
    if (st) kstat_flush(acc, s_st, st);
}

// ------------------------------------------------------------------ host pipeline
int select_flags(sg_ctx *c, const uint8_t *flags, uint32_t n, uint32_t *out_idx, uint32_t *count) {
    return run_select2(c, "select", FlagPred{flags}, n, out_idx, (uint32_t *)nullptr, count, nullptr);
}

// Records recs[0..count) (ids into spans), in list order, '\n'-terminated: the emit
// machinery (count -> tile scan -> LDS-window copy), with one host sync for the size.
static int emit_records(sg_ctx *c, const uint8_t *d_buf, const uint2 *spans, const uint32_t *recs, uint32_t count,
                        int out_slot, uint8_t *dst, size_t dst_cap, uint8_t **d_out, uint64_t *bytes) {
    *bytes = 0;
    const uint32_t ntiles = (count + EM_TILE - 1) / EM_TILE;
    if (ntiles == 0) {
        if (!dst) SG_TRY(slot(c, out_slot, 16, d_out));
        else *d_out = dst;
        return SG_OK;
    }
    uint64_t *tp;  // tot[ntiles] | pre[ntiles] | total
    SG_TRY(slot(c, S_EMIT, 2 * (size_t)ntiles + 4, &tp));
    uint64_t *tot = tp, *pre = tp + ntiles, *total = tp + 2 * (size_t)ntiles;
    uint2 *cache;
    SG_TRY(slot(c, S_ECACHE, (size_t)count + 1, &cache));
    const PermItem item{recs, spans};
    SG_LAUNCH(c, "emit_lines.count", k_emit_count<PermItem>, ntiles, EM_BLOCK, 0, item, count, cache, tot);
    SG_TRY(tile_scan(c, tot, ntiles, pre, total));
    uint64_t tv = 0;
    SG_TRY(ctx_readback(c, &tv, total, 8));
    const uint64_t nb = (uint32_t)tv;
    if (dst) {
        if (nb > dst_cap) { set_error("output capacity %zu < %llu", dst_cap, (unsigned long long)nb); return SG_E_CAP; }
        *d_out = dst;
    } else {
        SG_TRY(slot(c, out_slot, nb + 16, d_out));
    }
    // model: each output byte read once and written once, plus the cached (start, len)
    SG_LAUNCH_B(c, "emit_lines", 2.0 * nb + 8.0 * count, k_emit_apply, ntiles, EM_BLOCK, 0, cache, count, pre, d_buf,
                *d_out, (uint2 *)nullptr, (const uint64_t *)nullptr, (uint64_t *)nullptr);
    *bytes = nb;
    return SG_OK;
}

int serialize(sg_ctx *c, const uint8_t *d_buf, const uint2 *spans,
              const uint32_t *recs, const uint32_t * /*map*/, uint32_t count, int out_slot,
              uint8_t **d_out, uint64_t *bytes) {
    return emit_records(c, d_buf, spans, recs, count, out_slot, nullptr, 0, d_out, bytes);
}

// Records recs[0..count) of d_buf, '\n'-terminated, written from dst_base + shift on (no
// host sync: the caller knows the byte count).
int emit_into(sg_ctx *c, const uint8_t *d_buf, const uint2 *spans, const uint32_t *recs, uint32_t count,
              uint8_t *dst_base, uint32_t shift) {
    uint64_t *tot;
    return run_emit(c, k_emit_apply, "part_emit", "part_emit.count", S_EMIT, PermItem{recs, spans}, count, d_buf, dst_base,
                    nullptr, nullptr, nullptr, &tot, 0.0, shift);
}

int serialize_into(sg_ctx *c, const uint8_t *d_buf, const uint2 *spans,
                   const uint32_t *recs, uint32_t count, uint8_t *dst, size_t dst_cap, uint64_t *bytes) {
    uint8_t *o;
    return emit_records(c, d_buf, spans, recs, count, 0, dst, dst_cap, &o, bytes);
}


// Order-preserving packing of a round's chunk keys (7 big-endian bytes + tag): each byte is
// replaced by its rank in the alphabet the keys use (0 always present: the filler past a
// record's end), s bits per byte, the tag kept in the low 4 bits. IP or digit-heavy chunks
// (13 symbols: 4 bits) then sort in 4 radix passes instead of 8.
__global__ __launch_bounds__(256) void k_alpha_mask(const uint64_t *__restrict__ K, uint32_t M, uint32_t *__restrict__ mask) {
    __shared__ unsigned long long s_m[4];
    if (threadIdx.x < 4) s_m[threadIdx.x] = threadIdx.x == 0 ? 1ull : 0ull;
    __syncthreads();
    // per thread in registers (selects, no indexed arrays), then OR-reduced over the wave
    uint64_t m0 = 0, m1 = 0, m2 = 0, m3 = 0;
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < M; j += gridDim.x * blockDim.x) {
        const uint64_t k = K[j];
#pragma unroll
        for (int b = 1; b < 8; ++b) {
            const uint32_t v = (uint32_t)(k >> (8 * b)) & 0xffu;
            const uint64_t bit = 1ull << (v & 63u);
            const uint32_t q = v >> 6;
            m0 |= q == 0 ? bit : 0ull;
            m1 |= q == 1 ? bit : 0ull;
            m2 |= q == 2 ? bit : 0ull;
            m3 |= q == 3 ? bit : 0ull;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        m0 |= __shfl_xor((unsigned long long)m0, o, 64);
        m1 |= __shfl_xor((unsigned long long)m1, o, 64);
        m2 |= __shfl_xor((unsigned long long)m2, o, 64);
        m3 |= __shfl_xor((unsigned long long)m3, o, 64);
    }
    if (lane_id() == 0) {
        atomicOr(&s_m[0], (unsigned long long)m0);
        atomicOr(&s_m[1], (unsigned long long)m1);
        atomicOr(&s_m[2], (unsigned long long)m2);
        atomicOr(&s_m[3], (unsigned long long)m3);
    }
    __syncthreads();
    if (threadIdx.x < 8) {
        const uint32_t w = (uint32_t)(s_m[threadIdx.x >> 1] >> (32 * (threadIdx.x & 1)));
        if (w) atomicOr(&mask[threadIdx.x], w);
    }
}

// RG (optional): each row's group index placed above the packed key (bit kb on), so one
// sort orders rows by (group, chunk).
__global__ __launch_bounds__(256) void k_alpha_pack(uint64_t *__restrict__ K, uint32_t M, const uint8_t *__restrict__ rank,
                                                    uint32_t sbits, const uint32_t *__restrict__ RG, uint32_t kb) {
    __shared__ uint8_t s_r[256];
    s_r[threadIdx.x] = rank[threadIdx.x];
    __syncthreads();
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < M; j += gridDim.x * blockDim.x) {
        const uint64_t k = K[j];
        uint64_t p = 0;
#pragma unroll
        for (int b = 7; b >= 1; --b) p = (p << sbits) | s_r[(k >> (8 * b)) & 0xffu];
        p = (p << 4) | (k & 0xfu);
        K[j] = RG ? (((uint64_t)RG[j] << kb) | p) : p;
    }
}

// ------------------------------------------------------------------ big-group rounds
// Positions GS[g]..GE[g] (g < B) are groups of > 64 records sharing their first `off`
// bytes. Each round sorts every group's members by the next 7-byte chunk (stable), marks
// sub-segment heads in brk, and keeps the sub-segments that are still > 64 records.
template <typename VT>
static int refine_big_groups(sg_ctx *c, const uint8_t *d_buf, const uint2 *spans, VT *V, uint8_t *brk,
                             uint32_t *GS, uint32_t *GE, uint32_t B, uint32_t bk) {
    uint32_t off = (bk & 0xffffu) + (bk >> 16);
    while (B > 0) {
        uint64_t *goff;
        SG_TRY(slot(c, S_R_OFF, (size_t)B + 1, &goff));
        uint64_t M64 = 0;
        SG_TRY(run_scan64(c, "scan_groups", GroupSizeFn{GS, GE}, B, goff, &M64));
        const uint32_t M = (uint32_t)M64;
        uint64_t *RK, *RK2;
        uint32_t *RG, *RP, *RV, *RV2;
        SG_TRY(slot(c, S_R_KEY, M, &RK));
        SG_TRY(slot(c, S_R_KEY2, M, &RK2));
        SG_TRY(slot(c, S_R_GID, M, &RG));
        SG_TRY(slot(c, S_R_POS, M, &RP));
        SG_TRY(slot(c, S_R_VAL, M, &RV));
        SG_TRY(slot(c, S_R_VAL2, M, &RV2));
        SG_LAUNCH(c, "round_expand", k_expand<VT>, (M + 4 * EXP_ROWS - 1) / (4 * EXP_ROWS), 256, 0, d_buf, spans, GS, goff,
                  B, V, M, off, RK, RG, RP);
        // the chunk keys' byte alphabet: packed keys when it is small enough to save passes
        uint32_t *amask;
        SG_TRY(slot(c, S_R_ALPHA, 8 + 64, &amask));
        SG_HIP(hipMemsetAsync(amask, 0, 32, c->stream));
        SG_LAUNCH(c, "round_alpha", k_alpha_mask, std::min<uint32_t>(grid_for(M, 256), 512u), 256, 0, RK, M, amask);
        uint32_t hm[8];
        SG_TRY(ctx_readback(c, hm, amask, 32));
        uint8_t rank[256];
        uint32_t na = 0;
        for (uint32_t v = 0; v < 256; ++v) {
            rank[v] = (uint8_t)na;
            if ((hm[v >> 5] >> (v & 31)) & 1u) ++na;
        }
        uint32_t sbits = 1;
        while ((1u << sbits) < na) ++sbits;
        int gbits = 1;
        while (gbits < 32 && (1u << gbits) < B) ++gbits;
        int kbits = 64;
        bool joint = false;  // (group, packed chunk) in one key: one sort, no group pass
        if (7 * sbits + 4 <= 56) {  // at least one radix pass fewer
            kbits = (int)(7 * sbits + 4);
            joint = kbits + gbits <= 64;
            uint8_t *drank = reinterpret_cast<uint8_t *>(amask + 8);
            SG_TRY(ctx_upload(c, drank, rank, 256));  // staged: the stack copy may go
            SG_LAUNCH(c, "round_alpha", k_alpha_pack, std::min<uint32_t>(grid_for(M, 256), 2048u), 256, 0, RK, M, drank,
                      sbits, joint ? RG : (const uint32_t *)nullptr, (uint32_t)kbits);
        }
        uint64_t *FK;
        uint32_t *perm2, *Tfree;
        uint64_t *FKw;  // the round_gather's key output (null: FK = the sorted packed keys)
        if (joint) {
            uint64_t *SK;
            SG_TRY(radix_sort(c, RK, RV, RK2, RV2, M, 0, kbits + gbits, true, &SK, &perm2, "rs_pass_refine"));
            Tfree = (perm2 == RV) ? RV2 : RV;
            FK = SK;  // (group, packed chunk): equal iff same group and same chunk; tag in bits 0..3
            FKw = nullptr;
        } else {
            uint64_t *SK;
            uint32_t *perm;
            SG_TRY(radix_sort(c, RK, RV, RK2, RV2, M, 0, kbits, true, &SK, &perm, "rs_pass_refine"));
            // stable by group index on top: keys = gid of each row in current order
            uint64_t *GK = (SK == RK) ? RK2 : RK;
            uint32_t *pv_alt = (perm == RV) ? RV2 : RV;
            SG_LAUNCH(c, "round_gid", k_gid_keys, grid_for(M, 256), 256, 0, RG, perm, GK, M);
            uint64_t *GK2 = (GK == RK) ? RK2 : RK;
            uint64_t *FKs;
            SG_TRY(radix_sort(c, GK, perm, GK2, pv_alt, M, 0, gbits, false, &FKs, &perm2, "rs_pass_refine"));
            Tfree = (perm2 == perm) ? pv_alt : perm;
            FK = (FKs == GK) ? GK2 : GK;
            FKw = FK;
        }
        VT *T;
        if constexpr (sizeof(VT) == 4) T = Tfree;
        else SG_TRY(slot(c, S_R_T2, M, &T));
        SG_LAUNCH(c, "round_gather", k_round_gather<VT>, grid_for(M, 256), 256, 0, d_buf, spans, V, RP, perm2, M, off, T, FKw);
        SG_LAUNCH(c, "round_scatter", k_round_scatter<VT>, grid_for(M, 256), 256, 0, T, RP, M, V);
        // perm2 and the free id buffer are reusable after the scatter (same stream)
        uint32_t *NS = perm2, *NE = Tfree;
        uint32_t B3 = 0, B4 = 0;
        SG_TRY(run_select2(c, "round_mark", RoundGroupPred{FK, RG, RP, brk, M, joint ? 0xfull : 0xffull}, M, NS, NE, &B3,
                           &B4));
        if (B3 != B4) { set_error("round group mismatch %u/%u", B3, B4); return SG_E_HIP; }
        if (B3) {
            SG_LAUNCH(c, "round_pos", k_pos_of, grid_for(B3, 256), 256, 0, NS, RP, B3, GS);
            SG_LAUNCH(c, "round_pos", k_pos_of, grid_for(B3, 256), 256, 0, NE, RP, B3, GE);
        }
        B = B3;
        off += 7;
    }
    return SG_OK;
}

// ------------------------------------------------------------------ unique view
// The sorted unique records of one buffer: serialized ('\n'-terminated, byte order) with
// per-record spans into `buf` and key0. For a prior that is already strictly increasing
// the view is the input itself.
struct UView {
    const uint8_t *buf = nullptr;
    const uint2 *spans = nullptr;
    const uint64_t *keys = nullptr;
    uint32_t n = 0;
    uint64_t bytes = 0;
    uint32_t in_records = 0;
};

struct ViewSlots {
    SlotSet lines;
    int ubuf, uspans, ukeys;
};

static const ViewSlots CUR_VIEW = {CUR_SLOTS, S_OUT_UNIQ, S_U_SPANS, S_U_KEYS};
static const ViewSlots PRIOR_VIEW = {PRIOR_SLOTS, S_P_UBUF, S_P_USPANS, S_P_UKEYS};

// `pre`: the buffer's lines already parsed (and, for a trusted view, `trust_sorted` already
// decided by the caller's check_sorted), so no parse or sortedness check is queued here.
// A caller output (dst, capacity >= n + 1) replaces the unique-view slot: the unique records
// are written from dst on (the view's buf is dst rounded down to 16 B, its spans shifted).
struct OutBuf {
    uint8_t *p = nullptr;
    size_t cap = 0;
    uint8_t *base() const { return reinterpret_cast<uint8_t *>((uintptr_t)p & ~(uintptr_t)15); }
    uint32_t shift() const { return (uint32_t)((uintptr_t)p & 15); }
};

static int build_unique(sg_ctx *c, const uint8_t *d_buf, uint64_t n, const ViewSlots &vs, bool trust_sorted,
                        UView *uv, const Lines *pre = nullptr, uint32_t base = make_bk(0u, 7u), const OutBuf *dst = nullptr,
                        const KeyStats *ks = nullptr) {
    *uv = UView{};
    Lines L;
    if (pre) L = *pre;
    else SG_TRY(run_lines(c, d_buf, n, vs.lines, &L));
    const uint32_t R = L.n_rec;
    uv->in_records = R;
    if (R >= (1u << 30)) { set_error("%u records exceed the 2^30 per-call limit", R); return SG_E_TOO_LARGE; }
    if (trust_sorted && R > 1 && !pre) {
        uint32_t *flag;
        SG_TRY(slot(c, S_M_CNT, 4, &flag));
        SG_HIP(hipMemsetAsync(flag, 0, 4, c->stream));
        SG_LAUNCH_B(c, "check_sorted", 8.0 * R, k_check_sorted, grid_for(R - 1, 256), 256, 0, d_buf, L.spans, L.keys, R, flag,
                    base);
        uint32_t f = 1;
        SG_TRY(ctx_readback(c, &f, flag, 4));
        trust_sorted = (f == 0);
    }
    if (trust_sorted || R <= 1) {
        if (R == 1 || trust_sorted) {
            uv->buf = d_buf;
            uv->spans = L.spans;
            uv->keys = L.keys;
            uv->n = R;
            uv->bytes = R ? (uint64_t)0 : 0;  // not used for an input view
            if (!trust_sorted) {
                // a single record: serialize it (the caller may return this view); its key
                // narrowed here (a sort would have done it on its first pass)
                if ((base >> 16) < 7u)
                    SG_LAUNCH(c, "narrow_keys", k_narrow_keys, 1, 256, 0, L.keys, R, base >> 16);
                uint8_t *ub;
                uint2 *us;
                uint64_t *uk;
                if (dst) ub = dst->base();
                else SG_TRY(slot(c, vs.ubuf, (size_t)n + 64, &ub));
                SG_TRY(slot(c, vs.uspans, 1, &us));
                SG_TRY(slot(c, vs.ukeys, 1, &uk));
                uint64_t *cnt;
                SG_TRY(run_emit(c, k_emit_uniq, "emit_uniq", "emit_uniq.count", S_EMIT2, PermItem{nullptr, L.spans}, R, d_buf, ub,
                                us, L.keys, uk, &cnt, 0.0, dst ? dst->shift() : 0u));
                uint64_t t = 0;
                SG_TRY(ctx_readback(c, &t, cnt, 8));
                *uv = UView{ub, us, uk, (uint32_t)(t >> 32), (uint32_t)t, R};
            }
            return SG_OK;
        }
        uint8_t *ub;
        if (dst) ub = dst->base();
        else SG_TRY(slot(c, vs.ubuf, 64, &ub));
        uv->buf = ub;
        return SG_OK;  // R == 0
    }

    // sort (key0, span) pairs: the spans come out in sorted order (the records' ids are
    // never needed, so no gather of spans by id afterwards)
    // (the parse's span array is the first ping-pong buffer: nothing reads it afterwards)
    uint64_t *k2;
    uint2 *v2;
    SG_TRY(slot(c, vs.lines.keys2, R, &k2));
    SG_TRY(slot(c, vs.lines.vals2, R, &v2));
    uint64_t *K;
    uint2 *V;
    // the key narrowing to kw bytes happens in the sort's first pass; with the key histograms
    // on the host the sort may finish its low digits per group in LDS (lerr: checked with
    // the group counts below, before anything trusts the order)
    // segbad (a flag per position), then the counters read back together: the three list
    // counters (zeroed with the head marks), the segment-head select's total, the local
    // sort's overflow word
    const size_t cnt_off = ((size_t)R + 15) & ~(size_t)15;
    uint8_t *segbad;
    SG_TRY(slot(c, S_BAD, cnt_off + 32, &segbad));
    uint32_t *acnt = reinterpret_cast<uint32_t *>(segbad + cnt_off);
    uint64_t *stot_at = reinterpret_cast<uint64_t *>(acnt + 4);
    uint32_t *lerr = nullptr;
    SG_TRY(radix_sort_spans(c, L.keys, L.spans, k2, v2, R, 0, 64, &K, &V, "rs_pass", ks,
                            (base >> 16) < 7u ? base >> 16 : 0u, ks ? &lerr : nullptr, acnt + 6));
    if (lerr) c->last_flags |= 1u;

    // key0 groups -> brk; groups of > 64 records sharing 7 bytes -> refinement rounds
    uint8_t *brk;
    SG_TRY(slot(c, S_BRK, (size_t)R + 32, &brk));  // + the 16-B windows of the brk scans
    uint32_t *GS, *GE;
    SG_TRY(slot(c, S_GS, R / 64 + 16, &GS));
    SG_TRY(slot(c, S_GE, R / 64 + 16, &GE));
    uint32_t B = 0;
    uint32_t ns = 0, nb = 0;
    uint32_t *hs, *hb;
    uint8_t *dup;
    SG_TRY(slot(c, S_DUP, R, &dup));
    SG_TRY(slot(c, S_SEL, (size_t)R / 2 + 16, &hs));
    SG_TRY(slot(c, S_R_VAL, (size_t)R / 17 + 16, &hb));
    const AdjLists AL{hs, hb, GS, GE, acnt, R / 2 + 16, R / 17 + 16, R / 64 + 16};
    // adjacent equality inside segments; segments holding two different records -> sort.
    // model: key0 + brk + span per record, both records' bytes where compared, dup out
    uint64_t *stot = nullptr;
    // All-segments mode: when the last call on this context kept few of its records (most
    // records repeat, and their groups hold near-duplicates: host:port scans, where a host's
    // ports share key0 — C5), the adjacent pass compares no bytes and every segment of two
    // or more records goes to the segment sorts, which rank its members and mark their
    // duplicates: each grouped record is gathered once (by its segment sort) instead of twice
    // (the adjacent compare, then the sort). Results are the same either way.
    const int sa = sw_seg_all();
    const bool seg_all = sa == 2 || (sa == 1 && c->last_uniq_frac < SEG_ALL_UNIQ);
    if (seg_all) c->last_flags |= 8u;
    auto adjacent = [&](bool keys, bool with_dup, const uint8_t *Sb, const uint2 *SSp) -> int {
        SG_HIP(hipMemsetAsync(segbad, 0, cnt_off + 16, c->stream));  // head marks + list counters
        // (keys only: after refinement rounds a segment of more than 64 identical records may
        // remain — rounds stop where the records end — which only the byte compare marks)
        if (seg_all && with_dup && keys) {
            SG_LAUNCH_B(c, "mark_groups", 10.0 * R, (k_adjacent2<true, false, true>), grid_for(R, 256), 256, 0, Sb, SSp, K,
                        brk, R, dup, segbad, AL, base);
            SG_TRY(run_select2_nb(c, "seg_heads", SegPred{brk, segbad, R}, R, hs, hb, S_COUNT2, &stot, stot_at));
            return SG_OK;
        }
        if (keys && with_dup)
            SG_LAUNCH_B(c, "adjacent", 19.0 * R + (double)n, (k_adjacent2<true, true>), grid_for(R, 256), 256, 0, Sb, SSp, K,
                        brk, R, dup, segbad, AL, base);
        else if (keys)
            SG_LAUNCH_B(c, "mark_groups", 9.0 * R, (k_adjacent2<true, false>), grid_for(R, 256), 256, 0, Sb, SSp, K, brk, R,
                        dup, segbad, AL, base);
        else
            SG_LAUNCH_B(c, "adjacent", 19.0 * R + (double)n, (k_adjacent2<false, true>), grid_for(R, 256), 256, 0, Sb, SSp, K,
                        brk, R, dup, segbad, AL, base);
        if (with_dup) SG_TRY(run_select2_nb(c, "seg_heads", SegPred{brk, segbad, R}, R, hs, hb, S_COUNT2, &stot, stot_at));
        return SG_OK;
    };
    uint32_t lerr_v = 0;
    // the big-group count, the segment-head select's counts and the local sort's overflow
    // word with one host sync
    auto read_counts = [&](bool with_heads) -> int {
        uint8_t *pin = (uint8_t *)c->pinned;
        SG_HIP(hipMemcpyAsync(pin, acnt, 32, hipMemcpyDeviceToHost, c->stream));  // acnt | stot | lerr[2]
        SG_HIP(hipStreamSynchronize(c->stream));
        uint32_t v[3];
        memcpy(v, pin, 12);
        lerr_v = 0;
        if (lerr) {
            uint32_t fixed = 0;
            memcpy(&lerr_v, pin + 24, 4);  // big groups listed by the local sort's fix-up pass
            memcpy(&fixed, pin + 28, 4);   // tiles that pass redid
            if (fixed) c->last_flags |= 4u;
        }
        B = v[2];
        if (with_heads) {
            uint64_t t = 0;
            memcpy(&t, pin + 16, 8);
            ns = (uint32_t)(t >> 31);
            nb = (uint32_t)(t & 0x7fffffffu);
        }
        if (B > R / 64 + 16) { set_error("adjacent: big-group list overflow (%u)", B); return SG_E_HIP; }
        return SG_OK;
    };
    // With narrowed keys (kw < 7: few big groups) the adjacent compare runs before the group
    // count comes back (one host sync for everything); when big groups exist (the 7-byte key
    // was kept: low-entropy text) the groups are marked first and compared after refinement.
    // In the all-segments mode the keys pass compares no bytes either way, so it marks the
    // segments at once; only when big groups come back does the byte pass follow refinement.
    const bool speculate = (base >> 16) < 7u;
    const bool first_dup = speculate || seg_all;
    bool fix_tried = false;
    for (;;) {
        SG_TRY(adjacent(true, first_dup, d_buf, V));
        SG_TRY(read_counts(first_dup));
        if (!lerr_v) break;
        uint64_t *Ka = (K == L.keys) ? k2 : L.keys;
        uint2 *Va = (V == L.spans) ? v2 : L.spans;
        if (!fix_tried) {
            // a group larger than any LDS window (its pairs are intact, unsorted; the tiles
            // around it were already redone in the sort's own stream): the big groups' members
            // sorted by one radix sort from the local sort's input (Ka, Va still hold it; a
            // record repeated thousands of times), then the adjacent pass again
            fix_tried = true;
            SG_TRY(lsort_fixup_big(c, Ka, Va, K, V, R, lerr_v));
            SG_HIP(hipMemsetAsync(lerr, 0, 4, c->stream));
            c->last_flags |= 4u;
            continue;
        }
        // (not reached unless the fix-up flags again) the plain LSD sort of the same pairs
        // (keys already narrowed, histograms unchanged)
        SG_TRY(radix_sort_spans(c, K, V, Ka, Va, R, 0, 64, &K, &V, "rs_pass", ks, 0u, nullptr));
        lerr = nullptr;
        c->last_flags |= 2u;
    }
    if (B) SG_TRY(refine_big_groups(c, d_buf, L.spans, V, brk, GS, GE, B, base));

    // The records in this order: SS = the input spans in sorted order (the sort's payload),
    // S = the input itself; the later passes (adjacent compare, segment sort, unique emit)
    // gather from the input. Measured cheaper than materialising a sorted copy first (C2
    // 2.51 -> 2.30 ms, X1 4.37 -> 3.97 ms): the copy gathered every record once and the
    // unique emit copied ~2/3 of them again, where gathering only the unique records reads
    // each kept record once.
    uint8_t *Sb = const_cast<uint8_t *>(d_buf);
    uint2 *SS = V;  // the segment sorts permute it in place
    if (!first_dup || B) {
        SG_TRY(adjacent(false, true, Sb, SS));
        SG_TRY(read_counts(true));
    }
    // the run-sort error word beside the unique emit's total (that slot at its final size
    // now, so run_emit finds it in place): one copy brings both back
    uint32_t *err;
    {
        const uint32_t ent = (R + EM_TILE - 1) / EM_TILE;
        uint64_t *etp;
        SG_TRY(slot(c, S_EMIT2, 2 * (size_t)ent + 4, &etp));
        err = reinterpret_cast<uint32_t *>(etp + 2 * (size_t)ent + 1);
    }
    if (nb) SG_HIP(hipMemsetAsync(err, 0, 4, c->stream));
    // long records (mean >= 48 B: httpx lines) compare their tails with wide loads
    const bool wide_cmp = n >= 48ull * R;
    if (ns) {
        if (wide_cmp) SG_LAUNCH(c, "seg_small", k_seg_small<true>, grid_for(ns, 16), 256, 0, Sb, SS, brk, dup, hs, ns, R, base);
        else SG_LAUNCH(c, "seg_small", k_seg_small<false>, grid_for(ns, 16), 256, 0, Sb, SS, brk, dup, hs, ns, R, base);
    }
    if (nb) {
        if (wide_cmp)
            SG_LAUNCH(c, "seg_wave", k_seg_wave<true>, grid_for((nb + 1) / 2, 4), 256, 0, Sb, SS, brk, dup, hb, nb, R, err, base);
        else
            SG_LAUNCH(c, "seg_wave", k_seg_wave<false>, grid_for((nb + 1) / 2, 4), 256, 0, Sb, SS, brk, dup, hb, nb, R, err, base);
    }
    if (c->profile && c->prof_only.empty() && (ns || nb)) {  // full-profile steps only
        // byte model: per member its span read + written, ~4 chunk keys of record bytes, flag
        unsigned long long *mc;
        SG_TRY(slot(c, S_M_CNT, 4, &mc));
        SG_HIP(hipMemsetAsync(mc, 0, 16, c->stream));
        if (ns) SG_LAUNCH(c, "seg_members", k_seg_members, std::min<uint32_t>(grid_for(ns, 256), 1024u), 256, 0, brk, hs,
                          ns, R, mc);
        if (nb) SG_LAUNCH(c, "seg_members", k_seg_members, std::min<uint32_t>(grid_for(nb, 256), 1024u), 256, 0, brk, hb,
                          nb, R, mc + 1);
        unsigned long long m[2];
        SG_TRY(ctx_readback(c, m, mc, 16));
        prof_bytes(c, "seg_small", 45.0 * (double)m[0]);
        prof_bytes(c, "seg_wave", 45.0 * (double)m[1]);
    }

    // compact the unique records
    uint8_t *ub;
    uint2 *us;
    uint64_t *uk;
    if (dst) ub = dst->base();
    else SG_TRY(slot(c, vs.ubuf, (size_t)n + 64, &ub));
    SG_TRY(slot(c, vs.uspans, R, &us));
    SG_TRY(slot(c, vs.ukeys, R, &uk));
    uint64_t *uc;
    // short records: the small-window emit (more blocks per CU for the random gather)
    const EmitApplyFn uk_kern = (n <= 40ull * R) ? k_emit_uniq_s : k_emit_uniq;
    SG_TRY(run_emit(c, uk_kern, "emit_uniq", "emit_uniq.count", S_EMIT2, FlagItem{SS, dup, 0}, R, Sb, ub, us, K, uk, &uc,
                    0.0, dst ? dst->shift() : 0u));
    // the output count and the run-sort error word come back with one host sync
    uint8_t *pin = (uint8_t *)c->pinned;
    if (nb && reinterpret_cast<uint32_t *>(uc + 1) != err) { set_error("emit: status slot moved"); return SG_E_HIP; }
    SG_HIP(hipMemcpyAsync(pin, uc, nb ? 12 : 8, hipMemcpyDeviceToHost, c->stream));
    SG_HIP(hipStreamSynchronize(c->stream));
    uint64_t tt = 0;
    memcpy(&tt, pin, 8);
    const uint32_t t1 = (uint32_t)(tt >> 32), t2 = (uint32_t)tt;
    // model: cached span per record; kept bytes read + written; span + key0 per kept record
    if (c->profile) prof_bytes(c, "emit_uniq", 8.0 * R + 2.0 * t2 + 24.0 * t1);
    if (nb) {
        uint32_t e = 0;
        memcpy(&e, pin + 8, 4);
        if (e) { set_error("run sort: segment bound violated (0x%x)", e); return SG_E_HIP; }
    }
    *uv = UView{ub, us, uk, t1, t2, R};
    if (vs.ubuf == CUR_VIEW.ubuf) c->last_uniq_frac = R ? (float)t1 / (float)R : 1.0f;
    return SG_OK;
}


// cur_lcp (with cur_pre): a device word already holding the common prefix of cur's records
// vs cur's first record (computed where the records were gathered), so cur is not scanned
// again for it.
static int dev_dedup_diff_radix(sg_ctx *c, const uint8_t *d_cur, uint64_t n_cur, const uint8_t *d_prior,
                                uint64_t n_prior, bool want_fresh, sg_dev_result *res, const Lines *cur_pre = nullptr,
                                const OutBuf *ou = nullptr, const OutBuf *of = nullptr,
                                const uint32_t *cur_lcp = nullptr) {
    *res = sg_dev_result{};
    UView pv;
    const bool have_prior = want_fresh && d_prior && n_prior;
    // Both parses first: the prior's sortedness flag rides back to the host with the current
    // buffer's record count (one host sync instead of two). Then the prior's view (the input
    // itself when strictly increasing), then the current scan's sort -u.
    Lines Lp, Lc;
    bool prior_sorted = true;
    // dflag: [0] prior not strictly increasing, [1] common prefix length, then the cur keys'
    // KeyStatD from byte 0 ([4..10)) and after a rekey at the common prefix ([12..18))
    // (the front of one slot with the sample histograms and the stat partials after it: the
    // flags, the stats and the histograms come back in one copy)
    uint32_t *dflag;
    // [32, 32 + 2048): the sample histograms of the keys from byte 0, then those of the
    // speculative keys at the last common prefix, then the key-stat partials
    constexpr size_t DF_CHK = 32 + 2 * 8 * 256 + 2 * 2048 * sizeof(KeyStatD) / 4;  // handover check partials
    SG_TRY(slot(c, S_HIST, DF_CHK + 2048 * sizeof(SpanChkPart) / 4, &dflag));
    KeyStatD *st0 = reinterpret_cast<KeyStatD *>(dflag + 4), *st1 = reinterpret_cast<KeyStatD *>(dflag + 12);
    {
        uint32_t init[20] = {0u, 255u};
        const KeyStatD z{0ull, ~0ull, 255u, 0u};
        memcpy(init + 4, &z, sizeof z);
        memcpy(init + 12, &z, sizeof z);
        SG_HIP(hipMemcpyAsync(dflag, init, sizeof init, hipMemcpyHostToDevice, c->stream));
    }
    if (cur_lcp) SG_HIP(hipMemcpyAsync(dflag + 1, cur_lcp, 4, hipMemcpyDeviceToDevice, c->stream));
    if (have_prior) {
        if (!cur_pre) SG_TRY(run_lines2(c, d_prior, n_prior, PRIOR_VIEW.lines, &Lp, d_cur, n_cur, CUR_VIEW.lines, &Lc));
        else SG_TRY(run_lines(c, d_prior, n_prior, PRIOR_VIEW.lines, &Lp));
    }
    // The prior's sortedness (dflag[0]): keys from byte 0 decide it exactly like keys from the
    // common prefix would (a separate launch: fused into the prior's common-prefix scan, whose
    // grid is capped for its atomics, the byte compares of equal keys ran 40 µs longer on C2).
    // With speculative keys (below) the check runs on the prior's keys at the last common
    // prefix instead, after the prior's prefix scan wrote them: URL-like priors share their
    // first bytes, so keys from byte 0 all tie and every pair would be compared bytewise.
    // Those keys decide it only if the prefix comes out the same (checked after the read-back).
    auto check_prior = [&](const uint64_t *keys, uint32_t bk) -> int {
        const uint32_t R = Lp.n_rec;
        if (R > 1 && R < (1u << 30))
            SG_LAUNCH_B(c, "check_sorted", 8.0 * R, k_check_sorted, grid_for(R - 1, 256), 256, 0, d_prior, Lp.spans, keys,
                        R, dflag, bk);
        return SG_OK;
    };
    if (cur_pre) Lc = *cur_pre;
    else if (!have_prior) SG_TRY(run_lines(c, d_cur, n_cur, CUR_VIEW.lines, &Lc));
    // common prefix of every record (reference: the first record of cur, else of prior)
    const bool ref_cur = Lc.n_rec > 0;
    const uint8_t *rbuf = ref_cur ? d_cur : d_prior;
    const uint2 *rsp = ref_cur ? Lc.spans : (have_prior ? Lp.spans : nullptr);
    const uint64_t *rkeys = ref_cur ? Lc.keys : (have_prior ? Lp.keys : nullptr);
    // the sort's key statistics (KeyStats): exact varying bits, sampled digit histograms
    const bool want_hist = Lc.n_rec >= 4096;
    uint32_t *shist = nullptr, hist_n = 0;
    KeyStatD *parts = nullptr;  // per-block partials (k_lcp / k_key_stats / k_rekey blocks)
    // (2048 blocks: 512 left C2's 10M-key prefix scan at 2 waves per SIMD)
    const uint32_t g_cur = std::min<uint32_t>(grid_for(Lc.n_rec, 256), 2048u);
    const uint32_t g_rekey = std::min<uint32_t>(grid_for(Lc.n_rec, 256), 2048u);
    if (want_hist) {
        shist = dflag + 32;
        parts = reinterpret_cast<KeyStatD *>(shist + 2 * 8 * 256);
        SG_HIP(hipMemsetAsync(shist, 0, 2 * 8 * 256 * 4, c->stream));
    }
    // Speculation: when the last call's records shared a prefix of >= 8 bytes (URL lists),
    // the prefix scans also write the keys at that offset, so a common prefix that comes out
    // the same needs no re-key pass (and its second key-statistics pass reads these keys).
    // (cur gathered elsewhere, cur_lcp: its gatherer wrote the speculative keys, Lines::spec_*)
    const bool cur_spec = !cur_lcp || (Lc.spec_keys && Lc.spec_off == c->last_base);
    const uint32_t Ls = (c->last_base >= 8u && rsp && want_hist && cur_spec) ? c->last_base : 0u;
    uint64_t *kLc = nullptr, *kLp = nullptr;
    KeyStatD *partsL = nullptr;
    uint32_t npartsL = 0;
    if (Ls) {
        if (cur_lcp) {
            kLc = Lc.spec_keys;
            partsL = const_cast<KeyStatD *>(Lc.spec_parts);
            npartsL = Lc.spec_nparts;
        } else {
            SG_TRY(slot(c, S_KEYSL, (size_t)Lc.n_rec + 1, &kLc));
            partsL = parts + 2048;
            npartsL = g_cur;
        }
        if (have_prior && Lp.n_rec) SG_TRY(slot(c, S_KEYSL2, (size_t)Lp.n_rec + 1, &kLp));
    }
    const bool spec_chk = have_prior && kLp && rsp;  // the prior's check on its keys at Ls
    if (have_prior && !spec_chk) SG_TRY(check_prior(Lp.keys, make_bk(0u, 7u)));
    // a handed-over parse (Lc.chk) is checked by the cur scan, and nothing reads bytes through
    // an unchecked reference span (rnb) before the check's result comes back with the flags
    const bool chk = Lc.chk && Lc.n_rec;
    const uint32_t rnb = chk && ref_cur ? (uint32_t)n_cur : 0u;
    SpanChkPart *chk_parts = reinterpret_cast<SpanChkPart *>(dflag + DF_CHK);
    if (rsp && Lc.n_rec && !cur_lcp) {
        if (chk) {
            // model: key + span per record (the sampled byte checks are not credited)
            SG_HIP(hipMemsetAsync(dflag + 22, 0, 4, c->stream));
            SG_LAUNCH_B(c, "lcp", 16.0 * Lc.n_rec, k_lcp<true>, g_cur, 256, 0, d_cur, Lc.spans, Lc.keys, Lc.n_rec, rbuf,
                        rsp, rkeys, dflag + 1, parts, kLc, Ls, partsL, rnb, chk_parts, (uint32_t)n_cur, dflag + 22);
            SG_LAUNCH(c, "chk_combine", k_chk_combine, 1, 256, 0, chk_parts, g_cur, dflag + 20);
            const uint32_t ns = (Lc.n_rec + CHK_SAMPLE - 1) / CHK_SAMPLE;
            SG_LAUNCH(c, "chk_sample", k_chk_sample, (ns + 255) / 256, 256, 0, d_cur, Lc.spans, Lc.keys, Lc.n_rec,
                      (uint32_t)n_cur, dflag + 22);
        } else {
            SG_LAUNCH_B(c, "lcp", 8.0 * Lc.n_rec, k_lcp<false>, g_cur, 256, 0, d_cur, Lc.spans, Lc.keys, Lc.n_rec, rbuf,
                        rsp, rkeys, dflag + 1, parts, kLc, Ls, partsL, 0u, (SpanChkPart *)nullptr, 0u, (uint32_t *)nullptr);
        }
    } else if (want_hist) {  // (not reached with a handed-over parse: it always has cur_lcp null)
        SG_LAUNCH_B(c, "key_stats", 8.0 * Lc.n_rec, k_key_stats, g_cur, 256, 0, Lc.keys, Lc.n_rec, parts);
    }
    if (rsp && have_prior && Lp.n_rec)
        SG_LAUNCH_B(c, "lcp", 8.0 * Lp.n_rec, k_lcp<false>, std::min<uint32_t>(grid_for(Lp.n_rec, 256), 2048u), 256, 0,
                    d_prior, Lp.spans, Lp.keys, Lp.n_rec, rbuf, rsp, rkeys, dflag + 1, (KeyStatD *)nullptr, kLp, Ls,
                    (KeyStatD *)nullptr, rnb, (SpanChkPart *)nullptr, 0u, (uint32_t *)nullptr);
    if (spec_chk) SG_TRY(check_prior(kLp, make_bk(Ls, 7u)));
    // the sample histograms (and the combined partials) come back with the flags; they stay
    // valid when the common prefix turns out to be empty
    if (want_hist) SG_TRY(key_sample_hist(c, Lc.keys, Lc.n_rec, shist, &hist_n, parts, g_cur, st0));
    // with speculative keys, their sample histograms and combined statistics too: when the
    // common prefix comes out where they were taken (the usual case for URL-like lists), the
    // sort's plan needs no second round trip (X1, URLs: one host sync fewer per call)
    const bool spec_hist = want_hist && Ls;
    uint32_t hist_n2 = 0;
    if (spec_hist) SG_TRY(key_sample_hist(c, kLc, Lc.n_rec, shist + 8 * 256, &hist_n2, partsL, npartsL, st1));
    uint32_t *hh = c->hist_host;
    uint32_t fl[32] = {0u};
    uint8_t *pin = (uint8_t *)c->pinned;
    auto read_stats = [&](uint32_t words, uint32_t nhist) -> int {
        SG_HIP(hipMemcpyAsync(pin, dflag, nhist ? 128 + nhist * 8 * 256 * 4 : 4 * words, hipMemcpyDeviceToHost, c->stream));
        SG_HIP(hipStreamSynchronize(c->stream));
        memcpy(fl, pin, 4 * words);
        if (nhist) memcpy(hh, pin + 128, 8 * 256 * 4);
        return SG_OK;
    };
    SG_TRY(read_stats(chk ? 24u : (spec_hist ? 20u : (want_hist ? 12u : 2u)), spec_hist ? 2u : (shist ? 1u : 0u)));
    if (chk) {  // before any kernel indexes the bytes through the handed-over spans
        uint64_t sum = 0;
        memcpy(&sum, fl + 20, 8);
        if (fl[22] || sum != Lc.chk_sum) {
            set_error("handed-over parse does not match the buffer: %u of %u records out of place, checksum %016llx "
                      "(expected %016llx)", fl[22], Lc.n_rec, (unsigned long long)sum, (unsigned long long)Lc.chk_sum);
            return SG_E_CORRUPT;
        }
    }
    const uint32_t base = (rsp && (Lc.n_rec || (have_prior && Lp.n_rec))) ? fl[1] : 0u;
    if (spec_chk && base != Ls) {  // the prefix moved: the check again on keys from byte 0
        SG_HIP(hipMemsetAsync(dflag, 0, 4, c->stream));
        SG_TRY(check_prior(Lp.keys, make_bk(0u, 7u)));
        SG_TRY(ctx_readback(c, fl, dflag, 4));
    }
    prior_sorted = fl[0] == 0;
    if (base) {
        const bool spec = Ls && base == Ls;
        if (want_hist && !spec) SG_HIP(hipMemsetAsync(shist, 0, 8 * 256 * 4, c->stream));
        if (spec) {  // the speculative keys are every record's keys at the common prefix
            Lc.keys = kLc;
            if (kLp) Lp.keys = kLp;
        } else {
            SG_LAUNCH(c, "rekey", k_rekey, g_rekey, 256, 0, d_cur, Lc.spans, Lc.n_rec, base, Lc.keys, parts);
            if (have_prior && Lp.n_rec)
                SG_LAUNCH(c, "rekey", k_rekey, std::min<uint32_t>(grid_for(Lp.n_rec, 256), 2048u), 256, 0, d_prior,
                          Lp.spans, Lp.n_rec, base, Lp.keys, (KeyStatD *)nullptr);
        }
        if (want_hist && spec) {  // keys changed: their statistics, already read back
            memcpy(hh, pin + 128 + 8 * 256 * 4, 8 * 256 * 4);
            hist_n = hist_n2;
            memcpy(fl + 4, fl + 12, sizeof(KeyStatD));
        } else if (want_hist) {
            SG_TRY(key_sample_hist(c, Lc.keys, Lc.n_rec, shist, &hist_n, parts, g_rekey, st1));
            SG_TRY(read_stats(20u, 1u));
            memcpy(fl + 4, fl + 12, sizeof(KeyStatD));
        }
    }
    c->last_base = base;
    // Key width: the cur keys' sampled digit histograms give each byte position's entropy;
    // when the first 6 (or 5) key bytes already carry well over as many bits as there are
    // records (expected << 1 record per key value, so few tie segments), the keys are
    // narrowed to those bytes and the sort runs 1 (or 2) fewer passes. IP-like text (few
    // distinct bytes per position) keeps the 7-byte key.
    uint32_t kw = 7;
    KeyStats ks;
    if (want_hist) {
        const double N = (double)hist_n;
        double H[8] = {0};
        for (int p = 0; p < 8; ++p)
            for (int d = 0; d < 256; ++d)
                if (hh[p * 256 + d]) {
                    const double q = hh[p * 256 + d] / N;
                    H[p] -= q * std::log2(q);
                }
        // margins measured on C2/X1: a 5-byte key saved 2 radix passes but its tie segments
        // (distinct records sharing 5 bytes) cost the segment sort about as much again
        const double lg = std::log2((double)Lc.n_rec);
        const double h5 = H[7] + H[6] + H[5] + H[4] + H[3], h6 = h5 + H[2];
        KeyStatD k0;
        memcpy(&k0, fl + 4, sizeof k0);
        uint64_t vary = (uint64_t)(k0.o ^ k0.a);
        // the passes narrowing removes must be live (a sampled zero entropy may miss a rare
        // digit: the exact varying bits decide)
        const bool live2 = (vary >> 16) & 0xffu, live1 = (vary >> 8) & 0xffu;
        if (h5 >= lg + 4.0 && (live2 || live1)) kw = 5;
        else if (h6 >= lg + 2.0 && live1) kw = 6;
        if (kw < 7) {
            // the cur keys are narrowed by the sort's first pass (build_unique); the prior's
            // as the diff reads them (key_narrow: its view is the input itself when sorted)
            // the narrowed keys' histograms: bytes kw..6 are zero, the tag is clamped to kw + 1
            for (int p = 1; p <= 7 - (int)kw; ++p) {
                for (int d = 0; d < 256; ++d) hh[p * 256 + d] = 0;
                hh[p * 256] = hist_n;
                vary &= ~(0xffull << (8 * p));
            }
            uint32_t tg[256] = {0};
            for (int d = 0; d < 256; ++d) tg[d < (int)kw + 1 ? d : (int)kw + 1] += hh[d];
            for (int d = 0; d < 256; ++d) hh[d] = tg[d];
        }
        const uint32_t cl = kw + 1;  // the (narrowed) tag varies iff its clamped range does
        vary &= ~0xffull;
        if (std::min(k0.tmin, cl) != std::min(k0.tmax, cl)) vary |= 0xffull;
        ks = KeyStats{vary, hh, hist_n};
    }
    c->last_kw = kw;
    const uint32_t bk = make_bk(base, kw);
    if (have_prior) SG_TRY(build_unique(c, d_prior, n_prior, PRIOR_VIEW, prior_sorted, &pv, &Lp, bk));
    UView cu;
    SG_TRY(build_unique(c, d_cur, n_cur, CUR_VIEW, false, &cu, &Lc, bk, ou, want_hist ? &ks : nullptr));
    res->in_records = cu.in_records;
    res->uniq = ou ? ou->p : const_cast<uint8_t *>(cu.buf);
    res->uniq_bytes = cu.bytes;
    res->uniq_records = cu.n;
    if (!want_fresh) return SG_OK;
    res->prior_records = pv.in_records;
    if (pv.n == 0 || cu.n == 0) {
        res->fresh = res->uniq;
        res->fresh_bytes = res->uniq_bytes;
        res->fresh_records = res->uniq_records;
        if (of && res->fresh_bytes) {  // caller outputs: the new records are all of them, copied
            SG_HIP(hipMemcpyAsync(of->p, res->uniq, res->fresh_bytes, hipMemcpyDeviceToDevice, c->stream));
            // every other route returns after a host sync: the caller may hand the buffer
            // to another stream (or free it) as soon as this returns
            SG_HIP(hipStreamSynchronize(c->stream));
            res->fresh = of->p;
        } else if (of) {
            res->fresh = of->p;
        }
        return SG_OK;
    }
    uint8_t *fresh;
    SG_TRY(slot(c, S_FRESHF, (size_t)cu.n + 1, &fresh));
    RecSet U{cu.buf, cu.spans, cu.keys, cu.n};
    RecSet P{pv.buf, pv.spans, pv.keys, pv.n};
    const uint32_t ntiles = (cu.n + DF_TILE - 1) / DF_TILE;
    uint32_t *jb;
    SG_TRY(slot(c, S_R_OFF, (size_t)ntiles + 2, &jb));
    SG_LAUNCH(c, "diff_split", k_diff_split, grid_for(ntiles + 1, 4), 256, 0, cu.keys, cu.n, pv.keys, pv.n, ntiles + 1, jb,
              bk >> 16);
    // model: key + span of every unique cur record, key of every prior record, the compared
    // bytes of both sides (~ the unique output + the prior), one flag per cur record
    SG_LAUNCH_B(c, "diff_tile", 16.0 * cu.n + 8.0 * pv.n + (double)cu.bytes + cu.n, k_diff_tile, ntiles, 256, 0,
                U, P, jb, fresh, bk);
    uint8_t *fout;
    if (of) fout = of->base();
    else SG_TRY(slot(c, S_OUT_FRESH, (size_t)cu.bytes + 64, &fout));
    uint64_t *fc;
    SG_TRY(run_emit(c, k_emit_fresh, "emit_fresh", "emit_fresh.count", S_EMIT3, FlagItem{cu.spans, fresh, 1}, cu.n, cu.buf, fout,
                    nullptr, nullptr, nullptr, &fc, 0.0, of ? of->shift() : 0u));
    uint64_t tt = 0;
    SG_TRY(ctx_readback(c, &tt, fc, 8));
    if (c->profile) prof_bytes(c, "emit_fresh", 8.0 * cu.n + 2.0 * (double)(uint32_t)tt);
    res->fresh = of ? of->p : fout;
    res->fresh_bytes = (uint32_t)tt;
    res->fresh_records = (uint32_t)(tt >> 32);
    return SG_OK;
}

int dev_dedup_diff_into(sg_ctx *c, const uint8_t *d_cur, uint64_t n_cur, const uint8_t *d_prior, uint64_t n_prior,
                        uint8_t *d_uniq, size_t uniq_cap, uint8_t *d_fresh, size_t fresh_cap, sg_dev_result *res) {
    if (uniq_cap < n_cur + 1 || (d_fresh && fresh_cap < n_cur + 1)) {
        set_error("output capacities must be >= n_cur + 1 (%llu)", (unsigned long long)(n_cur + 1));
        return SG_E_CAP;
    }
    c->last_path = 0;
    c->last_flags = 0;
    const OutBuf ou{d_uniq, uniq_cap}, of{d_fresh, fresh_cap};
    return dev_dedup_diff_radix(c, d_cur, n_cur, d_prior, n_prior, true, res, nullptr, &ou, d_fresh ? &of : nullptr);
}

int dev_dedup_diff_into_lines(sg_ctx *c, const uint8_t *d_cur, uint64_t n_cur, const Lines &cur, const uint8_t *d_prior,
                              uint64_t n_prior, uint8_t *d_uniq, size_t uniq_cap, uint8_t *d_fresh, size_t fresh_cap,
                              sg_dev_result *res) {
    if (uniq_cap < n_cur + 1 || (d_fresh && fresh_cap < n_cur + 1)) {
        set_error("output capacities must be >= n_cur + 1 (%llu)", (unsigned long long)(n_cur + 1));
        return SG_E_CAP;
    }
    c->last_path = 0;
    c->last_flags = 0;
    const OutBuf ou{d_uniq, uniq_cap}, of{d_fresh, fresh_cap};
    return dev_dedup_diff_radix(c, d_cur, n_cur, d_prior, n_prior, true, res, &cur, &ou, d_fresh ? &of : nullptr);
}

int dev_dedup_diff_lines(sg_ctx *c, const uint8_t *d_cur, uint64_t n_cur, const Lines &cur, const uint8_t *d_prior,
                         uint64_t n_prior, sg_dev_result *res, const uint32_t *cur_lcp) {
    c->last_path = 0;
    c->last_flags = 0;
    return dev_dedup_diff_radix(c, d_cur, n_cur, d_prior, n_prior, true, res, &cur, nullptr, nullptr, cur_lcp);
}

// Dedup+diff entry (the radix pipeline above).
int dev_dedup_diff(sg_ctx *c, const uint8_t *d_cur, uint64_t n_cur, const uint8_t *d_prior,
                   uint64_t n_prior, bool want_fresh, sg_dev_result *res) {
    c->last_path = 0;
    c->last_flags = 0;
    return dev_dedup_diff_radix(c, d_cur, n_cur, d_prior, n_prior, want_fresh, res);
}

}  // namespace sg
