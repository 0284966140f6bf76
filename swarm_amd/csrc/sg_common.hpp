// sg_common.hpp — shared host/device infrastructure for libswarmgpu (gfx950 only).
//
// Host side: thread-local error text, the sg_ctx (device, stream, grow-only HBM buffer
// slots, optional per-kernel HIP-event timing) and a launch wrapper.
// Device side: wave64/block scans, the one-block tile scan declaration shared by every
// reduce-then-scan kernel pair (count pass -> tile scan -> apply pass), and record
// compare/key helpers. No kernel waits on another block: single-pass decoupled look-back
// was measured slower on MI355X (a cross-XCD round trip per tile).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdarg.h>

#include <mutex>
#include <string>
#include <vector>

#include "../../include/swarmgpu.h"
#include "sg_switches.hpp"

#define SG_PINNED_BYTES 32768

namespace sg {

// ------------------------------------------------------------------ errors
void set_error(const char *fmt, ...);
const char *get_error();

#define SG_HIP(call)                                                                   \
    do {                                                                               \
        hipError_t e_ = (call);                                                        \
        if (e_ != hipSuccess) {                                                        \
            ::sg::set_error("%s:%d %s: %s", __FILE__, __LINE__, #call,                 \
                            hipGetErrorString(e_));                                    \
            return SG_E_HIP;                                                           \
        }                                                                              \
    } while (0)

#define SG_TRY(expr)                  \
    do {                              \
        int rc_ = (expr);             \
        if (rc_ != SG_OK) return rc_; \
    } while (0)

// ------------------------------------------------------------------ context
enum Slot : int {
    // line split of the current buffer
    S_STARTS, S_ENDS, S_KEYS, S_KEYS2, S_VALS, S_VALS2, S_LB, S_COUNT,
    // dedup / refinement
    S_UNIQ, S_GS, S_GE, S_SEL, S_OFFS, S_OUT_UNIQ, S_OUT_FRESH, S_FRESH_IDX,
    S_R_POS, S_R_KEY, S_R_KEY2, S_R_VAL, S_R_VAL2, S_R_GID, S_R_OFF,
    S_HIST, S_ALIGN,
    // prior
    S_P_STARTS, S_P_ENDS, S_P_KEYS, S_P_REC, S_P_FLAG, S_P_KEYS2, S_P_VALS, S_P_VALS2,
    S_P_UNIQ, S_P_SORTED_KEYS,
    // partition / match
    S_PART, S_PART_OUT, S_M_HITS, S_M_SIG, S_M_LINES, S_M_TMP, S_M_TMP2, S_M_CNT,
    S_IN, S_IN2, S_CUR_UR, S_CUR_UK,
    // sorted materialisation (shared temporaries) and per-view outputs
    S_SBUF, S_SSPANS, S_DUP, S_BAD, S_BRK, S_MIRROR, S_EMIT, S_EMIT2, S_EMIT3, S_ERR,
    S_U_SPANS, S_U_KEYS, S_P_UBUF, S_P_USPANS, S_P_UKEYS, S_FRESHF, S_ECACHE, S_TILES, S_RS_TCNT, S_RS_DIGITS,
    // module-output formats (nmap -oN, httpx -json) and template evaluation
    S_F_SPANS, S_F_LB, S_F_A, S_F_B, S_F_DESC, S_F_OFFS, S_F_OUT, S_F_REC, S_F_KEY, S_F_KEYS,
    S_T_HITS, S_T_EXP, S_T_K2, S_T_V1, S_T_V2, S_T_OUT, S_T_SEL, S_T_E, S_T_E2, S_T_SEG, S_T_FLAG, S_T_O,
    S_T_REC, S_T_TID,
    S_M_FLAG, S_M_SP2, S_M_K2, S_R_T2, S_COUNT2,
    S_R_ALPHA,  // refinement rounds: byte alphabet mask + rank table of the chunk keys
    // hit sort by record buckets (sg_match.hip)
    S_HB_CNT, S_HB_OFF, S_HB_OUT, S_HB_ERR, S_HB_SEL2,
    S_TS2,  // two-level tile scan scratch
    S_PT_CNT, S_PT_PRE, S_PT_BASE,  // piece partition multi-split
    S_PT_SP, S_PT_KEYS,             // piece partition: spans and parts kept from pass 1 for pass 2
    S_PT_LTP,                       // piece partition: every piece's parse tile counts and prefixes
    S_PT_RCNT, S_PT_RPRE, S_PT_SPOUT, S_PT_KOUT,  // piece partition: the parts' record spans/keys out
    S_PT_SUMS,                      // piece partition: per-(part, tile) handover checksums, per-part totals
    S_LS_ERR, S_LS_BOUNDS,  // hybrid radix sort: overflow flag, local-sort tile bounds
    S_LS_LIST, S_LF_OFF, S_LF_KEY, S_LF_KEY2, S_LF_VAL, S_LF_VAL2, S_LF_POS,  // its overflow fix-up
    S_KEYSL, S_KEYSL2,  // dedup: cur / prior keys at the last call's common prefix (speculative)
    S_SPEC_PARTS,       // X1: the speculative keys' KeyStatD partials
    S_M_K0, S_M_R7,     // X1: every record's key0 and bytes 7..14, written by the literal scan
    S_NSLOTS
};

struct KStat {
    const char *name;
    uint64_t launches;
    double ms;
    double bytes;  // algorithmic bytes (SURVEY.md §8(d) model) of the timed launches
};

struct sg_ctx_impl;
}  // namespace sg

struct sg_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    bool owns_stream = false;
    void *slot_ptr[sg::S_NSLOTS] = {};
    size_t slot_cap[sg::S_NSLOTS] = {};
    void *pinned = nullptr;   // host pinned staging for small readbacks (SG_PINNED_BYTES)
    int last_path = 0;        // dedup/diff pipeline of the last call: 0 = the radix pipeline (the only one)
    uint32_t last_flags = 0;  // dedup of the last call: bit 0 hybrid sort (local LDS sort), bit 1 its overflow
                              // re-sort, bit 2 its overflow fix-up, bit 3 all-segments mode
    uint32_t last_kw = 7;     // dedup: key width (bytes) the last radix sort used
    float last_uniq_frac = 1.0f;  // dedup: unique / input records of the last sort -u (all-segments mode)
    uint32_t last_base = 0;       // dedup: the last call's common prefix (keys taken there speculatively)
    uint32_t hist_host[8 * 256] = {};  // dedup: digit histograms of the current keys (host copy)
    // the last hybrid radix sort's local-sort plan (lsort_fixup redoes its flagged tiles)
    struct LsLast {
        bool on = false;
        uint64_t gmask = 0;
        uint32_t lpos = 0, nloc = 0, ntiles = 0, cap = 0;
        uint32_t *bounds = nullptr;
        uint32_t *gs = nullptr, *ge = nullptr;  // the big groups the fix-up pass listed
    } ls_last;
    // the piece partition's pass 0 (record counts per piece) kept from sg_dev_partition_pieces_count
    // for the next partition call on the same pieces (its tile scans stay in slot S_PT_LTP)
    struct PtPrep {
        bool on = false;
        std::vector<const uint8_t *> ptrs;
        std::vector<size_t> lens;
        std::vector<uint32_t> Rj;
    } pt_prep;
    // pinned staging for host-to-device uploads on the context stream (ctx_upload): grown on
    // demand; up_ev marks the last upload's copy so the buffer is not rewritten under it
    void *up_pin = nullptr;
    size_t up_cap = 0;
    hipEvent_t up_ev = nullptr;
    // profiling
    bool profile = false;
    std::string prof_only;  // non-empty: time only launches with this name
    std::vector<sg::KStat> stats;
    struct Pending { int stat; hipEvent_t a, b; };
    std::vector<Pending> pending;
    std::vector<hipEvent_t> free_events;
};

namespace sg {

int ctx_slot(sg_ctx *c, int slot, size_t bytes, void **out);
template <class T>
inline int slot(sg_ctx *c, int s, size_t count, T **out) {
    void *p = nullptr;
    int rc = ctx_slot(c, s, count * sizeof(T) + 64, &p);
    *out = (T *)p;
    return rc;
}
// Element capacity a slot already holds for T (0 if unallocated): callers that size an
// output by an upper bound reuse a larger existing slot without growing it (slot() adds
// its own headroom, so feeding slot_cap back into a request would compound).
template <class T>
inline uint64_t slot_elems(const sg_ctx *c, int s) {
    return c->slot_cap[s] > 64 ? (c->slot_cap[s] - 64) / sizeof(T) : 0;
}
int ctx_readback(sg_ctx *c, void *host, const void *dev, size_t bytes);  // sync on stream
// Async host-to-device copy on the context stream through pinned staging: the host bytes
// may be reused as soon as it returns, and nothing waits on the device (or the null stream).
int ctx_upload(sg_ctx *c, void *dev, const void *host, size_t bytes);
int ctx_harvest(sg_ctx *c);
int prof_begin(sg_ctx *c, const char *name, int *stat, hipEvent_t *a);
void prof_end(sg_ctx *c, int stat, hipEvent_t a);
inline bool prof_wanted(sg_ctx *c, const char *name) { return c->prof_only.empty() || c->prof_only == name; }
// Credit algorithmic bytes to the named kernel (no-op unless profiling).
void prof_bytes(sg_ctx *c, const char *name, double bytes);

// Launch with optional HIP-event timing on the context stream.
#define SG_LAUNCH(ctx, name, kernel, grid, block, lds, ...)                          \
    do {                                                                              \
        int st_ = -1;                                                                 \
        hipEvent_t ea_ = nullptr;                                                     \
        if ((ctx)->profile && ::sg::prof_wanted((ctx), (name)))                        \
            ::sg::prof_begin((ctx), (name), &st_, &ea_);                              \
        hipLaunchKernelGGL(kernel, dim3(grid), dim3(block), (lds), (ctx)->stream,     \
                           __VA_ARGS__);                                              \
        hipError_t le_ = hipGetLastError();                                           \
        if (le_ != hipSuccess) {                                                      \
            ::sg::set_error("launch %s: %s", (name), hipGetErrorString(le_));         \
            return SG_E_HIP;                                                          \
        }                                                                             \
        if (st_ >= 0) ::sg::prof_end((ctx), st_, ea_);                                \
        if (::sg::sw_sync_check()) {                                                  \
            hipError_t se_ = hipStreamSynchronize((ctx)->stream);                     \
            if (se_ != hipSuccess) {                                                  \
                ::sg::set_error("kernel %s: %s", (name), hipGetErrorString(se_));     \
                return SG_E_HIP;                                                      \
            }                                                                         \
        }                                                                             \
    } while (0)

// Same, crediting `bytes` algorithmic bytes to the kernel's roofline accounting.
#define SG_LAUNCH_B(ctx, name, bytes, kernel, grid, block, lds, ...)                 \
    do {                                                                              \
        SG_LAUNCH(ctx, name, kernel, grid, block, lds, __VA_ARGS__);                  \
        if ((ctx)->profile) ::sg::prof_bytes((ctx), (name), (double)(bytes));         \
    } while (0)

// ------------------------------------------------------------------ limits
constexpr uint64_t MAX_BYTES = 0xFFFF0000ull;  // 32-bit record offsets with headroom

// ------------------------------------------------------------------ device helpers
__device__ __forceinline__ int lane_id() { return __lane_id(); }

template <class T>
__device__ __forceinline__ T wave_incl_scan_shfl(T v) {
    const int lane = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        T t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    return v;
}

// DPP move of a 32- or 64-bit value (lanes without a source, and rows outside RM, read 0).
template <int CTRL, int RM, class T>
__device__ __forceinline__ T dpp_mov0(T v) {
    static_assert(sizeof(T) == 4 || sizeof(T) == 8, "32- or 64-bit");
    if constexpr (sizeof(T) == 4) {
        return (T)(uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, CTRL, RM, 0xf, true);
    } else {
        const uint64_t u = (uint64_t)v;
        const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, CTRL, RM, 0xf, true);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), CTRL, RM, 0xf, true);
        return (T)((uint64_t)lo | ((uint64_t)hi << 32));
    }
}

// Inclusive wave64 scan by DPP: row_shr 1, 2, 4, 8 inside each 16-lane row, then row_bcast:15
// (rows 1, 3 add the previous row's last lane) and row_bcast:31 (rows 2, 3 add lane 31): no
// LDS round trips (the __shfl_up form costs a ds_bpermute round trip per step). Every lane
// of the wave must be active (block-uniform call sites); wave_incl_scan_shfl otherwise.
template <class T>
__device__ __forceinline__ T wave_incl_scan(T v) {
    v += dpp_mov0<0x111, 0xf>(v);
    v += dpp_mov0<0x112, 0xf>(v);
    v += dpp_mov0<0x114, 0xf>(v);
    v += dpp_mov0<0x118, 0xf>(v);
    v += dpp_mov0<0x142, 0xa>(v);
    v += dpp_mov0<0x143, 0xc>(v);
    return v;
}

// Lane `lane`'s value in every lane (v_readlane: `lane` must be wave-uniform).
template <class T>
__device__ __forceinline__ T wave_bcast(T v, int lane) {
    static_assert(sizeof(T) == 4 || sizeof(T) == 8, "32- or 64-bit");
    if constexpr (sizeof(T) == 4) {
        return (T)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, lane);
    } else {
        const uint64_t u = (uint64_t)v;
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, lane);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), lane);
        return (T)((uint64_t)lo | ((uint64_t)hi << 32));
    }
}

// Wave sum in every lane: the DPP scan's last lane (every lane active; wave_sum_shfl otherwise).
template <class T>
__device__ __forceinline__ T wave_sum(T v) {
    return wave_bcast(wave_incl_scan(v), 63);
}

template <class T>
__device__ __forceinline__ T wave_sum_shfl(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Exclusive block scan, BLOCK threads (multiple of 64). lds: >= BLOCK/64 elements.
template <int BLOCK, class T>
__device__ __forceinline__ T block_excl_scan(T v, T *total, T *lds) {
    const int lane = lane_id(), wid = threadIdx.x >> 6;
    T inc = wave_incl_scan(v);
    if (lane == 63) lds[wid] = inc;
    __syncthreads();
    T woff = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < BLOCK / 64; ++w) {
        T s = lds[w];
        woff += (w < wid) ? s : T(0);
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return woff + inc - v;
}

// Exclusive scan of per-tile aggregates (u64 whose packed fields never carry), ONE block:
// the middle step of every reduce-then-scan kernel pair (count pass -> this -> apply pass).
// On MI355X a single-pass decoupled look-back over small tiles waits a cross-XCD round trip
// per tile; reading the per-item input twice is cheaper (tools/c2_probe.py measurements).
constexpr int TS_BLOCK = 1024;
constexpr int TS_ITEMS = 4;
__global__ __launch_bounds__(TS_BLOCK) void k_tile_scan(const uint64_t *__restrict__ tot, uint32_t nt,
                                                        uint64_t *__restrict__ pre, uint64_t *__restrict__ total);

// Bytewise compare of two records starting `off` bytes in (both have > off bytes or
// not — lengths decide). Returns <0, 0, >0 like memcmp-then-length.
__device__ __forceinline__ int rec_cmp(const uint8_t *buf_a, uint32_t sa, uint32_t ea,
                                       const uint8_t *buf_b, uint32_t sb, uint32_t eb,
                                       uint32_t off) {
    uint32_t la = ea - sa, lb = eb - sb;
    uint32_t m = la < lb ? la : lb;
    for (uint32_t i = off; i < m; ++i) {
        uint32_t x = buf_a[sa + i], y = buf_b[sb + i];
        if (x != y) return (int)x - (int)y;
    }
    return (la < lb) ? -1 : (la > lb ? 1 : 0);
}

// Prefix key of a record at byte offset `off`: bytes [off, off+7) big-endian in bits
// 63..8 (zero past the record end) and tag = min(remaining, 8) in bits 7..0. Ordering
// of (key) == bytewise ordering of the suffixes when the tags differ or tag < 8;
// equal keys with tag 8 need the next chunk.
// Word-granular: at most two naturally aligned 8-byte loads (buf must be 8-byte aligned;
// an aligned word that holds an in-bounds byte never crosses a page).
__device__ __forceinline__ uint64_t chunk_key(const uint8_t *buf, uint32_t s, uint32_t e, uint32_t off) {
    const uint32_t len = e - s;
    const uint32_t rem = (len > off) ? (len - off) : 0u;
    const uint64_t tag = rem < 8u ? rem : 8u;
    if (rem == 0) return 0;
    const uint32_t take = rem < 7u ? rem : 7u;
    const uint32_t p = s + off;
    const uint32_t a = p & ~7u;
    const uint32_t sh = (p - a) * 8u;
    uint64_t v = *reinterpret_cast<const uint64_t *>(buf + a) >> sh;
    if (p + take > a + 8u) v |= *reinterpret_cast<const uint64_t *>(buf + a + 8) << (64u - sh);
    v &= (1ull << (8u * take)) - 1ull;  // take <= 7
    return (__builtin_bswap64(v) & ~0xffull) | tag;
}

// One record's term of the handover checksum (include/swarmgpu.h sg_span_sum): its length
// (end - start) and its first-chunk key, mixed by one odd multiply and an xor-shift (both
// bijective: a change of one record's key or length always changes the sum). The checksum is
// the sum of the terms mod 2^64, so producers add them in any order (per tile, per part).
__host__ __device__ __forceinline__ uint64_t span_mix(uint32_t len, uint64_t key) {
    const uint64_t h = (key + (uint64_t)len * 0x9E3779B97F4A7C15ull) * 0xBF58476D1CE4E5B9ull;
    return h ^ (h >> 31);
}

// Bytes [lo, hi) of the little-endian dword v stored at p (p 4-byte aligned, 0 <= lo <= hi
// <= 4): at most a byte, a 16-bit and a byte store (a partial dword shared with a
// neighbouring lane's bytes).
__device__ __forceinline__ void put_edge(uint8_t *p, uint32_t v, uint32_t lo, uint32_t hi) {
    if (lo < hi && (lo & 1u)) { p[lo] = (uint8_t)(v >> (8u * lo)); ++lo; }
    if (hi >= lo + 2u) { *reinterpret_cast<uint16_t *>(p + lo) = (uint16_t)(v >> (8u * lo)); lo += 2u; }
    if (lo < hi) p[lo] = (uint8_t)(v >> (8u * lo));
}

// Bytes [p, p+t) (t <= 8) little-endian in a u64, zero above; buf 8-byte aligned.
__device__ __forceinline__ uint64_t load_le(const uint8_t *buf, uint32_t p, uint32_t t) {
    const uint32_t a = p & ~7u;
    const uint32_t sh = (p - a) * 8u;
    uint64_t v = *reinterpret_cast<const uint64_t *>(buf + a) >> sh;
    if (p + t > a + 8u) v |= *reinterpret_cast<const uint64_t *>(buf + a + 8) << (64u - sh);
    return t >= 8u ? v : (v & ((1ull << (8u * t)) - 1ull));
}

// Byte equality of two records from offset `off` (lengths must match). Loads of a
// 32-byte block are issued together; one branch per block.
__device__ __forceinline__ bool rec_equal(const uint8_t *ba, uint32_t sa, uint32_t ea, const uint8_t *bb,
                                          uint32_t sb, uint32_t eb, uint32_t off) {
    const uint32_t la = ea - sa;
    if (la != eb - sb) return false;
    for (uint32_t o = off; o < la; o += 32) {
        uint64_t d = 0;
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) {
            const uint32_t oo = o + 8 * q;
            if (oo < la) {
                const uint32_t t = (la - oo) < 8u ? (la - oo) : 8u;
                d |= load_le(ba, sa + oo, t) ^ load_le(bb, sb + oo, t);
            }
        }
        if (d) return false;
    }
    return true;
}

// The 52 bytes starting at window byte sh (0..15) of four 16-B chunks, as dwords r[0..12]:
// a dword barrel shift by sh>>2 (mask blends: a select between elements of one array would
// be folded into a dynamically indexed load and spill the array to scratch) and a byte
// funnel shift by sh&3.
__device__ __forceinline__ void normalize52(const uint4 (&c)[4], uint32_t sh, uint32_t (&r)[13]) {
    const uint32_t dw[18] = {c[0].x, c[0].y, c[0].z, c[0].w, c[1].x, c[1].y, c[1].z, c[1].w,
                             c[2].x, c[2].y, c[2].z, c[2].w, c[3].x, c[3].y, c[3].z, c[3].w, 0u, 0u};
    const uint32_t t = sh >> 2, e = sh & 3u;
    const uint32_t m2 = (t & 2u) ? ~0u : 0u, m1 = (t & 1u) ? ~0u : 0u;
    uint32_t s1[16], s2[15];
#pragma unroll
    for (int o = 0; o < 16; ++o) s1[o] = dw[o] ^ ((dw[o] ^ dw[o + 2]) & m2);
#pragma unroll
    for (int o = 0; o < 15; ++o) s2[o] = s1[o] ^ ((s1[o] ^ s1[o + 1]) & m1);
#pragma unroll
    for (int o = 0; o < 13; ++o) r[o] = __builtin_amdgcn_alignbyte(s2[o + 1], s2[o], e);
}

// Aligned 16-B chunks covering bytes [p, p + cl) of buf (cl <= 48): chunk k loaded only when
// it holds some of them.
__device__ __forceinline__ void load_chunks(const uint8_t *buf, uint32_t p, uint32_t cl, uint4 (&c)[4]) {
    const uint32_t q0 = p & ~15u, sh = p - q0;
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k)
        c[k] = (16u * k < sh + cl) ? *reinterpret_cast<const uint4 *>(buf + q0 + 16u * k) : make_uint4(0u, 0u, 0u, 0u);
}

// rec_equal with wide loads: the compared span (len - off) goes in windows of 48 bytes,
// each side taking at most four 16-B loads per window, and a window's comparison is a masked
// XOR of normalised dwords (long records — URLs with titles — cost 16-B loads instead of
// 8-B load pairs). Buffers must be 16-byte aligned.
__device__ __forceinline__ bool rec_equal_w(const uint8_t *ba, uint32_t sa, uint32_t ea, const uint8_t *bb,
                                            uint32_t sb, uint32_t eb, uint32_t off) {
    const uint32_t la = ea - sa;
    if (la != eb - sb) return false;
    for (uint32_t o = off; o < la; o += 48u) {
        const uint32_t cl = (la - o) < 48u ? (la - o) : 48u;
        uint4 ca[4], cb[4];
        load_chunks(ba, sa + o, cl, ca);
        load_chunks(bb, sb + o, cl, cb);
        uint32_t ra[13], rb[13];
        normalize52(ca, (sa + o) & 15u, ra);
        normalize52(cb, (sb + o) & 15u, rb);
        uint32_t d = 0;
#pragma unroll
        for (uint32_t q = 0; q < 12; ++q) {
            if (4u * q < cl) {
                const uint32_t k = cl - 4u * q;
                const uint32_t m = k >= 4u ? ~0u : ((1u << (8u * k)) - 1u);
                d |= (ra[q] ^ rb[q]) & m;
            }
        }
        if (d) return false;
    }
    return true;
}

// Bytewise compare of the suffixes from `off` by 7-byte chunk keys (memcmp-then-length).
__device__ __forceinline__ int rec_cmp_k(const uint8_t *ba, uint32_t sa, uint32_t ea, const uint8_t *bb,
                                         uint32_t sb, uint32_t eb, uint32_t off) {
    for (;;) {
        const uint64_t x = chunk_key(ba, sa, ea, off), y = chunk_key(bb, sb, eb, off);
        if (x != y) return x < y ? -1 : 1;
        if ((x & 0xffu) < 8u) return 0;
        off += 7;
    }
}

// rec_cmp_k's order (memcmp of the suffixes from `off`, then length) from one set of wide
// loads when the common suffix is <= 48 bytes: the first differing byte of the normalised
// words decides, else the shorter suffix is smaller.
__device__ __forceinline__ int rec_cmp_w(const uint8_t *ba, uint32_t sa, uint32_t ea, const uint8_t *bb,
                                         uint32_t sb, uint32_t eb, uint32_t off) {
    const uint32_t la = ea - sa, lb = eb - sb;
    const uint32_t ma = la > off ? la - off : 0u, mb = lb > off ? lb - off : 0u;
    const uint32_t cm = ma < mb ? ma : mb;
    const int by_len = ma < mb ? -1 : (ma > mb ? 1 : 0);
    for (uint32_t o = 0; o < cm; o += 48u) {  // 48-byte windows of 16-B loads
        const uint32_t cl = (cm - o) < 48u ? (cm - o) : 48u;
        uint4 ca[4], cb[4];
        load_chunks(ba, sa + off + o, cl, ca);
        load_chunks(bb, sb + off + o, cl, cb);
        uint32_t ra[13], rb[13];
        normalize52(ca, (sa + off + o) & 15u, ra);
        normalize52(cb, (sb + off + o) & 15u, rb);
#pragma unroll
        for (uint32_t q = 0; q < 12; ++q) {
            if (4u * q < cl) {
                const uint32_t k = cl - 4u * q;
                const uint32_t m = k >= 4u ? ~0u : ((1u << (8u * k)) - 1u);
                const uint32_t x = (ra[q] ^ rb[q]) & m;
                if (x) {
                    const uint32_t sh = (uint32_t)__builtin_ctz(x) & ~7u;
                    return ((ra[q] >> sh) & 0xffu) < ((rb[q] >> sh) & 0xffu) ? -1 : 1;
                }
            }
        }
    }
    return by_len;
}

}  // namespace sg
