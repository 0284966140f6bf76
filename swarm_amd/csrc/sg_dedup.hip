// sg_dedup.hip — A7 sort -u dedup and A8 new-record diff on HBM-resident text.
//
// Pipeline (one stream):
//   lines   -> (start, end, key0) per record, key0 = chunk_key(rec, 0)
//   sort    -> LSD radix sort of (key0, rec id)
//   mark    -> equal-key groups; a group with tag < 8 is a run of identical records
//              (keep the first); a tag-8 group of >= 2 records shares 7 bytes and
//              continues, so it is refined:
//   refine  -> groups of <= 8 records: one thread ranks members by full byte compare
//              (stable; later equal members are duplicates). Larger groups: a radix
//              round on the next 7-byte chunk (stable sort by chunk, then by group),
//              repeated until every group is resolved. Exact for any input, including
//              64-bit-hash collisions, NULs and long shared prefixes.
//   select  -> unique positions in byte order -> serialize '\n'-terminated output.
//   diff    -> each unique record binary-searches the prior's sorted keys inside the
//              key range its 256-record block spans (full compare on 8-byte ties).
#include "sg_internal.hpp"
#include "sg_prims.hpp"

namespace sg {

const SlotSet CUR_SLOTS = {S_STARTS, S_ENDS, S_KEYS, S_KEYS2, S_VALS, S_VALS2, S_UNIQ, S_LB};
const SlotSet PRIOR_SLOTS = {S_P_STARTS, S_P_ENDS, S_P_KEYS, S_P_KEYS2, S_P_VALS, S_P_VALS2, S_P_UNIQ, S_P_FLAG};

constexpr uint32_t EQ_GROUP = 4096;
constexpr uint32_t WAVE_GROUP = 64;

// ------------------------------------------------------------------ launch helpers
template <class Pred>
static int run_select2(sg_ctx *c, const char *name, Pred pred, uint32_t n, uint32_t *outA,
                       uint32_t *outB, uint32_t *cntA, uint32_t *cntB) {
    *cntA = 0;
    if (cntB) *cntB = 0;
    if (n == 0) return SG_OK;
    const uint32_t ntiles = (n + SEL_TILE - 1) / SEL_TILE;
    uint64_t *status;
    SG_TRY(slot(c, S_COUNT, (size_t)ntiles + 4, &status));
    uint32_t *counter = reinterpret_cast<uint32_t *>(status + ntiles);
    SG_HIP(hipMemsetAsync(status, 0, ((size_t)ntiles + 4) * 8, c->stream));
    SG_LAUNCH(c, name, k_select2<Pred>, ntiles, SEL_BLOCK, 0, pred, n, outA, outB, status, counter, ntiles);
    uint32_t cnt[3];
    SG_TRY(ctx_readback(c, cnt, counter, 12));
    *cntA = cnt[1];
    if (cntB) *cntB = cnt[2];
    // model: the predicate reads ~8 B per item; 4 B written per selected index
    prof_bytes(c, name, 8.0 * n + 4.0 * (cnt[1] + (cntB ? cnt[2] : 0)));
    return SG_OK;
}

template <class Fn>
static int run_scan64(sg_ctx *c, const char *name, Fn fn, uint32_t n, uint64_t *out, uint64_t *total) {
    *total = 0;
    if (n == 0) return SG_OK;
    const uint32_t ntiles = (n + SCAN_TILE - 1) / SCAN_TILE;
    uint64_t *status;
    SG_TRY(slot(c, S_COUNT, (size_t)ntiles + 4, &status));
    uint32_t *counter = reinterpret_cast<uint32_t *>(status + ntiles);
    SG_HIP(hipMemsetAsync(status, 0, ((size_t)ntiles + 4) * 8, c->stream));
    SG_LAUNCH_B(c, name, 12.0 * n, k_scan64<Fn>, ntiles, SCAN_BLOCK, 0, fn, n, out, status, counter, ntiles);
    uint32_t cnt[3];
    SG_TRY(ctx_readback(c, cnt, counter, 12));
    *total = (uint64_t)cnt[1] | ((uint64_t)cnt[2] << 32);
    return SG_OK;
}

static inline uint32_t grid_for(uint64_t n, uint32_t block, uint32_t cap = 0x7fffffffu) {
    uint64_t g = (n + block - 1) / block;
    if (g == 0) g = 1;
    return (uint32_t)(g < cap ? g : cap);
}

// ------------------------------------------------------------------ predicates / functors
struct FlagPred {
    const uint8_t *f;
    __device__ uint32_t operator()(uint32_t i) const { return f[i] ? 1u : 0u; }
};

// Over sorted keys: uniq[i] = head(i); A = start of a multi-record tag-8 group,
// B = its last record.
struct GroupPred {
    const uint64_t *K;
    uint8_t *uniq;
    uint32_t n;
    __device__ uint32_t operator()(uint32_t i) const {
        const uint64_t k = K[i];
        const bool head = (i == 0) || K[i - 1] != k;
        const bool tail = (i + 1 == n) || K[i + 1] != k;
        uniq[i] = head ? 1 : 0;
        const bool t8 = (k & 0xffu) == 8u;
        return (t8 && head && !tail ? 1u : 0u) | (t8 && tail && !head ? 2u : 0u);
    }
};

// Over the final order of a refinement round: sub-groups by (gid, chunk key).
struct RoundGroupPred {
    const uint64_t *FK;     // chunk key, final order
    const uint32_t *G;      // group index, final order
    const uint32_t *P;      // global position, final order
    uint8_t *uniq;
    uint32_t n;
    __device__ uint32_t operator()(uint32_t i) const {
        const uint64_t k = FK[i];
        const uint32_t g = G[i];
        const bool head = (i == 0) || FK[i - 1] != k || G[i - 1] != g;
        const bool tail = (i + 1 == n) || FK[i + 1] != k || G[i + 1] != g;
        uniq[P[i]] = head ? 1 : 0;
        const bool t8 = (k & 0xffu) == 8u;
        return (t8 && head && !tail ? 1u : 0u) | (t8 && tail && !head ? 2u : 0u);
    }
};

struct BigGroupPred {
    const uint32_t *GS, *GE;
    __device__ uint32_t operator()(uint32_t i) const { return (GE[i] - GS[i] + 1u > WAVE_GROUP) ? 1u : 0u; }
};

struct DenseLenFn {
    const uint32_t *L;
    __device__ uint64_t operator()(uint32_t i) const { return L[i]; }
};

struct GroupSizeFn {
    const uint32_t *GS, *GE, *big;
    __device__ uint64_t operator()(uint32_t i) const {
        const uint32_t g = big[i];
        return (uint64_t)(GE[g] - GS[g] + 1u);
    }
};

__device__ __forceinline__ int key_cmp_full(const uint8_t *buf, const uint2 *spans,
                                            uint64_t ka, uint32_t ra, uint64_t kb, uint32_t rb, uint32_t off) {
    if (ka != kb) return ka < kb ? -1 : 1;
    if ((ka & 0xffu) < 8u) return 0;
    return rec_cmp_k(buf, spans[ra].x, spans[ra].y, buf, spans[rb].x, spans[rb].y, off + 7);
}

// ------------------------------------------------------------------ refinement kernels
// Every group (records sharing `off` bytes, >= 2 members): one thread checks whether all
// members are byte-identical to the first (the common case: duplicates). If so the first
// stays unique and the rest are duplicates, order unchanged. Otherwise (or above
// EQ_GROUP members) the group is flagged for ranking.
__global__ __launch_bounds__(256) void k_refine_eq(const uint8_t *__restrict__ buf,
                                                   const uint2 *__restrict__ spans,
                                                   const uint32_t *__restrict__ GS,
                                                   const uint32_t *__restrict__ GE, uint32_t G,
                                                   const uint32_t *__restrict__ V, uint8_t *uniq,
                                                   uint32_t off, uint8_t *unresolved) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= G) return;
    const uint32_t s = GS[g], k = GE[g] - s + 1u;
    bool same = k <= EQ_GROUP;
    if (same) {
        const uint32_t m0 = V[s];
        const uint32_t s0 = spans[m0].x, e0 = spans[m0].y;
        for (uint32_t a = 1; a < k; ++a) {
            const uint32_t m = V[s + a];
            if (!rec_equal(buf, s0, e0, buf, spans[m].x, spans[m].y, off)) { same = false; break; }
        }
    }
    if (same)
        for (uint32_t a = 1; a < k; ++a) uniq[s + a] = 0;
    unresolved[g] = same ? 0 : 1;
}

// Unresolved groups of <= 64 records: one wave per group, one member per lane; each lane counts the
// members that precede it (stable), duplicates are members equal to an earlier one.
__global__ __launch_bounds__(256) void k_refine_wave(const uint8_t *__restrict__ buf,
                                                     const uint2 *__restrict__ spans,
                                                     const uint32_t *__restrict__ GS,
                                                     const uint32_t *__restrict__ GE, uint32_t G,
                                                     uint32_t *V, uint8_t *uniq, uint32_t off) {
    const uint32_t g = blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t lane = lane_id();
    if (g >= G) return;
    const uint32_t s = GS[g], k = GE[g] - s + 1u;
    if (k > WAVE_GROUP) return;
    const bool act = lane < k;
    const uint32_t m = act ? V[s + lane] : 0u;
    const uint64_t key = act ? chunk_key(buf, spans[m].x, spans[m].y, off) : ~0ull;
    uint32_t rank = 0;
    bool dup = false;
    for (uint32_t j = 0; j < k; ++j) {
        const uint64_t kb = __shfl(key, (int)j, 64);
        const uint32_t mb = __shfl(m, (int)j, 64);
        if (act && j != lane) {
            const int c = key_cmp_full(buf, spans, key, m, kb, mb, off);
            if (c > 0 || (c == 0 && j < lane)) rank++;
            if (c == 0 && j < lane) dup = true;
        }
    }
    if (act) {
        V[s + rank] = m;
        uniq[s + rank] = dup ? 0 : 1;
    }
}

// Expand big groups into member rows: row j -> group index (into big list), global
// position, and the record's chunk key at `off`.
__global__ __launch_bounds__(256) void k_expand(const uint8_t *__restrict__ buf,
                                                const uint2 *__restrict__ spans,
                                                const uint32_t *__restrict__ GS,
                                                const uint32_t *__restrict__ big,
                                                const uint64_t *__restrict__ goff, uint32_t B,
                                                const uint32_t *__restrict__ V, uint32_t M,
                                                uint32_t off, uint64_t *RK, uint32_t *RG,
                                                uint32_t *RP) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= M) return;
    uint32_t lo = 0, hi = B;  // last k with goff[k] <= j
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (goff[mid] <= j) lo = mid; else hi = mid;
    }
    const uint32_t pos = GS[big[lo]] + (j - (uint32_t)goff[lo]);
    const uint32_t r = V[pos];
    RK[j] = chunk_key(buf, spans[r].x, spans[r].y, off);
    RG[j] = lo;
    RP[j] = pos;
}

__global__ void k_gather_pair(const uint32_t *__restrict__ idx, const uint32_t *__restrict__ A,
                              const uint32_t *__restrict__ B, uint32_t n, uint32_t *A2, uint32_t *B2) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t q = idx[i];
    A2[i] = A[q];
    B2[i] = B[q];
}

__global__ void k_gid_keys(const uint32_t *__restrict__ RG, const uint32_t *__restrict__ perm,
                           uint64_t *GK, uint32_t M) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < M) GK[i] = RG[perm[i]];
}

// Final order of a round: T[i] = record now at final index i; FK its chunk key.
__global__ void k_round_gather(const uint8_t *__restrict__ buf, const uint2 *__restrict__ spans, const uint32_t *__restrict__ V,
                               const uint32_t *__restrict__ RP, const uint32_t *__restrict__ perm,
                               uint32_t M, uint32_t off, uint32_t *T, uint64_t *FK) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= M) return;
    const uint32_t r = V[RP[perm[i]]];
    T[i] = r;
    FK[i] = chunk_key(buf, spans[r].x, spans[r].y, off);
}

__global__ void k_round_scatter(const uint32_t *__restrict__ T, const uint32_t *__restrict__ RP,
                                uint32_t M, uint32_t *V) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < M) V[RP[i]] = T[i];
}

__global__ void k_pos_of(const uint32_t *__restrict__ idx, const uint32_t *__restrict__ RP, uint32_t n,
                         uint32_t *out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = RP[idx[i]];
}

// ------------------------------------------------------------------ gathers / output
// Selected positions -> record id, key0 and serialized length (len + 1) per record.
__global__ void k_gather_sel(const uint32_t *__restrict__ sel, const uint32_t *__restrict__ V,
                             const uint64_t *__restrict__ K, const uint2 *__restrict__ spans, uint32_t n, uint32_t *UR, uint64_t *UK,
                             uint32_t *UL) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t p = sel[i];
    const uint32_t r = V ? V[p] : p;
    UR[i] = r;
    if (UK) UK[i] = K[p];
    UL[i] = spans[r].y - spans[r].x + 1u;
}

__global__ void k_gather_rl(const uint32_t *__restrict__ idx, const uint32_t *__restrict__ R,
                            const uint32_t *__restrict__ L, uint32_t n, uint32_t *R2, uint32_t *L2) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t q = idx[i];
    R2[i] = R[q];
    L2[i] = L[q];
}

constexpr uint32_t CP_WAVE_BYTES = 8192;

// Records (list order) -> out at offs[i], each '\n'-terminated. Each wave owns 64
// consecutive list entries, whose output is one contiguous span. The wave assembles that
// span in an LDS window: groups of 16 lanes copy one record at a time with coalesced
// aligned word loads (the record's bytes are contiguous in the source), then the whole
// wave writes the window with 16-byte stores. Spans wider than the window (records longer
// than CP_WAVE_BYTES / 64 on average) are copied the same way straight to HBM.
__global__ __launch_bounds__(256) void k_copy_records(const uint8_t *__restrict__ buf,
                                                      const uint2 *__restrict__ spans,
                                                      const uint32_t *__restrict__ recs,
                                                      const uint64_t *__restrict__ offs, uint32_t n,
                                                      uint8_t *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint8_t s_buf[4][CP_WAVE_BYTES];
    __shared__ uint32_t s_src[4][64], s_len[4][64], s_dst[4][64];
    const uint32_t wid = threadIdx.x >> 6, lane = lane_id();
    const uint32_t wfirst = (blockIdx.x * 4 + wid) * 64u;
    if (wfirst >= n) return;
    const uint32_t i = wfirst + lane;
    const bool act = i < n;
    const uint32_t r = act ? recs[i] : 0u;
    const uint2 sp = act ? spans[r] : make_uint2(0, 0);
    const uint32_t s = sp.x, len = sp.y - sp.x;
    const uint64_t o = act ? offs[i] : 0ull;
    const uint32_t last = (n - wfirst) < 64u ? (n - wfirst - 1u) : 63u;
    const uint64_t o0 = __shfl(o, 0, 64);
    const uint64_t oend = __shfl(o + len + 1u, (int)last, 64);
    const uint64_t base = o0 & ~15ull;
    const uint64_t span = oend - base;
    const bool in_lds = span <= CP_WAVE_BYTES;
    s_src[wid][lane] = s;
    s_len[wid][lane] = len;
    s_dst[wid][lane] = (uint32_t)(o - base);  // < 4 GiB: one call's output
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const uint32_t g = lane >> 4, gl = lane & 15;
    uint8_t *L = s_buf[wid];
    for (uint32_t j = g; j <= last; j += 4) {
        const uint32_t sj = s_src[wid][j], lj = s_len[wid][j];
        const uint32_t ej = sj + lj;
        const uint32_t a0 = sj & ~3u;
        uint8_t *dst = (in_lds ? L : out + base) + s_dst[wid][j];
        for (uint32_t a = a0 + 4 * gl; a < ej; a += 64) {
            const uint32_t x = *reinterpret_cast<const uint32_t *>(buf + a);
#pragma unroll
            for (uint32_t b = 0; b < 4; ++b) {
                const uint32_t p = a + b;
                if (p >= sj && p < ej) dst[p - sj] = (uint8_t)(x >> (8 * b));
            }
        }
        if (gl == 0) dst[lj] = 0x0a;
    }
    if (!in_lds) return;
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const uint32_t nch = (uint32_t)((span + 15) / 16);
    for (uint32_t ch = lane; ch < nch; ch += 64) {
        const uint64_t ga = base + 16ull * ch;
        if (ga >= o0 && ga + 16 <= oend) {
            *reinterpret_cast<uint4 *>(out + ga) = *reinterpret_cast<const uint4 *>(L + 16 * ch);
        } else {
#pragma unroll
            for (uint32_t b = 0; b < 16; ++b) {
                const uint64_t ad = ga + b;
                if (ad >= o0 && ad < oend) out[ad] = L[16 * ch + b];
            }
        }
    }
}

// Prior check: flag[0] = 1 if records are not strictly increasing.
__global__ void k_check_sorted(const uint8_t *__restrict__ buf, const uint2 *__restrict__ spans, const uint64_t *__restrict__ K,
                               uint32_t n, uint32_t *flag) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x + 1;
    if (i >= n) return;
    if (key_cmp_full(buf, spans, K[i - 1], i - 1, K[i], i, 0) >= 0) atomicOr(flag, 1u);
}

// ------------------------------------------------------------------ diff (merge path)
struct RecSet {
    const uint8_t *buf;
    const uint2 *sp;
    const uint32_t *ids;  // position -> record id (null = identity)
    const uint64_t *K;    // key0 per position
    uint32_t n;
    __device__ uint32_t id(uint32_t i) const { return ids ? ids[i] : i; }
};

__device__ __forceinline__ int set_cmp(const RecSet &A, uint64_t ka, uint32_t ra, const RecSet &B, uint64_t kb,
                                       uint32_t rb) {
    if (ka != kb) return ka < kb ? -1 : 1;
    if ((ka & 0xffu) < 8u) return 0;
    return rec_cmp_k(A.buf, A.sp[ra].x, A.sp[ra].y, B.buf, B.sp[rb].x, B.sp[rb].y, 7);
}

constexpr uint32_t MP_TILE = 2048;

// Merge-path split of diagonal t*MP_TILE over (U, P), U first on ties: split[t] = i.
__global__ void k_merge_split(RecSet U, RecSet P, uint32_t ntiles, uint32_t *split) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t > ntiles) return;
    const uint64_t tot = (uint64_t)U.n + P.n;
    const uint64_t d64 = (uint64_t)t * MP_TILE < tot ? (uint64_t)t * MP_TILE : tot;
    const uint32_t d = (uint32_t)d64;
    uint32_t lo = d > P.n ? d - P.n : 0u, hi = d < U.n ? d : U.n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        const uint32_t j = d - mid - 1;
        if (set_cmp(U, U.K[mid], U.id(mid), P, P.K[j], P.id(j)) <= 0) lo = mid + 1;
        else hi = mid;
    }
    split[t] = lo;
}

// fresh[i] = 1 if U[i] is absent from P. Inside the tile's P range (keys staged in LDS)
// find the run of P keys equal to U[i]'s key0: a tag < 8 key is the whole record, so the
// run decides; a tag-8 run (usually one record) is checked with a wide byte compare. The
// run may continue past the tile into P[j1...] (ties go to U first in the merge order).
__global__ __launch_bounds__(256) void k_diff_tile(RecSet U, RecSet P, const uint32_t *__restrict__ split,
                                                   uint8_t *fresh) {
    __shared__ uint64_t s_k[MP_TILE];
    __shared__ uint32_t s_r[MP_TILE];
    const uint32_t t = blockIdx.x;
    const uint64_t tot = (uint64_t)U.n + P.n;
    const uint32_t d0 = (uint32_t)((uint64_t)t * MP_TILE);
    const uint32_t d1 = (uint32_t)((uint64_t)(t + 1) * MP_TILE < tot ? (uint64_t)(t + 1) * MP_TILE : tot);
    const uint32_t i0 = split[t], i1 = split[t + 1];
    const uint32_t j0 = d0 - i0, j1 = d1 - i1;
    const uint32_t np = j1 - j0;
    for (uint32_t q = threadIdx.x; q < np; q += blockDim.x) {
        s_k[q] = P.K[j0 + q];
        s_r[q] = P.id(j0 + q);
    }
    __syncthreads();
    for (uint32_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
        const uint64_t ku = U.K[i];
        uint32_t lo = 0, hi = np;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (s_k[mid] < ku) lo = mid + 1;
            else hi = mid;
        }
        bool present = false;
        const bool whole = (ku & 0xffu) < 8u;
        uint32_t ru = 0, us = 0, ue = 0;
        if (!whole) { ru = U.id(i); us = U.sp[ru].x; ue = U.sp[ru].y; }
        for (uint32_t q = j0 + lo; q < P.n; ++q) {
            const uint32_t lq = q - j0;
            const uint64_t kp = (lq < np) ? s_k[lq] : P.K[q];
            if (kp != ku) break;
            if (whole) { present = true; break; }
            const uint32_t rp = (lq < np) ? s_r[lq] : P.id(q);
            if (rec_equal(U.buf, us, ue, P.buf, P.sp[rp].x, P.sp[rp].y, 7)) { present = true; break; }
        }
        fresh[i] = present ? 0 : 1;
    }
}

// ------------------------------------------------------------------ host pipeline
int select_flags(sg_ctx *c, const uint8_t *flags, uint32_t n, uint32_t *out_idx, uint32_t *count) {
    return run_select2(c, "select", FlagPred{flags}, n, out_idx, (uint32_t *)nullptr, count, nullptr);
}

// recs/lens: record ids and serialized lengths (len + 1) in output order.
static int serialize_dense(sg_ctx *c, const uint8_t *d_buf, const uint2 *spans,
                           const uint32_t *recs, const uint32_t *lens, uint32_t count, int out_slot,
                           uint8_t *dst, size_t dst_cap, uint8_t **d_out, uint64_t *bytes) {
    *bytes = 0;
    uint64_t *offs;
    SG_TRY(slot(c, S_OFFS, (size_t)count + 1, &offs));
    uint64_t total = 0;
    SG_TRY(run_scan64(c, "scan_len", DenseLenFn{lens}, count, offs, &total));
    if (dst) {
        if (total > dst_cap) { set_error("output capacity %zu < %llu", dst_cap, (unsigned long long)total); return SG_E_CAP; }
        *d_out = dst;
    } else {
        SG_TRY(slot(c, out_slot, (size_t)total + 16, d_out));
    }
    // model: each output byte read once and written once, plus id/start/end/offset per record
    if (count) SG_LAUNCH_B(c, "copy_records", 2.0 * total + 20.0 * count, k_copy_records, grid_for(count, 256), 256, 0, d_buf, spans, recs, offs, count, *d_out);
    *bytes = total;
    return SG_OK;
}

__global__ void k_lens_of(const uint32_t *__restrict__ recs, const uint2 *__restrict__ spans, uint32_t n, uint32_t *L) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) { const uint32_t r = recs[i]; L[i] = spans[r].y - spans[r].x + 1u; }
}

int serialize(sg_ctx *c, const uint8_t *d_buf, const uint2 *spans,
              const uint32_t *recs, const uint32_t * /*map*/, uint32_t count, int out_slot,
              uint8_t **d_out, uint64_t *bytes) {
    uint32_t *L;
    SG_TRY(slot(c, S_M_TMP2, (size_t)count + 1, &L));
    if (count) SG_LAUNCH(c, "lens", k_lens_of, grid_for(count, 256), 256, 0, recs, spans, count, L);
    return serialize_dense(c, d_buf, spans, recs, L, count, out_slot, nullptr, 0, d_out, bytes);
}

int serialize_into(sg_ctx *c, const uint8_t *d_buf, const uint2 *spans,
                   const uint32_t *recs, uint32_t count, uint8_t *dst, size_t dst_cap, uint64_t *bytes) {
    uint32_t *L;
    SG_TRY(slot(c, S_M_TMP2, (size_t)count + 1, &L));
    if (count) SG_LAUNCH(c, "lens", k_lens_of, grid_for(count, 256), 256, 0, recs, spans, count, L);
    uint8_t *o;
    return serialize_dense(c, d_buf, spans, recs, L, count, 0, dst, dst_cap, &o, bytes);
}

int sort_records(sg_ctx *c, const uint8_t *d_buf, const Lines &L, const SlotSet &ss, SortedSet *out) {
    const uint32_t R = L.n_rec;
    out->n = R;
    uint64_t *k2;
    uint32_t *v1, *v2;
    SG_TRY(slot(c, ss.keys2, R, &k2));
    SG_TRY(slot(c, ss.vals, R, &v1));
    SG_TRY(slot(c, ss.vals2, R, &v2));
    uint8_t *uniq;
    SG_TRY(slot(c, ss.uniq, R, &uniq));
    out->uniq = uniq;
    if (R == 0) { out->keys = L.keys; out->recs = v1; return SG_OK; }
    uint64_t *K;
    uint32_t *V;
    SG_TRY(radix_sort(c, L.keys, v1, k2, v2, R, 0, 64, true, &K, &V));
    out->keys = K;
    out->recs = V;

    // groups of the first chunk
    uint32_t *GS, *GE;
    SG_TRY(slot(c, S_GS, R / 2 + 16, &GS));
    SG_TRY(slot(c, S_GE, R / 2 + 16, &GE));
    uint32_t G = 0, G2 = 0;
    SG_TRY(run_select2(c, "mark_groups", GroupPred{K, uniq, R}, R, GS, GE, &G, &G2));
    if (G != G2) { set_error("group start/end mismatch %u/%u", G, G2); return SG_E_HIP; }

    uint32_t off = 7;
    while (G > 0) {
        uint8_t *unres;
        SG_TRY(slot(c, S_M_TMP, (size_t)G + 16, &unres));
        // model: per group GS/GE + flag; per member id, start, end and ~26 record bytes twice
        SG_LAUNCH_B(c, "refine_eq", 9.0 * G + 64.0 * 2.0 * G, k_refine_eq, grid_for(G, 256), 256, 0, d_buf, L.spans, GS, GE, G, V, uniq, off, unres);
        uint32_t *ulist;
        SG_TRY(slot(c, S_SEL, (size_t)G + 16, &ulist));
        uint32_t Ux = 0;
        SG_TRY(select_flags(c, unres, G, ulist, &Ux));
        if (Ux == 0) break;
        uint32_t *GS2, *GE2;
        SG_TRY(slot(c, S_R_GID, (size_t)Ux + 16, &GS2));
        SG_TRY(slot(c, S_R_POS, (size_t)Ux + 16, &GE2));
        SG_LAUNCH(c, "gather_groups", k_gather_pair, grid_for(Ux, 256), 256, 0, ulist, GS, GE, Ux, GS2, GE2);
        SG_LAUNCH(c, "refine_wave", k_refine_wave, grid_for(Ux, 4), 256, 0, d_buf, L.spans, GS2, GE2, Ux, V, uniq, off);
        // unresolved groups above one wave -> a radix round on the next chunk
        uint32_t *big;
        SG_TRY(slot(c, S_SEL, Ux + 16, &big));
        uint32_t B = 0;
        SG_TRY(run_select2(c, "select_big", BigGroupPred{GS2, GE2}, Ux, big, (uint32_t *)nullptr, &B, nullptr));
        if (B == 0) break;
        SG_HIP(hipMemcpyAsync(GS, GS2, (size_t)Ux * 4, hipMemcpyDeviceToDevice, c->stream));
        SG_HIP(hipMemcpyAsync(GE, GE2, (size_t)Ux * 4, hipMemcpyDeviceToDevice, c->stream));
        uint64_t *goff;
        SG_TRY(slot(c, S_R_OFF, (size_t)B + 1, &goff));
        uint64_t M64 = 0;
        SG_TRY(run_scan64(c, "scan_groups", GroupSizeFn{GS, GE, big}, B, goff, &M64));
        const uint32_t M = (uint32_t)M64;
        uint64_t *RK, *RK2, *GK;
        uint32_t *RG, *RP, *RV, *RV2, *T;
        SG_TRY(slot(c, S_R_KEY, M, &RK));
        SG_TRY(slot(c, S_R_KEY2, M, &RK2));
        SG_TRY(slot(c, S_R_GID, M, &RG));
        SG_TRY(slot(c, S_R_POS, M, &RP));
        SG_TRY(slot(c, S_R_VAL, M, &RV));
        SG_TRY(slot(c, S_R_VAL2, M, &RV2));
        SG_LAUNCH(c, "round_expand", k_expand, grid_for(M, 256), 256, 0, d_buf, L.spans, GS, big, goff, B, V, M, off, RK, RG, RP);
        uint64_t *SK;
        uint32_t *perm;
        SG_TRY(radix_sort(c, RK, RV, RK2, RV2, M, 0, 64, true, &SK, &perm, "rs_pass_refine"));
        // stable by group index on top: keys = gid of each row in current order
        GK = (SK == RK) ? RK2 : RK;
        uint32_t *pv_alt = (perm == RV) ? RV2 : RV;
        SG_LAUNCH(c, "round_gid", k_gid_keys, grid_for(M, 256), 256, 0, RG, perm, GK, M);
        int gbits = 1;
        while (gbits < 32 && (1u << gbits) < B) ++gbits;
        uint64_t *GK2 = (GK == RK) ? RK2 : RK;
        uint64_t *FKs;
        uint32_t *perm2;
        SG_TRY(radix_sort(c, GK, perm, GK2, pv_alt, M, 0, gbits, false, &FKs, &perm2, "rs_pass_refine"));
        T = (perm2 == perm) ? pv_alt : perm;
        uint64_t *FK = (FKs == GK) ? GK2 : GK;
        SG_LAUNCH(c, "round_gather", k_round_gather, grid_for(M, 256), 256, 0, d_buf, L.spans, V, RP, perm2, M, off, T, FK);
        SG_LAUNCH(c, "round_scatter", k_round_scatter, grid_for(M, 256), 256, 0, T, RP, M, V);
        // sub-groups: RG is the group index of final row i as well (same row ranges);
        // perm2/T are free again after the scatter (same stream)
        uint32_t *NS = perm2, *NE = T;
        uint32_t G3 = 0, G4 = 0;
        SG_TRY(run_select2(c, "round_mark", RoundGroupPred{FK, RG, RP, uniq, M}, M, NS, NE, &G3, &G4));
        if (G3 != G4) { set_error("round group mismatch"); return SG_E_HIP; }
        if (G3) {
            SG_LAUNCH(c, "round_pos", k_pos_of, grid_for(G3, 256), 256, 0, NS, RP, G3, GS);
            SG_LAUNCH(c, "round_pos", k_pos_of, grid_for(G3, 256), 256, 0, NE, RP, G3, GE);
        }
        G = G3;
        off += 7;
    }
    return SG_OK;
}

// Parsed + sorted-unique view of one buffer.
struct UniqView {
    Lines L;
    uint32_t *UR = nullptr;  // record ids, byte order (null = identity 0..U-1)
    uint64_t *UK = nullptr;  // key0 per unique record
    uint32_t *UL = nullptr;  // serialized length per unique record (may be null)
    uint32_t U = 0;
};

static int unique_view(sg_ctx *c, const uint8_t *d_buf, uint64_t n, const SlotSet &ss, int ur_slot,
                       int uk_slot, int ul_slot, bool trust_sorted, UniqView *uv) {
    SG_TRY(run_lines(c, d_buf, n, ss, &uv->L));
    const uint32_t R = uv->L.n_rec;
    if (trust_sorted && R > 1) {
        uint32_t *flag;
        SG_TRY(slot(c, S_M_CNT, 4, &flag));
        SG_HIP(hipMemsetAsync(flag, 0, 4, c->stream));
        SG_LAUNCH_B(c, "check_sorted", 8.0 * R, k_check_sorted, grid_for(R - 1, 256), 256, 0, d_buf, uv->L.spans, uv->L.keys, R, flag);
        uint32_t f = 1;
        SG_TRY(ctx_readback(c, &f, flag, 4));
        trust_sorted = (f == 0);
    }
    if (trust_sorted) {
        uv->UR = nullptr;
        uv->UK = uv->L.keys;
        uv->UL = nullptr;
        uv->U = R;
        return SG_OK;
    }
    SortedSet S;
    SG_TRY(sort_records(c, d_buf, uv->L, ss, &S));
    uint32_t *sel;
    SG_TRY(slot(c, S_SEL, R + 16, &sel));
    uint32_t U = 0;
    SG_TRY(select_flags(c, S.uniq, R, sel, &U));
    SG_TRY(slot(c, ur_slot, (size_t)U + 1, &uv->UR));
    SG_TRY(slot(c, uk_slot, (size_t)U + 1, &uv->UK));
    SG_TRY(slot(c, ul_slot, (size_t)U + 1, &uv->UL));
    if (U) SG_LAUNCH_B(c, "gather_uniq", 40.0 * U, k_gather_sel, grid_for(U, 256), 256, 0, sel, S.recs, S.keys, uv->L.spans, U, uv->UR, uv->UK, uv->UL);
    uv->U = U;
    return SG_OK;
}

int dev_dedup_diff(sg_ctx *c, const uint8_t *d_cur, uint64_t n_cur, const uint8_t *d_prior,
                   uint64_t n_prior, bool want_fresh, sg_dev_result *res) {
    *res = sg_dev_result{};
    UniqView cu;
    SG_TRY(unique_view(c, d_cur, n_cur, CUR_SLOTS, S_CUR_UR, S_CUR_UK, S_FRESH_IDX, false, &cu));
    res->in_records = cu.L.n_rec;
    uint8_t *uout;
    uint64_t ubytes = 0;
    SG_TRY(serialize_dense(c, d_cur, cu.L.spans, cu.UR, cu.UL, cu.U, S_OUT_UNIQ, nullptr, 0, &uout, &ubytes));
    res->uniq = uout;
    res->uniq_bytes = ubytes;
    res->uniq_records = cu.U;
    if (!want_fresh) return SG_OK;

    UniqView pv;
    if (d_prior && n_prior) {
        SG_TRY(unique_view(c, d_prior, n_prior, PRIOR_SLOTS, S_P_REC, S_P_SORTED_KEYS, S_P_FLAG, true, &pv));
    }
    res->prior_records = pv.L.n_rec;
    if (pv.U == 0 || cu.U == 0) {
        res->fresh = res->uniq;
        res->fresh_bytes = res->uniq_bytes;
        res->fresh_records = res->uniq_records;
        return SG_OK;
    }
    uint8_t *fresh;
    SG_TRY(slot(c, S_M_TMP, (size_t)cu.U + 1, &fresh));
    RecSet U{d_cur, cu.L.spans, cu.UR, cu.UK, cu.U};
    RecSet P{d_prior, pv.L.spans, pv.UR, pv.UK, pv.U};
    const uint32_t ntiles = (uint32_t)(((uint64_t)cu.U + pv.U + MP_TILE - 1) / MP_TILE);
    uint32_t *split;
    SG_TRY(slot(c, S_R_OFF, (size_t)ntiles + 2, &split));
    SG_LAUNCH(c, "merge_split", k_merge_split, grid_for(ntiles + 1, 256), 256, 0, U, P, ntiles, split);
    // model: key+id of every unique cur and prior record, one flag per cur record
    SG_LAUNCH_B(c, "diff_tile", 12.0 * (cu.U + (double)pv.U) + cu.U, k_diff_tile, ntiles, 256, 0, U, P, split, fresh);
    uint32_t *fidx;
    SG_TRY(slot(c, S_SEL, (size_t)cu.U + 16, &fidx));
    uint32_t F = 0;
    SG_TRY(select_flags(c, fresh, cu.U, fidx, &F));
    uint32_t *FR, *FL;
    SG_TRY(slot(c, S_R_VAL, (size_t)F + 1, &FR));
    SG_TRY(slot(c, S_R_GID, (size_t)F + 1, &FL));
    if (F) SG_LAUNCH(c, "gather_fresh", k_gather_rl, grid_for(F, 256), 256, 0, fidx, cu.UR, cu.UL, F, FR, FL);
    uint8_t *fout;
    uint64_t fbytes = 0;
    SG_TRY(serialize_dense(c, d_cur, cu.L.spans, FR, FL, F, S_OUT_FRESH, nullptr, 0, &fout, &fbytes));
    res->fresh = fout;
    res->fresh_bytes = fbytes;
    res->fresh_records = F;
    return SG_OK;
}

}  // namespace sg
