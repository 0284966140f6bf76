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

constexpr uint32_t SMALL_GROUP = 8;

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
    SG_LAUNCH(c, name, k_scan64<Fn>, ntiles, SCAN_BLOCK, 0, fn, n, out, status, counter, ntiles);
    uint32_t cnt[3];
    SG_TRY(ctx_readback(c, cnt, counter, 12));
    *total = (uint64_t)cnt[1] | ((uint64_t)cnt[2] << 32);
    return SG_OK;
}

static inline uint32_t grid_for(uint64_t n, uint32_t block, uint32_t cap = 65535u * 4) {
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
    __device__ uint32_t operator()(uint32_t i) const { return (GE[i] - GS[i] + 1u > SMALL_GROUP) ? 1u : 0u; }
};

struct RecLenFn {
    const uint32_t *starts, *ends, *recs;
    __device__ uint64_t operator()(uint32_t i) const {
        const uint32_t r = recs[i];
        return (uint64_t)(ends[r] - starts[r]) + 1ull;
    }
};

struct GroupSizeFn {
    const uint32_t *GS, *GE, *big;
    __device__ uint64_t operator()(uint32_t i) const {
        const uint32_t g = big[i];
        return (uint64_t)(GE[g] - GS[g] + 1u);
    }
};

// ------------------------------------------------------------------ kernels
// Groups of <= 8 records sharing `off` bytes: rank by full compare, stable; duplicates
// (equal to an earlier member) lose uniq.
__global__ __launch_bounds__(256) void k_refine_small(const uint8_t *__restrict__ buf,
                                                      const uint32_t *__restrict__ starts,
                                                      const uint32_t *__restrict__ ends,
                                                      const uint32_t *__restrict__ GS,
                                                      const uint32_t *__restrict__ GE, uint32_t G,
                                                      uint32_t *V, uint8_t *uniq, uint32_t off) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= G) return;
    const uint32_t s = GS[g], k = GE[g] - s + 1u;
    if (k > SMALL_GROUP) return;
    uint32_t m[SMALL_GROUP], rs[SMALL_GROUP], re[SMALL_GROUP], rank[SMALL_GROUP];
    bool dup[SMALL_GROUP];
#pragma unroll
    for (uint32_t a = 0; a < SMALL_GROUP; ++a) {
        if (a < k) {
            m[a] = V[s + a];
            rs[a] = starts[m[a]];
            re[a] = ends[m[a]];
        }
        rank[a] = 0;
        dup[a] = false;
    }
#pragma unroll
    for (uint32_t a = 0; a < SMALL_GROUP; ++a) {
#pragma unroll
        for (uint32_t b = a + 1; b < SMALL_GROUP; ++b) {
            if (b < k) {
                const int cmp = rec_cmp(buf, rs[a], re[a], buf, rs[b], re[b], off);
                // stable: a precedes b when a <= b
                if (cmp <= 0) rank[b]++; else rank[a]++;
                if (cmp == 0) dup[b] = true;
            }
        }
    }
#pragma unroll
    for (uint32_t a = 0; a < SMALL_GROUP; ++a) {
        if (a < k) {
            V[s + rank[a]] = m[a];
            uniq[s + rank[a]] = dup[a] ? 0 : 1;
        }
    }
}

// Expand big groups into member rows: row j -> group index (into big list), global
// position, and the record's chunk key at `off`.
__global__ __launch_bounds__(256) void k_expand(const uint8_t *__restrict__ buf,
                                                const uint32_t *__restrict__ starts,
                                                const uint32_t *__restrict__ ends,
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
    RK[j] = chunk_key(buf, starts[r], ends[r], off);
    RG[j] = lo;
    RP[j] = pos;
}

__global__ void k_gid_keys(const uint32_t *__restrict__ RG, const uint32_t *__restrict__ perm,
                           uint64_t *GK, uint32_t M) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < M) GK[i] = RG[perm[i]];
}

// Final order of a round: T[i] = record now at final index i; FK its chunk key.
__global__ void k_round_gather(const uint8_t *__restrict__ buf, const uint32_t *__restrict__ starts,
                               const uint32_t *__restrict__ ends, const uint32_t *__restrict__ V,
                               const uint32_t *__restrict__ RP, const uint32_t *__restrict__ perm,
                               uint32_t M, uint32_t off, uint32_t *T, uint64_t *FK) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= M) return;
    const uint32_t r = V[RP[perm[i]]];
    T[i] = r;
    FK[i] = chunk_key(buf, starts[r], ends[r], off);
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

__global__ void k_gather_u32(const uint32_t *__restrict__ src, const uint32_t *__restrict__ idx,
                             uint32_t n, uint32_t *out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = src[idx[i]];
}

__global__ void k_gather_u64(const uint64_t *__restrict__ src, const uint32_t *__restrict__ idx,
                             uint32_t n, uint64_t *out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = src[idx[i]];
}

// Copy records (list order) to out at offs[i]; each followed by '\n'.
__global__ __launch_bounds__(256) void k_copy_records(const uint8_t *__restrict__ buf,
                                                      const uint32_t *__restrict__ starts,
                                                      const uint32_t *__restrict__ ends,
                                                      const uint32_t *__restrict__ recs,
                                                      const uint64_t *__restrict__ offs, uint32_t n,
                                                      uint8_t *__restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t r = recs[i];
    const uint32_t s = starts[r], e = ends[r];
    uint8_t *d = out + offs[i];
    for (uint32_t p = s; p < e; ++p) *d++ = buf[p];
    *d = 0x0a;
}

// Prior check: flag[0] = 1 if records are not strictly increasing.
__global__ void k_check_sorted(const uint8_t *__restrict__ buf, const uint32_t *__restrict__ starts,
                               const uint32_t *__restrict__ ends, const uint64_t *__restrict__ K,
                               uint32_t n, uint32_t *flag) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x + 1;
    if (i >= n) return;
    const uint64_t a = K[i - 1], b = K[i];
    bool bad;
    if (a != b) bad = a > b;
    else if ((a & 0xffu) < 8u) bad = true;  // identical records
    else bad = rec_cmp(buf, starts[i - 1], ends[i - 1], buf, starts[i], ends[i], 7) >= 0;
    if (bad) atomicOr(flag, 1u);
}

__device__ __forceinline__ int cmp_rec_key(const uint8_t *ub, uint32_t us, uint32_t ue, uint64_t uk,
                                           const uint8_t *pb, uint32_t ps, uint32_t pe, uint64_t pk) {
    if (uk != pk) return uk < pk ? -1 : 1;
    if ((uk & 0xffu) < 8u) return 0;
    return rec_cmp(ub, us, ue, pb, ps, pe, 7);
}

// fresh[i] = unique cur record i (sorted) is absent from the prior (sorted unique).
__global__ __launch_bounds__(256) void k_diff_mark(
    const uint8_t *__restrict__ cbuf, const uint32_t *__restrict__ cst, const uint32_t *__restrict__ cen,
    const uint32_t *__restrict__ UR, const uint64_t *__restrict__ UK, uint32_t U,
    const uint8_t *__restrict__ pbuf, const uint32_t *__restrict__ pst, const uint32_t *__restrict__ pen,
    const uint32_t *__restrict__ PR, const uint64_t *__restrict__ PK, uint32_t P, uint8_t *fresh) {
    __shared__ uint32_t s_lo, s_hi;
    const uint32_t i0 = blockIdx.x * blockDim.x;
    const uint32_t i = i0 + threadIdx.x;
    auto prec = [&](uint32_t j) { return PR ? PR[j] : j; };
    auto lower = [&](uint32_t r, uint64_t k, uint32_t lo, uint32_t hi) {
        const uint32_t us = cst[r], ue = cen[r];
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            const uint32_t q = prec(mid);
            if (cmp_rec_key(cbuf, us, ue, k, pbuf, pst[q], pen[q], PK[mid]) > 0) lo = mid + 1;
            else hi = mid;
        }
        return lo;
    };
    if (threadIdx.x == 0) {
        const uint32_t last = (i0 + blockDim.x <= U) ? i0 + blockDim.x - 1 : U - 1;
        s_lo = lower(UR[i0], UK[i0], 0, P);
        s_hi = lower(UR[last], UK[last], s_lo, P);
    }
    __syncthreads();
    if (i >= U) return;
    const uint32_t r = UR[i];
    const uint64_t k = UK[i];
    const uint32_t j = lower(r, k, s_lo, s_hi);
    bool present = false;
    if (j < P) {
        const uint32_t q = prec(j);
        present = cmp_rec_key(cbuf, cst[r], cen[r], k, pbuf, pst[q], pen[q], PK[j]) == 0;
    }
    fresh[i] = present ? 0 : 1;
}

// ------------------------------------------------------------------ host pipeline
int select_flags(sg_ctx *c, const uint8_t *flags, uint32_t n, uint32_t *out_idx, uint32_t *count) {
    return run_select2(c, "select", FlagPred{flags}, n, out_idx, (uint32_t *)nullptr, count, nullptr);
}

int serialize(sg_ctx *c, const uint8_t *d_buf, const uint32_t *starts, const uint32_t *ends,
              const uint32_t *recs, const uint32_t * /*map*/, uint32_t count, int out_slot,
              uint8_t **d_out, uint64_t *bytes) {
    *bytes = 0;
    uint64_t *offs;
    SG_TRY(slot(c, S_OFFS, (size_t)count + 1, &offs));
    uint64_t total = 0;
    SG_TRY(run_scan64(c, "scan_len", RecLenFn{starts, ends, recs}, count, offs, &total));
    SG_TRY(slot(c, out_slot, (size_t)total + 16, d_out));
    if (count) SG_LAUNCH(c, "copy_records", k_copy_records, grid_for(count, 256), 256, 0, d_buf, starts, ends, recs, offs, count, *d_out);
    *bytes = total;
    return SG_OK;
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
        SG_LAUNCH(c, "refine_small", k_refine_small, grid_for(G, 256), 256, 0, d_buf, L.starts, L.ends, GS, GE, G, V, uniq, off);
        // big groups -> a radix round on the next chunk
        uint32_t *big;
        SG_TRY(slot(c, S_SEL, G + 16, &big));
        uint32_t B = 0;
        SG_TRY(run_select2(c, "select_big", BigGroupPred{GS, GE}, G, big, (uint32_t *)nullptr, &B, nullptr));
        if (B == 0) break;
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
        SG_LAUNCH(c, "round_expand", k_expand, grid_for(M, 256), 256, 0, d_buf, L.starts, L.ends, GS, big, goff, B, V, M, off, RK, RG, RP);
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
        // GK2 is the key currently holding sorted chunk keys (no longer needed).
        SG_TRY(radix_sort(c, GK, perm, GK2, pv_alt, M, 0, gbits, false, &FKs, &perm2, "rs_pass_refine"));
        // T and FK into the arrays not holding perm2
        T = (perm2 == perm) ? pv_alt : perm;
        uint64_t *FK = (FKs == GK) ? GK2 : GK;
        SG_LAUNCH(c, "round_gather", k_round_gather, grid_for(M, 256), 256, 0, d_buf, L.starts, L.ends, V, RP, perm2, M, off, T, FK);
        SG_LAUNCH(c, "round_scatter", k_round_scatter, grid_for(M, 256), 256, 0, T, RP, M, V);
        // sub-groups: RG is the group index of final row i as well (same row ranges)
        uint32_t *NS = perm2, *NE = T;  // reuse (T consumed by scatter above; perm2 no longer needed)
        // NOTE: NS/NE are written after the scatter kernel on the same stream.
        uint32_t G3 = 0, G4 = 0;
        SG_TRY(run_select2(c, "round_mark", RoundGroupPred{FK, RG, RP, uniq, M}, M, NS, NE, &G3, &G4));
        if (G3 != G4) { set_error("round group mismatch"); return SG_E_HIP; }
        // rows -> global positions into GS/GE
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
    uint32_t U = 0;
};

static int unique_view(sg_ctx *c, const uint8_t *d_buf, uint64_t n, const SlotSet &ss, int ur_slot,
                       int uk_slot, bool trust_sorted, UniqView *uv) {
    SG_TRY(run_lines(c, d_buf, n, ss, &uv->L));
    const uint32_t R = uv->L.n_rec;
    if (trust_sorted && R > 1) {
        uint32_t *flag;
        SG_TRY(slot(c, S_M_CNT, 4, &flag));
        SG_HIP(hipMemsetAsync(flag, 0, 4, c->stream));
        SG_LAUNCH(c, "check_sorted", k_check_sorted, grid_for(R - 1, 256), 256, 0, d_buf, uv->L.starts, uv->L.ends, uv->L.keys, R, flag);
        uint32_t f = 1;
        SG_TRY(ctx_readback(c, &f, flag, 4));
        trust_sorted = (f == 0);
    }
    if (trust_sorted) {
        uv->UR = nullptr;
        uv->UK = uv->L.keys;
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
    if (U) {
        SG_LAUNCH(c, "gather", k_gather_u32, grid_for(U, 256), 256, 0, S.recs, sel, U, uv->UR);
        SG_LAUNCH(c, "gather", k_gather_u64, grid_for(U, 256), 256, 0, S.keys, sel, U, uv->UK);
    }
    uv->U = U;
    return SG_OK;
}

int dev_dedup_diff(sg_ctx *c, const uint8_t *d_cur, uint64_t n_cur, const uint8_t *d_prior,
                   uint64_t n_prior, bool want_fresh, sg_dev_result *res) {
    *res = sg_dev_result{};
    UniqView cu;
    SG_TRY(unique_view(c, d_cur, n_cur, CUR_SLOTS, S_CUR_UR, S_CUR_UK, false, &cu));
    uint32_t *UR = cu.UR;
    uint64_t *UK = cu.UK;
    res->in_records = cu.L.n_rec;
    uint8_t *uout;
    uint64_t ubytes = 0;
    SG_TRY(serialize(c, d_cur, cu.L.starts, cu.L.ends, UR, nullptr, cu.U, S_OUT_UNIQ, &uout, &ubytes));
    res->uniq = uout;
    res->uniq_bytes = ubytes;
    res->uniq_records = cu.U;
    if (!want_fresh) return SG_OK;

    UniqView pv;
    if (d_prior && n_prior) {
        SG_TRY(unique_view(c, d_prior, n_prior, PRIOR_SLOTS, S_P_REC, S_P_SORTED_KEYS, true, &pv));
    }
    res->prior_records = pv.L.n_rec;
    if (pv.U == 0) {
        res->fresh = res->uniq;
        res->fresh_bytes = res->uniq_bytes;
        res->fresh_records = res->uniq_records;
        return SG_OK;
    }
    uint8_t *fresh;
    SG_TRY(slot(c, S_M_TMP, (size_t)cu.U + 1, &fresh));
    if (cu.U) {
        SG_LAUNCH(c, "diff_mark", k_diff_mark, grid_for(cu.U, 256), 256, 0, d_cur, cu.L.starts, cu.L.ends, UR, UK, cu.U,
                  d_prior, pv.L.starts, pv.L.ends, pv.UR, pv.UK, pv.U, fresh);
    }
    uint32_t *fidx;
    SG_TRY(slot(c, S_SEL, (size_t)cu.U + 16, &fidx));
    uint32_t F = 0;
    SG_TRY(select_flags(c, fresh, cu.U, fidx, &F));
    uint32_t *FR;
    SG_TRY(slot(c, S_M_TMP2, (size_t)F + 1, &FR));
    if (F) SG_LAUNCH(c, "gather", k_gather_u32, grid_for(F, 256), 256, 0, UR, fidx, F, FR);
    uint8_t *fout;
    uint64_t fbytes = 0;
    SG_TRY(serialize(c, d_cur, cu.L.starts, cu.L.ends, FR, nullptr, F, S_OUT_FRESH, &fout, &fbytes));
    res->fresh = fout;
    res->fresh_bytes = fbytes;
    res->fresh_records = F;
    return SG_OK;
}

}  // namespace sg
