// EXPERIMENT (not built): the round-2 "probe path" of sg_dedup.hip — a sorted prior scan as
// a segmented hash table, the current records looked up by bytes, only the new ones sorted,
// the unique output merged from two sources. Bit-exact, but measured slower than the radix
// pipeline (C2 2.46 vs 2.10 ms), so it left libswarmgpu.so in round 3. Kept
// verbatim for reference; it depends on sg_dedup.hip internals as of commit 5828609
// (k_diff_tile_t<INS>, run_select2_nb, run_emit, RecSet, OutBuf, UView) and the S_PB_* slots.
// Its GPU tests are tools/experiments/test_gpu_probe.py.
__global__ __launch_bounds__(256) void k_ins_tile(RecSet U, RecSet P, const uint32_t *__restrict__ jb,
                                                  uint32_t *__restrict__ ins, uint32_t base) {
    diff_tile_body<true>(U, P, jb, nullptr, ins, base);
}

// ------------------------------------------------------------------ probe path
// When the prior scan is sorted and duplicate-free (the previous run's sort -u output), the
// current scan's records are looked up in a hash table of the prior instead of sorting all
// of them: a record found there belongs to the output at the prior record's place, so only
// the records NOT in the prior (the new ones, ~10 % on a recurring scan) are sorted. The
// unique output is the prior's found records merged with the sorted new records (each new
// record's insertion point in the prior from the same key0 search the diff uses); the new
// records ARE the diff. Equality is decided by bytes (the hash only picks the candidate).
//
// Table: 2^tb 16-B slots {fp, start, record index, length} (fp 0 = empty) in segments of
// 2^sb slots (sb <= 12: one segment is 64 KB of LDS). A record's segment is the top bits of
// its first hash, its home slot the low sb bits; linear probing wraps inside the segment.
// fp = the second hash's top 20 bits | the home slot (never 0).
// No global atomics: device-scope atomics execute memory-side on MI355X (one CAS per prior
// record took 0.49 ms for 5.7M records, an atomicOr per found record 0.77 ms). Instead the
// prior records are partitioned by segment (count pass with LDS ranks -> scan -> scatter) and
// one block per segment fills its 64 KB of slots with LDS atomics, then writes them out.
constexpr uint32_t PB_SB = 12;           // max log2 slots per segment
constexpr uint32_t PB_THREADS = 1024;    // count/scatter pass block
constexpr uint32_t PB_PER = 16;          // records per thread in the count/scatter passes
constexpr uint32_t PB_BLK = PB_THREADS * PB_PER;
constexpr uint32_t PB_MAXSEG = 16384;    // LDS histogram bound of the count pass

__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
    h ^= h >> 16;
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
    h *= 0xC2B2AE35u;
    h ^= h >> 16;
    return h;
}

// Two 32-bit hashes of the record's bytes (48-byte windows of 16-B loads).
__device__ __forceinline__ uint2 rec_hash(const uint8_t *__restrict__ buf, uint32_t s, uint32_t len) {
    uint32_t h1 = 0x9E3779B9u ^ len, h2 = 0x7F4A7C15u + len * 0x85EBCA77u;
    for (uint32_t o = 0; o < len; o += 48u) {
        const uint32_t cl = (len - o) < 48u ? (len - o) : 48u;
        uint4 c[4];
        load_chunks(buf, s + o, cl, c);
        uint32_t r[13];
        normalize52(c, (s + o) & 15u, r);
#pragma unroll
        for (uint32_t q = 0; q < 12; ++q) {
            if (4u * q < cl) {
                const uint32_t k = cl - 4u * q;
                const uint32_t w = r[q] & (k >= 4u ? ~0u : ((1u << (8u * k)) - 1u));
                h1 = __builtin_rotateleft32(h1 ^ w, 13) * 0x9E3779B1u;
                h2 = (h2 + w) * 0xC2B2AE3Du;
                h2 ^= h2 >> 15;
            }
        }
    }
    return make_uint2(fmix32(h1), fmix32(h2 ^ (h1 >> 7)));
}

// Table geometry: tb = log2 slots, sb = log2 slots per segment; fpm masks the fingerprint
// (tests narrow it so every probe takes the byte compare).
struct PbGeom {
    uint32_t tb, sb, fpm;
    __device__ uint32_t seg(uint32_t hx) const { return tb > sb ? hx >> (32u - (tb - sb)) : 0u; }
    __device__ uint32_t home(uint32_t hx) const { return hx & ((1u << sb) - 1u); }
    __device__ uint32_t fp(uint2 h) const {
        const uint32_t t = h.y & fpm & 0xFFFFF000u;
        return (t ? t : 0x1000u) | home(h.x);
    }
};

// Count pass: per record its hash pair and its rank among the block's records of the same
// segment (LDS atomics); per (segment, block) the count, segment-major for the scan.
__global__ __launch_bounds__(PB_THREADS) void k_pb_count(const uint8_t *__restrict__ P, const uint2 *__restrict__ sp,
                                                          uint32_t n, PbGeom g, uint2 *__restrict__ H,
                                                          uint16_t *__restrict__ rk, uint32_t *__restrict__ cnt,
                                                          uint32_t nblk) {
    extern __shared__ uint32_t s_h[];
    const uint32_t nseg = 1u << (g.tb - g.sb);
    for (uint32_t x = threadIdx.x; x < nseg; x += PB_THREADS) s_h[x] = 0;
    __syncthreads();
    const uint32_t b0 = blockIdx.x * PB_BLK;
#pragma unroll 4
    for (uint32_t r = 0; r < PB_PER; ++r) {
        const uint32_t i = b0 + r * PB_THREADS + threadIdx.x;
        if (i >= n) break;
        const uint2 x = sp[i];
        const uint2 h = rec_hash(P, x.x, x.y - x.x);
        H[i] = h;
        rk[i] = (uint16_t)atomicAdd(&s_h[g.seg(h.x)], 1u);
    }
    __syncthreads();
    for (uint32_t x = threadIdx.x; x < nseg; x += PB_THREADS) cnt[(size_t)x * nblk + blockIdx.x] = s_h[x];
}

struct U32AsU64 {
    const uint32_t *v;
    __device__ uint64_t operator()(uint32_t i) const { return v[i]; }
};

// Scatter pass: record -> its segment's slice of E (order inside a segment is immaterial).
__global__ __launch_bounds__(PB_THREADS) void k_pb_scatter(const uint2 *__restrict__ sp, uint32_t n, PbGeom g,
                                                            const uint2 *__restrict__ H, const uint16_t *__restrict__ rk,
                                                            const uint64_t *__restrict__ off, uint32_t nblk,
                                                            uint4 *__restrict__ E) {
    const uint32_t b0 = blockIdx.x * PB_BLK;
#pragma unroll 4
    for (uint32_t r = 0; r < PB_PER; ++r) {
        const uint32_t i = b0 + r * PB_THREADS + threadIdx.x;
        if (i >= n) break;
        const uint2 h = H[i];
        const uint2 x = sp[i];
        const uint64_t pos = off[(size_t)g.seg(h.x) * nblk + blockIdx.x] + rk[i];
        E[pos] = make_uint4(g.fp(h), x.x, i, x.y - x.x);
    }
}

// Fill pass: one block per segment inserts the segment's records into its LDS slots, then
// writes all 2^sb slots (empty ones as zeros: the table needs no memset). A segment with no
// free slot left sets *err (the caller falls back to the radix pipeline).
__global__ __launch_bounds__(256) void k_pb_fill(const uint4 *__restrict__ E, const uint64_t *__restrict__ off,
                                                 uint32_t nblk, uint32_t n, PbGeom g, uint4 *__restrict__ T,
                                                 uint32_t *__restrict__ err) {
    __shared__ uint32_t s_fp[1u << PB_SB], s_st[1u << PB_SB], s_ix[1u << PB_SB], s_ln[1u << PB_SB];
    const uint32_t S = 1u << g.sb, seg = blockIdx.x, nseg = 1u << (g.tb - g.sb);
    for (uint32_t x = threadIdx.x; x < S; x += 256) s_fp[x] = 0;
    __syncthreads();
    const uint64_t e0 = off[(size_t)seg * nblk];
    const uint64_t e1 = (seg + 1 < nseg) ? off[(size_t)(seg + 1) * nblk] : (uint64_t)n;
    if (e1 - e0 >= S) {
        if (threadIdx.x == 0) *err = 1u;
        return;
    }
    for (uint64_t q = e0 + threadIdx.x; q < e1; q += 256) {
        const uint4 e = E[q];
        uint32_t at = e.x & (S - 1u);
        for (;;) {
            if (atomicCAS(&s_fp[at], 0u, e.x) == 0u) break;
            at = (at + 1u) & (S - 1u);
        }
        s_st[at] = e.y;
        s_ix[at] = e.z;
        s_ln[at] = e.w;
    }
    __syncthreads();
    uint4 *out = T + (size_t)seg * S;
    for (uint32_t x = threadIdx.x; x < S; x += 256)
        out[x] = s_fp[x] ? make_uint4(s_fp[x], s_st[x], s_ix[x], s_ln[x]) : make_uint4(0u, 0u, 0u, 0u);
}

// new[i] = record i of cur is not in the prior; a found prior record j gets pflag[j] = 1
// (plain byte stores: every writer stores the same value).
__global__ __launch_bounds__(256) void k_probe_lookup(const uint8_t *__restrict__ C, const uint2 *__restrict__ csp,
                                                      uint32_t n, const uint8_t *__restrict__ P, PbGeom g,
                                                      const uint4 *__restrict__ T, uint8_t *__restrict__ pflag,
                                                      uint8_t *__restrict__ fresh) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint2 x = csp[i];
    const uint32_t len = x.y - x.x;
    const uint2 h = rec_hash(C, x.x, len);
    const uint32_t fp = g.fp(h), S = 1u << g.sb;
    const uint4 *seg = T + (size_t)g.seg(h.x) * S;
    uint32_t at = g.home(h.x);
    bool found = false;
    for (uint32_t k = 0; k < S; ++k) {  // a segment always keeps a free slot (k_pb_fill)
        const uint4 e = seg[at];
        if (e.x == 0u) break;
        if (e.x == fp && e.w == len && rec_equal_w(C, x.x, x.y, P, e.y, e.y + len, 0u)) {
            found = true;
            pflag[e.z] = 1;
            break;
        }
        at = (at + 1u) & (S - 1u);
    }
    fresh[i] = found ? 0 : 1;
}

__global__ __launch_bounds__(256) void k_gather_sk(const uint32_t *__restrict__ idx, uint32_t n,
                                                   const uint2 *__restrict__ sp, const uint64_t *__restrict__ K,
                                                   uint2 *__restrict__ osp, uint64_t *__restrict__ oK) {
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
        const uint32_t i = idx[k];
        osp[k] = sp[i];
        oK[k] = K[i];
    }
}

// Merged output order: prior record j (kept iff its bit is set) and new record k placed
// right before prior record ins[k] (ins non-decreasing, n_p = after the last), so new record
// k sits at merged position pos(k) = k + ins[k] (strictly increasing). kb[t] = the number
// of new records before merged position t * EM_TILE: one wave per tile boundary, a 64-ary
// search over pos (as k_diff_split).
__global__ __launch_bounds__(256) void k_merge_split(const uint32_t *__restrict__ ins, uint32_t nu, uint32_t nb,
                                                     uint32_t *__restrict__ kb) {
    const uint32_t t = blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t lane = lane_id();
    if (t >= nb) return;
    const uint64_t m0 = (uint64_t)t * EM_TILE;
    uint32_t lo = 0, hi = nu;  // first k with pos(k) >= m0, in [lo, hi]
    while (hi > lo) {
        const uint32_t span = hi - lo;
        if (span <= 64) {
            const uint32_t p = lo + lane;
            const bool ge = (p >= hi) || (uint64_t)p + ins[p] >= m0;
            const uint64_t m = __ballot(ge);
            lo = m ? lo + (uint32_t)(__ffsll((long long)m) - 1) : hi;  // span 64, all below: hi
            break;
        }
        const uint32_t p = lo + (uint32_t)(((uint64_t)span * (lane + 1)) / 65);
        const bool ge = (uint64_t)p + ins[p] >= m0;
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
    if (lane == 0) kb[t] = lo;
}

// One block per EM_TILE merged positions: each position's item (start | source bit, length)
// or a dropped prior record, written as the emit cache, and the tile's (count, bytes) total
// (k_emit_count's job, so the merged output goes straight to the emit apply pass).
constexpr uint32_t MG_PER = EM_TILE / 256;
__global__ __launch_bounds__(256) void k_merge_items(const uint2 *__restrict__ psp, uint32_t np,
                                                     const uint8_t *__restrict__ pflag, const uint2 *__restrict__ usp,
                                                     const uint32_t *__restrict__ ins, const uint32_t *__restrict__ kb,
                                                     uint32_t M, uint2 *__restrict__ cache, uint64_t *__restrict__ tot) {
    __shared__ uint8_t s_take[EM_TILE];
    __shared__ uint32_t s_red[4];
    __shared__ uint64_t s_r64[4];
    const uint32_t t = threadIdx.x, tile = blockIdx.x;
    const uint32_t m0 = tile * EM_TILE;
    const uint32_t k0 = kb[tile], k1 = kb[tile + 1];
    for (uint32_t x = t; x < EM_TILE; x += 256) s_take[x] = 0;
    __syncthreads();
    for (uint32_t k = k0 + t; k < k1; k += 256) s_take[k + ins[k] - m0] = 1;
    __syncthreads();
    // thread t: positions m0 + MG_PER*t .. + MG_PER - 1
    uint32_t tk = 0;
#pragma unroll
    for (uint32_t q = 0; q < MG_PER; ++q) tk += s_take[MG_PER * t + q];
    uint32_t ttot;
    uint32_t before = block_excl_scan<256>(tk, &ttot, s_red);  // new records before my first
    uint64_t sum = 0;
#pragma unroll
    for (uint32_t q = 0; q < MG_PER; ++q) {
        const uint32_t lm = MG_PER * t + q, m = m0 + lm;
        if (m >= M) break;
        uint2 it;
        if (s_take[lm]) {
            const uint2 u = usp[k0 + before];
            it = make_uint2(u.x | 0x80000000u, u.y - u.x);
            ++before;
        } else {
            const uint32_t j = (m0 - k0) + (lm - before);
            const uint2 p = psp[j];
            const bool keep = pflag[j] != 0;
            it = make_uint2(p.x, keep ? p.y - p.x : EM_DROP);
        }
        cache[m] = it;
        sum += (it.y != EM_DROP) ? (EM_ONE | (uint64_t)(it.y + 1u)) : 0ull;
    }
    sum = wave_sum(sum);
    if (lane_id() == 0) s_r64[t >> 6] = sum;
    __syncthreads();
    if (t == 0) tot[tile] = s_r64[0] + s_r64[1] + s_r64[2] + s_r64[3];
}

template <uint32_t WIN>
__global__ __launch_bounds__(EM_BLOCK) void k_emit_merge(const uint2 *__restrict__ cache, uint32_t n,
                                                         const uint64_t *__restrict__ pre, const uint8_t *__restrict__ srcP,
                                                         const uint8_t *__restrict__ srcU, uint8_t *__restrict__ dst) {
    emit_apply_body<true, WIN, true>(cache, n, pre, srcP, srcU, dst, nullptr, nullptr, nullptr, 0);
}


// The probe path (see the kernels above). Lc/Lp: both buffers parsed, keyed with bk (the
// common prefix and key width every later compare uses); the prior is strictly increasing.
// *used = false: the prior does not fit the table's bounds (a segment without a free slot,
// more segments than the count pass's LDS histogram): nothing was changed, the caller runs
// the radix pipeline.
static int probe_dedup_diff(sg_ctx *c, const uint8_t *d_cur, uint64_t n_cur, const Lines &Lc, const uint8_t *d_prior,
                            uint64_t n_prior, const Lines &Lp, uint32_t bk, sg_dev_result *res, const OutBuf *ou,
                            const OutBuf *of, bool *used) {
    *used = false;
    const uint32_t R = Lc.n_rec, NP = Lp.n_rec;
    // table slots per prior record (>= 1.25: a load <= 0.8, so the longest probe runs stay
    // short) and the fingerprint mask: tests shrink both (SG_PROBE_SLOTS, SG_PROBE_FPMASK)
    const char *e_sl = getenv("SG_PROBE_SLOTS"), *e_fp = getenv("SG_PROBE_FPMASK");
    const double load = e_sl ? std::max(1.01, atof(e_sl)) : 1.25;
    PbGeom g;
    g.fpm = e_fp ? (uint32_t)strtoul(e_fp, nullptr, 0) : 0xffffffffu;
    g.tb = 4;
    while ((double)(1ull << g.tb) < load * NP + 1.0) ++g.tb;
    const char *e_sb = getenv("SG_PROBE_SEGBITS");  // tests: tiny segments overflow -> radix
    g.sb = std::min(g.tb, e_sb ? std::max(1u, std::min(PB_SB, (uint32_t)atoi(e_sb))) : PB_SB);
    const uint32_t nseg = 1u << (g.tb - g.sb);
    if (g.tb > 31 || nseg > PB_MAXSEG) return SG_OK;
    const uint32_t nblk = (NP + PB_BLK - 1) / PB_BLK;
    const size_t nc = (size_t)nseg * nblk;
    uint4 *T, *E;
    uint2 *H;
    uint16_t *rk;
    uint32_t *cnt, *err;
    uint64_t *off;
    uint8_t *pflag, *nf;
    SG_TRY(slot(c, S_PB_TAB, (size_t)1 << g.tb, &T));
    SG_TRY(slot(c, S_PB_E, NP, &E));
    SG_TRY(slot(c, S_PB_H, NP, &H));
    SG_TRY(slot(c, S_PB_RK, NP, &rk));
    SG_TRY(slot(c, S_PB_CNT, nc, &cnt));
    SG_TRY(slot(c, S_PB_OFF, nc, &off));
    SG_TRY(slot(c, S_PB_ERR, 1, &err));
    SG_TRY(slot(c, S_PB_BITS, NP, &pflag));
    SG_TRY(slot(c, S_PB_NEW, R, &nf));
    SG_HIP(hipMemsetAsync(err, 0, 4, c->stream));
    SG_HIP(hipMemsetAsync(pflag, 0, NP, c->stream));
    // model: prior records + spans read, hash pair + rank written
    SG_LAUNCH_B(c, "probe_count", (double)n_prior + 18.0 * NP, k_pb_count, nblk, PB_THREADS, nseg * 4, d_prior, Lp.spans,
                NP, g, H, rk, cnt, nblk);
    {
        const uint32_t nt = (uint32_t)((nc + SCAN_TILE - 1) / SCAN_TILE);
        uint64_t *tp;
        SG_TRY(slot(c, S_TILES, 2 * (size_t)nt + 4, &tp));
        SG_LAUNCH(c, "scan.count", k_scan64_count<U32AsU64>, nt, SCAN_BLOCK, 0, U32AsU64{cnt}, (uint32_t)nc, tp);
        SG_TRY(tile_scan(c, tp, nt, tp + nt, tp + 2 * (size_t)nt));
        SG_LAUNCH(c, "scan.apply", k_scan64_apply<U32AsU64>, nt, SCAN_BLOCK, 0, U32AsU64{cnt}, (uint32_t)nc, tp + nt, off);
    }
    // model: hash pair + rank + span read, one 16-B entry written
    SG_LAUNCH_B(c, "probe_scatter", 34.0 * NP, k_pb_scatter, nblk, PB_THREADS, 0, Lp.spans, NP, g, H, rk, off, nblk, E);
    // model: entries read, the whole table written
    SG_LAUNCH_B(c, "probe_fill", 16.0 * NP + 16.0 * (double)(1ull << g.tb), k_pb_fill, nseg, 256, 0, E, off, nblk, NP, g, T,
                err);
    // model: cur records + spans read, a 16-B slot and the prior record per found record, a flag
    SG_LAUNCH_B(c, "probe_lookup", (double)n_cur + 25.0 * R, k_probe_lookup, grid_for(R, 256), 256, 0, d_cur, Lc.spans, R,
                d_prior, g, T, pflag, nf);
    // the new records (not in the prior): their count comes back with the table's error word
    uint32_t *idx;
    SG_TRY(slot(c, S_PB_IDX, R, &idx));
    uint64_t *stot;
    SG_TRY(run_select2_nb(c, "probe_select", FlagPred{nf}, R, idx, nullptr, S_PB_STAT, &stot));
    uint32_t nn = 0;
    {
        uint8_t *pin = (uint8_t *)c->pinned;
        SG_HIP(hipMemcpyAsync(pin, stot, 8, hipMemcpyDeviceToHost, c->stream));
        SG_HIP(hipMemcpyAsync(pin + 8, err, 4, hipMemcpyDeviceToHost, c->stream));
        SG_HIP(hipStreamSynchronize(c->stream));
        uint64_t tv = 0;
        uint32_t ev = 0;
        memcpy(&tv, pin, 8);
        memcpy(&ev, pin + 8, 4);
        if (ev) return SG_OK;  // a full segment: the radix pipeline instead
        nn = (uint32_t)(tv >> 31);
    }
    *used = true;
    // the new records, sorted and deduplicated: the fresh output (into the caller's buffer)
    OutBuf fo;
    if (of) {
        fo = *of;
    } else {
        uint8_t *fb;
        SG_TRY(slot(c, S_OUT_FRESH, (size_t)n_cur + 64, &fb));
        fo = OutBuf{fb, (size_t)n_cur + 64};
    }
    UView nu;
    nu.buf = fo.base();
    if (nn) {
        Lines Ls;
        SG_TRY(slot(c, S_PB_SP, nn, &Ls.spans));
        SG_TRY(slot(c, S_PB_K, nn, &Ls.keys));
        Ls.n_rec = nn;
        SG_LAUNCH_B(c, "probe_gather", 20.0 * nn, k_gather_sk, grid_for(nn, 256, 4096), 256, 0, idx, nn, Lc.spans, Lc.keys,
                    Ls.spans, Ls.keys);
        SG_TRY(build_unique(c, d_cur, n_cur, CUR_VIEW, false, &nu, &Ls, bk, &fo, nullptr));
    }
    if ((uint64_t)nu.bytes + 16 >= (1ull << 31)) { set_error("probe: new records exceed 2 GiB"); return SG_E_TOO_LARGE; }
    // each new record's insertion point in the prior
    uint32_t *ins;
    SG_TRY(slot(c, S_PB_INS, (size_t)nu.n + 1, &ins));
    if (nu.n) {
        const uint32_t ntiles = (nu.n + DF_TILE - 1) / DF_TILE;
        uint32_t *jb;
        SG_TRY(slot(c, S_R_OFF, (size_t)ntiles + 2, &jb));
        SG_LAUNCH(c, "diff_split", k_diff_split, grid_for(ntiles + 1, 4), 256, 0, nu.keys, nu.n, Lp.keys, NP, ntiles + 1, jb);
        RecSet U{nu.buf, nu.spans, nu.keys, nu.n};
        RecSet P{d_prior, Lp.spans, Lp.keys, NP};
        SG_LAUNCH_B(c, "ins_tile", 16.0 * nu.n + 8.0 * NP, k_ins_tile, ntiles, 256, 0, U, P, jb, ins, bk);
    }
    // the merged unique output
    const uint32_t M = NP + nu.n;
    const uint32_t mt = (M + EM_TILE - 1) / EM_TILE;
    uint32_t *kb;
    SG_TRY(slot(c, S_PB_KB, (size_t)mt + 2, &kb));
    SG_LAUNCH(c, "merge_split", k_merge_split, grid_for(mt + 1, 4), 256, 0, ins, nu.n, mt + 1, kb);
    uint2 *cache;
    SG_TRY(slot(c, S_PB_MI, (size_t)M + 1, &cache));
    uint64_t *tp;
    SG_TRY(slot(c, S_PB_STAT, 2 * (size_t)mt + 4, &tp));
    uint64_t *tot = tp, *pre = tp + mt, *total = tp + 2 * (size_t)mt;
    SG_LAUNCH_B(c, "merge_items", 13.0 * M, k_merge_items, mt, 256, 0, Lp.spans, NP, pflag, nu.spans, ins, kb, M,
                cache, tot);
    SG_TRY(tile_scan(c, tot, mt, pre, total, ou ? ou->shift() : 0u));
    uint8_t *ub;
    if (ou) ub = ou->base();
    else SG_TRY(slot(c, S_OUT_UNIQ, (size_t)n_cur + 64, &ub));
    const bool shortr = n_prior <= 40ull * NP;
    if (shortr)
        SG_LAUNCH(c, "emit_merge", k_emit_merge<EM_WIN_S>, mt, EM_BLOCK, 0, cache, M, pre, d_prior, nu.buf, ub);
    else
        SG_LAUNCH(c, "emit_merge", k_emit_merge<EM_WIN>, mt, EM_BLOCK, 0, cache, M, pre, d_prior, nu.buf, ub);
    uint64_t tt = 0;
    SG_TRY(ctx_readback(c, &tt, total, 8));
    if (c->profile) prof_bytes(c, "emit_merge", 8.0 * M + 2.0 * (double)(uint32_t)tt);
    res->in_records = R;
    res->uniq = ou ? ou->p : ub;
    res->uniq_bytes = (uint32_t)tt;
    res->uniq_records = (uint32_t)(tt >> 32);
    res->prior_records = NP;
    res->fresh = of ? of->p : fo.base();
    res->fresh_bytes = nu.bytes;
    res->fresh_records = nu.n;
    c->last_path = SG_PATH_PROBE;
    return SG_OK;
}
