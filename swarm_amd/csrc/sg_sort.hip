// sg_sort.hip — stable LSD radix sort of (u64 key, u32 value) pairs, onesweep style.
//
// One histogram kernel reads the keys once and counts all 8-bit digit positions; each
// pass is then ONE kernel: a tile of 4096 pairs is ranked per wave64 with 8 ballots per
// item (wave-local match of the digit), the tile's 256 digit counts are published to a
// per-(tile, digit) look-back granule, and the pairs are re-ordered through LDS so the
// global writes of each digit run are contiguous. Passes whose digit is identical for
// every key are skipped. Algorithmic bytes per pass: 12 B read + 12 B written per pair.
#include "sg_internal.hpp"

namespace sg {

constexpr int RS_BLOCK = 256;
constexpr int RS_ITEMS = 16;
constexpr int RS_TILE = RS_BLOCK * RS_ITEMS;
constexpr int RS_WAVES = RS_BLOCK / 64;
constexpr int RS_MAXPASS = 8;

__global__ __launch_bounds__(256) void k_rs_hist(const uint64_t *__restrict__ keys, uint32_t n,
                                                 int begin_bit, int npasses, uint32_t *hist) {
    __shared__ uint32_t h[RS_MAXPASS][256];
    for (int i = threadIdx.x; i < RS_MAXPASS * 256; i += 256) (&h[0][0])[i] = 0;
    __syncthreads();
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        const uint64_t k = keys[i];
        for (int p = 0; p < npasses; ++p) atomicAdd(&h[p][(k >> (begin_bit + 8 * p)) & 255u], 1u);
    }
    __syncthreads();
    for (int p = 0; p < npasses; ++p) {
        uint32_t v = h[p][threadIdx.x];
        if (v) atomicAdd(&hist[p * 256 + threadIdx.x], v);
    }
}

// One block per pass: exclusive digit offsets, and trivial[p] = 1 if one digit holds all.
__global__ __launch_bounds__(256) void k_rs_scan(const uint32_t *hist, uint32_t *offs, uint32_t *trivial,
                                                 uint32_t n) {
    __shared__ uint32_t s_red[4];
    const int p = blockIdx.x;
    const uint32_t v = hist[p * 256 + threadIdx.x];
    uint32_t total;
    const uint32_t ex = block_excl_scan<256>(v, &total, s_red);
    offs[p * 256 + threadIdx.x] = ex;
    const int all = __syncthreads_or(v == n);
    if (threadIdx.x == 0) trivial[p] = all ? 1u : 0u;
}

__global__ void k_iota(uint32_t *v, uint32_t n) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) v[i] = i;
}

template <bool IOTA>
__global__ __launch_bounds__(RS_BLOCK) void k_rs_pass(const uint64_t *__restrict__ kin,
                                                      const uint32_t *__restrict__ vin,
                                                      uint64_t *__restrict__ kout,
                                                      uint32_t *__restrict__ vout, uint32_t n,
                                                      int shift, const uint32_t *__restrict__ goffs,
                                                      uint64_t *status, uint32_t *counter) {
    __shared__ uint64_t s_k[RS_TILE];  // keys, then (aliased) values
    uint32_t *s_v = reinterpret_cast<uint32_t *>(s_k);
    __shared__ uint32_t s_wh[RS_WAVES][256];
    __shared__ uint32_t s_dstart[256];
    __shared__ uint32_t s_gbase[256];
    __shared__ uint32_t s_red[RS_WAVES];
    __shared__ uint32_t s_tile;

    const int tid = threadIdx.x, lane = lane_id(), wid = tid >> 6;
#pragma unroll
    for (int w = 0; w < RS_WAVES; ++w) s_wh[w][tid] = 0;
    const uint32_t tile = take_ticket(counter, &s_tile);  // includes a barrier
    const uint32_t tbase = tile * RS_TILE;
    const uint32_t wbase = tbase + wid * (RS_ITEMS * 64);
    const uint64_t lt_mask = (1ull << lane) - 1ull;

    uint64_t k[RS_ITEMS];
    uint32_t v[RS_ITEMS];
    uint32_t r[RS_ITEMS];
#pragma unroll
    for (int i = 0; i < RS_ITEMS; ++i) {
        const uint32_t pos = wbase + i * 64 + lane;
        const bool valid = pos < n;
        k[i] = valid ? kin[pos] : ~0ull;
        v[i] = IOTA ? pos : (valid ? vin[pos] : 0u);
    }
#pragma unroll
    for (int i = 0; i < RS_ITEMS; ++i) {
        const bool valid = (wbase + i * 64 + lane) < n;
        const uint32_t d = (uint32_t)(k[i] >> shift) & 255u;
        uint64_t m = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const uint64_t bb = __ballot((d >> b) & 1u);
            m &= ((d >> b) & 1u) ? bb : ~bb;
        }
        const uint32_t lt = __popcll(m & lt_mask);
        const uint32_t cnt = s_wh[wid][d];
        r[i] = cnt + lt;
        if (valid && lt == 0) s_wh[wid][d] = cnt + (uint32_t)__popcll(m);
    }
    __syncthreads();

    // thread tid owns digit tid
    uint32_t c[RS_WAVES];
    uint32_t tot_d = 0;
#pragma unroll
    for (int w = 0; w < RS_WAVES; ++w) { c[w] = s_wh[w][tid]; tot_d += c[w]; }
    uint32_t run = 0;
#pragma unroll
    for (int w = 0; w < RS_WAVES; ++w) { s_wh[w][tid] = run; run += c[w]; }
    uint32_t blk_total;
    const uint32_t dstart = block_excl_scan<RS_BLOCK>(tot_d, &blk_total, s_red);
    s_dstart[tid] = dstart;

    uint64_t excl = 0;
    uint64_t *st = status + (uint64_t)tile * 256 + tid;
    if (tile == 0) {
        lb_store(st, LB_FLAG_INC, tot_d);
    } else {
        lb_store(st, LB_FLAG_AGG, tot_d);
        const uint64_t *q = st - 256;
        uint32_t spins = 0;
        while (true) {
            const uint64_t s = lb_load(q);
            const uint32_t f = (uint32_t)(s >> 62);
            if (f == 0) {
                if (++spins > 32) __builtin_amdgcn_s_sleep(1);
                continue;
            }
            excl += s & LB_VAL_MASK;
            if (f == LB_FLAG_INC) break;
            q -= 256;
        }
        lb_store(st, LB_FLAG_INC, excl + tot_d);
    }
    s_gbase[tid] = goffs[tid] + (uint32_t)excl - dstart;
    __syncthreads();

    // block-local destination of each item; keys then values go through LDS so the
    // global writes of each digit run are contiguous
    uint32_t dst[RS_ITEMS];
#pragma unroll
    for (int i = 0; i < RS_ITEMS; ++i) {
        const bool valid = (wbase + i * 64 + lane) < n;
        const uint32_t d = (uint32_t)(k[i] >> shift) & 255u;
        dst[i] = valid ? s_dstart[d] + s_wh[wid][d] + r[i] : 0xffffffffu;
        if (valid) s_k[dst[i]] = k[i];
    }
    __syncthreads();
    const uint32_t tile_n = (n - tbase) < (uint32_t)RS_TILE ? (n - tbase) : (uint32_t)RS_TILE;
    uint32_t g[RS_ITEMS];
#pragma unroll
    for (int j = 0; j < RS_ITEMS; ++j) {
        const uint32_t p = j * RS_BLOCK + tid;
        g[j] = 0xffffffffu;
        if (p < tile_n) {
            const uint64_t kk = s_k[p];
            const uint32_t d = (uint32_t)(kk >> shift) & 255u;
            g[j] = s_gbase[d] + p;
            kout[g[j]] = kk;
        }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < RS_ITEMS; ++i)
        if (dst[i] != 0xffffffffu) s_v[dst[i]] = v[i];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < RS_ITEMS; ++j)
        if (g[j] != 0xffffffffu) vout[g[j]] = s_v[j * RS_BLOCK + tid];
}

int radix_sort(sg_ctx *c, uint64_t *keys, uint32_t *vals, uint64_t *keys_alt, uint32_t *vals_alt,
               uint32_t n, int begin_bit, int end_bit, bool iota_vals, uint64_t **keys_out,
               uint32_t **vals_out, const char *pass_name) {
    *keys_out = keys;
    *vals_out = vals;
    if (n == 0) return SG_OK;
    const int npasses = (end_bit - begin_bit + 7) / 8;
    if (npasses <= 0 || npasses > RS_MAXPASS) { set_error("radix_sort: bad bit range"); return SG_E_INVAL; }
    uint32_t *hist;
    SG_TRY(slot(c, S_HIST, RS_MAXPASS * 256 * 2 + RS_MAXPASS, &hist));
    uint32_t *offs = hist + RS_MAXPASS * 256;
    uint32_t *triv = offs + RS_MAXPASS * 256;
    SG_HIP(hipMemsetAsync(hist, 0, RS_MAXPASS * 256 * 4, c->stream));
    uint32_t hgrid = (n + 256 * 16 - 1) / (256 * 16);
    if (hgrid > 2048) hgrid = 2048;
    SG_LAUNCH_B(c, "rs_hist", 8.0 * n, k_rs_hist, hgrid, 256, 0, keys, n, begin_bit, npasses, hist);
    SG_LAUNCH(c, "rs_scan", k_rs_scan, npasses, 256, 0, hist, offs, triv, n);
    uint32_t trivial[RS_MAXPASS];
    SG_TRY(ctx_readback(c, trivial, triv, npasses * 4));

    const uint32_t ntiles = (n + RS_TILE - 1) / RS_TILE;
    uint64_t *status;
    SG_TRY(slot(c, S_RS_STATUS, (size_t)ntiles * 256 + 8, &status));
    uint32_t *counter = reinterpret_cast<uint32_t *>(status + (size_t)ntiles * 256);

    uint64_t *ck = keys, *ak = keys_alt;
    uint32_t *cv = vals, *av = vals_alt;
    bool iota_pending = iota_vals;
    for (int p = 0; p < npasses; ++p) {
        if (trivial[p]) continue;
        SG_HIP(hipMemsetAsync(status, 0, ((size_t)ntiles * 256 + 8) * 8, c->stream));
        const int shift = begin_bit + 8 * p;
        if (iota_pending) {
            SG_LAUNCH(c, pass_name, k_rs_pass<true>, ntiles, RS_BLOCK, 0, ck, cv, ak, av, n, shift,
                      offs + p * 256, status, counter);
        } else {
            SG_LAUNCH(c, pass_name, k_rs_pass<false>, ntiles, RS_BLOCK, 0, ck, cv, ak, av, n, shift,
                      offs + p * 256, status, counter);
        }
        // 12 B read (8 B key + 4 B value; 8 B with implied iota values) + 12 B written per pair
        prof_bytes(c, pass_name, (iota_pending ? 20.0 : 24.0) * n);
        iota_pending = false;
        uint64_t *tk = ck; ck = ak; ak = tk;
        uint32_t *tv = cv; cv = av; av = tv;
    }
    if (iota_pending) {
        uint32_t g = (n + 255) / 256;
        if (g > 4096) g = 4096;
        SG_LAUNCH(c, "iota", k_iota, g, 256, 0, cv, n);
    }
    *keys_out = ck;
    *vals_out = cv;
    return SG_OK;
}

}  // namespace sg
