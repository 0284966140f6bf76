// sg_sort.hip — stable LSD radix sort of (u64 key, u32 value) pairs (see below).
//
// Design and measurements: the block comment at the top of namespace sg below.
#include "sg_internal.hpp"
#include "sg_prims_host.hpp"

#include <stdlib.h>

#include <cmath>

namespace sg {

// sg_sort: stable LSD radix sort of (u64 key, u32 value) pairs, reduce-then-scan.
//
//   k_rs_hist  : all 8 digit histograms in ONE read of the keys (per-wave LDS histograms,
//                a wave whose lanes share a digit adds once) -> per-pass digit bases and
//                "trivial" passes (one digit holds every key) that are skipped. A caller
//                that knows the keys' varying bits (KeyStats: the dedup gathers them while
//                it reads the keys anyway) skips this pass and its read-back: each pass's
//                digit bases then come from its own tile counts (k_rs_dsum).
//   per pass   : k_rs_up    per-tile digit counts (per-wave LDS histograms)
//                k_rs_cscan per digit, exclusive over tiles + the digit base
//                k_rs_down  rank in tile (wave64 8-ballot digit match, stable), keys then
//                           values staged through one LDS buffer so each digit run is
//                           written contiguously
// No inter-block waits (a single-pass look-back over 4096-item tiles waited cross-XCD
// round trips per tile on MI355X: 88 µs/pass vs 55 µs for this downsweep at 10M pairs).
// Algorithmic bytes per pass: 8 B key + the value read and written per pair (the dedup
// carries the 8-B span: 16 B read + 16 B written; iota ids: 12 B written).

constexpr int RS_MAXPASS = 8;

// The dedup's key narrowing (sg_dedup.hip k_narrow_keys), applied while the first live pass
// reads the keys (kw 0: none): bytes kw..6 cleared, the tag clamped to kw + 1.
__device__ __forceinline__ uint64_t rs_narrow(uint64_t k, uint32_t kw) {
    if (!kw) return k;
    const uint64_t top = ~0ull << (64u - 8u * kw);
    const uint64_t t = k & 0xffu;
    return (k & top) | (t < kw + 1u ? t : (uint64_t)(kw + 1u));
}
constexpr int RS_HBLOCK = 256;

__global__ __launch_bounds__(RS_HBLOCK) void k_rs_hist(const uint64_t *__restrict__ keys, uint32_t n,
                                                       int begin_bit, int npasses, uint32_t *hist, uint32_t kw) {
    __shared__ uint32_t h[RS_HBLOCK / 64][RS_MAXPASS][256];
    for (int i = threadIdx.x; i < (RS_HBLOCK / 64) * RS_MAXPASS * 256; i += RS_HBLOCK) (&h[0][0][0])[i] = 0;
    __syncthreads();
    const int wid = threadIdx.x >> 6;
    constexpr int HU = 4;
    const uint32_t stride = gridDim.x * RS_HBLOCK * HU;
    for (uint32_t i0 = blockIdx.x * RS_HBLOCK * HU; i0 < n; i0 += stride) {
        uint64_t k[HU];
#pragma unroll
        for (int u = 0; u < HU; ++u) {
            const uint32_t i = i0 + u * RS_HBLOCK + threadIdx.x;
            k[u] = (i < n) ? rs_narrow(keys[i], kw) : 0ull;
        }
#pragma unroll
        for (int u = 0; u < HU; ++u) {
            const bool valid = i0 + u * RS_HBLOCK + threadIdx.x < n;
            const uint32_t cnt = (uint32_t)__popcll(__ballot(valid));
            const uint64_t kk = k[u] >> begin_bit;
#pragma unroll
            for (int p = 0; p < RS_MAXPASS; ++p) {
                if (p >= npasses) break;
                const uint32_t d = (uint32_t)(kk >> (8 * p)) & 255u;
                const uint32_t d0 = wave_bcast(d, 0);
                if (__all(!valid || d == d0)) {
                    if (lane_id() == 0 && cnt) h[wid][p][d0] += cnt;
                } else if (valid) {
                    atomicAdd(&h[wid][p][d], 1u);
                }
            }
        }
    }
    __syncthreads();
    for (int x = threadIdx.x; x < npasses * 256; x += RS_HBLOCK) {
        uint32_t v = 0;
#pragma unroll
        for (int w = 0; w < RS_HBLOCK / 64; ++w) v += (&h[w][0][0])[x];
        if (v) atomicAdd(&hist[x], v);
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

// Digit histograms of a sample of the keys: the 64-key rows r with r % rstride == 0, one
// wave per row (8 waves per block). Planning only (key width, hybrid split): the counts
// are not the sort's offsets.
__global__ __launch_bounds__(512) void k_key_sample(const uint64_t *__restrict__ keys, uint32_t n, uint32_t rstride,
                                                    uint32_t *__restrict__ hist, const KeyStatD *__restrict__ parts,
                                                    uint32_t nparts, KeyStatD *__restrict__ st) {
    __shared__ uint32_t h[8][256];
    if (parts && blockIdx.x == 0) {  // combine the KeyStatD partials (512 threads, 8 waves)
        __shared__ KeyStatD s_p[8];
        uint64_t o = 0, a = ~0ull;
        uint32_t tmin = 255u, tmax = 0u;
        for (uint32_t b = threadIdx.x; b < nparts; b += 512) {
            const KeyStatD q = parts[b];
            o |= q.o;
            a &= q.a;
            tmin = min(tmin, q.tmin);
            tmax = max(tmax, q.tmax);
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            o |= (uint64_t)__shfl_xor((long long)o, off, 64);
            a &= (uint64_t)__shfl_xor((long long)a, off, 64);
            tmin = min(tmin, (uint32_t)__shfl_xor((int)tmin, off, 64));
            tmax = max(tmax, (uint32_t)__shfl_xor((int)tmax, off, 64));
        }
        if (lane_id() == 0) s_p[threadIdx.x >> 6] = KeyStatD{o, a, tmin, tmax};
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int w = 1; w < 8; ++w) {
                o |= s_p[w].o;
                a &= s_p[w].a;
                tmin = min(tmin, s_p[w].tmin);
                tmax = max(tmax, s_p[w].tmax);
            }
            *st = KeyStatD{o, a, tmin, tmax};
        }
    }
    for (int x = threadIdx.x; x < 8 * 256; x += 512) (&h[0][0])[x] = 0;
    __syncthreads();
    const uint32_t nrows = (n + 63) / 64;
    constexpr int KS_U = 8;  // rows in flight per wave (the loads are independent)
    const uint32_t jstep = gridDim.x * 8;
    for (uint32_t j0 = blockIdx.x * 8 + (threadIdx.x >> 6); (uint64_t)j0 * rstride < nrows; j0 += jstep * KS_U) {
        uint64_t k[KS_U];
        bool ok[KS_U];
#pragma unroll
        for (int u = 0; u < KS_U; ++u) {
            const uint64_t i = ((uint64_t)(j0 + u * jstep) * rstride) * 64 + lane_id();
            ok[u] = i < n;
            k[u] = ok[u] ? keys[i] : 0ull;
        }
#pragma unroll
        for (int u = 0; u < KS_U; ++u)
            if (ok[u]) {
#pragma unroll
                for (int p = 0; p < 8; ++p) atomicAdd(&h[p][(uint32_t)(k[u] >> (8 * p)) & 255u], 1u);
            }
    }
    __syncthreads();
    for (int x = threadIdx.x; x < 8 * 256; x += 512) {
        const uint32_t v = (&h[0][0])[x];
        if (v) atomicAdd(&hist[x], v);
    }
}

__global__ void k_iota(uint32_t *v, uint32_t n) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) v[i] = i;
}

// XCD-aware tile order: blocks are dispatched round-robin over the 8 XCDs (block b on XCD
// b % 8), so block b takes tile (b % 8) * per + b / 8 — each XCD works a contiguous eighth of
// the tiles, and the per-tile digit counts of 16 neighbouring tiles (one 64-B line of a
// digit's row) are written through one L2 instead of eight partial lines in eight L2s.
__device__ __forceinline__ uint32_t rs_tile_of(uint32_t b, uint32_t ntiles) {
    const uint32_t per = (ntiles + 7u) / 8u;
    return (b & 7u) * per + (b >> 3);
}

#ifndef SG_RD_BLOCK
#define SG_RD_BLOCK 512
#endif
constexpr int RD_BLOCK = SG_RD_BLOCK;  // 256 or 512 threads per 4096-pair tile (digit owners: tid < 256)
constexpr int RD_ITEMS = 4096 / RD_BLOCK;
constexpr int RD_TILE = RD_BLOCK * RD_ITEMS;
constexpr int RD_WAVES = RD_BLOCK / 64;

// Tile digit counts -> cnt[d * ntiles + tile]: per-wave LDS histograms (atomics), a
// wave-row whose lanes share one digit adds once (skewed digits: '.' or 't' at fixed
// positions of host names).
__global__ __launch_bounds__(RD_BLOCK) void k_rs_up(const uint64_t *__restrict__ keys, uint32_t n, int shift,
                                                    uint32_t ntiles, uint32_t *__restrict__ cnt, uint32_t kw, bool xcd) {
    __shared__ uint32_t h[RD_WAVES][256];
    const int wid = threadIdx.x >> 6;
    const uint32_t tile = xcd ? rs_tile_of(blockIdx.x, ntiles) : blockIdx.x;
    if (tile >= ntiles) return;
    for (int x = threadIdx.x; x < RD_WAVES * 256; x += RD_BLOCK) (&h[0][0])[x] = 0;
    __syncthreads();
    const uint32_t wbase = tile * RD_TILE + wid * (RD_ITEMS * 64);
    uint32_t dd[RD_ITEMS];
#pragma unroll
    for (int i = 0; i < RD_ITEMS; ++i) {
        const uint32_t pos = wbase + i * 64 + lane_id();
        dd[i] = (pos < n) ? ((uint32_t)(rs_narrow(keys[pos], kw) >> shift) & 255u) : 256u;
    }
#pragma unroll
    for (int i = 0; i < RD_ITEMS; ++i) {
        const uint32_t d = dd[i];
        const uint32_t d0 = wave_bcast(d, 0);
        if (__all(d == d0 || d == 256u)) {
            const uint32_t cnt = (uint32_t)__popcll(__ballot(d < 256u));
            if (lane_id() == 0 && d0 < 256u) h[wid][d0] += cnt;
        } else if (d < 256u) {
            atomicAdd(&h[wid][d], 1u);
        }
    }
    __syncthreads();
    if (threadIdx.x < 256) {
        uint32_t v = 0;
#pragma unroll
        for (int w = 0; w < RD_WAVES; ++w) v += h[w][threadIdx.x];
        cnt[(size_t)threadIdx.x * ntiles + tile] = v;
    }
}

// k_rs_up from the digit bytes the previous pass's downsweep wrote beside the keys (dig[i] =
// the digit of the pair now at position i): 1 B read per pair instead of the 8-B key. Eight
// consecutive digits per thread (one 8-B load), per-wave LDS histograms.
__global__ __launch_bounds__(RD_BLOCK) void k_rs_up8(const uint8_t *__restrict__ dig, uint32_t n, uint32_t ntiles,
                                                     uint32_t *__restrict__ cnt, bool xcd) {
    static_assert(RD_ITEMS == 8, "eight digits per thread");
    __shared__ uint32_t h[RD_WAVES][256];
    const int wid = threadIdx.x >> 6;
    const uint32_t tile = xcd ? rs_tile_of(blockIdx.x, ntiles) : blockIdx.x;
    if (tile >= ntiles) return;
    for (int x = threadIdx.x; x < RD_WAVES * 256; x += RD_BLOCK) (&h[0][0])[x] = 0;
    __syncthreads();
    const uint32_t base = tile * RD_TILE + threadIdx.x * 8u;
    uint64_t w = 0;
    uint32_t m = 0;
    if (base + 8u <= n) {
        w = *reinterpret_cast<const uint64_t *>(dig + base);
        m = 8u;
    } else if (base < n) {
        m = n - base;
        for (uint32_t j = 0; j < m; ++j) w |= (uint64_t)dig[base + j] << (8u * j);
    }
#pragma unroll
    for (uint32_t j = 0; j < 8u; ++j)
        if (j < m) atomicAdd(&h[wid][(uint32_t)(w >> (8u * j)) & 255u], 1u);
    __syncthreads();
    if (threadIdx.x < 256) {
        uint32_t v = 0;
#pragma unroll
        for (int ww = 0; ww < RD_WAVES; ++ww) v += h[ww][threadIdx.x];
        cnt[(size_t)threadIdx.x * ntiles + tile] = v;
    }
}

// One block per digit d: the digit's total over the tiles (the pass's digit bases without a
// key histogram: KeyStats sorts).
__global__ __launch_bounds__(256) void k_rs_dsum(const uint32_t *__restrict__ cnt, uint32_t ntiles,
                                                 uint32_t *__restrict__ dtot) {
    __shared__ uint32_t s_red[4];
    const uint32_t *row = cnt + (size_t)blockIdx.x * ntiles;
    uint32_t v = 0;
    for (uint32_t i = threadIdx.x; i < ntiles; i += 256) v += row[i];
    uint32_t tot;
    block_excl_scan<256>(v, &tot, s_red);
    if (threadIdx.x == 0) dtot[blockIdx.x] = tot;
}

// One block per digit d: cnt[d][t] -> exclusive prefix over tiles + the digit base (goffs[d],
// or with dtot the sum of the digit totals below d).
__global__ __launch_bounds__(256) void k_rs_cscan(uint32_t *__restrict__ cnt, uint32_t ntiles,
                                                  const uint32_t *__restrict__ goffs,
                                                  const uint32_t *__restrict__ dtot) {
    __shared__ uint32_t s_red[4];
    __shared__ uint32_t s_base;
    const uint32_t d = blockIdx.x;
    uint32_t *row = cnt + (size_t)d * ntiles;
    uint32_t carry;
    if (dtot) {
        uint32_t tot;
        const uint32_t ex = block_excl_scan<256>(dtot[threadIdx.x], &tot, s_red);
        if (threadIdx.x == d) s_base = ex;
        __syncthreads();
        carry = s_base;
    } else {
        carry = goffs[d];
    }
    for (uint32_t b = 0; b < ntiles; b += 256 * 4) {
        const uint32_t i0 = b + threadIdx.x * 4;
        uint32_t v[4], sum = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) { v[j] = (i0 + j < ntiles) ? row[i0 + j] : 0u; sum += v[j]; }
        uint32_t tot;
        const uint32_t ex = block_excl_scan<256>(sum, &tot, s_red);
        uint32_t run = carry + ex;
#pragma unroll
        for (int j = 0; j < 4; ++j) { if (i0 + j < ntiles) row[i0 + j] = run; run += v[j]; }
        carry += tot;
    }
}

// VT: u32 record ids (IOTA: generated on the first pass) or uint2 spans carried along, so
// the sorted spans need no gather afterwards (sg_dedup.hip build_unique).
// dnext (optional): each pair's digit for the next pass (at shift_next), written beside its
// key at its output position, so the next pass's tile counts read 1 B per pair (k_rs_up8).
template <bool IOTA, typename VT = uint32_t>
__global__ __launch_bounds__(RD_BLOCK) void k_rs_down(const uint64_t *__restrict__ kin,
                                                      const VT *__restrict__ vin,
                                                      uint64_t *__restrict__ kout, VT *__restrict__ vout,
                                                      uint32_t n, int shift, uint32_t ntiles,
                                                      const uint32_t *__restrict__ toffs, uint32_t kw, bool xcd,
                                                      uint8_t *__restrict__ dnext, int shift_next) {
    static_assert(sizeof(VT) <= sizeof(uint64_t), "values staged in the key buffer");
    __shared__ uint64_t s_k[RD_TILE];  // keys, then (aliased) values
    VT *s_v = reinterpret_cast<VT *>(s_k);
    __shared__ uint32_t s_wh[RD_WAVES][256];
    __shared__ uint32_t s_dstart[256];
    __shared__ uint32_t s_gbase[256];
    __shared__ uint32_t s_red[RD_WAVES];

    const int tid = threadIdx.x, lane = lane_id(), wid = tid >> 6;
    for (int x = tid; x < RD_WAVES * 256; x += RD_BLOCK) (&s_wh[0][0])[x] = 0;
    __syncthreads();
    const uint32_t tile = xcd ? rs_tile_of(blockIdx.x, ntiles) : blockIdx.x;
    if (tile >= ntiles) return;
    const uint32_t tbase = tile * RD_TILE;
    const uint32_t wbase = tbase + wid * (RD_ITEMS * 64);
    const uint64_t lt_mask = (1ull << lane) - 1ull;

    uint64_t k[RD_ITEMS];
    uint32_t r[RD_ITEMS];  // rank inside (wave, digit), then the LDS slot
#pragma unroll
    for (int i = 0; i < RD_ITEMS; ++i) {
        const uint32_t pos = wbase + i * 64 + lane;
        k[i] = (pos < n) ? rs_narrow(kin[pos], kw) : ~0ull;
    }
#pragma unroll
    for (int i = 0; i < RD_ITEMS; ++i) {
        const bool valid = (wbase + i * 64 + lane) < n;
        const uint32_t d = (uint32_t)(k[i] >> shift) & 255u;
        uint64_t m = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const uint64_t bb = __ballot((d >> b) & 1u);
            m &= ((d >> b) & 1u) ? bb : ~bb;
        }
        const uint32_t ltc = __popcll(m & lt_mask);
        const uint32_t c = s_wh[wid][d];
        r[i] = c + ltc;
        if (valid && ltc == 0) s_wh[wid][d] = c + (uint32_t)__popcll(m);
    }
    __syncthreads();
    // thread tid owns digit tid
    uint32_t run = 0;
    if (tid < 256) {
#pragma unroll
        for (int w = 0; w < RD_WAVES; ++w) { const uint32_t x = s_wh[w][tid]; s_wh[w][tid] = run; run += x; }
    }
    uint32_t blk_total;
    const uint32_t dstart = block_excl_scan<RD_BLOCK>(run, &blk_total, s_red);
    if (tid < 256) {
        s_dstart[tid] = dstart;
        s_gbase[tid] = toffs[(size_t)tid * ntiles + tile] - dstart;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < RD_ITEMS; ++i) {
        const bool valid = (wbase + i * 64 + lane) < n;
        const uint32_t d = (uint32_t)(k[i] >> shift) & 255u;
        r[i] = valid ? s_dstart[d] + s_wh[wid][d] + r[i] : 0xffffffffu;
        if (valid) s_k[r[i]] = k[i];
    }
    __syncthreads();
    const uint32_t tile_n = (n - tbase) < (uint32_t)RD_TILE ? (n - tbase) : (uint32_t)RD_TILE;
    uint32_t dg[RD_ITEMS / 4];  // digit of LDS slot j*RD_BLOCK+tid, 4 per word
#pragma unroll
    for (int q = 0; q < RD_ITEMS / 4; ++q) dg[q] = 0;
#pragma unroll
    for (int j = 0; j < RD_ITEMS; ++j) {
        const uint32_t p = j * RD_BLOCK + tid;
        if (p < tile_n) {
            const uint64_t kk = s_k[p];
            const uint32_t d = (uint32_t)(kk >> shift) & 255u;
            dg[j >> 2] |= d << (8 * (j & 3));
            kout[s_gbase[d] + p] = kk;
            if (dnext) dnext[s_gbase[d] + p] = (uint8_t)(kk >> shift_next);
        }
    }
    VT v[RD_ITEMS];
#pragma unroll
    for (int i = 0; i < RD_ITEMS; ++i) {
        const uint32_t pos = wbase + i * 64 + lane;
        if constexpr (IOTA) v[i] = pos;
        else v[i] = (pos < n) ? vin[pos] : VT{};
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < RD_ITEMS; ++i)
        if (r[i] != 0xffffffffu) s_v[r[i]] = v[i];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < RD_ITEMS; ++j) {
        const uint32_t p = j * RD_BLOCK + tid;
        if (p < tile_n) {
            const uint32_t d = (dg[j >> 2] >> (8 * (j & 3))) & 255u;
            vout[s_gbase[d] + p] = s_v[p];
        }
    }
}

// ------------------------------------------------------------------ hybrid: top digits globally, the rest in LDS
// When the keys' top m live digits already split them into small groups (expected group
// size <= 2^HY_SLACK_BITS by the digit entropies), only those m digits get global LSD
// passes; every group is then finished inside one block's LDS by the remaining live digits
// (<= 4, packed into a u32 local key). A global pass moves 16 B + 16 B per pair and its
// up-sweep reads 8 B more; the local sort reads each pair once and writes it once.
// The result equals the full LSD sort's, ties included (both sorts are stable).
//
// Tiles: groups (runs of equal top-m digits) that start in [t * LS_T, (t + 1) * LS_T) are
// block t's: it sorts [s_t, e_t), s_t = head(t * LS_T), e_t = head((t + 1) * LS_T), where
// head(x) = the first group start in [x, x + LS_CAP] (else x + LS_CAP, clamped to n). head
// is monotone, so the tiles partition [0, n) whatever the data; a tile over LS_CAP pairs
// (a group too large for the LDS) is copied unsorted and flagged, and the caller re-sorts.
#ifndef SG_LS_BLOCK
#define SG_LS_BLOCK 512
#endif
constexpr int LS_BLOCK = SG_LS_BLOCK;  // 256 or 512 (digit owners: the first 256 threads)
constexpr int LS_CAP = 4096;           // pairs sorted in one block's LDS
#ifndef SG_LS_T
#define SG_LS_T 3072
#endif
constexpr int LS_T = SG_LS_T;          // base tile (LS_CAP - LS_T: room for the last group)
constexpr int LS_ITEMS = LS_CAP / LS_BLOCK;
constexpr int LS_WCH = LS_ITEMS * 64;  // positions per wave (wave-major, row, lane)

// The first group start in [x, min(x + LS_CAP, n)) (n past the end, 0 at 0); *real = 0 when
// none was found (a group of >= LS_CAP pairs: the tile cannot be sorted in LDS).
__device__ __forceinline__ uint32_t ls_head(const uint64_t *__restrict__ K, uint32_t n, uint32_t x, uint64_t gmask,
                                            uint32_t *real) {
    const uint32_t lane = lane_id();
    *real = 1;
    if (x >= n) return n;
    if (x == 0) return 0;
    const uint32_t lim = min(n, x + (uint32_t)LS_CAP);
    for (uint32_t i0 = x; i0 < lim; i0 += 64) {
        const uint32_t i = i0 + lane;
        const bool h = i < lim && ((K[i] ^ K[i - 1]) & gmask) != 0;
        const uint64_t m = __ballot(h);
        if (m) return i0 + (uint32_t)(__ffsll((long long)m) - 1);
    }
    *real = lim == n ? 1u : 0u;
    return lim;
}

// bounds[t] = head(t * LS_T) | real << 31, t = 0 .. ntiles (one wave per boundary): the group
// search runs as its own launch, many waves in flight, instead of at the head of every
// local-sort block.
// (err[0]: the big-group count of the local sort's fix-up, err[1]: its flagged-tile count;
// zeroed here instead of by a memset launch)
__global__ __launch_bounds__(256) void k_rs_lbounds(const uint64_t *__restrict__ K, uint32_t n, uint64_t gmask,
                                                    uint32_t nb, uint32_t *__restrict__ bounds, uint32_t *__restrict__ err) {
    if (blockIdx.x == 0 && threadIdx.x < 2) err[threadIdx.x] = 0u;
    const uint32_t t = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (t >= nb) return;
    uint32_t real;
    const uint32_t h = ls_head(K, n, t * (uint32_t)LS_T, gmask, &real);
    if (lane_id() == 0) bounds[t] = h | (real << 31);
}

// lpos: the local key's digit positions (byte q of lpos = key byte of local digit q, LSD
// order), nloc of them. A window holds several groups: its pairs are sorted by the local key,
// then (stable) by their group ordinal in the window (1 or 2 more digits), which restores the
// groups' order with each group sorted inside. Whole block, uniform call; [s, s + nt) holds
// whole groups and nt <= LS_CAP.
struct LsShared {
    uint32_t key[LS_CAP];
    uint32_t ig[LS_CAP];  // window offset | group ordinal << 16
    uint32_t wh[LS_BLOCK / 64][256];
    uint32_t dstart[256];
    uint32_t red[LS_BLOCK / 64];
    uint32_t bits[2][LS_BLOCK / 64];
};

__device__ __forceinline__ void ls_sort_window(const uint64_t *__restrict__ K, const uint2 *__restrict__ V,
                                               uint64_t *__restrict__ Ko, uint2 *__restrict__ Vo, uint32_t s,
                                               uint32_t nt, uint64_t gmask, uint32_t lpos, uint32_t nloc,
                                               LsShared &sh_) {
    uint32_t *s_key = sh_.key, *s_ig = sh_.ig, *s_dstart = sh_.dstart, *s_red = sh_.red;
    auto &s_wh = sh_.wh;
    auto &s_bits = sh_.bits;
    const int tid = threadIdx.x, lane = lane_id(), wid = tid >> 6;
    __syncthreads();  // a previous window of this block may still read the shared arrays
    for (int x = tid; x < (LS_BLOCK / 64) * 256; x += LS_BLOCK) (&s_wh[0][0])[x] = 0;
    // touch the tile's spans now (one load per 128-B line): the sorted-order gather at the
    // end then hits L2 instead of waiting on HBM after the last pass
    uint32_t touch = 0;
    if ((uint32_t)tid * 16u < nt) touch = V[s + (uint32_t)tid * 16u].x;
    const uint64_t lt_mask = (1ull << lane) - 1ull;
    const uint32_t wbase = (uint32_t)wid * LS_WCH;
    uint32_t lk[LS_ITEMS], ig[LS_ITEMS];
    uint32_t wheads = 0;              // group starts in this wave's earlier rows
    uint32_t kor = 0, kand = ~0u;     // local-key bits that vary over the tile
#pragma unroll
    for (int i = 0; i < LS_ITEMS; ++i) {
        const uint32_t pos = wbase + i * 64 + lane;
        uint32_t v = 0;
        bool head = false;
        if (pos < nt) {
            const uint64_t k = K[s + pos];
            head = pos == 0 || ((k ^ K[s + pos - 1]) & gmask) != 0;
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (q < (int)nloc) v |= (uint32_t)((k >> (8 * ((lpos >> (8 * q)) & 255u))) & 255u) << (8 * q);
            kor |= v;
            kand &= v;
        }
        const uint64_t hm = __ballot(head);
        ig[i] = pos | ((wheads + (uint32_t)__popcll(hm & (lt_mask | (1ull << lane)))) << 16);  // inclusive, this wave
        wheads += (uint32_t)__popcll(hm);
        lk[i] = v;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        kor |= (uint32_t)__shfl_xor((int)kor, o, 64);
        kand &= (uint32_t)__shfl_xor((int)kand, o, 64);
    }
    if (lane == 0) { s_red[wid] = wheads; s_bits[0][wid] = kor; s_bits[1][wid] = kand; }
    __syncthreads();
    uint32_t before = 0, ngroups = 0;
    kor = 0;
    kand = ~0u;
#pragma unroll
    for (int w = 0; w < LS_BLOCK / 64; ++w) {
        const uint32_t x = s_red[w];
        before += (w < wid) ? x : 0u;
        ngroups += x;
        kor |= s_bits[0][w];
        kand &= s_bits[1][w];
    }
#pragma unroll
    for (int i = 0; i < LS_ITEMS; ++i) ig[i] = ig[i] + ((before - 1u) << 16);  // group ordinal in the tile
    __syncthreads();  // s_red is reused by the scans below
    const uint32_t lvary = kor ^ kand;
    const uint32_t npass = nloc + (ngroups > 1 ? (ngroups > 256 ? 2u : 1u) : 0u);
    for (uint32_t q = 0; q < npass; ++q) {
        const bool on_grp = q >= nloc;
        const int sh = on_grp ? 16 + 8 * (int)(q - nloc) : 8 * (int)q;
        // digit bits that vary over the tile (block-uniform): only those need a ballot
        const uint32_t gh = on_grp ? (ngroups - 1u) >> (sh - 16) : 0u;  // highest group ordinal's digit
        const uint32_t vb = on_grp ? (gh >= 128u ? 0xffu : (2u << (31 - __builtin_clz(gh | 1u))) - 1u)
                                   : ((lvary >> sh) & 255u);
        if (!on_grp && vb == 0) continue;  // a local digit constant over the tile
        uint32_t r[LS_ITEMS];
#pragma unroll
        for (int i = 0; i < LS_ITEMS; ++i) {
            if (wbase + i * 64 >= nt) { r[i] = 0; continue; }  // wave-uniform: row past the tile
            const bool valid = (wbase + i * 64 + lane) < nt;
            const uint32_t d = ((on_grp ? ig[i] : lk[i]) >> sh) & 255u;
            uint64_t m = __ballot(valid);
#pragma unroll
            for (int b = 0; b < 8; ++b) {
                if (!((vb >> b) & 1u)) continue;
                const uint64_t bb = __ballot((d >> b) & 1u);
                m &= ((d >> b) & 1u) ? bb : ~bb;
            }
            const uint32_t ltc = (uint32_t)__popcll(m & lt_mask);
            const uint32_t c = s_wh[wid][d];
            r[i] = c + ltc;
            if (valid && ltc == 0) s_wh[wid][d] = c + (uint32_t)__popcll(m);
        }
        __syncthreads();
        uint32_t run = 0;
        if (tid < 256) {
#pragma unroll
            for (int w = 0; w < LS_BLOCK / 64; ++w) { const uint32_t x = s_wh[w][tid]; s_wh[w][tid] = run; run += x; }
        }
        uint32_t tot;
        const uint32_t dst = block_excl_scan<LS_BLOCK>(run, &tot, s_red);
        if (tid < 256) s_dstart[tid] = dst;
        __syncthreads();
#pragma unroll
        for (int i = 0; i < LS_ITEMS; ++i) {
            if ((wbase + i * 64 + lane) < nt) {
                const uint32_t d = ((on_grp ? ig[i] : lk[i]) >> sh) & 255u;
                const uint32_t slot_i = s_dstart[d] + s_wh[wid][d] + r[i];
                s_key[slot_i] = lk[i];
                s_ig[slot_i] = ig[i];
            }
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < LS_ITEMS; ++i) {
            const uint32_t pos = wbase + i * 64 + lane;
            if (pos < nt) { lk[i] = s_key[pos]; ig[i] = s_ig[pos]; }
        }
        for (int x = tid; x < (LS_BLOCK / 64) * 256; x += LS_BLOCK) (&s_wh[0][0])[x] = 0;
        __syncthreads();
    }
    // pairs out in sorted order, fetched by their tile offset (the tile was just read: L2)
#pragma unroll
    for (int i = 0; i < LS_ITEMS; ++i) {
        const uint32_t pos = wbase + i * 64 + lane;
        if (pos < nt) {
            const uint32_t ix = ig[i] & 0xffffu;
            Ko[s + pos] = K[s + ix];
            Vo[s + pos] = V[s + ix];
        }
    }
    asm volatile("" ::"v"(touch));  // keeps the touch load (its result is not needed)
}

// Block-wide max of one value per thread (every thread gets the result).
__device__ __forceinline__ uint32_t ls_blk_max(uint32_t v, uint32_t *s_agg) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o, 64));
    __syncthreads();
    if (lane_id() == 0) s_agg[threadIdx.x >> 6] = v;
    __syncthreads();
#pragma unroll
    for (int w = 0; w < LS_BLOCK / 64; ++w) v = max(v, s_agg[w]);
    return v;
}

// flist / fcnt: the tiles this sort could not do in one window (over LS_CAP pairs: a group
// straddles the tile's end boundary far enough, or is larger than the LDS), listed for
// k_rs_lsort_fix, which the host launches right behind this kernel (no read-back between).
__global__ __launch_bounds__(LS_BLOCK) void k_rs_lsort(const uint64_t *__restrict__ K, const uint2 *__restrict__ V,
                                                       uint64_t *__restrict__ Ko, uint2 *__restrict__ Vo, uint32_t n,
                                                       uint64_t gmask, uint32_t lpos, uint32_t nloc,
                                                       const uint32_t *__restrict__ bounds, uint32_t *__restrict__ flist,
                                                       uint32_t *__restrict__ fcnt) {
    __shared__ LsShared sh_;
    const uint32_t t = blockIdx.x;
    const uint32_t b0 = bounds[t], b1 = bounds[t + 1];
    const uint32_t s = b0 & 0x7fffffffu, e = max(b1 & 0x7fffffffu, s);
    const uint32_t nt = e - s;
    if (nt == 0) return;
    if (nt > (uint32_t)LS_CAP || !(b0 >> 31) || !(b1 >> 31)) {
        if (threadIdx.x == 0) flist[atomicAdd(fcnt, 1u)] = t;
        return;
    }
    ls_sort_window(K, V, Ko, Vo, s, nt, gmask, lpos, nloc, sh_);
}

// The tiles k_rs_lsort listed (a group of equal top digits larger than the LDS lies in them,
// or the tile edge cuts one far enough), redone from the same input right behind it, a few
// blocks walking the list (cost proportional to the listed tiles, no host round trip):
// windows of whole groups (<= LS_CAP pairs) are sorted in LDS as usual; every group too large
// for a window ("big group", e.g. one record repeated thousands of times) is copied and listed
// (gs, ge: its position range, appended by the block that holds its first position; the
// blocks its tail reaches skip it; cnt: how many), and lsort_fixup_big sorts the listed
// groups' members by one global radix sort on (group, local digits) — the only case the host
// sees (cnt comes back with the dedup's counts).
__device__ void ls_fix_tile(const uint64_t *__restrict__ K, const uint2 *__restrict__ V, uint64_t *__restrict__ Ko,
                            uint2 *__restrict__ Vo, uint32_t n, uint64_t gmask, uint32_t lpos, uint32_t nloc, uint32_t b0,
                            uint32_t b1, uint32_t *__restrict__ gs, uint32_t *__restrict__ ge, uint32_t cap,
                            uint32_t *__restrict__ cnt, LsShared &sh_, uint32_t *s_agg) {
    const uint32_t tid = threadIdx.x;
    const uint32_t s = b0 & 0x7fffffffu, e = max(b1 & 0x7fffffffu, s);
    const bool e_real = (b1 >> 31) != 0;
    auto is_head = [&](uint32_t i) -> bool { return i >= n || ((K[i] ^ K[i - 1]) & gmask) != 0; };
    // the first group start in [from, lim) (lim when none); from >= 1
    auto first_head = [&](uint32_t from, uint32_t lim) -> uint32_t {
        for (uint32_t b = from; b < lim; b += LS_BLOCK) {
            const uint32_t i = b + tid;
            const uint32_t m = ~ls_blk_max((i < lim && is_head(i)) ? ~i : 0u, s_agg);
            if (m != 0xffffffffu) return m;
        }
        return lim;
    };
    uint32_t p = s;
    bool p_real = (b0 >> 31) != 0;
    while (p < e) {
        if (!p_real) {  // the tail of a big group listed by an earlier block
            const uint32_t q = first_head(p + 1, e);
            p = q;
            p_real = q < e || e_real;
            continue;
        }
        uint32_t h;
        if (e - p <= (uint32_t)LS_CAP && e_real) {
            h = e;
        } else {
            const uint32_t lim = min(p + (uint32_t)LS_CAP, e);  // window ends: group starts in (p, lim]
            uint32_t best = 0;
            for (uint32_t i = p + 1 + tid; i <= lim; i += LS_BLOCK)
                if (i == e ? e_real : is_head(i)) best = max(best, i);
            h = ls_blk_max(best, s_agg);
        }
        if (h > p) {
            ls_sort_window(K, V, Ko, Vo, p, h - p, gmask, lpos, nloc, sh_);
            p = h;
            continue;
        }
        // a big group starts at p: its end may lie in a later tile
        const uint32_t q = first_head(p + (uint32_t)LS_CAP + 1u, n);
        for (uint32_t i = p + tid; i < q; i += LS_BLOCK) { Ko[i] = K[i]; Vo[i] = V[i]; }
        if (tid == 0) {
            const uint32_t k = atomicAdd(cnt, 1u);
            if (k < cap) { gs[k] = p; ge[k] = q; }
        }
        p = q;  // >= e ends the tile
    }
}

__global__ __launch_bounds__(LS_BLOCK) void k_rs_lsort_fix(const uint64_t *__restrict__ K, const uint2 *__restrict__ V,
                                                           uint64_t *__restrict__ Ko, uint2 *__restrict__ Vo, uint32_t n,
                                                           uint64_t gmask, uint32_t lpos, uint32_t nloc,
                                                           const uint32_t *__restrict__ bounds,
                                                           const uint32_t *__restrict__ flist,
                                                           const uint32_t *__restrict__ fcnt, uint32_t *__restrict__ gs,
                                                           uint32_t *__restrict__ ge, uint32_t cap, uint32_t *__restrict__ cnt) {
    __shared__ LsShared sh_;
    __shared__ uint32_t s_agg[LS_BLOCK / 64];
    const uint32_t nf = *fcnt;  // final: k_rs_lsort completed before this launch
    for (uint32_t j = blockIdx.x; j < nf; j += gridDim.x) {
        const uint32_t t = flist[j];
        ls_fix_tile(K, V, Ko, Vo, n, gmask, lpos, nloc, bounds[t], bounds[t + 1], gs, ge, cap, cnt, sh_, s_agg);
    }
}

// Big groups -> member rows: row j -> its group g (goff: exclusive row offsets), position
// gs[g] + (j - goff[g]), key = g << 32 | the position's local digits (as k_rs_lsort packs
// them). One wave per 1024 consecutive rows (groups hold > LS_CAP rows).
__global__ __launch_bounds__(256) void k_lfix_expand(const uint64_t *__restrict__ K, const uint32_t *__restrict__ gs,
                                                     const uint64_t *__restrict__ goff, uint32_t B, uint32_t M,
                                                     uint32_t lpos, uint32_t nloc, uint64_t *__restrict__ RK,
                                                     uint32_t *__restrict__ RP) {
    const uint32_t j0 = (blockIdx.x * 4u + (threadIdx.x >> 6)) * 1024u;
    if (j0 >= M) return;
    uint32_t g = 0, hi = B;  // last g with goff[g] <= j0
    while (hi - g > 1) {
        const uint32_t mid = (g + hi) >> 1;
        if (goff[mid] <= j0) g = mid; else hi = mid;
    }
    const uint32_t je = min(M, j0 + 1024u);
    for (uint32_t j = j0 + lane_id(); j < je; j += 64) {
        while (g + 1 < B && goff[g + 1] <= j) ++g;
        const uint32_t pos = gs[g] + (j - (uint32_t)goff[g]);
        const uint64_t k = K[pos];
        uint32_t v = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (q < (int)nloc) v |= (uint32_t)((k >> (8 * ((lpos >> (8 * q)) & 255u))) & 255u) << (8 * q);
        RK[j] = ((uint64_t)g << 32) | v;
        RP[j] = pos;
    }
}

// Sorted rows -> the big groups' positions: row j's position takes the pair of the row that
// sorted to j (rows are group-major, so row j's position lies in its sorted group).
__global__ void k_lfix_apply(const uint64_t *__restrict__ K, const uint2 *__restrict__ V, const uint32_t *__restrict__ RP,
                             const uint32_t *__restrict__ perm, uint32_t M, uint64_t *__restrict__ Ko,
                             uint2 *__restrict__ Vo) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= M) return;
    const uint32_t src = RP[perm[j]];
    Ko[RP[j]] = K[src];
    Vo[RP[j]] = V[src];
}

struct LfixSizeFn {
    const uint32_t *gs, *ge;
    __device__ uint64_t operator()(uint32_t g) const { return (uint64_t)(ge[g] - gs[g]); }
};

// Host plan: the top live digits (in descending significance) until their entropy leaves
// groups of about 2^HY_SLACK_BITS pairs; hybrid only when 2..4 live digits remain below
// them (each one a global pass saved). top[]: the global passes (LSD order), lpos/nloc: the
// local key's digit positions.
// 10 bits (round 6; 8 before): C5's 52M-record parts take 4 global passes instead of 5 and
// finish groups of ~600 pairs in LDS (one more local pass, ~2.7 ms per step, against ~6 ms per
// global pass); with 3,072-pair base tiles no C5 tile outgrows a window (3,584: ~2 % did, and
// the fix-up pass then cost 1.7 ms). C5 179.9 -> 173.9 ms, C2 unchanged (1.596 / 1.592).
#ifndef SG_HY_SLACK
#define SG_HY_SLACK 10.0
#endif
constexpr double HY_SLACK_BITS = SG_HY_SLACK;
struct HybridPlan {
    bool on = false;
    int top[RS_MAXPASS];
    int ntop = 0;
    uint32_t lpos = 0, nloc = 0;
    uint64_t gmask = 0;
};

static HybridPlan plan_hybrid(const uint32_t *hh, uint32_t hn, uint32_t n, const int *live, int nlive) {
    HybridPlan hp;
    if (n < (1u << 20) || nlive < 3) return hp;
    const double need = std::log2((double)n) - HY_SLACK_BITS;
    double acc = 0;
    int q = nlive;  // live[q..nlive) are the top digits taken
    while (q > 0 && acc < need) {
        --q;
        const int p = live[q];
        double H = 0;
        for (int d = 0; d < 256; ++d)
            if (hh[p * 256 + d]) {
                const double f = hh[p * 256 + d] / (double)hn;
                H -= f * std::log2(f);
            }
        acc += H;
    }
    if (acc < need) return hp;
    const int nl = q;  // live digits below the top ones: sorted locally
    if (nl < 2 || nl > 4) return hp;
    hp.on = true;
    for (int i = q; i < nlive; ++i) hp.top[hp.ntop++] = live[i];
    for (int i = 0; i < nl; ++i) hp.lpos |= (uint32_t)live[i] << (8 * i);
    hp.nloc = (uint32_t)nl;
    hp.gmask = ~0ull << (8 * live[q]);
    return hp;
}

int key_sample_hist(sg_ctx *c, const uint64_t *keys, uint32_t n, uint32_t *dev_hist, uint32_t *sample_n,
                    const KeyStatD *parts, uint32_t nparts, KeyStatD *st) {
    *sample_n = 0;
    if (n == 0) return SG_OK;
    const uint32_t nrows = (n + 63) / 64;
    // about 2^16 sampled keys: the plug-in entropy estimate's bias is ~0.003 bit per digit
    // (the LDS atomics of 2^18 sampled keys cost 12 µs on 64 CUs)
    uint32_t rs = 1;
    while (rs < 1024 && (uint64_t)(nrows / (rs * 2)) * 64 >= (1u << 16)) rs *= 2;
    const uint32_t srows = (nrows + rs - 1) / rs;
    const uint32_t grid = std::min<uint32_t>((srows + 7) / 8, 64u);
    SG_LAUNCH_B(c, "key_sample", 8.0 * srows * 64, k_key_sample, grid, 512, 0, keys, n, rs, dev_hist, parts,
                nparts, st);
    const uint32_t last = (srows - 1) * rs;  // the last sampled row may be partial
    *sample_n = (srows - 1) * 64 + std::min<uint32_t>(64u, n - last * 64);
    return SG_OK;
}

// ks (optional, bits [0, 64)): the keys' varying bits (exact: the trivial passes are known
// without a histogram pass or a read-back; each pass's digit bases then come from its own
// tile counts) and sampled digit histograms (the hybrid plan).
template <typename VT>
static int radix_sort_t(sg_ctx *c, uint64_t *keys, VT *vals, uint64_t *keys_alt, VT *vals_alt,
                        uint32_t n, int begin_bit, int end_bit, bool iota_vals, uint64_t **keys_out,
                        VT **vals_out, const char *pass_name, const KeyStats *ks = nullptr,
                        uint32_t narrow_kw = 0, uint32_t **lsort_err = nullptr, uint32_t *err_at = nullptr) {
    if (lsort_err) *lsort_err = nullptr;
    *keys_out = keys;
    *vals_out = vals;
    if (n == 0) return SG_OK;
    const int npasses = (end_bit - begin_bit + 7) / 8;
    if (npasses <= 0 || npasses > RS_MAXPASS) { set_error("radix_sort: bad bit range"); return SG_E_INVAL; }
    if (ks && (begin_bit != 0 || npasses != RS_MAXPASS)) { set_error("radix_sort: key stats cover 64 bits"); return SG_E_INVAL; }
    uint32_t *hist;
    SG_TRY(slot(c, S_HIST, RS_MAXPASS * 256 * 2 + RS_MAXPASS, &hist));
    uint32_t *offs = hist + RS_MAXPASS * 256;
    uint32_t *triv = offs + RS_MAXPASS * 256;
    uint32_t *dtot = nullptr;  // KeyStats sorts: per-pass digit totals (in the histogram area)
    uint32_t trivial[RS_MAXPASS];
    if (ks) {
        dtot = hist;
        for (int p = 0; p < npasses; ++p) trivial[p] = ((ks->vary >> (8 * p)) & 0xffu) == 0;
    } else {
        SG_HIP(hipMemsetAsync(hist, 0, RS_MAXPASS * 256 * 4, c->stream));
        uint32_t hgrid = (n + RS_HBLOCK * 16 - 1) / (RS_HBLOCK * 16);
        if (hgrid > 1024) hgrid = 1024;
        SG_LAUNCH_B(c, "rs_hist", 8.0 * n, k_rs_hist, hgrid, RS_HBLOCK, 0, keys, n, begin_bit, npasses, hist,
                    narrow_kw);
        SG_LAUNCH(c, "rs_scan", k_rs_scan, npasses, 256, 0, hist, offs, triv, n);
        SG_TRY(ctx_readback(c, trivial, triv, npasses * 4));
    }
    int live[RS_MAXPASS], nlive = 0;
    for (int p = 0; p < npasses; ++p)
        if (!trivial[p]) live[nlive++] = p;

    const uint32_t ntiles = (n + RD_TILE - 1) / RD_TILE;
    uint32_t *tcnt;
    SG_TRY(slot(c, S_RS_TCNT, (size_t)ntiles * 256 + 64, &tcnt));
    uint64_t *ck = keys, *ak = keys_alt;
    VT *cv = vals, *av = vals_alt;
    bool iota_pending = iota_vals;
    constexpr double VB = (double)sizeof(VT);
    const bool xcd = true;  // XCD-aware tile order
    const uint32_t grid = xcd ? 8u * ((ntiles + 7u) / 8u) : ntiles;
    if (narrow_kw && begin_bit != 0) { set_error("radix_sort: narrowing needs the keys' bit 0"); return SG_E_INVAL; }
    if (narrow_kw && nlive == 0) live[nlive++] = 0;  // one (no-op) pass still writes the narrowed keys
    // hybrid (spans payload, host histograms, a caller that checks the local sort's flag):
    // global passes over the top digits only, the rest sorted per group in LDS
    HybridPlan hp;
    if constexpr (sizeof(VT) == 8) {
        if (ks && ks->hist && ks->hist_n && lsort_err) hp = plan_hybrid(ks->hist, ks->hist_n, n, live, nlive);
    }
    const int *passes = hp.on ? hp.top : live;
    const int npass = hp.on ? hp.ntop : nlive;
    // every pass after the first counts its tiles from the digit bytes its predecessor wrote
    uint8_t *dig = nullptr;
    if (npass > 1) SG_TRY(slot(c, S_RS_DIGITS, (size_t)n + 16, &dig));
    for (int q = 0; q < npass; ++q) {
        const int p = passes[q];
        const int shift = begin_bit + 8 * p;
        const uint32_t kw = q == 0 ? narrow_kw : 0u;  // the first pass narrows as it reads
        if (q == 0 || !dig) SG_LAUNCH_B(c, "rs_up", 8.0 * n, k_rs_up, grid, RD_BLOCK, 0, ck, n, shift, ntiles, tcnt, kw, xcd);
        else SG_LAUNCH_B(c, "rs_up", 1.0 * n, k_rs_up8, grid, RD_BLOCK, 0, dig, n, ntiles, tcnt, xcd);
        if (dtot) SG_LAUNCH(c, "rs_dsum", k_rs_dsum, 256, 256, 0, tcnt, ntiles, dtot);
        SG_LAUNCH(c, "rs_cscan", k_rs_cscan, 256, 256, 0, tcnt, ntiles, offs + p * 256, dtot);
        uint8_t *dn = q + 1 < npass ? dig : nullptr;
        const int shn = q + 1 < npass ? begin_bit + 8 * passes[q + 1] : 0;
        if constexpr (sizeof(VT) == 4) {
            if (iota_pending)
                SG_LAUNCH(c, pass_name, (k_rs_down<true, VT>), grid, RD_BLOCK, 0, ck, cv, ak, av, n, shift, ntiles, tcnt, kw, xcd,
                          dn, shn);
            else
                SG_LAUNCH(c, pass_name, (k_rs_down<false, VT>), grid, RD_BLOCK, 0, ck, cv, ak, av, n, shift, ntiles, tcnt, kw,
                          xcd, dn, shn);
        } else {
            SG_LAUNCH(c, pass_name, (k_rs_down<false, VT>), grid, RD_BLOCK, 0, ck, cv, ak, av, n, shift, ntiles, tcnt, kw, xcd,
                      dn, shn);
        }
        // 8 B key + the value read (implied for iota ids) and both written, per pair (+ the
        // next pass's digit byte)
        prof_bytes(c, pass_name, (iota_pending ? 16.0 + VB : 16.0 + 2.0 * VB) * n + (dn ? 1.0 * n : 0.0));
        iota_pending = false;
        uint64_t *tk = ck; ck = ak; ak = tk;
        VT *tv = cv; cv = av; av = tv;
    }
    if constexpr (sizeof(VT) == 8) {
        if (hp.on) {
            // err[0]: big groups the fix-up listed (the caller reads it back), err[1]: tiles
            // it redid
            uint32_t *err = err_at;
            if (!err) SG_TRY(slot(c, S_LS_ERR, 2, &err));
            const uint32_t g = (n + LS_T - 1) / LS_T;
            uint32_t *bounds;
            SG_TRY(slot(c, S_LS_BOUNDS, (size_t)g + 1, &bounds));
            // the fix-up's lists: flagged tiles (g), big groups' ranges (cap each)
            const uint32_t cap = g + 16;
            uint32_t *lst;
            SG_TRY(slot(c, S_LS_LIST, (size_t)g + 2 * (size_t)cap + 16, &lst));
            uint32_t *flist = lst, *gs = lst + g, *ge = gs + cap;
            SG_LAUNCH(c, "rs_lbounds", k_rs_lbounds, (g + 1 + 3) / 4, 256, 0, ck, n, hp.gmask, g + 1, bounds, err);
            // model: key read, key + span fetched in sorted order, both written
            SG_LAUNCH_B(c, "rs_lsort", 40.0 * n, k_rs_lsort, g, LS_BLOCK, 0, ck, cv, ak, av, n, hp.gmask, hp.lpos, hp.nloc,
                        bounds, flist, err + 1);
            // the listed tiles redone from the same input by a few blocks walking the list (64:
            // the launch costs ~7 us at 256 blocks when, as usual, no tile is listed; folding it
            // into k_rs_lsort as a call took that kernel to 184 VGPRs)
            SG_LAUNCH(c, "rs_lfix", k_rs_lsort_fix, std::min<uint32_t>(g, 64u), LS_BLOCK, 0, ck, cv, ak, av, n, hp.gmask,
                      hp.lpos, hp.nloc, bounds, flist, err + 1, gs, ge, cap, err);
            c->ls_last.on = true;
            c->ls_last.gmask = hp.gmask;
            c->ls_last.lpos = hp.lpos;
            c->ls_last.nloc = hp.nloc;
            c->ls_last.ntiles = g;
            c->ls_last.bounds = bounds;
            c->ls_last.gs = gs;
            c->ls_last.ge = ge;
            c->ls_last.cap = cap;
            uint64_t *tk = ck; ck = ak; ak = tk;
            VT *tv = cv; cv = av; av = tv;
            *lsort_err = err;
        }
    }
    if constexpr (sizeof(VT) == 4) {
        if (iota_pending) {
            uint32_t g = (n + 255) / 256;
            if (g > 4096) g = 4096;
            SG_LAUNCH(c, "iota", k_iota, g, 256, 0, cv, n);
        }
    }
    *keys_out = ck;
    *vals_out = cv;
    return SG_OK;
}

int lsort_fixup_big(sg_ctx *c, const uint64_t *Kin, const uint2 *Vin, uint64_t *Ko, uint2 *Vo, uint32_t n, uint32_t B) {
    const auto &P = c->ls_last;
    if (!P.on) { set_error("lsort_fixup: no hybrid sort to fix"); return SG_E_INVAL; }
    if (B > P.cap) { set_error("lsort_fixup: %u big groups (list of %u)", B, P.cap); return SG_E_HIP; }
    if (!B) return SG_OK;
    const uint32_t *gs = P.gs, *ge = P.ge;
    // the big groups' members: one stable radix sort on (group, local digits)
    uint64_t *goff;
    SG_TRY(slot(c, S_LF_OFF, (size_t)B + 1, &goff));
    uint64_t M64 = 0;
    SG_TRY(run_scan64(c, "lfix_scan", LfixSizeFn{gs, ge}, B, goff, &M64));
    const uint32_t M = (uint32_t)M64;
    uint64_t *RK, *RK2, *SK;
    uint32_t *RV, *RV2, *RP, *perm;
    SG_TRY(slot(c, S_LF_KEY, M, &RK));
    SG_TRY(slot(c, S_LF_KEY2, M, &RK2));
    SG_TRY(slot(c, S_LF_VAL, M, &RV));
    SG_TRY(slot(c, S_LF_VAL2, M, &RV2));
    SG_TRY(slot(c, S_LF_POS, M, &RP));
    SG_LAUNCH(c, "lfix_expand", k_lfix_expand, (M + 4095) / 4096, 256, 0, Kin, gs, goff, B, M, P.lpos, P.nloc, RK, RP);
    int gbits = 1;
    while (gbits < 31 && (1u << gbits) < B) ++gbits;
    SG_TRY(radix_sort(c, RK, RV, RK2, RV2, M, 0, 32 + gbits, true, &SK, &perm, "rs_lfix_pass"));
    SG_LAUNCH(c, "lfix_apply", k_lfix_apply, (M + 255) / 256, 256, 0, Kin, Vin, RP, perm, M, Ko, Vo);
    return SG_OK;
}

int radix_sort(sg_ctx *c, uint64_t *keys, uint32_t *vals, uint64_t *keys_alt, uint32_t *vals_alt,
               uint32_t n, int begin_bit, int end_bit, bool iota_vals, uint64_t **keys_out,
               uint32_t **vals_out, const char *pass_name) {
    return radix_sort_t<uint32_t>(c, keys, vals, keys_alt, vals_alt, n, begin_bit, end_bit, iota_vals, keys_out,
                                  vals_out, pass_name);
}

int radix_sort_spans(sg_ctx *c, uint64_t *keys, uint2 *spans, uint64_t *keys_alt, uint2 *spans_alt, uint32_t n,
                     int begin_bit, int end_bit, uint64_t **keys_out, uint2 **spans_out, const char *pass_name,
                     const KeyStats *ks, uint32_t narrow_kw, uint32_t **lsort_err, uint32_t *err_at) {
    return radix_sort_t<uint2>(c, keys, spans, keys_alt, spans_alt, n, begin_bit, end_bit, false, keys_out, spans_out,
                               pass_name, ks, narrow_kw, lsort_err, err_at);
}

}  // namespace sg
