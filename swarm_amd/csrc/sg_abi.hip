// sg_abi.hip — the exported C entry points of libswarmgpu.so (include/swarmgpu.h) and the
// multi-GPU record partition.
#include "sg_internal.hpp"
#include "sg_prims.hpp"
#define SG_EMIT_DEVICE_ONLY
#include "sg_emit.hpp"
#include "sg_route.hpp"

#include <string.h>

namespace sg {

int dev_dedup_diff(sg_ctx *c, const uint8_t *d_cur, uint64_t n_cur, const uint8_t *d_prior,
                   uint64_t n_prior, bool want_fresh, sg_dev_result *res);

// ------------------------------------------------------------------ record hash
// Shared host/device definition (oracle: tests restate it in Python).
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

template <class Load>
__host__ __device__ __forceinline__ uint64_t hash_words(Load ld, uint32_t len) {
    uint64_t h = 0x9e3779b97f4a7c15ull ^ ((uint64_t)len * 0xff51afd7ed558ccdull);
    for (uint32_t o = 0; o < len; o += 8) {
        uint64_t w = 0;
        const uint32_t take = (len - o) < 8u ? (len - o) : 8u;
        for (uint32_t j = 0; j < take; ++j) w |= (uint64_t)ld(o + j) << (8 * j);
        h = (h ^ mix64(w)) * 0x9fb21c651e98df25ull;
        h ^= h >> 29;
    }
    return mix64(h);
}

// hash_words over buf[s, e) with aligned 8-byte loads (bit-identical): word o is bytes
// [s+o, s+o+8) little-endian, joined from at most two aligned words. buf is 8-B aligned; a
// second word is read only when it holds a byte of the record.
__device__ __forceinline__ uint64_t hash_record(const uint8_t *__restrict__ buf, uint32_t s, uint32_t e) {
    const uint32_t len = e - s;
    uint64_t h = 0x9e3779b97f4a7c15ull ^ ((uint64_t)len * 0xff51afd7ed558ccdull);
    const uint32_t sh = (s & 7u) * 8u;
    const uint64_t *wp = reinterpret_cast<const uint64_t *>(buf + (s & ~7u));
    uint64_t lo = wp[0];
    for (uint32_t o = 0; o < len; o += 8) {
        const uint32_t take = (len - o) < 8u ? (len - o) : 8u;
        uint64_t w = lo >> sh;
        if (sh && (s & 7u) + take > 8u) {
            const uint64_t hi = wp[(o >> 3) + 1];
            w |= hi << (64u - sh);
            lo = hi;
        } else if (sh == 0 && o + 8u < len) {
            lo = wp[(o >> 3) + 1];
        }
        if (take < 8u) w &= (1ull << (8u * take)) - 1ull;
        h = (h ^ mix64(w)) * 0x9fb21c651e98df25ull;
        h ^= h >> 29;
    }
    return mix64(h);
}

__host__ __device__ __forceinline__ uint32_t part_of(uint64_t h, uint32_t parts) {
    return (uint32_t)(((h >> 32) * (uint64_t)parts) >> 32);
}

// Add (1 record, `bytes`) to counter slot `q` of the block's LDS histogram: one LDS
// atomic pair per wave when the whole wave routes to one part (sorted inputs, few
// parts), else one per lane (LDS atomics spread over the parts' addresses).
__device__ __forceinline__ void wave_count(unsigned long long *s_c, uint32_t stride, bool act, uint32_t q,
                                           uint32_t bytes) {
    const uint64_t am = __ballot(act);
    if (!am) return;
    const int leader = __ffsll((long long)am) - 1;
    const uint32_t lq = (uint32_t)__shfl((int)q, leader, 64);
    if (__ballot(act && q != lq) == 0) {
        const uint64_t b = wave_sum<uint64_t>(act ? (uint64_t)bytes : 0ull);
        if (lane_id() == leader) {
            atomicAdd(&s_c[lq], (unsigned long long)__popcll(am));
            atomicAdd(&s_c[stride + lq], (unsigned long long)b);
        }
    } else if (act) {
        atomicAdd(&s_c[q], 1ull);
        atomicAdd(&s_c[stride + q], (unsigned long long)bytes);
    }
}

__global__ __launch_bounds__(256) void k_part_keys(const uint8_t *__restrict__ buf,
                                                   const uint2 *__restrict__ spans, uint32_t R,
                                                   uint32_t parts, uint8_t *keys,
                                                   unsigned long long *cnt /* [2*parts] */) {
    __shared__ unsigned long long s_c[2 * 256];
    for (int i = threadIdx.x; i < 2 * 256; i += blockDim.x) s_c[i] = 0;
    __syncthreads();
    // grid-stride (a bounded grid): each block flushes its histogram once, so the global
    // counters see ~grid x parts atomics instead of one burst per 256 records
    for (uint32_t i0 = blockIdx.x * blockDim.x; i0 < R; i0 += gridDim.x * blockDim.x) {
        const uint32_t i = i0 + threadIdx.x;
        uint32_t q = 0, bytes = 0;
        if (i < R) {
            const uint32_t s = spans[i].x, e = spans[i].y;
            const uint64_t h = hash_record(buf, s, e);
            q = part_of(h, parts);
            keys[i] = (uint8_t)q;
            bytes = e - s + 1;
        }
        wave_count(s_c, 256, i < R, q, bytes);
    }
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < parts; q += blockDim.x) {
        if (s_c[q]) atomicAdd(&cnt[q], s_c[q]);
        if (s_c[256 + q]) atomicAdd(&cnt[parts + q], s_c[256 + q]);
    }
}

// Range routing (order-preserving shards): part = number of splitters <= key0(record).
// key0 order is consistent with byte order, and equal key0 values share a
// part, so part p holds only records below every record of part p+1: the per-part sort -u
// outputs concatenated in part order are the global sort -u output.
__global__ __launch_bounds__(256) void k_range_keys(const uint64_t *__restrict__ key0, const uint2 *__restrict__ spans,
                                                    uint32_t R, const uint64_t *__restrict__ split, uint32_t ns,
                                                    uint8_t *keys, unsigned long long *cnt /* [2*parts] */) {
    __shared__ unsigned long long s_c[2 * 256];
    __shared__ uint64_t s_split[256];
    for (int i = threadIdx.x; i < 2 * 256; i += blockDim.x) s_c[i] = 0;
    for (uint32_t i = threadIdx.x; i < ns; i += blockDim.x) s_split[i] = split[i];
    __syncthreads();
    for (uint32_t i0 = blockIdx.x * blockDim.x; i0 < R; i0 += gridDim.x * blockDim.x) {
        const uint32_t i = i0 + threadIdx.x;
        uint32_t lo = 0, bytes = 0;
        if (i < R) {
            const uint64_t k = key0[i];
            uint32_t hi = ns;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (s_split[mid] <= k) lo = mid + 1; else hi = mid;
            }
            keys[i] = (uint8_t)lo;
            bytes = spans[i].y - spans[i].x + 1;
        }
        wave_count(s_c, 256, i < R, lo, bytes);
    }
    __syncthreads();
    for (uint32_t q = threadIdx.x; q <= ns; q += blockDim.x) {
        if (s_c[q]) atomicAdd(&cnt[q], s_c[q]);
        if (s_c[256 + q]) atomicAdd(&cnt[ns + 1 + q], s_c[256 + q]);
    }
}

// Byte-string splitters: sg_route.hpp.
// Ordering by key0 first: record key0 vs splitter key0 (both the first 7 bytes + min(len, 8))
// decides unless they are equal with tag 8; only then are the first 64 bytes loaded and
// compared word by word (host:port records: one or two 8-B loads per record instead of
// eight; URL records share key0 and take the word compare).
__global__ __launch_bounds__(256) void k_range_bytes(const uint8_t *__restrict__ buf, const uint2 *__restrict__ spans,
                                                     uint32_t R, const uint64_t *__restrict__ split_w,
                                                     const uint32_t *__restrict__ split_len, uint32_t ns,
                                                     uint8_t *keys, unsigned long long *cnt /* [2*parts] */) {
    __shared__ unsigned long long s_c[2 * 256];
    __shared__ uint64_t s_w[255 * SPL_WORDS];
    __shared__ uint64_t s_k0[256];
    __shared__ uint32_t s_len[256];
    for (int i = threadIdx.x; i < 2 * 256; i += blockDim.x) s_c[i] = 0;
    for (uint32_t i = threadIdx.x; i < ns * SPL_WORDS; i += blockDim.x) s_w[i] = split_w[i];
    for (uint32_t i = threadIdx.x; i < ns; i += blockDim.x) {
        const uint32_t l = split_len[i];
        s_len[i] = l;
        s_k0[i] = (split_w[i * SPL_WORDS] & ~0xffull) | (uint64_t)(l < 8u ? l : 8u);
    }
    __syncthreads();
    for (uint32_t i0 = blockIdx.x * blockDim.x; i0 < R; i0 += gridDim.x * blockDim.x) {
        const uint32_t i = i0 + threadIdx.x;
        uint32_t lo = 0, bytes = 0;
        if (i < R) {
            const uint2 x = spans[i];
            lo = route_record(buf, ~0ull, x.x, x.y, chunk_key(buf, x.x, x.y, 0), s_k0, ns, s_w, s_len);
            keys[i] = (uint8_t)lo;
            bytes = x.y - x.x + 1;
        }
        wave_count(s_c, 256, i < R, lo, bytes);
    }
    __syncthreads();
    for (uint32_t q = threadIdx.x; q <= ns; q += blockDim.x) {
        if (s_c[q]) atomicAdd(&cnt[q], s_c[q]);
        if (s_c[256 + q]) atomicAdd(&cnt[ns + 1 + q], s_c[256 + q]);
    }
}

// m evenly spaced records' first 64 bytes (zero-filled) and min(len, 64).
__global__ __launch_bounds__(256) void k_head_sample(const uint8_t *__restrict__ buf, const uint2 *__restrict__ spans,
                                                     uint32_t R, uint32_t m, uint64_t *__restrict__ heads,
                                                     uint32_t *__restrict__ lens) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= m) return;
    const uint2 x = spans[(uint32_t)(((uint64_t)k * R) / m)];
    uint64_t w[SPL_WORDS];
    head_words(buf, x.x, x.y, w);
#pragma unroll
    for (uint32_t j = 0; j < SPL_WORDS; ++j) heads[(size_t)k * SPL_WORDS + j] = w[j];
    lens[k] = min(x.y - x.x, SPL_W);
}

__global__ __launch_bounds__(256) void k_key_sample(const uint64_t *__restrict__ key0, uint32_t R, uint32_t m,
                                                    uint64_t *__restrict__ out) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < m) out[k] = key0[(uint32_t)(((uint64_t)k * R) / m)];
}

struct Acq {
    sg_ctx *c = nullptr;
    ~Acq() { if (c) pool_release(c); }
};

static int acquire(Acq *a) {
    int dev = 0;
    SG_TRY(pick_device(&dev));
    SG_TRY(pool_acquire(dev, &a->c));
    SG_HIP(hipSetDevice(dev));
    return SG_OK;
}

static int upload(sg_ctx *c, int s, const uint8_t *host, size_t n, uint8_t **d) {
    SG_TRY(slot(c, s, n + 16, d));
    if (n) SG_HIP(hipMemcpyAsync(*d, host, n, hipMemcpyHostToDevice, c->stream));
    return SG_OK;
}

static int aligned_in(sg_ctx *c, int s, const uint8_t *d, size_t n, const uint8_t **out) {
    if (((uintptr_t)d & 15) == 0) { *out = d; return SG_OK; }
    uint8_t *a;
    SG_TRY(slot(c, s, n + 16, &a));
    if (n) SG_HIP(hipMemcpyAsync(a, d, n, hipMemcpyDeviceToDevice, c->stream));
    *out = a;
    return SG_OK;
}

static int host_dedup_diff(const uint8_t *const *chunks, const size_t *lens, size_t k,
                           const uint8_t *prior, size_t n_prior, bool want_uniq, bool want_fresh,
                           uint8_t *uniq, size_t ucap, size_t *un, uint8_t *fresh, size_t fcap,
                           size_t *fn) {
    uint64_t n = 0;
    for (size_t i = 0; i < k; ++i) {
        if (!chunks[i] && lens[i]) { set_error("chunk %zu is NULL", i); return SG_E_INVAL; }
        n += lens[i];
    }
    if (n > MAX_BYTES || n_prior > MAX_BYTES) { set_error("input exceeds 4 GiB per call"); return SG_E_TOO_LARGE; }
    Acq a;
    SG_TRY(acquire(&a));
    sg_ctx *c = a.c;
    uint8_t *d_cur;
    SG_TRY(slot(c, S_IN, n + 16, &d_cur));
    uint64_t o = 0;
    for (size_t i = 0; i < k; ++i) {
        if (lens[i]) SG_HIP(hipMemcpyAsync(d_cur + o, chunks[i], lens[i], hipMemcpyHostToDevice, c->stream));
        o += lens[i];
    }
    uint8_t *d_prior = nullptr;
    if (want_fresh && n_prior) SG_TRY(upload(c, S_IN2, prior, n_prior, &d_prior));
    sg_dev_result r;
    SG_TRY(dev_dedup_diff(c, d_cur, n, d_prior, want_fresh ? n_prior : 0, want_fresh, &r));
    int rc = SG_OK;
    if (want_uniq) {
        *un = r.uniq_bytes;
        if (r.uniq_bytes > ucap) rc = SG_E_CAP;
    }
    if (want_fresh) {
        *fn = r.fresh_bytes;
        if (r.fresh_bytes > fcap) rc = SG_E_CAP;
    }
    if (rc == SG_E_CAP) { set_error("output capacity too small"); SG_HIP(hipStreamSynchronize(c->stream)); return rc; }
    if (want_uniq && r.uniq_bytes) SG_HIP(hipMemcpyAsync(uniq, r.uniq, r.uniq_bytes, hipMemcpyDeviceToHost, c->stream));
    if (want_fresh && r.fresh_bytes) SG_HIP(hipMemcpyAsync(fresh, r.fresh, r.fresh_bytes, hipMemcpyDeviceToHost, c->stream));
    SG_HIP(hipStreamSynchronize(c->stream));
    return SG_OK;
}

// Byte splitters packed for k_range_bytes: BE words of the first 64 bytes + lengths.
struct ByteSplit {
    uint64_t w[255 * SPL_WORDS];
    uint32_t len[256];
};

// Splitter q = splitters[split_offs[q] .. split_offs[q+1]) cut to SPL_W bytes, packed as BE
// words; the cut splitters must be non-decreasing in byte order.
static int pack_byte_splitters(const uint8_t *splitters, const uint32_t *split_offs, uint32_t n_parts, ByteSplit *bs) {
    memset(bs, 0, sizeof(*bs));
    for (uint32_t q = 0; q + 1 < n_parts; ++q) {
        if (split_offs[q + 1] < split_offs[q]) { set_error("split_offs must be non-decreasing"); return SG_E_INVAL; }
        const uint32_t len = std::min<uint32_t>(split_offs[q + 1] - split_offs[q], SPL_W);
        uint8_t b[SPL_W] = {0};
        memcpy(b, splitters + split_offs[q], len);
        for (uint32_t k = 0; k < SPL_WORDS; ++k) {
            uint64_t v = 0;
            for (uint32_t j = 0; j < 8; ++j) v = (v << 8) | b[8 * k + j];
            bs->w[q * SPL_WORDS + k] = v;
        }
        bs->len[q] = len;
        if (q > 0) {
            const uint64_t *a = bs->w + (q - 1) * SPL_WORDS, *w = bs->w + q * SPL_WORDS;
            int r = 0;
            for (uint32_t k = 0; k < SPL_WORDS && !r; ++k)
                if (a[k] != w[k]) r = a[k] < w[k] ? -1 : 1;
            if (r > 0 || (r == 0 && bs->len[q - 1] > len)) {
                set_error("splitters must be non-decreasing in byte order (splitter %u)", q);
                return SG_E_INVAL;
            }
        }
    }
    return SG_OK;
}

// Hash routing (split == null), range routing by key0 splitters, or by byte splitters
// (bsplit) — parts - 1 of them.
// ------------------------------------------------------------------ part multi-split
// Pass 2 of the piece partition, one tile of PT_TILE records per block (the piece's records in
// input order): each record's part (k_range_bytes' key), a stable rank by part inside the tile
// (8 wave64 ballots per item, as the radix downsweep), the records' bytes scanned in part
// order, and each record copied by its own lane to part base + tile offset + offset in the
// part's run — consecutive lanes write consecutive bytes of one part, and the reads stay
// inside the tile's ~100 KB of input. Replaces a radix sort of the record ids by part and one
// gather-emit per part (random 27-B reads: C5's part_emit ran at ~1.6 TB/s).
constexpr int PT_BLOCK = 256;
#ifndef SG_PT_ITEMS
#define SG_PT_ITEMS 2
#endif
#ifndef SG_PT_IMG
#define SG_PT_IMG 19456
#endif
constexpr int PT_ITEMS = SG_PT_ITEMS;
constexpr uint32_t PT_TILE = PT_BLOCK * PT_ITEMS;
constexpr uint32_t PT_IMG = SG_PT_IMG;  // LDS image of a tile's output (records of <= ~38 B on average)

// bytes (record + '\n') per (part, tile), part-major: cnt[q * ntiles + t]
// Optional span output of k_part_apply (sp null: none): rpre = exclusive prefix of the
// per-(part, tile) record counts (part-major), rbase[p] = index of part p's first record of
// this piece among all parts' records, pstart[p] = part p's start in the output.
// sums (optional, with sp): per (part, tile), part-major, the sum of the tile's span_mix terms
// of that part's records (the handover checksum, sg_span_sum), reduced per part by k_part_sums.
struct PartSpansOut {
    const uint64_t *rpre = nullptr, *rbase = nullptr, *pstart = nullptr;
    uint2 *sp = nullptr;
    uint64_t *keys = nullptr;
    uint64_t *sums = nullptr;
};

__global__ __launch_bounds__(PT_BLOCK) void k_part_count(const uint2 *__restrict__ spans, const uint8_t *__restrict__ part,
                                                          uint32_t R, uint32_t nparts, uint32_t ntiles,
                                                          uint32_t *__restrict__ cnt, uint32_t *__restrict__ rcnt) {
    __shared__ uint32_t s_b[256], s_r[256];
    s_b[threadIdx.x] = 0;
    s_r[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t t0 = blockIdx.x * PT_TILE;
#pragma unroll 4
    for (int j = 0; j < PT_ITEMS; ++j) {
        const uint32_t i = t0 + j * PT_BLOCK + threadIdx.x;
        if (i < R) {
            const uint2 x = spans[i];
            atomicAdd(&s_b[(uint32_t)part[i]], x.y - x.x + 1u);
            if (rcnt) atomicAdd(&s_r[(uint32_t)part[i]], 1u);
        }
    }
    __syncthreads();
    if (threadIdx.x < nparts) {
        cnt[(size_t)threadIdx.x * ntiles + blockIdx.x] = s_b[threadIdx.x];
        if (rcnt) rcnt[(size_t)threadIdx.x * ntiles + blockIdx.x] = s_r[threadIdx.x];
    }
}

// Per part q, this piece's record and byte totals from the per-(part, tile) counts and their
// exclusive scans (part-major): cnt[q] = records, cnt[nparts + q] = bytes.
__global__ __launch_bounds__(256) void k_part_totals(const uint32_t *__restrict__ pcnt, const uint64_t *__restrict__ ppre,
                                                     const uint32_t *__restrict__ rcnt, const uint64_t *__restrict__ rpre,
                                                     uint32_t nparts, uint32_t ntiles, unsigned long long *cnt) {
    const uint32_t q = threadIdx.x;
    if (q >= nparts) return;
    const size_t a = (size_t)q * ntiles, z = a + ntiles - 1;
    cnt[q] = rpre[z] + rcnt[z] - rpre[a];
    cnt[nparts + q] = ppre[z] + pcnt[z] - ppre[a];
}

// Part q's handover checksum over this piece's tiles (per-(part, tile) sums, part-major),
// added into tot[q]: block (x, q) sums tiles [x * PS_CHUNK, + PS_CHUNK) of part q's row.
constexpr uint32_t PS_CHUNK = 4096;
__global__ __launch_bounds__(256) void k_part_sums(const uint64_t *__restrict__ sums, uint32_t ntiles,
                                                   unsigned long long *__restrict__ tot) {
    __shared__ uint64_t s[4];
    const uint64_t *row = sums + (size_t)blockIdx.y * ntiles;
    const uint32_t t0 = blockIdx.x * PS_CHUNK, t1 = min(ntiles, t0 + PS_CHUNK);
    uint64_t v = 0;
    for (uint32_t t = t0 + threadIdx.x; t < t1; t += 256u) v += row[t];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += (uint64_t)__shfl_xor((long long)v, o, 64);
    if (lane_id() == 0) s[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(&tot[blockIdx.y], (unsigned long long)(s[0] + s[1] + s[2] + s[3]));
}

struct U32AsU64P {
    const uint32_t *v;
    __device__ uint64_t operator()(uint32_t i) const { return v[i]; }
};

// Bytes [lo, hi) of the 16-B aligned chunk at p, from v: whole dwords as dword stores, the
// partial ones as byte + 16-bit stores (a byte loop issued up to 15 byte stores).
__device__ __forceinline__ void put_chunk_part(uint8_t *p, const uint4 &v, uint32_t lo, uint32_t hi) {
    const uint32_t dw[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
        const uint32_t a = max(lo, 4u * k), e = min(hi, 4u * k + 4u);
        if (a >= e) continue;
        if (a == 4u * k && e == 4u * k + 4u) *reinterpret_cast<uint32_t *>(p + 4u * k) = dw[k];
        else put_edge(p + 4u * k, dw[k], a - 4u * k, e - 4u * k);
    }
}

// pre: exclusive prefix of cnt (flat, part-major); pbase[q]: where part q's bytes of this
// piece start in the output (null: a single buffer, parts back to back from offset 0).
__global__ __launch_bounds__(PT_BLOCK) void k_part_apply(const uint8_t *__restrict__ buf, const uint2 *__restrict__ spans,
                                                          const uint8_t *__restrict__ part, uint32_t R, uint32_t ntiles,
                                                          uint32_t nparts, const uint64_t *__restrict__ pre,
                                                          const uint64_t *__restrict__ pbase, uint8_t *__restrict__ out,
                                                          const PartSpansOut so) {
    constexpr int NW = PT_BLOCK / 64;
    __shared__ uint32_t s_dstart[256];
    __shared__ uint64_t s_dst[256];
    __shared__ uint64_t s_g0[256];
    __shared__ uint32_t s_rel0[256];  // span of sorted position q inside its part: s_rel0[part] + s_off[q]
    __shared__ uint32_t s_red[NW];
    __shared__ uint2 s_sp[PT_TILE];
    __shared__ uint32_t s_off[PT_TILE];
    __shared__ uint8_t s_pq[PT_TILE];  // part of each sorted position
    // the tile's output, part runs aligned as in `out`; before it is written, the ranking's
    // per-wave part counters (LDS per block decides the resident tiles per CU)
    __shared__ __attribute__((aligned(16))) uint8_t s_img[PT_IMG > NW * 1024 ? PT_IMG : NW * 1024];
    uint32_t(*s_wh)[256] = reinterpret_cast<uint32_t(*)[256]>(s_img);
    __shared__ uint32_t s_lp[256], s_le[256];  // image offset - tile offset of part p's run; its image end
    __shared__ uint32_t s_red2[NW];
    __shared__ uint64_t s_k0[PT_TILE];  // key0 of each sorted position (written out in sorted order)
    __shared__ uint64_t s_sum[256];     // per part: the tile's handover checksum terms
    const int tid = threadIdx.x, lane = lane_id(), wid = tid >> 6;
    if (so.sums) s_sum[tid] = 0;
    for (int x = tid; x < NW * 256; x += PT_BLOCK) (&s_wh[0][0])[x] = 0;
    const uint32_t tile = blockIdx.x, tbase = tile * PT_TILE;
    const uint32_t wbase = tbase + wid * (PT_ITEMS * 64);
    const uint64_t lt = (1ull << lane) - 1ull;
    // The tile's loads that need no ranking are issued here, before it: the per-part offsets
    // (thread p: part p) and each item's span (round 5 before: each behind a block phase).
    uint64_t p_pre = 0, p_pre0 = 0, p_pb = 0, p_r = 0, p_r0 = 0, p_rb = 0, p_ps = 0;
    if ((uint32_t)tid < nparts) {
        p_pre = pre[(size_t)tid * ntiles + tile];
        if (pbase) { p_pre0 = pre[(size_t)tid * ntiles]; p_pb = pbase[tid]; }
        if (so.sp) {
            p_r = so.rpre[(size_t)tid * ntiles + tile];
            p_r0 = so.rpre[(size_t)tid * ntiles];
            p_rb = so.rbase[tid];
            p_ps = so.pstart[tid];
        }
    }
    uint32_t d[PT_ITEMS], r[PT_ITEMS];
    uint2 sp[PT_ITEMS];
#pragma unroll
    for (int i = 0; i < PT_ITEMS; ++i) {
        const uint32_t pos = wbase + i * 64 + lane;
        d[i] = pos < R ? (uint32_t)part[pos] : 0u;
        sp[i] = pos < R ? spans[pos] : make_uint2(0u, 0u);
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < PT_ITEMS; ++i) {
        const bool valid = (wbase + i * 64 + lane) < R;
        uint64_t m = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const uint64_t bb = __ballot((d[i] >> b) & 1u);
            m &= ((d[i] >> b) & 1u) ? bb : ~bb;
        }
        const uint32_t ltc = (uint32_t)__popcll(m & lt);
        const uint32_t c = s_wh[wid][d[i]];
        r[i] = c + ltc;
        if (valid && ltc == 0) s_wh[wid][d[i]] = c + (uint32_t)__popcll(m);
    }
    __syncthreads();
    uint32_t run = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) { const uint32_t x = s_wh[w][tid]; s_wh[w][tid] = run; run += x; }
    uint32_t tot;
    const uint32_t dstart = block_excl_scan<PT_BLOCK>(run, &tot, s_red);
    s_dstart[tid] = dstart;
    s_dst[tid] = 0;
    __syncthreads();
    uint32_t qi[PT_ITEMS];
#pragma unroll
    for (int i = 0; i < PT_ITEMS; ++i) {
        const uint32_t pos = wbase + i * 64 + lane;
        qi[i] = s_dstart[d[i]] + s_wh[wid][d[i]] + r[i];
        if (pos < R) {
            s_sp[qi[i]] = sp[i];
            s_pq[qi[i]] = (uint8_t)d[i];
        }
    }
    __syncthreads();
    // bytes in part order: thread tid scans sorted positions tid*PT_ITEMS .. + PT_ITEMS - 1
    const uint32_t n_t = min(PT_TILE, R - tbase);
    uint32_t ln[PT_ITEMS], sum = 0;
#pragma unroll
    for (int j = 0; j < PT_ITEMS; ++j) {
        const uint32_t q = tid * PT_ITEMS + j;
        ln[j] = q < n_t ? s_sp[q].y - s_sp[q].x + 1u : 0u;
        sum += ln[j];
    }
    uint32_t btot;
    uint32_t o = block_excl_scan<PT_BLOCK>(sum, &btot, s_red);
#pragma unroll
    for (int j = 0; j < PT_ITEMS; ++j) { s_off[tid * PT_ITEMS + j] = o; o += ln[j]; }
    __syncthreads();
    // destination of each part's run: its piece base + this tile's prefix inside the part,
    // minus the tile-local byte offset where the part's run starts
    const bool present = (uint32_t)tid < nparts && s_dstart[tid] < n_t && (tid == 255 || s_dstart[tid + 1] > s_dstart[tid]);
    uint32_t npresent;
    const uint32_t prank = block_excl_scan<PT_BLOCK>(present ? 1u : 0u, &npresent, s_red2);
    // the tile's output assembled in LDS when it fits: part p's run at image offset l_p with
    // l_p = its global address mod 16 (runs in part order, at most 15 bytes apart)
    const bool use_img = btot + 16u * npresent <= PT_IMG;  // block-uniform
    if (present) {
        // pbase null: one buffer, parts in part order (pre is already the global offset)
        const uint32_t o_s = s_off[s_dstart[tid]];
        const uint32_t e = tid == 255 ? n_t : s_dstart[tid + 1];
        const uint32_t o_e = e < n_t ? s_off[e] : btot;
        const uint64_t g = p_pb + (p_pre - p_pre0);  // the run's first byte in out
        s_dst[tid] = g - o_s;
        const uint32_t S = o_s + 16u * prank;
        const uint32_t l = S + (((uint32_t)((uintptr_t)out + g) - S) & 15u);
        s_lp[tid] = l - o_s;
        s_le[tid] = l + (o_e - o_s);
        if (so.sp) {  // record index of sorted position q = s_g0[part] + q; span base = part start
            s_g0[tid] = p_rb + (p_r - p_r0) - s_dstart[tid];
            s_rel0[tid] = (uint32_t)(s_dst[tid] - p_ps);
        }
    }
    __syncthreads();
    auto finish = [&](uint32_t q, uint32_t lo, uint2 x, uint64_t k0) {
        if (so.sp) {  // also the record's span inside its part and its key, at its index in the parts
            const uint64_t g = s_g0[lo] + q;
            const uint32_t rel = s_rel0[lo] + s_off[q];
            so.sp[g] = make_uint2(rel, rel + (x.y - x.x));
            so.keys[g] = k0;
        }
    };
    if (!use_img) {  // long records: each lane stores its own record
        for (uint32_t q = tid; q < n_t; q += PT_BLOCK) {
            const uint32_t lo = s_pq[q];
            const uint2 x = s_sp[q];
            const uint64_t dst = s_dst[lo] + s_off[q];
            uint64_t k0 = 0;
            if (so.sp) put_medium<true, true>(buf, out + (dst & ~3ull), (uint32_t)(dst & 3u), x.x, x.y - x.x, &k0);
            else put_medium<false, true>(buf, out + (dst & ~3ull), (uint32_t)(dst & 3u), x.x, x.y - x.x);
            finish(q, lo, x, k0);
            if (so.sums) atomicAdd((unsigned long long *)&s_sum[lo], (unsigned long long)span_mix(x.y - x.x, k0));
        }
        if (so.sums) {
            __syncthreads();
            if ((uint32_t)tid < nparts) so.sums[(size_t)tid * ntiles + tile] = s_sum[tid];
        }
        return;
    }
    // Each lane places its own records in the image (LDS stores), then every 16-B chunk of a
    // part run leaves as one aligned 16-B store, by the lane whose sorted position holds the
    // chunk's first byte: consecutive lanes store consecutive chunks (a lane-per-record global
    // copy issued 16/8/4-byte, 16-bit and byte stores at every record's own alignment). The
    // spans and keys leave in sorted order too (consecutive lanes, consecutive slots).
#pragma unroll
    for (int i = 0; i < PT_ITEMS; ++i) {
        if (wbase + i * 64 + lane >= R) continue;
        const uint32_t q = qi[i], lo = d[i];
        const uint2 x = sp[i];
        const uint32_t li = s_lp[lo] + s_off[q];
        uint64_t k0 = 0;
        if (so.sp) put_medium<true, false>(buf, s_img, li, x.x, x.y - x.x, &k0);
        else put_medium<false, false>(buf, s_img, li, x.x, x.y - x.x);
        if (so.sp) s_k0[q] = k0;
        if (so.sums) atomicAdd((unsigned long long *)&s_sum[lo], (unsigned long long)span_mix(x.y - x.x, k0));
    }
    __syncthreads();
    if (so.sums && (uint32_t)tid < nparts) so.sums[(size_t)tid * ntiles + tile] = s_sum[tid];
    for (uint32_t q = tid; q < n_t; q += PT_BLOCK) {
        const uint32_t lo = s_pq[q];
        const uint2 x = s_sp[q];
        const uint32_t li = s_lp[lo] + s_off[q], le = li + (x.y - x.x) + 1u;  // the record's image bytes
        const uint32_t pe = s_le[lo];                                          // its run's image end
        uint8_t *g = out + (s_dst[lo] - s_lp[lo]);                             // image offset b -> g + b
        if (so.sp) {  // the record's span inside its part and its key, at its index in the parts
            const uint64_t gi = s_g0[lo] + q;
            const uint32_t rel = s_rel0[lo] + s_off[q];
            so.sp[gi] = make_uint2(rel, rel + (x.y - x.x));
            so.keys[gi] = s_k0[q];
        }
        if (q == s_dstart[lo] && (li & 15u)) {  // the run's unaligned head
            const uint32_t hb = li & ~15u;
            put_chunk_part(g + hb, *reinterpret_cast<const uint4 *>(s_img + hb), li - hb, min(16u, pe - hb));
        }
        for (uint32_t b = (li + 15u) & ~15u; b < le; b += 16u) {
            const uint4 v = *reinterpret_cast<const uint4 *>(s_img + b);
            if (b + 16u <= pe) *reinterpret_cast<uint4 *>(g + b) = v;
            else put_chunk_part(g + b, v, 0u, pe - b);  // the run's tail (the next tile's run shares the chunk)
        }
    }
}

// Spans received from several sources (a multi-GPU exchange round: each source's spans are
// relative to the start of its own bytes) rebased to the receive buffer: records
// [first[s], first[s + 1]) get + off[s]. The transfer is checked on the first and last
// SG_REBASE_CHECK records of every source: each must end right before a '\n' of the buffer
// (the routing wrote every record '\n'-terminated), so a message that arrived short or
// stale (this image's RCCL left the upper half of a 1.5 GB message unwritten) is reported in
// *bad instead of deduped — without reading every record's bytes (a per-record check touched
// the whole buffer: 8.7 ms per 1B records).
constexpr uint32_t SG_REBASE_CHECK = 256;
struct RebaseSegs {
    uint32_t first[SG_REBASE_SEGS + 1];
    uint32_t off[SG_REBASE_SEGS];
    uint32_t nseg;
};

__device__ __forceinline__ bool span_ends_at_nl(uint2 x, const uint8_t *__restrict__ buf, uint32_t n) {
    return x.x <= x.y && x.y < n && buf[x.y] == 0x0a;
}

// every record of one batch of sources (records [sg_.first[0], sg_.first[nseg])) rebased; the
// sampled ones checked
__global__ __launch_bounds__(256) void k_rebase_spans(uint2 *__restrict__ sp, const uint8_t *__restrict__ buf,
                                                      uint32_t n, const RebaseSegs sg_, unsigned long long *__restrict__ bad) {
    const uint32_t i = sg_.first[0] + blockIdx.x * 256u + threadIdx.x;
    bool ok = true;
    if (i < sg_.first[sg_.nseg]) {
        uint32_t lo = 0, hi = sg_.nseg;  // last segment whose first record <= i
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (sg_.first[mid] <= i) lo = mid; else hi = mid;
        }
        uint2 x = sp[i];
        const uint32_t o = sg_.off[lo];
        x.x += o;
        x.y += o;
        sp[i] = x;
        if (i - sg_.first[lo] < SG_REBASE_CHECK || sg_.first[lo + 1] - i <= SG_REBASE_CHECK) ok = span_ends_at_nl(x, buf, n);
    }
    const uint64_t m = __ballot(!ok);
    if (m && lane_id() == 0) atomicAdd(bad, (unsigned long long)__popcll(m));
}

// spans already relative to the buffer (one source at offset 0): the sampled records only
__global__ __launch_bounds__(256) void k_check_spans(const uint2 *__restrict__ sp, const uint8_t *__restrict__ buf, uint32_t n,
                                                     const RebaseSegs sg_, unsigned long long *__restrict__ bad) {
    const uint32_t t = blockIdx.x * 256u + threadIdx.x;
    const uint32_t s = t / (2 * SG_REBASE_CHECK), j = t % (2 * SG_REBASE_CHECK);
    bool ok = true;
    if (s < sg_.nseg) {
        const uint32_t a = sg_.first[s], e = sg_.first[s + 1];
        const uint32_t i = j < SG_REBASE_CHECK ? a + j : e - (2 * SG_REBASE_CHECK - j);
        if (i >= a && i < e && (j < SG_REBASE_CHECK || e - a > SG_REBASE_CHECK)) ok = span_ends_at_nl(sp[i], buf, n);
    }
    const uint64_t m = __ballot(!ok);
    if (m && lane_id() == 0) atomicAdd(bad, (unsigned long long)__popcll(m));
}

int dev_partition(sg_ctx *c, const uint8_t *d_buf, uint64_t n, uint32_t parts, uint8_t *d_out,
                  size_t out_cap, uint64_t *part_bytes, uint64_t *part_records, const uint64_t *split = nullptr,
                  const ByteSplit *bsplit = nullptr) {
    if (parts == 0 || parts > 256) { set_error("n_parts must be in 1..256"); return SG_E_INVAL; }
    if (split)
        for (uint32_t q = 1; q + 1 < parts; ++q)
            if (split[q] < split[q - 1]) { set_error("splitters must be non-decreasing"); return SG_E_INVAL; }
    Lines L;
    SG_TRY(run_lines(c, d_buf, n, CUR_SLOTS, &L));
    const uint32_t R = L.n_rec;
    unsigned long long *cnt;
    SG_TRY(slot(c, S_M_CNT, 2 * 256, &cnt));
    SG_HIP(hipMemsetAsync(cnt, 0, 2 * 256 * 8, c->stream));
    uint8_t *keys;  // part of each record
    SG_TRY(slot(c, S_KEYS2, R, &keys));
    if (R && bsplit) {
        uint64_t *d_w;
        SG_TRY(slot(c, S_M_TMP2, sizeof(ByteSplit) / 8, &d_w));
        SG_HIP(hipMemcpyAsync(d_w, bsplit, sizeof(ByteSplit), hipMemcpyHostToDevice, c->stream));
        SG_LAUNCH_B(c, "range_bytes", 24.0 * R, k_range_bytes, std::min<uint32_t>((R + 255) / 256, 2048u), 256, 0, d_buf,
                    L.spans, R, d_w, reinterpret_cast<const uint32_t *>(d_w + 255 * SPL_WORDS), parts - 1, keys, cnt);
    } else if (R && !split) {
        SG_LAUNCH(c, "part_keys", k_part_keys, std::min<uint32_t>((R + 255) / 256, 2048u), 256, 0, d_buf, L.spans, R,
                  parts, keys, cnt);
    } else if (R) {
        uint64_t *d_split;
        SG_TRY(slot(c, S_M_TMP2, 256, &d_split));
        if (parts > 1) SG_HIP(hipMemcpyAsync(d_split, split, 8 * (parts - 1), hipMemcpyHostToDevice, c->stream));
        SG_LAUNCH_B(c, "range_keys", 24.0 * R, k_range_keys, std::min<uint32_t>((R + 255) / 256, 2048u), 256, 0, L.keys, L.spans, R,
                  d_split, parts - 1, keys, cnt);
    }
    // the multi-split: per-tile part byte counts, their scan (= each part's offset in the
    // output), every record copied straight to its place (no sort of ids by part, no gather)
    if (R) {
        if (out_cap < n + 1) { set_error("output capacity %zu < %llu", out_cap, (unsigned long long)(n + 1)); return SG_E_CAP; }
        const uint32_t ntiles = (R + PT_TILE - 1) / PT_TILE;
        const size_t nflat = (size_t)parts * ntiles;
        uint32_t *pcnt;
        uint64_t *ppre;
        SG_TRY(slot(c, S_PT_CNT, nflat, &pcnt));
        SG_TRY(slot(c, S_PT_PRE, nflat, &ppre));
        SG_LAUNCH_B(c, "part_count", 16.0 * R, k_part_count, ntiles, PT_BLOCK, 0, L.spans, keys, R, parts, ntiles, pcnt,
                    (uint32_t *)nullptr);
        const uint32_t nt = (uint32_t)((nflat + SCAN_TILE - 1) / SCAN_TILE);
        uint64_t *tp;
        SG_TRY(slot(c, S_TILES, 2 * (size_t)nt + 4, &tp));
        SG_LAUNCH(c, "scan.count", k_scan64_count<U32AsU64P>, nt, SCAN_BLOCK, 0, U32AsU64P{pcnt}, (uint32_t)nflat, tp);
        SG_TRY(tile_scan(c, tp, nt, tp + nt, tp + 2 * (size_t)nt));
        SG_LAUNCH(c, "scan.apply", k_scan64_apply<U32AsU64P>, nt, SCAN_BLOCK, 0, U32AsU64P{pcnt}, (uint32_t)nflat, tp + nt, ppre);
        SG_LAUNCH_B(c, "part_emit", 16.0 * R + 2.0 * (double)n, k_part_apply, ntiles, PT_BLOCK, 0, d_buf, L.spans, keys, R,
                    ntiles, parts, ppre, (const uint64_t *)nullptr, d_out, PartSpansOut{});
    }
    uint64_t h[2 * 256];
    SG_TRY(ctx_readback(c, h, cnt, 2 * parts * 8));
    for (uint32_t q = 0; q < parts; ++q) {
        if (part_records) part_records[q] = h[q];
        if (part_bytes) part_bytes[q] = h[parts + q];
    }
    return SG_OK;
}

}  // namespace sg

using namespace sg;

extern "C" {

uint64_t sg_hash64(const uint8_t *rec, size_t len) {
    return hash_words([&](uint32_t j) { return rec[j]; }, (uint32_t)len);
}

uint64_t sg_span_sum(const uint32_t *spans, const uint64_t *keys, size_t n_rec) {
    uint64_t s = 0;
    for (size_t i = 0; i < n_rec; ++i) s += span_mix(spans[2 * i + 1] - spans[2 * i], keys[i]);
    return s;
}

int sg_lines(const uint8_t *buf, size_t n, uint64_t *spans, size_t cap, size_t *n_rec) {
    if ((!buf && n) || !n_rec) { set_error("sg_lines: bad arguments"); return SG_E_INVAL; }
    if (n > MAX_BYTES) { set_error("input exceeds 4 GiB per call"); return SG_E_TOO_LARGE; }
    Acq a;
    SG_TRY(acquire(&a));
    sg_ctx *c = a.c;
    uint8_t *d;
    SG_TRY(upload(c, S_IN, buf, n, &d));
    Lines L;
    SG_TRY(run_lines(c, d, n, CUR_SLOTS, &L));
    *n_rec = L.n_rec;
    if (L.n_rec > cap) { set_error("span capacity too small"); return SG_E_CAP; }
    std::vector<uint2> sp(L.n_rec);
    if (L.n_rec) SG_HIP(hipMemcpyAsync(sp.data(), L.spans, L.n_rec * 8ull, hipMemcpyDeviceToHost, c->stream));
    SG_HIP(hipStreamSynchronize(c->stream));
    for (uint32_t i = 0; i < L.n_rec; ++i) { spans[2 * i] = sp[i].x; spans[2 * i + 1] = sp[i].y; }
    return SG_OK;
}

int sg_dedup(const uint8_t *buf, size_t n, uint8_t *out, size_t cap, size_t *out_n) {
    if ((!buf && n) || !out_n) { set_error("sg_dedup: bad arguments"); return SG_E_INVAL; }
    const uint8_t *ch[1] = {buf};
    size_t ln[1] = {n};
    return host_dedup_diff(ch, ln, 1, nullptr, 0, true, false, out, cap, out_n, nullptr, 0, nullptr);
}

int sg_dedup_chunks(const uint8_t *const *chunks, const size_t *lens, size_t k, uint8_t *out, size_t cap,
                    size_t *out_n) {
    if ((!chunks && k) || (!lens && k) || !out_n) { set_error("sg_dedup_chunks: bad arguments"); return SG_E_INVAL; }
    return host_dedup_diff(chunks, lens, k, nullptr, 0, true, false, out, cap, out_n, nullptr, 0, nullptr);
}

int sg_diff(const uint8_t *cur, size_t n_cur, const uint8_t *prior, size_t n_prior, uint8_t *out, size_t cap,
            size_t *out_n) {
    if ((!cur && n_cur) || (!prior && n_prior) || !out_n) { set_error("sg_diff: bad arguments"); return SG_E_INVAL; }
    const uint8_t *ch[1] = {cur};
    size_t ln[1] = {n_cur};
    return host_dedup_diff(ch, ln, 1, prior, n_prior, false, true, nullptr, 0, nullptr, out, cap, out_n);
}

int sg_dedup_diff(const uint8_t *cur, size_t n_cur, const uint8_t *prior, size_t n_prior, uint8_t *uniq,
                  size_t uniq_cap, size_t *uniq_n, uint8_t *fresh, size_t fresh_cap, size_t *fresh_n) {
    if ((!cur && n_cur) || (!prior && n_prior) || !uniq_n || !fresh_n) { set_error("sg_dedup_diff: bad arguments"); return SG_E_INVAL; }
    const uint8_t *ch[1] = {cur};
    size_t ln[1] = {n_cur};
    return host_dedup_diff(ch, ln, 1, prior, n_prior, true, true, uniq, uniq_cap, uniq_n, fresh, fresh_cap, fresh_n);
}

int sg_dev_dedup_diff(sg_ctx *c, const uint8_t *d_cur, size_t n_cur, const uint8_t *d_prior, size_t n_prior,
                      sg_dev_result *res) {
    if (!c || !res || (!d_cur && n_cur) || (!d_prior && n_prior)) { set_error("sg_dev_dedup_diff: bad arguments"); return SG_E_INVAL; }
    SG_HIP(hipSetDevice(c->device));
    const uint8_t *cur, *prior = nullptr;
    SG_TRY(aligned_in(c, S_IN, d_cur, n_cur, &cur));
    if (n_prior) SG_TRY(aligned_in(c, S_IN2, d_prior, n_prior, &prior));
    return dev_dedup_diff(c, cur, n_cur, prior, n_prior, true, res);
}

int sg_dev_dedup_diff_into(sg_ctx *c, const uint8_t *d_cur, size_t n_cur, const uint8_t *d_prior, size_t n_prior,
                           uint8_t *d_uniq, size_t uniq_cap, uint8_t *d_fresh, size_t fresh_cap, sg_dev_result *res) {
    if (!c || !res || (!d_cur && n_cur) || (!d_prior && n_prior) || !d_uniq) {
        set_error("sg_dev_dedup_diff_into: bad arguments");
        return SG_E_INVAL;
    }
    if (n_cur > MAX_BYTES || n_prior > MAX_BYTES) { set_error("input exceeds 4 GiB per call"); return SG_E_TOO_LARGE; }
    SG_HIP(hipSetDevice(c->device));
    const uint8_t *cur, *prior = nullptr;
    SG_TRY(aligned_in(c, S_IN, d_cur, n_cur, &cur));
    if (n_prior) SG_TRY(aligned_in(c, S_IN2, d_prior, n_prior, &prior));
    return dev_dedup_diff_into(c, cur, n_cur, prior, n_prior, d_uniq, uniq_cap, d_fresh, fresh_cap, res);
}

int sg_dev_partition_range(sg_ctx *c, const uint8_t *d_buf, size_t n, const uint64_t *splitters, uint32_t n_parts,
                           uint8_t *d_out, size_t out_cap, uint64_t *part_bytes, uint64_t *part_records) {
    if (!c || (!d_out && n) || (!d_buf && n) || (!splitters && n_parts > 1)) {
        set_error("sg_dev_partition_range: bad arguments");
        return SG_E_INVAL;
    }
    if (n > MAX_BYTES) { set_error("input exceeds 4 GiB per call"); return SG_E_TOO_LARGE; }
    SG_HIP(hipSetDevice(c->device));
    const uint8_t *b;
    SG_TRY(aligned_in(c, S_IN, d_buf, n, &b));
    static const uint64_t none = 0;
    return dev_partition(c, b, n, n_parts, d_out, out_cap, part_bytes, part_records, n_parts > 1 ? splitters : &none);
}

int sg_dev_partition_bytes(sg_ctx *c, const uint8_t *d_buf, size_t n, const uint8_t *splitters,
                           const uint32_t *split_offs, uint32_t n_parts, uint8_t *d_out, size_t out_cap,
                           uint64_t *part_bytes, uint64_t *part_records) {
    if (!c || (!d_out && n) || (!d_buf && n) || ((!splitters || !split_offs) && n_parts > 1)) {
        set_error("sg_dev_partition_bytes: bad arguments");
        return SG_E_INVAL;
    }
    if (n_parts == 0 || n_parts > 256) { set_error("n_parts must be in 1..256"); return SG_E_INVAL; }
    if (n > MAX_BYTES) { set_error("input exceeds 4 GiB per call"); return SG_E_TOO_LARGE; }
    static thread_local ByteSplit bs;
    SG_TRY(pack_byte_splitters(splitters, split_offs, n_parts, &bs));
    SG_HIP(hipSetDevice(c->device));
    const uint8_t *b;
    SG_TRY(aligned_in(c, S_IN, d_buf, n, &b));
    return dev_partition(c, b, n, n_parts, d_out, out_cap, part_bytes, part_records, nullptr, &bs);
}

}  // extern "C"

// a16: part q starts at the 16-byte aligned offset after part q - 1 (parts usable in place
// by the dedup, which takes 16-byte aligned buffers).
// rounds > 1 (multi-GPU exchange rounds): n_parts = G x rounds, part q = g * rounds + p is
// range p of rank g, and the parts are laid out round-major: round p's parts (0, p), (1, p),
// ..., (G - 1, p) back to back (one contiguous all-to-all send buffer per round), each round
// starting at a 16-byte aligned offset.
// Pass 0 of the piece partition: every piece's record count (count pass + tile scan per
// piece into slot S_PT_LTP, one read-back). Kept in c->pt_prep for the next partition call on
// the same pieces (sg_dev_partition_pieces_count: the caller sizes its span buffers first).
// prep: the context's kept pass 0 may be used (taken, and cleared, by the caller on entry, so
// a call that fails before reaching here never leaves it for a later one).
static int pieces_pass0(sg_ctx *c, const uint8_t *const *d_pieces, const size_t *lens, size_t k,
                        std::vector<uint32_t> &lnt, std::vector<size_t> &loff, uint64_t **ltp_out,
                        std::vector<uint32_t> &Rj, bool prep) {
    lnt.assign(k, 0);
    loff.assign(k, 0);
    Rj.assign(k, 0);
    size_t ltot = 0;
    for (size_t j = 0; j < k; ++j) {
        if (!lens[j]) continue;
        lnt[j] = lines_tiles(lens[j]);
        loff[j] = ltot;
        ltot += 2 * (size_t)lnt[j] + 4;
    }
    uint64_t *ltp = nullptr;
    if (ltot) SG_TRY(slot(c, S_PT_LTP, ltot, &ltp));
    *ltp_out = ltp;
    auto &P = c->pt_prep;
    if (prep && P.ptrs.size() == k && std::equal(P.lens.begin(), P.lens.end(), lens) &&
        std::equal(P.ptrs.begin(), P.ptrs.end(), d_pieces)) {
        Rj = P.Rj;  // the counts and tile scans of sg_dev_partition_pieces_count
        return SG_OK;
    }
    uint8_t *pin = (uint8_t *)c->pinned;
    if (8 * k > SG_PINNED_BYTES) { set_error("partition: %zu pieces exceed the read-back staging", k); return SG_E_INVAL; }
    // (a piece that is not 16-byte aligned is copied to the aligned staging slot before each
    // of its passes: the slot holds one piece at a time)
    for (size_t j = 0; j < k; ++j) {
        if (!lens[j]) continue;
        const uint8_t *pb = nullptr;
        SG_TRY(aligned_in(c, S_IN, d_pieces[j], lens[j], &pb));
        SG_TRY(lines_count_scan(c, pb, lens[j], ltp + loff[j]));
        SG_HIP(hipMemcpyAsync(pin + 8 * j, ltp + loff[j] + 2 * (size_t)lnt[j], 8, hipMemcpyDeviceToHost, c->stream));
    }
    SG_HIP(hipStreamSynchronize(c->stream));
    for (size_t j = 0; j < k; ++j) {
        if (!lens[j]) continue;
        uint64_t tv;
        memcpy(&tv, pin + 8 * j, 8);
        Rj[j] = (uint32_t)(tv >> 31);
        if (Rj[j] != (uint32_t)(tv & 0x7fffffffu)) { set_error("run_lines: start/end count mismatch"); return SG_E_HIP; }
    }
    return SG_OK;
}

// user_sp / user_k (rec_cap records): the span and key outputs in caller buffers (any
// rounds), records in the same part order as the bytes (round-major with rounds > 1).
static int partition_pieces(sg_ctx *c, const uint8_t *const *d_pieces, const size_t *lens, size_t k,
                            const uint8_t *splitters, const uint32_t *split_offs, uint32_t n_parts, uint8_t *d_out,
                            size_t out_cap, uint64_t *part_bytes, uint64_t *part_records, bool a16,
                            const uint2 **sp_out = nullptr, const uint64_t **k_out = nullptr, uint32_t rounds = 1,
                            uint2 *user_sp = nullptr, uint64_t *user_k = nullptr, size_t rec_cap = 0,
                            uint64_t *part_sums = nullptr) {
    // the kept pass 0 of sg_dev_partition_pieces_count serves this call only, whatever happens
    const bool prep = c && c->pt_prep.on;
    if (c) c->pt_prep.on = false;
    if (!c || (k && (!d_pieces || !lens)) || ((!splitters || !split_offs) && n_parts > 1)) {
        set_error("sg_dev_partition_bytes_pieces: bad arguments");
        return SG_E_INVAL;
    }
    if (n_parts == 0 || n_parts > 256) { set_error("n_parts must be in 1..256"); return SG_E_INVAL; }
    if (rounds == 0 || n_parts % rounds || (rounds > 1 && sp_out)) {
        set_error("n_parts (%u) must be a multiple of rounds (%u)", n_parts, rounds);
        return SG_E_INVAL;
    }
    if ((user_sp != nullptr) != (user_k != nullptr)) { set_error("partition: span and key buffers go together"); return SG_E_INVAL; }
    uint64_t total_in = 0;
    for (size_t j = 0; j < k; ++j) {
        if (!d_pieces[j] && lens[j]) { set_error("piece %zu is NULL", j); return SG_E_INVAL; }
        if (lens[j] > MAX_BYTES) { set_error("piece %zu exceeds 4 GiB", j); return SG_E_TOO_LARGE; }
        total_in += lens[j];
    }
    if (total_in && !d_out) { set_error("sg_dev_partition_bytes_pieces: d_out is NULL"); return SG_E_INVAL; }
    static thread_local ByteSplit bs;
    SG_TRY(pack_byte_splitters(splitters, split_offs, n_parts, &bs));
    SG_HIP(hipSetDevice(c->device));
    const uint32_t ns = n_parts - 1;
    uint64_t *d_w;
    SG_TRY(slot(c, S_M_TMP2, sizeof(ByteSplit) / 8, &d_w));
    SG_HIP(hipMemcpyAsync(d_w, &bs, sizeof(ByteSplit), hipMemcpyHostToDevice, c->stream));
    const uint32_t *d_len = reinterpret_cast<const uint32_t *>(d_w + 255 * SPL_WORDS);
    // pass 0: every piece's record count (count pass + tile scan per piece), one read-back
    std::vector<const uint8_t *> pb_in(k, nullptr);
    std::vector<uint32_t> lnt, Rj;
    std::vector<size_t> loff;
    uint64_t *ltp = nullptr;
    SG_TRY(pieces_pass0(c, d_pieces, lens, k, lnt, loff, &ltp, Rj, prep));
    std::vector<uint64_t> roff(k, 0);
    uint64_t all_rec = 0;
    for (size_t j = 0; j < k; ++j) {
        roff[j] = all_rec;
        all_rec += Rj[j];
    }
    // pass 1 per piece: parse + route (spans and a part byte per record, kept for pass 2),
    // the per-(part, tile) byte and record counts and their scans (kept per piece), and the
    // piece's per-part totals; one read-back of all pieces' totals
    uint2 *keep_sp;
    uint8_t *keep_k;
    SG_TRY(slot(c, S_PT_SP, all_rec + 1, &keep_sp));
    SG_TRY(slot(c, S_PT_KEYS, all_rec + 16, &keep_k));
    std::vector<uint32_t> ptn(k, 0);
    std::vector<size_t> poff(k, 0);
    size_t ptot = 0;
    for (size_t j = 0; j < k; ++j) {
        if (!Rj[j]) continue;
        ptn[j] = (Rj[j] + PT_TILE - 1) / PT_TILE;
        poff[j] = ptot;
        ptot += (size_t)n_parts * ptn[j];
    }
    uint32_t *pcnt_all = nullptr, *rcnt_all = nullptr;
    uint64_t *ppre_all = nullptr, *rpre_all = nullptr;
    if (ptot) {
        SG_TRY(slot(c, S_PT_CNT, 2 * ptot, &pcnt_all));
        SG_TRY(slot(c, S_PT_PRE, 2 * ptot, &ppre_all));
        rcnt_all = pcnt_all + ptot;
        rpre_all = ppre_all + ptot;
    }
    unsigned long long *cnt;
    SG_TRY(slot(c, S_PART, (size_t)std::max<size_t>(k, 1) * 512, &cnt));
    SG_HIP(hipMemsetAsync(cnt, 0, std::max<size_t>(k, 1) * 512 * 8, c->stream));
    for (size_t j = 0; j < k; ++j) {
        if (!Rj[j]) continue;
        SG_TRY(aligned_in(c, S_IN, d_pieces[j], lens[j], &pb_in[j]));
        SG_TRY(lines_route_apply(c, pb_in[j], lens[j], ltp + loff[j], Rj[j], keep_sp + roff[j], d_w, d_len, ns,
                                 keep_k + roff[j]));
        const uint32_t ntiles = ptn[j];
        const size_t nflat = (size_t)n_parts * ntiles;
        uint32_t *pcnt = pcnt_all + poff[j], *rcnt = rcnt_all + poff[j];
        uint64_t *ppre = ppre_all + poff[j], *rpre = rpre_all + poff[j];
        SG_LAUNCH_B(c, "part_count", 9.0 * Rj[j], k_part_count, ntiles, PT_BLOCK, 0, keep_sp + roff[j], keep_k + roff[j],
                    Rj[j], n_parts, ntiles, pcnt, rcnt);
        const uint32_t nt = (uint32_t)((nflat + SCAN_TILE - 1) / SCAN_TILE);
        uint64_t *tp;
        SG_TRY(slot(c, S_TILES, 2 * (size_t)nt + 4, &tp));
        for (int pass = 0; pass < 2; ++pass) {
            const U32AsU64P src{pass ? rcnt : pcnt};
            SG_LAUNCH(c, "scan.count", k_scan64_count<U32AsU64P>, nt, SCAN_BLOCK, 0, src, (uint32_t)nflat, tp);
            SG_TRY(tile_scan(c, tp, nt, tp + nt, tp + 2 * (size_t)nt));
            SG_LAUNCH(c, "scan.apply", k_scan64_apply<U32AsU64P>, nt, SCAN_BLOCK, 0, src, (uint32_t)nflat, tp + nt,
                      pass ? rpre : ppre);
        }
        SG_LAUNCH(c, "part_totals", k_part_totals, 1, 256, 0, pcnt, ppre, rcnt, rpre, n_parts, ntiles, cnt + 512 * j);
    }
    std::vector<uint64_t> h(std::max<size_t>(k, 1) * 512, 0);
    SG_TRY(ctx_readback(c, h.data(), cnt, h.size() * 8));
    // destinations: part p = pieces' part-p records in piece order
    std::vector<uint64_t> pbase(n_parts, 0), pbytes(n_parts, 0), prec(n_parts, 0);
    for (uint32_t q = 0; q < n_parts; ++q)
        for (size_t j = 0; j < k; ++j) { prec[q] += h[512 * j + q]; pbytes[q] += h[512 * j + n_parts + q]; }
    uint64_t end = 0;
    if (rounds > 1) {
        const uint32_t G = n_parts / rounds;
        for (uint32_t p = 0; p < rounds; ++p) {
            end = (end + 15) & ~15ull;
            for (uint32_t g = 0; g < G; ++g) {
                pbase[g * rounds + p] = end;
                end += pbytes[g * rounds + p];
            }
        }
    } else {
        for (uint32_t q = 0; q < n_parts; ++q) {
            pbase[q] = end;
            end += pbytes[q];
            if (a16 && q + 1 < n_parts) end = (end + 15) & ~15ull;
        }
    }
    if (end > out_cap) {
        set_error("output capacity %zu < %llu", out_cap, (unsigned long long)end);
        return SG_E_CAP;
    }
    for (uint32_t q = 0; q < n_parts; ++q) {
        if (part_bytes) part_bytes[q] = pbytes[q];
        if (part_records) part_records[q] = prec[q];
    }
    // destinations of every (piece, part): part q's bytes of piece j follow those of pieces
    // 0..j-1
    std::vector<uint64_t> acc(pbase);
    std::vector<uint64_t> pb_all((size_t)k * n_parts, 0);
    for (size_t j = 0; j < k; ++j) {
        for (uint32_t q = 0; q < n_parts; ++q) {
            pb_all[j * n_parts + q] = acc[q];
            acc[q] += h[512 * j + n_parts + q];
        }
    }
    // span output: part q's records at [rstart[q], rstart[q + 1]) of the parts' records;
    // piece j's part-q records from rb_all[j][q] on
    const bool want_sp = sp_out != nullptr || user_sp != nullptr;
    uint2 *d_sp = nullptr;
    uint64_t *d_k = nullptr;
    if (want_sp) {
        // part q's records start at racc[q] of the span output, parts in the order of the
        // byte layout (round-major with rounds > 1)
        uint64_t rtot = 0;
        std::vector<uint64_t> racc(n_parts);
        if (rounds > 1) {
            const uint32_t G = n_parts / rounds;
            for (uint32_t p = 0; p < rounds; ++p)
                for (uint32_t g = 0; g < G; ++g) { racc[g * rounds + p] = rtot; rtot += prec[g * rounds + p]; }
        } else {
            for (uint32_t q = 0; q < n_parts; ++q) { racc[q] = rtot; rtot += prec[q]; }
        }
        for (size_t j = 0; j < k; ++j)
            for (uint32_t q = 0; q < n_parts; ++q) {
                pb_all.push_back(racc[q]);
                racc[q] += h[512 * j + q];
            }
        for (uint32_t q = 0; q < n_parts; ++q) pb_all.push_back(pbase[q]);
        if (user_sp) {
            if (rtot > rec_cap) {
                set_error("span capacity %zu < %llu records", rec_cap, (unsigned long long)rtot);
                return SG_E_CAP;
            }
            d_sp = user_sp;
            d_k = user_k;
        } else {
            SG_TRY(slot(c, S_PT_SPOUT, rtot + 1, &d_sp));
            SG_TRY(slot(c, S_PT_KOUT, rtot + 1, &d_k));
            *sp_out = d_sp;
            *k_out = d_k;
        }
    }
    uint64_t *d_pb;
    SG_TRY(slot(c, S_PT_BASE, pb_all.size(), &d_pb));
    SG_TRY(ctx_upload(c, d_pb, pb_all.data(), pb_all.size() * 8));
    const uint64_t *d_rb = d_pb + (size_t)k * n_parts, *d_pstart = d_pb + 2 * (size_t)k * n_parts;
    // the handover checksum per part (sg_span_sum of its records' spans and keys): per-(part,
    // tile) partials from the copy pass, then per part over every piece's tiles
    const bool want_sums = want_sp && part_sums;
    uint64_t *d_sums = nullptr;
    unsigned long long *d_stot = nullptr;
    if (want_sums) {
        SG_TRY(slot(c, S_PT_SUMS, ptot + n_parts + 1, &d_sums));
        d_stot = reinterpret_cast<unsigned long long *>(d_sums + ptot);
        SG_HIP(hipMemsetAsync(d_stot, 0, 8ull * n_parts, c->stream));
    }
    // pass 2 per piece: the multi-split copy with pass 1's spans, parts and scans
    for (size_t j = 0; j < k; ++j) {
        if (!Rj[j]) continue;
        SG_TRY(aligned_in(c, S_IN, d_pieces[j], lens[j], &pb_in[j]));
        PartSpansOut so;
        if (want_sp)
            so = PartSpansOut{rpre_all + poff[j], d_rb + j * n_parts, d_pstart, d_sp, d_k,
                              want_sums ? d_sums + poff[j] : nullptr};
        // model: span + part read, the record's bytes read and written (+ span and key out)
        SG_LAUNCH_B(c, "part_emit", (want_sp ? 25.0 : 9.0) * Rj[j] + 2.0 * (double)lens[j], k_part_apply, ptn[j],
                    PT_BLOCK, 0, pb_in[j], keep_sp + roff[j], keep_k + roff[j], Rj[j], ptn[j], n_parts, ppre_all + poff[j],
                    d_pb + j * n_parts, d_out, so);
        if (want_sums)
            SG_LAUNCH(c, "part_sums", k_part_sums, dim3((ptn[j] + PS_CHUNK - 1) / PS_CHUNK, n_parts), 256, 0,
                      d_sums + poff[j], ptn[j], d_stot);
    }
    if (want_sums) {  // (the host waits for the copy pass here: the sums travel with the sizes)
        std::vector<uint64_t> hs(n_parts, 0);
        SG_TRY(ctx_readback(c, hs.data(), d_stot, 8ull * n_parts));
        for (uint32_t q = 0; q < n_parts; ++q) part_sums[q] = hs[q];
    }
    return SG_OK;
}

extern "C" {

int sg_dev_partition_bytes_pieces(sg_ctx *c, const uint8_t *const *d_pieces, const size_t *lens, size_t k,
                                  const uint8_t *splitters, const uint32_t *split_offs, uint32_t n_parts, uint8_t *d_out,
                                  size_t out_cap, uint64_t *part_bytes, uint64_t *part_records) {
    return partition_pieces(c, d_pieces, lens, k, splitters, split_offs, n_parts, d_out, out_cap, part_bytes,
                            part_records, false);
}

int sg_dev_partition_bytes_pieces_a16(sg_ctx *c, const uint8_t *const *d_pieces, const size_t *lens, size_t k,
                                      const uint8_t *splitters, const uint32_t *split_offs, uint32_t n_parts,
                                      uint8_t *d_out, size_t out_cap, uint64_t *part_bytes, uint64_t *part_records) {
    return partition_pieces(c, d_pieces, lens, k, splitters, split_offs, n_parts, d_out, out_cap, part_bytes,
                            part_records, true);
}

int sg_dev_partition_bytes_pieces_spans(sg_ctx *c, const uint8_t *const *d_pieces, const size_t *lens, size_t k,
                                        const uint8_t *splitters, const uint32_t *split_offs, uint32_t n_parts,
                                        uint8_t *d_out, size_t out_cap, uint64_t *part_bytes, uint64_t *part_records,
                                        const uint32_t **d_spans, const uint64_t **d_keys, uint64_t *part_sums) {
    if (!d_spans || !d_keys) {
        if (c) c->pt_prep.on = false;
        set_error("sg_dev_partition_bytes_pieces_spans: bad arguments");
        return SG_E_INVAL;
    }
    *d_spans = nullptr;
    *d_keys = nullptr;
    const uint2 *sp = nullptr;
    SG_TRY(partition_pieces(c, d_pieces, lens, k, splitters, split_offs, n_parts, d_out, out_cap, part_bytes,
                            part_records, true, &sp, d_keys, 1, nullptr, nullptr, 0, part_sums));
    *d_spans = reinterpret_cast<const uint32_t *>(sp);
    return SG_OK;
}

int sg_dev_partition_bytes_pieces_rounds(sg_ctx *c, const uint8_t *const *d_pieces, const size_t *lens, size_t k,
                                         const uint8_t *splitters, const uint32_t *split_offs, uint32_t n_parts,
                                         uint32_t rounds, uint8_t *d_out, size_t out_cap, uint64_t *part_bytes,
                                         uint64_t *part_records) {
    return partition_pieces(c, d_pieces, lens, k, splitters, split_offs, n_parts, d_out, out_cap, part_bytes,
                            part_records, false, nullptr, nullptr, rounds);
}

int sg_dev_partition_pieces_count(sg_ctx *c, const uint8_t *const *d_pieces, const size_t *lens, size_t k,
                                  uint64_t *n_records) {
    if (!c || !n_records || (k && (!d_pieces || !lens))) { set_error("sg_dev_partition_pieces_count: bad arguments"); return SG_E_INVAL; }
    *n_records = 0;
    for (size_t j = 0; j < k; ++j) {
        if (!d_pieces[j] && lens[j]) { set_error("piece %zu is NULL", j); return SG_E_INVAL; }
        if (lens[j] > MAX_BYTES) { set_error("piece %zu exceeds 4 GiB", j); return SG_E_TOO_LARGE; }
    }
    SG_HIP(hipSetDevice(c->device));
    std::vector<uint32_t> lnt, Rj;
    std::vector<size_t> loff;
    uint64_t *ltp = nullptr;
    c->pt_prep.on = false;
    SG_TRY(pieces_pass0(c, d_pieces, lens, k, lnt, loff, &ltp, Rj, false));
    uint64_t tot = 0;
    for (uint32_t r : Rj) tot += r;
    *n_records = tot;
    auto &P = c->pt_prep;
    P.ptrs.assign(d_pieces, d_pieces + k);
    P.lens.assign(lens, lens + k);
    P.Rj = Rj;
    P.on = true;
    return SG_OK;
}

int sg_dev_partition_bytes_pieces_rounds_spans(sg_ctx *c, const uint8_t *const *d_pieces, const size_t *lens, size_t k,
                                               const uint8_t *splitters, const uint32_t *split_offs, uint32_t n_parts,
                                               uint32_t rounds, uint8_t *d_out, size_t out_cap, uint64_t *part_bytes,
                                               uint64_t *part_records, uint32_t *d_spans, uint64_t *d_keys,
                                               size_t rec_cap, uint64_t *part_sums) {
    if (!d_spans || !d_keys) {
        if (c) c->pt_prep.on = false;
        set_error("sg_dev_partition_bytes_pieces_rounds_spans: bad arguments");
        return SG_E_INVAL;
    }
    return partition_pieces(c, d_pieces, lens, k, splitters, split_offs, n_parts, d_out, out_cap, part_bytes,
                            part_records, false, nullptr, nullptr, rounds, reinterpret_cast<uint2 *>(d_spans), d_keys,
                            rec_cap, part_sums);
}

int sg_dev_rebase_spans(sg_ctx *c, const uint8_t *d_buf, size_t n, uint32_t *d_spans, size_t n_rec,
                        const uint64_t *seg_first, const uint64_t *seg_off, uint32_t nseg, uint64_t *bad) {
    if (!c || !bad || (n_rec && (!d_spans || !d_buf)) || (nseg && (!seg_first || !seg_off))) {
        set_error("sg_dev_rebase_spans: bad arguments");
        return SG_E_INVAL;
    }
    *bad = 0;
    if (!n_rec) return SG_OK;
    if (n > MAX_BYTES || n_rec >= (1ull << 32)) { set_error("sg_dev_rebase_spans: input exceeds 4 GiB"); return SG_E_TOO_LARGE; }
    SG_HIP(hipSetDevice(c->device));
    const uint32_t ns = nseg ? nseg : 1u;
    std::vector<uint32_t> F(ns + 1), O(ns);
    bool shift = false;
    for (uint32_t s = 0; s < ns; ++s) {
        const uint64_t f = nseg ? seg_first[s] : 0, o = nseg ? seg_off[s] : 0;
        if (o > n || f > n_rec || (s && f < F[s - 1]) || (!s && f)) {
            set_error("sg_dev_rebase_spans: bad segments");
            return SG_E_INVAL;
        }
        F[s] = (uint32_t)f;
        O[s] = (uint32_t)o;
        shift |= o != 0;
    }
    F[ns] = (uint32_t)n_rec;
    unsigned long long *d_bad;
    SG_TRY(slot(c, S_M_CNT, 4, &d_bad));
    SG_HIP(hipMemsetAsync(d_bad, 0, 8, c->stream));
    // one launch per batch of SG_REBASE_SEGS sources (a kernel argument holds one batch's table)
    for (uint32_t s0 = 0; s0 < ns; s0 += SG_REBASE_SEGS) {
        RebaseSegs sg_{};
        sg_.nseg = std::min<uint32_t>(SG_REBASE_SEGS, ns - s0);
        for (uint32_t s = 0; s < sg_.nseg; ++s) { sg_.first[s] = F[s0 + s]; sg_.off[s] = O[s0 + s]; }
        sg_.first[sg_.nseg] = F[s0 + sg_.nseg];
        const uint32_t nr = sg_.first[sg_.nseg] - sg_.first[0];
        if (shift && nr)
            SG_LAUNCH_B(c, "rebase_spans", 16.0 * (double)nr, k_rebase_spans, (nr + 255) / 256, 256, 0,
                        reinterpret_cast<uint2 *>(d_spans), d_buf, (uint32_t)n, sg_, d_bad);
        else if (!shift)
            SG_LAUNCH(c, "check_spans", k_check_spans, (sg_.nseg * 2 * SG_REBASE_CHECK + 255) / 256, 256, 0,
                      reinterpret_cast<const uint2 *>(d_spans), d_buf, (uint32_t)n, sg_, d_bad);
    }
    unsigned long long b = 0;
    SG_TRY(ctx_readback(c, &b, d_bad, 8));
    *bad = b;
    return SG_OK;
}

int sg_dev_dedup_diff_spans_into(sg_ctx *c, const uint8_t *d_cur, size_t n_cur, uint32_t *d_spans,
                                 uint64_t *d_keys, size_t n_rec, uint64_t span_sum, const uint8_t *d_prior,
                                 size_t n_prior, uint8_t *d_uniq, size_t uniq_cap, uint8_t *d_fresh, size_t fresh_cap,
                                 sg_dev_result *res) {
    if (!c || !res || (!d_cur && n_cur) || (!d_prior && n_prior) || !d_uniq || (n_rec && (!d_spans || !d_keys))) {
        set_error("sg_dev_dedup_diff_spans_into: bad arguments");
        return SG_E_INVAL;
    }
    if (((uintptr_t)d_cur & 15) != 0) { set_error("sg_dev_dedup_diff_spans_into: d_cur must be 16-byte aligned"); return SG_E_INVAL; }
    if (n_cur > MAX_BYTES || n_prior > MAX_BYTES || n_rec >= (1ull << 32)) {
        set_error("input exceeds 4 GiB per call");
        return SG_E_TOO_LARGE;
    }
    if (!n_rec && (n_cur || span_sum)) {  // records tile the buffer: no records, no bytes
        set_error("handed-over parse does not match the buffer: 0 records for %zu bytes, checksum %016llx", n_cur,
                  (unsigned long long)span_sum);
        return SG_E_CORRUPT;
    }
    SG_HIP(hipSetDevice(c->device));
    const uint8_t *prior = nullptr;
    if (n_prior) SG_TRY(aligned_in(c, S_IN2, d_prior, n_prior, &prior));
    Lines L;
    L.spans = reinterpret_cast<uint2 *>(d_spans);  // consumed: the sort works in place
    L.keys = d_keys;
    L.n_rec = (uint32_t)n_rec;
    L.chk = true;  // checked by the dedup's prefix scan before any byte is read through a span
    L.chk_sum = span_sum;
    return dev_dedup_diff_into_lines(c, d_cur, n_cur, L, prior, n_prior, d_uniq, uniq_cap, d_fresh, fresh_cap, res);
}

int sg_dev_record_sample(sg_ctx *c, const uint8_t *d_buf, size_t n, uint32_t m, uint8_t *heads, uint32_t *lens,
                         uint64_t *n_rec) {
    if (!c || (!heads && m) || (!lens && m) || (!d_buf && n)) {
        set_error("sg_dev_record_sample: bad arguments");
        return SG_E_INVAL;
    }
    if (n > MAX_BYTES) { set_error("input exceeds 4 GiB per call"); return SG_E_TOO_LARGE; }
    SG_HIP(hipSetDevice(c->device));
    const uint8_t *b;
    SG_TRY(aligned_in(c, S_IN, d_buf, n, &b));
    Lines L;
    SG_TRY(run_lines(c, b, n, CUR_SLOTS, &L));
    if (n_rec) *n_rec = L.n_rec;
    const uint32_t take = L.n_rec ? m : 0u;
    if (take) {
        uint64_t *d;
        SG_TRY(slot(c, S_M_TMP2, (size_t)take * (SPL_WORDS + 1), &d));
        uint32_t *dl = reinterpret_cast<uint32_t *>(d + (size_t)take * SPL_WORDS);
        SG_LAUNCH(c, "head_sample", k_head_sample, (take + 255) / 256, 256, 0, b, L.spans, L.n_rec, take, d, dl);
        SG_TRY(ctx_readback(c, heads, d, (size_t)take * SPL_W));
        SG_TRY(ctx_readback(c, lens, dl, 4ull * take));
    }
    return SG_OK;
}

int sg_dev_key_sample(sg_ctx *c, const uint8_t *d_buf, size_t n, uint32_t m, uint64_t *keys, uint64_t *n_rec) {
    if (!c || !keys || (!d_buf && n)) { set_error("sg_dev_key_sample: bad arguments"); return SG_E_INVAL; }
    if (n > MAX_BYTES) { set_error("input exceeds 4 GiB per call"); return SG_E_TOO_LARGE; }
    SG_HIP(hipSetDevice(c->device));
    const uint8_t *b;
    SG_TRY(aligned_in(c, S_IN, d_buf, n, &b));
    Lines L;
    SG_TRY(run_lines(c, b, n, CUR_SLOTS, &L));
    if (n_rec) *n_rec = L.n_rec;
    const uint32_t take = L.n_rec ? m : 0u;
    if (take) {
        uint64_t *d;
        SG_TRY(slot(c, S_M_TMP2, take, &d));
        SG_LAUNCH(c, "key_sample", k_key_sample, (take + 255) / 256, 256, 0, L.keys, L.n_rec, take, d);
        SG_TRY(ctx_readback(c, keys, d, 8ull * take));
    }
    for (uint32_t k = take; k < m; ++k) keys[k] = ~0ull;
    return SG_OK;
}

int sg_dev_partition(sg_ctx *c, const uint8_t *d_buf, size_t n, uint32_t n_parts, uint8_t *d_out,
                     size_t out_cap, uint64_t *part_bytes, uint64_t *part_records) {
    if (!c || (!d_out && n) || (!d_buf && n)) { set_error("sg_dev_partition: bad arguments"); return SG_E_INVAL; }
    SG_HIP(hipSetDevice(c->device));
    const uint8_t *b;
    SG_TRY(aligned_in(c, S_IN, d_buf, n, &b));
    return dev_partition(c, b, n, n_parts, d_out, out_cap, part_bytes, part_records);
}

}  // extern "C"
