// sg_runtime.hip — context lifetime, HBM buffer slots, HIP-event kernel timing, errors,
// and the per-device context pool behind the re-entrant host-buffer API.
#include "sg_common.hpp"
#include "sg_internal.hpp"
#include "sg_prims.hpp"

#include <string.h>

#include <algorithm>

namespace sg {

static thread_local std::string g_err;

void set_error(const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
}
const char *get_error() { return g_err.c_str(); }

int ctx_slot(sg_ctx *c, int s, size_t bytes, void **out) {
    if (bytes < 256) bytes = 256;
    if (c->slot_cap[s] < bytes) {
        if (c->slot_ptr[s]) {
            SG_HIP(hipStreamSynchronize(c->stream));
            SG_HIP(hipFree(c->slot_ptr[s]));
            c->slot_ptr[s] = nullptr;
            c->slot_cap[s] = 0;
        }
        size_t want = bytes + bytes / 8;  // headroom so small growth does not realloc
        if (hipMalloc(&c->slot_ptr[s], want) != hipSuccess) {
            (void)hipGetLastError();
            set_error("hipMalloc(%zu) failed for slot %d", want, s);
            return SG_E_NOMEM;
        }
        c->slot_cap[s] = want;
    }
    *out = c->slot_ptr[s];
    return SG_OK;
}

int ctx_readback(sg_ctx *c, void *host, const void *dev, size_t bytes) {
    if (bytes > SG_PINNED_BYTES) {
        SG_HIP(hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, c->stream));
        SG_HIP(hipStreamSynchronize(c->stream));
        return SG_OK;
    }
    SG_HIP(hipMemcpyAsync(c->pinned, dev, bytes, hipMemcpyDeviceToHost, c->stream));
    SG_HIP(hipStreamSynchronize(c->stream));
    memcpy(host, c->pinned, bytes);
    return SG_OK;
}

int ctx_upload(sg_ctx *c, void *dev, const void *host, size_t bytes) {
    if (!bytes) return SG_OK;
    if (c->up_ev) SG_HIP(hipEventSynchronize(c->up_ev));  // the previous upload has left the buffer
    if (bytes > c->up_cap) {
        if (c->up_pin) (void)hipHostFree(c->up_pin);
        c->up_pin = nullptr;
        c->up_cap = 0;
        const size_t want = std::max<size_t>(bytes + bytes / 2, 64 << 10);
        if (hipHostMalloc(&c->up_pin, want, hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            set_error("hipHostMalloc(%zu) failed for upload staging", want);
            return SG_E_NOMEM;
        }
        c->up_cap = want;
    }
    if (!c->up_ev) SG_HIP(hipEventCreateWithFlags(&c->up_ev, hipEventDisableTiming));
    memcpy(c->up_pin, host, bytes);
    SG_HIP(hipMemcpyAsync(dev, c->up_pin, bytes, hipMemcpyHostToDevice, c->stream));
    SG_HIP(hipEventRecord(c->up_ev, c->stream));
    return SG_OK;
}

int prof_begin(sg_ctx *c, const char *name, int *stat, hipEvent_t *a) {
    int idx = -1;
    for (size_t i = 0; i < c->stats.size(); ++i)
        if (c->stats[i].name == name || strcmp(c->stats[i].name, name) == 0) { idx = (int)i; break; }
    if (idx < 0) {
        c->stats.push_back(KStat{name, 0, 0.0, 0.0});
        idx = (int)c->stats.size() - 1;
    }
    hipEvent_t e;
    if (!c->free_events.empty()) { e = c->free_events.back(); c->free_events.pop_back(); }
    else if (hipEventCreate(&e) != hipSuccess) { (void)hipGetLastError(); return SG_E_HIP; }
    (void)hipEventRecord(e, c->stream);
    *stat = idx;
    *a = e;
    return SG_OK;
}

void prof_end(sg_ctx *c, int stat, hipEvent_t a) {
    hipEvent_t e;
    if (!c->free_events.empty()) { e = c->free_events.back(); c->free_events.pop_back(); }
    else if (hipEventCreate(&e) != hipSuccess) { (void)hipGetLastError(); return; }
    (void)hipEventRecord(e, c->stream);
    c->pending.push_back(sg_ctx::Pending{stat, a, e});
}

void prof_bytes(sg_ctx *c, const char *name, double bytes) {
    if (!c->profile || !prof_wanted(c, name)) return;
    for (auto &s : c->stats)
        if (s.name == name || strcmp(s.name, name) == 0) { s.bytes += bytes; return; }
    c->stats.push_back(KStat{name, 0, 0.0, bytes});
}

int ctx_harvest(sg_ctx *c) {
    if (c->pending.empty()) return SG_OK;
    SG_HIP(hipStreamSynchronize(c->stream));
    for (auto &p : c->pending) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
            c->stats[p.stat].ms += ms;
            c->stats[p.stat].launches += 1;
        } else {
            (void)hipGetLastError();
        }
        c->free_events.push_back(p.a);
        c->free_events.push_back(p.b);
    }
    c->pending.clear();
    return SG_OK;
}

// ------------------------------------------------------------------ context pool
struct Pool {
    std::mutex mu;
    std::vector<sg_ctx *> idle[64];
};
static Pool g_pool;

int pool_acquire(int device, sg_ctx **out) {
    {
        std::lock_guard<std::mutex> g(g_pool.mu);
        auto &v = g_pool.idle[device & 63];
        if (!v.empty()) { *out = v.back(); v.pop_back(); return SG_OK; }
    }
    return sg_ctx_create(device, nullptr, out);
}

void pool_release(sg_ctx *c) {
    std::lock_guard<std::mutex> g(g_pool.mu);
    g_pool.idle[c->device & 63].push_back(c);
}

int pick_device(int *dev) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        (void)hipGetLastError();
        set_error("no HIP device visible");
        return SG_E_NODEV;
    }
    SG_HIP(hipGetDevice(dev));
    return SG_OK;
}

}  // namespace sg

using namespace sg;

extern "C" {

const char *sg_last_error(void) { return get_error(); }
int sg_version(void) { return 10000; }

int sg_device_count(int *n) {
    if (!n) return SG_E_INVAL;
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) { (void)hipGetLastError(); c = 0; }
    *n = c;
    return SG_OK;
}

int sg_ctx_create(int device, void *stream, sg_ctx **out) {
    if (!out) return SG_E_INVAL;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        (void)hipGetLastError();
        set_error("no HIP device visible");
        return SG_E_NODEV;
    }
    if (device < 0 || device >= n) { set_error("device %d out of range", device); return SG_E_INVAL; }
    SG_HIP(hipSetDevice(device));
    sg_ctx *c = new sg_ctx();
    c->device = device;
    if (stream) {
        c->stream = stream == SG_NULL_STREAM ? (hipStream_t)0 : (hipStream_t)stream;
    } else {
        if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
            delete c;
            set_error("hipStreamCreate failed");
            return SG_E_HIP;
        }
        c->owns_stream = true;
    }
    if (hipHostMalloc(&c->pinned, SG_PINNED_BYTES, hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        if (c->owns_stream) (void)hipStreamDestroy(c->stream);
        delete c;
        set_error("hipHostMalloc failed");
        return SG_E_NOMEM;
    }
    *out = c;
    return SG_OK;
}

int sg_ctx_destroy(sg_ctx *c) {
    if (!c) return SG_OK;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    for (int s = 0; s < S_NSLOTS; ++s)
        if (c->slot_ptr[s]) (void)hipFree(c->slot_ptr[s]);
    for (auto &p : c->pending) { (void)hipEventDestroy(p.a); (void)hipEventDestroy(p.b); }
    for (auto e : c->free_events) (void)hipEventDestroy(e);
    if (c->pinned) (void)hipHostFree(c->pinned);
    if (c->up_pin) (void)hipHostFree(c->up_pin);
    if (c->up_ev) (void)hipEventDestroy(c->up_ev);
    if (c->owns_stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return SG_OK;
}

int sg_ctx_sync(sg_ctx *c) {
    if (!c) return SG_E_INVAL;
    SG_HIP(hipStreamSynchronize(c->stream));
    return SG_OK;
}

int sg_ctx_profile(sg_ctx *c, int enable) {
    if (!c) return SG_E_INVAL;
    c->profile = enable != 0;
    return SG_OK;
}

int sg_ctx_profile_only(sg_ctx *c, const char *name) {
    if (!c) return SG_E_INVAL;
    c->prof_only = name ? name : "";
    return SG_OK;
}

int sg_ctx_kernel_stat(sg_ctx *c, int idx, const char **name, uint64_t *launches, double *total_ms,
                       double *total_bytes) {
    if (!c) return SG_E_INVAL;
    SG_TRY(ctx_harvest(c));
    if (idx < 0 || idx >= (int)c->stats.size()) return SG_E_INVAL;
    if (name) *name = c->stats[idx].name;
    if (launches) *launches = c->stats[idx].launches;
    if (total_ms) *total_ms = c->stats[idx].ms;
    if (total_bytes) *total_bytes = c->stats[idx].bytes;
    return SG_OK;
}

int sg_ctx_memcpy(sg_ctx *c, void *dst, const void *src, size_t n) {
    if (!c || (n && (!dst || !src))) return SG_E_INVAL;
    if (!n) return SG_OK;
    SG_HIP(hipMemcpyAsync(dst, src, n, hipMemcpyDefault, c->stream));
    SG_HIP(hipStreamSynchronize(c->stream));
    return SG_OK;
}

int sg_ctx_last_path(sg_ctx *c, int *path, uint32_t *flags) {
    if (!c) return SG_E_INVAL;
    if (path) *path = c->last_path;
    if (flags) *flags = c->last_flags;
    return SG_OK;
}

int sg_ctx_last_key_width(sg_ctx *c, uint32_t *kw) {
    if (!c || !kw) return SG_E_INVAL;
    *kw = c->last_kw;
    return SG_OK;
}

int sg_ctx_reset_stats(sg_ctx *c) {
    if (!c) return SG_E_INVAL;
    SG_TRY(ctx_harvest(c));
    c->stats.clear();
    return SG_OK;
}

}  // extern "C"

namespace sg {

__global__ __launch_bounds__(TS_BLOCK) void k_tile_scan(const uint64_t *__restrict__ tot, uint32_t nt,
                                                        uint64_t *__restrict__ pre, uint64_t *__restrict__ total,
                                                        uint64_t init) {
    __shared__ uint64_t s_red[TS_BLOCK / 64];
    uint64_t carry = 0;
    for (uint32_t base = 0; base < nt; base += TS_BLOCK * TS_ITEMS) {
        const uint32_t i0 = base + threadIdx.x * TS_ITEMS;
        uint64_t v[TS_ITEMS];
        uint64_t sum = 0;
#pragma unroll
        for (int j = 0; j < TS_ITEMS; ++j) {
            v[j] = (i0 + j < nt) ? tot[i0 + j] : 0ull;
            sum += v[j];
        }
        uint64_t btot;
        const uint64_t ex = block_excl_scan<TS_BLOCK>(sum, &btot, s_red);
        uint64_t run = carry + ex;
#pragma unroll
        for (int j = 0; j < TS_ITEMS; ++j) {
            if (i0 + j < nt) pre[i0 + j] = init + run;
            run += v[j];
        }
        carry += btot;
    }
    if (threadIdx.x == 0) *total = carry;
}

// Large scans (> 32k tiles; a 4 GB parse has ~250k: 62 rounds of one block, ~90 us) go in two
// levels: per-chunk sums by many blocks, the one-block scan of those, then each chunk's
// exclusive prefixes from its chunk base.
constexpr uint32_t TS_CHUNK = TS_BLOCK * TS_ITEMS;

__global__ __launch_bounds__(TS_BLOCK) void k_ts_sum(const uint64_t *__restrict__ tot, uint32_t nt,
                                                     uint64_t *__restrict__ part) {
    __shared__ uint64_t s_red[TS_BLOCK / 64];
    const uint32_t i0 = blockIdx.x * TS_CHUNK + threadIdx.x * TS_ITEMS;
    uint64_t sum = 0;
#pragma unroll
    for (int j = 0; j < TS_ITEMS; ++j) sum += (i0 + j < nt) ? tot[i0 + j] : 0ull;
    sum = wave_sum(sum);
    if (lane_id() == 0) s_red[threadIdx.x >> 6] = sum;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t t = 0;
#pragma unroll
        for (int w = 0; w < TS_BLOCK / 64; ++w) t += s_red[w];
        part[blockIdx.x] = t;
    }
}

__global__ __launch_bounds__(TS_BLOCK) void k_ts_apply(const uint64_t *__restrict__ tot, uint32_t nt,
                                                       const uint64_t *__restrict__ ppre, uint64_t *__restrict__ pre,
                                                       uint64_t init) {
    __shared__ uint64_t s_red[TS_BLOCK / 64];
    const uint32_t i0 = blockIdx.x * TS_CHUNK + threadIdx.x * TS_ITEMS;
    uint64_t v[TS_ITEMS], sum = 0;
#pragma unroll
    for (int j = 0; j < TS_ITEMS; ++j) {
        v[j] = (i0 + j < nt) ? tot[i0 + j] : 0ull;
        sum += v[j];
    }
    uint64_t btot;
    uint64_t run = init + ppre[blockIdx.x] + block_excl_scan<TS_BLOCK>(sum, &btot, s_red);
#pragma unroll
    for (int j = 0; j < TS_ITEMS; ++j) {
        if (i0 + j < nt) pre[i0 + j] = run;
        run += v[j];
    }
}

int tile_scan(sg_ctx *c, const uint64_t *tot, uint32_t nt, uint64_t *pre, uint64_t *total, uint64_t init) {
    if (nt <= 8 * TS_CHUNK) {  // up to 8 rounds of one block beat 3 launches
        SG_LAUNCH(c, "tile_scan", k_tile_scan, 1, TS_BLOCK, 0, tot, nt, pre, total, init);
        return SG_OK;
    }
    const uint32_t nc = (nt + TS_CHUNK - 1) / TS_CHUNK;
    uint64_t *part;
    SG_TRY(slot(c, S_TS2, 2 * (size_t)nc, &part));
    SG_LAUNCH(c, "tile_scan", k_ts_sum, nc, TS_BLOCK, 0, tot, nt, part);
    SG_LAUNCH(c, "tile_scan", k_tile_scan, 1, TS_BLOCK, 0, part, nc, part + nc, total, 0ull);
    SG_LAUNCH(c, "tile_scan", k_ts_apply, nc, TS_BLOCK, 0, tot, nt, part + nc, pre, init);
    return SG_OK;
}

__global__ __launch_bounds__(SEL_BLOCK) void k_sel_apply(uint32_t n, const uint64_t *__restrict__ mA,
                                                         const uint64_t *__restrict__ mB,
                                                         const uint64_t *__restrict__ pre, uint32_t *__restrict__ outA,
                                                         uint32_t *__restrict__ outB) {
    __shared__ uint32_t s_ca[SEL_MASKS], s_cb[SEL_MASKS];
    __shared__ uint64_t s_ma[SEL_MASKS], s_mb[SEL_MASKS];  // the tile's masks, read once
    const int t = threadIdx.x, lane = lane_id(), wid = t >> 6;
    const uint32_t base = blockIdx.x * SEL_TILE;
    const uint64_t *ma = mA + (uint64_t)blockIdx.x * SEL_MASKS;
    const uint64_t *mb = mB + (uint64_t)blockIdx.x * SEL_MASKS;
    if (t < 64) {
        const uint64_t xa = ma[t], xb = mb[t];
        const uint32_t a = (uint32_t)__popcll(xa), b = (uint32_t)__popcll(xb);
        const uint32_t ia = wave_incl_scan(a), ib = wave_incl_scan(b);
        s_ca[t] = ia - a;
        s_cb[t] = ib - b;
        s_ma[t] = xa;
        s_mb[t] = xb;
    }
    __syncthreads();
    const uint64_t p0 = pre[blockIdx.x];
    const uint32_t preA = (uint32_t)(p0 >> 31), preB = (uint32_t)(p0 & 0x7fffffffu);
    const uint64_t lt = (1ull << lane) - 1ull;
#pragma unroll
    for (int j = 0; j < SEL_ROWS; ++j) {
        const uint32_t i = base + j * SEL_BLOCK + t;
        const uint64_t xa = s_ma[j * 4 + wid];
        if ((xa >> lane) & 1ull) outA[preA + s_ca[j * 4 + wid] + (uint32_t)__popcll(xa & lt)] = i;
        if (outB) {
            const uint64_t xb = s_mb[j * 4 + wid];
            if ((xb >> lane) & 1ull) outB[preB + s_cb[j * 4 + wid] + (uint32_t)__popcll(xb & lt)] = i;
        }
    }
}

}  // namespace sg
