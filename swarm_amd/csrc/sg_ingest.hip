// sg_ingest.hip — streamed merge ingestion.
//
// server/server.py:407-410 builds the /raw body with Python `str +=` over S3 bodies before
// anything can run on it. Here the server appends each chunk body (or any piece of one, as
// it arrives from the S3 stream) in the A5 key order; the bytes are copied into one of two
// pinned staging buffers and sent to HBM with an async H2D copy on the context stream
// while the caller reads the next piece, so the merged buffer is resident when the last
// body ends. Concatenation has no separator, exactly as A5. The device buffer grows
// geometrically (size_hint from the S3 listing sizes avoids any regrowth).
#include "sg_internal.hpp"

#include <string.h>

constexpr size_t IG_STAGE = 8u << 20;

struct sg_ingest {
    sg_ctx *c = nullptr;
    uint8_t *d = nullptr;
    uint64_t cap = 0, n = 0;
    uint8_t *stage[2] = {nullptr, nullptr};
    hipEvent_t ev[2] = {nullptr, nullptr};
    bool busy[2] = {false, false};
    int cur = 0;
    size_t fill = 0;
};

namespace sg {

static int ig_reserve(sg_ingest *s, uint64_t need) {
    if (need <= s->cap) return SG_OK;
    if (need > MAX_BYTES) { set_error("ingest: merged body exceeds 4 GiB per call"); return SG_E_TOO_LARGE; }
    const uint64_t cap = std::min<uint64_t>(std::max<uint64_t>(need, 2 * s->cap), MAX_BYTES);
    uint8_t *nd = nullptr;
    if (hipMalloc(&nd, cap + 64) != hipSuccess) { (void)hipGetLastError(); set_error("ingest: hipMalloc(%llu)", (unsigned long long)cap); return SG_E_NOMEM; }
    if (s->d) {
        if (s->n) SG_HIP(hipMemcpyAsync(nd, s->d, s->n, hipMemcpyDeviceToDevice, s->c->stream));
        SG_HIP(hipStreamSynchronize(s->c->stream));
        SG_HIP(hipFree(s->d));
    }
    s->d = nd;
    s->cap = cap;
    return SG_OK;
}

static int ig_flush(sg_ingest *s) {
    if (!s->fill) return SG_OK;
    SG_TRY(ig_reserve(s, s->n + s->fill));
    SG_HIP(hipMemcpyAsync(s->d + s->n, s->stage[s->cur], s->fill, hipMemcpyHostToDevice, s->c->stream));
    SG_HIP(hipEventRecord(s->ev[s->cur], s->c->stream));
    s->busy[s->cur] = true;
    s->n += s->fill;
    s->fill = 0;
    s->cur ^= 1;
    return SG_OK;
}

}  // namespace sg

using namespace sg;

extern "C" {

int sg_ingest_open(sg_ctx *c, size_t size_hint, sg_ingest **out) {
    if (!c || !out) { set_error("sg_ingest_open: bad arguments"); return SG_E_INVAL; }
    SG_HIP(hipSetDevice(c->device));
    sg_ingest *s = new sg_ingest();
    s->c = c;
    int rc = SG_OK;
    for (int i = 0; i < 2 && rc == SG_OK; ++i) {
        if (hipHostMalloc(&s->stage[i], IG_STAGE, hipHostMallocDefault) != hipSuccess ||
            hipEventCreateWithFlags(&s->ev[i], hipEventDisableTiming) != hipSuccess) {
            (void)hipGetLastError();
            set_error("sg_ingest_open: pinned staging allocation failed");
            rc = SG_E_NOMEM;
        }
    }
    if (rc == SG_OK && size_hint) rc = ig_reserve(s, size_hint);
    if (rc != SG_OK) { sg_ingest_close(s); return rc; }
    *out = s;
    return SG_OK;
}

int sg_ingest_append(sg_ingest *s, const uint8_t *data, size_t len) {
    if (!s || (!data && len)) { set_error("sg_ingest_append: bad arguments"); return SG_E_INVAL; }
    if (s->n + s->fill + len > MAX_BYTES) { set_error("ingest: merged body exceeds 4 GiB per call"); return SG_E_TOO_LARGE; }
    SG_HIP(hipSetDevice(s->c->device));
    while (len) {
        if (s->fill == 0 && s->busy[s->cur]) {
            SG_HIP(hipEventSynchronize(s->ev[s->cur]));  // the DMA out of this buffer is done
            s->busy[s->cur] = false;
        }
        const size_t take = std::min(len, IG_STAGE - s->fill);
        memcpy(s->stage[s->cur] + s->fill, data, take);
        s->fill += take;
        data += take;
        len -= take;
        if (s->fill == IG_STAGE) SG_TRY(ig_flush(s));
    }
    return SG_OK;
}

int sg_ingest_finish(sg_ingest *s, const uint8_t **d_buf, uint64_t *n) {
    if (!s || !d_buf || !n) { set_error("sg_ingest_finish: bad arguments"); return SG_E_INVAL; }
    SG_HIP(hipSetDevice(s->c->device));
    SG_TRY(ig_flush(s));
    SG_TRY(ig_reserve(s, 16));
    SG_HIP(hipStreamSynchronize(s->c->stream));
    s->busy[0] = s->busy[1] = false;
    *d_buf = s->d;
    *n = s->n;
    return SG_OK;
}

int sg_ingest_close(sg_ingest *s) {
    if (!s) return SG_OK;
    (void)hipSetDevice(s->c->device);
    (void)hipStreamSynchronize(s->c->stream);
    for (int i = 0; i < 2; ++i) {
        if (s->stage[i]) (void)hipHostFree(s->stage[i]);
        if (s->ev[i]) (void)hipEventDestroy(s->ev[i]);
    }
    if (s->d) (void)hipFree(s->d);
    delete s;
    return SG_OK;
}

}  // extern "C"
