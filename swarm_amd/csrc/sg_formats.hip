// sg_formats.hip — module-output formats on the GPU:
//
//   * nmap -oN  -> host:port records (worker/modules/nmap.json:2). Each record is one
//     line; a "Nmap scan report for HOST ..." line sets the host for the open-port lines
//     ("PORT/tcp open ...") that follow it. Classification is a two-predicate compaction
//     (report lines, open-port lines), each port finds its report by a binary search over
//     the report list (the last report before it), and the records are written with an
//     exclusive scan of their lengths. Output feeds A7 dedup unchanged (C5-style records).
//
//   * httpx -json -> field rows (worker/modules/http2.json:2, web.json:2). One thread per
//     JSON line reads it with aligned 16-byte loads and runs a byte state machine (string
//     and escape state, depth, whitespace framing). A colon at depth 1 names a top-level
//     key; it is compared with the requested keys (length + first byte prefilter; a key
//     written with escapes is decoded first, as json.loads would), and the span of each
//     requested key's last occurrence is kept in LDS (json.loads keeps the last
//     duplicate). The thread then measures each value (string decode length, array
//     elements), and the rows are written after one exclusive scan, one thread per
//     (record, key). (A wave-per-line walker over ballot masks of the structural bytes was
//     6x slower: one shuffle per structural event.) Rows are
//     '\n'-terminated decoded values — the buffer is itself a line buffer, so the A4
//     matchers run on it unchanged (part-scoped matching, §8(f) row 3).
#include "sg_internal.hpp"

#include <stdlib.h>
#include "sg_prims_host.hpp"

namespace sg {

static const SlotSet FMT_SLOTS = {S_F_SPANS, S_F_SPANS, S_F_A, S_F_A, S_F_B, S_F_B, S_F_B, S_F_LB};

// ------------------------------------------------------------------ nmap -oN
constexpr uint32_t NM_PREFIX_LEN = 21;  // "Nmap scan report for "

__device__ __forceinline__ bool nm_is_digit(uint8_t b) { return b >= '0' && b <= '9'; }
__device__ __forceinline__ bool nm_is_blank(uint8_t b) { return b == ' ' || b == '\t'; }

// bit 0: report line; bit 1: open-port line. Port line grammar (re.match):
//   [0-9]{1,5} / (tcp|udp|sctp) [ \t]+ open ([ \t] | end)
struct NmapPred {
    const uint8_t *buf;
    const uint2 *spans;
    __device__ uint32_t operator()(uint32_t i) const {
        const uint2 sp = spans[i];
        const uint8_t *p = buf + sp.x;
        const uint32_t len = sp.y - sp.x;
        if (len >= NM_PREFIX_LEN && p[0] == 'N') {
            const char *pre = "Nmap scan report for ";
            bool ok = true;
            for (uint32_t j = 1; j < NM_PREFIX_LEN && ok; ++j) ok = p[j] == (uint8_t)pre[j];
            return ok ? 1u : 0u;
        }
        uint32_t j = 0;
        while (j < len && j < 5 && nm_is_digit(p[j])) ++j;
        if (j == 0 || j >= len || p[j] != '/') return 0u;
        ++j;
        auto word = [&](const char *w, uint32_t wl) {
            if (j + wl > len) return false;
            for (uint32_t q = 0; q < wl; ++q)
                if (p[j + q] != (uint8_t)w[q]) return false;
            return true;
        };
        if (word("tcp", 3) || word("udp", 3)) j += 3;
        else if (word("sctp", 4)) j += 4;
        else return 0u;
        const uint32_t b0 = j;
        while (j < len && nm_is_blank(p[j])) ++j;
        if (j == b0 || !word("open", 4)) return 0u;
        j += 4;
        return (j == len || nm_is_blank(p[j])) ? 2u : 0u;
    }
};

// Per open-port line: {host start, host end, port start, port end} (host empty -> dropped).
__global__ __launch_bounds__(256) void k_nmap_prep(const uint8_t *__restrict__ buf, const uint2 *__restrict__ spans,
                                                   const uint32_t *__restrict__ reps, uint32_t nrep,
                                                   const uint32_t *__restrict__ ports, uint32_t nport,
                                                   uint4 *__restrict__ desc) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nport) return;
    const uint32_t r = ports[k];
    // last report record before r
    uint32_t lo = 0, hi = nrep;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (reps[mid] < r) lo = mid + 1; else hi = mid;
    }
    uint4 d = make_uint4(0, 0, 0, 0);
    if (lo > 0) {
        const uint2 rs = spans[reps[lo - 1]];
        uint32_t he = rs.x + NM_PREFIX_LEN;
        while (he < rs.y && buf[he] != ' ') ++he;
        const uint2 ps = spans[r];
        uint32_t pe = ps.x;
        while (nm_is_digit(buf[pe])) ++pe;
        if (he > rs.x + NM_PREFIX_LEN) d = make_uint4(rs.x + NM_PREFIX_LEN, he, ps.x, pe);
    }
    desc[k] = d;
}

struct NmapLen {
    const uint4 *desc;
    __device__ uint64_t operator()(uint32_t k) const {
        const uint4 d = desc[k];
        return d.y > d.x ? (uint64_t)(d.y - d.x) + 1 + (d.w - d.z) + 1 : 0ull;
    }
};

__global__ __launch_bounds__(256) void k_nmap_emit(const uint8_t *__restrict__ buf, const uint4 *__restrict__ desc,
                                                   const uint64_t *__restrict__ offs, uint32_t nport,
                                                   uint8_t *__restrict__ out) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nport) return;
    const uint4 d = desc[k];
    if (d.y <= d.x) return;
    uint8_t *o = out + offs[k];
    for (uint32_t q = d.x; q < d.y; ++q) *o++ = buf[q];
    *o++ = ':';
    for (uint32_t q = d.z; q < d.w; ++q) *o++ = buf[q];
    *o = '\n';
}

static int dev_nmap_ports(sg_ctx *c, const uint8_t *d_buf, uint64_t n, sg_dev_text *res) {
    *res = sg_dev_text{};
    Lines L;
    SG_TRY(run_lines(c, d_buf, n, FMT_SLOTS, &L, false));
    const uint32_t R = L.n_rec;
    res->in_records = R;
    if (R == 0) return SG_OK;
    uint32_t *reps, *ports;
    SG_TRY(slot(c, S_F_REC, (size_t)R + 16, &reps));
    SG_TRY(slot(c, S_F_KEY, (size_t)R + 16, &ports));
    uint32_t nrep = 0, nport = 0;
    SG_TRY(run_select2(c, "nmap_classify", NmapPred{d_buf, L.spans}, R, reps, ports, &nrep, &nport, 40.0));
    if (nport == 0) return SG_OK;
    uint4 *desc;
    uint64_t *offs;
    SG_TRY(slot(c, S_F_DESC, (size_t)nport + 1, &desc));
    SG_TRY(slot(c, S_F_OFFS, (size_t)nport + 1, &offs));
    SG_LAUNCH(c, "nmap_prep", k_nmap_prep, (nport + 255) / 256, 256, 0, d_buf, L.spans, reps, nrep, ports, nport, desc);
    uint64_t total = 0;
    SG_TRY(run_scan64(c, "nmap_scan", NmapLen{desc}, nport, offs, &total));
    uint8_t *out;
    SG_TRY(slot(c, S_F_OUT, total + 16, &out));
    SG_LAUNCH_B(c, "nmap_emit", 2.0 * total, k_nmap_emit, (nport + 255) / 256, 256, 0, d_buf, desc, offs, nport, out);
    res->data = out;
    res->bytes = total;
    // records = ports with a host (count from the descriptors: rows of nonzero length)
    uint64_t recs = 0;
    {
        // lengths are > 0 exactly for kept rows; count them on the host from a compaction
        uint32_t *tmp;
        SG_TRY(slot(c, S_F_A, (size_t)nport + 16, &tmp));
        uint32_t kept = 0;
        struct KeptPred {
            const uint4 *d;
            __device__ uint32_t operator()(uint32_t i) const { return d[i].y > d[i].x ? 1u : 0u; }
        };
        SG_TRY(run_select2(c, "nmap_kept", KeptPred{desc}, nport, tmp, (uint32_t *)nullptr, &kept, nullptr, 16.0));
        recs = kept;
    }
    res->records = recs;
    return SG_OK;
}

// ------------------------------------------------------------------ httpx -json
constexpr uint32_t JS_MAXKEYS = 64;
constexpr uint32_t JS_KEYBYTES = 4096;
constexpr uint32_t JS_NONE = 0xffffffffu;

struct JsonArgs {
    const uint8_t *buf;
    const uint2 *spans;
    uint32_t R;
    const uint8_t *keys;       // concatenated key bytes
    const uint32_t *key_offs;  // nkeys + 1
    uint32_t nkeys;
    uint4 *desc;               // R * nkeys: {value start, value end, rows, bytes}
};

__device__ __forceinline__ bool js_ws(uint8_t b) { return b == ' ' || b == '\t' || b == '\r' || b == '\n'; }

__device__ __forceinline__ int js_hex(uint8_t b) {
    if (b >= '0' && b <= '9') return b - '0';
    if (b >= 'a' && b <= 'f') return b - 'a' + 10;
    if (b >= 'A' && b <= 'F') return b - 'A' + 10;
    return -1;
}

// Decode the JSON string body [a, b) (between the quotes) into `put`. Escapes follow
// json.loads: \" \\ \/ \b \f \n \r \t and \uXXXX (a high+low surrogate pair combines into
// one code point; a lone surrogate is encoded as its 3-byte form, like Python's
// 'surrogatepass'). A decoded U+000A is written as the two bytes '\' 'n' so a row stays
// one line (KEY: as the byte 0x0a, the form a requested key is compared in). Malformed
// escapes are copied verbatim.
template <bool KEY = false, class Buf, class Put>
__device__ __forceinline__ void js_decode(const Buf &buf, uint32_t a, uint32_t b, Put &put) {
    auto put_cp = [&](uint32_t cp) {
        if (cp == 0x0a && !KEY) { put('\\'); put('n'); }
        else if (cp < 0x80) put((uint8_t)cp);
        else if (cp < 0x800) { put((uint8_t)(0xc0 | (cp >> 6))); put((uint8_t)(0x80 | (cp & 0x3f))); }
        else if (cp < 0x10000) {
            put((uint8_t)(0xe0 | (cp >> 12))); put((uint8_t)(0x80 | ((cp >> 6) & 0x3f))); put((uint8_t)(0x80 | (cp & 0x3f)));
        } else {
            put((uint8_t)(0xf0 | (cp >> 18))); put((uint8_t)(0x80 | ((cp >> 12) & 0x3f)));
            put((uint8_t)(0x80 | ((cp >> 6) & 0x3f))); put((uint8_t)(0x80 | (cp & 0x3f)));
        }
    };
    auto u4 = [&](uint32_t p, uint32_t *v) -> bool {
        if (p + 4 > b) return false;
        uint32_t x = 0;
        for (uint32_t q = 0; q < 4; ++q) {
            const int h = js_hex(buf[p + q]);
            if (h < 0) return false;
            x = (x << 4) | (uint32_t)h;
        }
        *v = x;
        return true;
    };
    uint32_t p = a;
    while (p < b) {
        const uint8_t ch = buf[p];
        if (ch != '\\' || p + 1 >= b) { put(ch); ++p; continue; }
        const uint8_t e = buf[p + 1];
        uint32_t v;
        switch (e) {
            case '"': case '\\': case '/': put(e); p += 2; break;
            case 'b': put(0x08); p += 2; break;
            case 'f': put(0x0c); p += 2; break;
            case 'n': if (KEY) put(0x0a); else { put('\\'); put('n'); } p += 2; break;
            case 'r': put(0x0d); p += 2; break;
            case 't': put(0x09); p += 2; break;
            case 'u':
                if (!u4(p + 2, &v)) { put(ch); ++p; break; }
                p += 6;
                if (v >= 0xd800 && v < 0xdc00 && p + 1 < b && buf[p] == '\\' && buf[p + 1] == 'u') {
                    uint32_t lo;
                    if (u4(p + 2, &lo) && lo >= 0xdc00 && lo < 0xe000) {
                        v = 0x10000 + ((v - 0xd800) << 10) + (lo - 0xdc00);
                        p += 6;
                    }
                }
                put_cp(v);
                break;
            default: put(ch); ++p; break;
        }
    }
}

// Walk one value [vs, ve) (already trimmed): a string -> one decoded row; an array ->
// one row per element (strings decoded, anything else its trimmed raw text); anything
// else -> its raw text. Empty rows are dropped. `row(begin)` / `put(byte)` / `end()`
// receive the output.
template <class Buf, class Sink>
__device__ __forceinline__ void js_value(const Buf &buf, uint32_t vs, uint32_t ve, Sink &sk) {
    auto emit_item = [&](uint32_t a, uint32_t b) {
        while (a < b && js_ws(buf[a])) ++a;
        while (b > a && js_ws(buf[b - 1])) --b;
        if (a >= b) return;
        if (buf[a] == '"' && b - a >= 2 && buf[b - 1] == '"') {
            if (b - a == 2) return;  // ""
            sk.begin();
            js_decode(buf, a + 1, b - 1, sk);
            sk.end();
        } else {
            sk.begin();
            for (uint32_t q = a; q < b; ++q) sk(buf[q]);
            sk.end();
        }
    };
    if (vs >= ve) return;
    if (buf[vs] != '[') { emit_item(vs, ve); return; }
    // array: split at depth-1 commas outside strings
    uint32_t depth = 0, start = vs + 1;
    bool in_str = false, esc = false;
    for (uint32_t p = vs; p < ve; ++p) {
        const uint8_t ch = buf[p];
        if (in_str) {
            if (esc) esc = false;
            else if (ch == '\\') esc = true;
            else if (ch == '"') in_str = false;
            continue;
        }
        if (ch == '"') { in_str = true; continue; }
        if (ch == '[' || ch == '{') { ++depth; continue; }
        if (ch == ']' || ch == '}') {
            if (depth == 1) { emit_item(start, p); start = p + 1; }
            --depth;
            continue;
        }
        if (ch == ',' && depth == 1) { emit_item(start, p); start = p + 1; }
    }
}

// js_value's (rows, bytes) for an array value [vs, ve) holding no backslash (its strings
// decode to themselves), 16 bytes per step: SWAR masks of the bytes js_value reacts to
// ('"', '[', '{', ']', '}', ',') and of the non-blank bytes, and only those events walked
// through js_value's state machine (same depth arithmetic, same item ends), each item's first
// and last non-blank bytes taken from the masks between events. The byte walk cost the JSON
// scan ~2.7 ms of its 10.5 per fields step (measured by walking every such value twice).
__device__ __forceinline__ uint32_t js_swar_eq(uint32_t x, uint32_t pat) {
    const uint32_t y = x ^ pat;
    const uint32_t z = ~(((y & 0x7f7f7f7fu) + 0x7f7f7f7fu) | y | 0x7f7f7f7fu);
    return (((z >> 7) & 0x01010101u) * 0x01020408u) >> 24;
}
// on_item(a, b, q): each item's trimmed text [a, b) (non-empty), as js_value's emit_item sees
// it; q: it starts and ends with a quote (2+ bytes)
template <class OnItem>
__device__ __forceinline__ void js_array_plain_items(const uint8_t *buf, uint32_t vs, uint32_t ve, OnItem on_item) {
    const uint4 *gb = reinterpret_cast<const uint4 *>(buf);
    uint32_t depth = 0;
    bool in_str = false;
    uint32_t fnw = 0xffffffffu, lnw = 0;  // the current item's first / last non-blank byte
    bool fq = false, lq = false;          // ... are quotes
    auto item_end = [&]() {
        if (fnw != 0xffffffffu) on_item(fnw, lnw + 1u, fq && lq && lnw > fnw);
        fnw = 0xffffffffu;
    };
    auto content = [&](uint32_t pos, bool q) {  // a non-blank byte of the current item
        if (fnw == 0xffffffffu) { fnw = pos; fq = q; }
        lnw = pos;
        lq = q;
    };
    for (uint32_t b0 = vs & ~15u; b0 < ve; b0 += 16u) {
        const uint4 v = gb[b0 >> 4];
        const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
        uint32_t qm = 0, om = 0, cm = 0, km = 0, wm = 0;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            const uint32_t x = wd[d], lx = x | 0x20202020u;
            qm |= js_swar_eq(x, 0x22222222u) << (4 * d);
            om |= js_swar_eq(lx, 0x7b7b7b7bu) << (4 * d);
            cm |= js_swar_eq(lx, 0x7d7d7d7du) << (4 * d);
            km |= js_swar_eq(x, 0x2c2c2c2cu) << (4 * d);
            wm |= (js_swar_eq(x, 0x20202020u) | js_swar_eq(x, 0x09090909u) | js_swar_eq(x, 0x0d0d0d0du) |
                   js_swar_eq(x, 0x0a0a0a0au)) << (4 * d);
        }
        const uint32_t lo = vs > b0 ? vs - b0 : 0u, hi = ve - b0 < 16u ? ve - b0 : 16u;
        const uint32_t rng = ((1u << hi) - 1u) & ~((1u << lo) - 1u);
        const uint32_t nw = ~wm & rng;
        uint32_t ev = (qm | om | cm | km) & rng, from = lo;
        while (ev) {
            const uint32_t j = (uint32_t)__builtin_ctz(ev);
            ev &= ev - 1u;
            const uint32_t seg = nw & ((1u << j) - 1u) & ~((1u << from) - 1u);  // plain bytes before it
            if (seg) {
                content(b0 + (uint32_t)__builtin_ctz(seg), false);
                lnw = b0 + 31u - (uint32_t)__builtin_clz(seg);
            }
            from = j + 1u;
            const uint32_t bit = 1u << j, pos = b0 + j;
            if (in_str) {  // only the closing quote ends it; the rest is the item's text
                if (qm & bit) in_str = false;
                content(pos, (qm & bit) != 0u);
                continue;
            }
            if (qm & bit) { in_str = true; content(pos, true); continue; }
            if (om & bit) { ++depth; if (pos != vs) content(pos, false); continue; }  // all but the array's own
            if (cm & bit) {
                if (depth == 1u) item_end();
                else content(pos, false);
                --depth;
                continue;
            }
            if (depth == 1u) item_end();  // ','
            else content(pos, false);
        }
        const uint32_t seg = nw & ~((1u << from) - 1u);
        if (seg) {
            content(b0 + (uint32_t)__builtin_ctz(seg), false);
            lnw = b0 + 31u - (uint32_t)__builtin_clz(seg);
        }
    }
}

// js_value's (rows, bytes) for such an array: an item "..." of 2+ bytes gives its text
// between the quotes (none when empty), any other item its raw text
__device__ __forceinline__ void js_count_array_plain(const uint8_t *buf, uint32_t vs, uint32_t ve, uint32_t *rows,
                                                     uint32_t *bytes) {
    uint32_t nrow = 0, nb = 0;
    js_array_plain_items(buf, vs, ve, [&](uint32_t a, uint32_t b, bool q) {
        const uint32_t len = q ? b - a - 2u : b - a;
        if (len) { ++nrow; nb += len + 1u; }
    });
    *rows = nrow;
    *bytes = nb;
}

// no backslash in [vs, ve) (16-byte steps)
__device__ __forceinline__ bool js_no_backslash(const uint8_t *buf, uint32_t vs, uint32_t ve) {
    const uint4 *gb = reinterpret_cast<const uint4 *>(buf);
    for (uint32_t b0 = vs & ~15u; b0 < ve; b0 += 16u) {
        const uint4 v = gb[b0 >> 4];
        const uint32_t m = js_swar_eq(v.x, 0x5c5c5c5cu) | (js_swar_eq(v.y, 0x5c5c5c5cu) << 4) |
                           (js_swar_eq(v.z, 0x5c5c5c5cu) << 8) | (js_swar_eq(v.w, 0x5c5c5c5cu) << 12);
        const uint32_t lo = vs > b0 ? vs - b0 : 0u, hi = ve - b0 < 16u ? ve - b0 : 16u;
        if (m & ((1u << hi) - 1u) & ~((1u << lo) - 1u)) return false;
    }
    return true;
}

// Compares a decoded key stream with one requested key.
struct JsKeyEq {
    const uint8_t *k;
    uint32_t n, i = 0;
    bool ok = true;
    __device__ void operator()(uint8_t ch) {
        ok = ok && i < n && k[i] == ch;
        ++i;
    }
    __device__ bool eq() const { return ok && i == n; }
};

struct JsCount {
    uint32_t rows = 0, bytes = 0, cur = 0;
    __device__ void begin() { cur = 0; }
    __device__ void operator()(uint8_t) { ++cur; }
    __device__ void end() { if (cur) { ++rows; bytes += cur + 1; } }
};

// One thread per record: the record is read with aligned 16-byte loads and walked byte by
// byte with a JSON state machine (string/escape state, depth, key at a
// depth-1 colon, value end at a depth-1 comma or the closing brace, whitespace-only
// framing). Per-thread key spans live in LDS. Requested keys are pre-filtered by length
// and first byte before a byte compare.
constexpr int JT_BLOCK = 128;
__global__ __launch_bounds__(JT_BLOCK) __attribute__((amdgpu_waves_per_eu(6))) void k_json_scan_t(JsonArgs a) {
    extern __shared__ uint2 s_span[];  // JT_BLOCK * nkeys
    __shared__ uint8_t s_keys[JS_KEYBYTES];
    __shared__ uint32_t s_koff[JS_MAXKEYS + 1];
    __shared__ uint32_t s_kid[JS_MAXKEYS];  // klen | first byte << 16
    for (uint32_t q = threadIdx.x; q <= a.nkeys; q += JT_BLOCK) s_koff[q] = a.key_offs[q];
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < s_koff[a.nkeys]; q += JT_BLOCK) s_keys[q] = a.keys[q];
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < a.nkeys; q += JT_BLOCK) {
        const uint32_t kl = s_koff[q + 1] - s_koff[q];
        s_kid[q] = kl | ((kl ? (uint32_t)s_keys[s_koff[q]] : 0x100u) << 16);
    }
    __syncthreads();
    const uint32_t nk = a.nkeys;
    uint2 *my = s_span + threadIdx.x * nk;
    for (uint32_t r = blockIdx.x * JT_BLOCK + threadIdx.x; r < a.R; r += gridDim.x * JT_BLOCK) {
        const uint2 sp = a.spans[r];
        for (uint32_t k = 0; k < nk; ++k) my[k] = make_uint2(JS_NONE, 0);
        uint32_t depth = 0, str_s = 0, str_e = 0, val_s = 0, open_pos = JS_NONE, close_pos = JS_NONE;
        uint32_t first_nws = JS_NONE, last_nws = 0, c0 = 0;
        int cur_key = -1;
        bool in_str = false, esc = false, kesc = false, bad = false, done = false;
        // vbs: a backslash (in or out of a string) inside the current member's value; escm:
        // per requested key, whether its (last) value held one — a value without any takes
        // the counting fast path below (its rows are its raw text, no byte walk)
        bool vbs = false;
        uint64_t escm = 0;
        // Per 16-byte chunk, SWAR masks of the event bytes (quote, backslash, { [ } ] : ,) and
        // only those positions walked through the state machine — JSON lines hold an event
        // every few bytes, and every other byte only matters for the line's first and last
        // non-blank bytes (found after the walk). Escapes act inside strings only, as in a
        // byte walk: a backslash escapes the next byte, whatever it is.
        uint32_t esc_pos = JS_NONE;
        // 64-byte steps: a lane's four 16-B loads of a step are issued together (a half cache
        // line per request instead of 16 B, so a line evicted between a lane's steps is
        // fetched 2x rather than 8x), and the next step's four are in flight while this one
        // is walked
        const uint4 *gb = reinterpret_cast<const uint4 *>(a.buf);
        const uint32_t w0 = sp.x & ~63u;
        uint4 n0, n1, n2, n3;
        {
            const uint32_t c = w0 >> 4;
            n0 = w0 + 16u > sp.x && w0 < sp.y ? gb[c] : make_uint4(0, 0, 0, 0);
            n1 = w0 + 32u > sp.x && w0 + 16u < sp.y ? gb[c + 1] : make_uint4(0, 0, 0, 0);
            n2 = w0 + 48u > sp.x && w0 + 32u < sp.y ? gb[c + 2] : make_uint4(0, 0, 0, 0);
            n3 = w0 + 64u > sp.x && w0 + 48u < sp.y ? gb[c + 3] : make_uint4(0, 0, 0, 0);
        }
        for (uint32_t w = w0; w < sp.y && !bad; w += 64) {
            const uint4 v0 = n0, v1 = n1, v2 = n2, v3 = n3;
            {
                const uint32_t wn = w + 64u, c = wn >> 4;
                n0 = wn < sp.y ? gb[c] : make_uint4(0, 0, 0, 0);
                n1 = wn + 16u < sp.y ? gb[c + 1] : make_uint4(0, 0, 0, 0);
                n2 = wn + 32u < sp.y ? gb[c + 2] : make_uint4(0, 0, 0, 0);
                n3 = wn + 48u < sp.y ? gb[c + 3] : make_uint4(0, 0, 0, 0);
            }
            uint64_t ev = 0;
            const uint32_t wd[16] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w,
                                     v2.x, v2.y, v2.z, v2.w, v3.x, v3.y, v3.z, v3.w};
#pragma unroll
            for (int d = 0; d < 16; ++d) {
                const uint32_t x = wd[d];
                auto eqm = [](uint32_t y) -> uint32_t {  // high bit of each zero byte of y
                    return ~(((y & 0x7f7f7f7fu) + 0x7f7f7f7fu) | y | 0x7f7f7f7fu);
                };
                const uint32_t lx = x | 0x20202020u;  // '[' -> '{', ']' -> '}'
                const uint32_t z = eqm(x ^ 0x22222222u) | eqm(x ^ 0x5c5c5c5cu) | eqm(lx ^ 0x7b7b7b7bu) |
                                   eqm(lx ^ 0x7d7d7d7du) | eqm(x ^ 0x3a3a3a3au) | eqm(x ^ 0x2c2c2c2cu);
                ev |= (uint64_t)(((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u)) << (4 * d);
            }
            if (w < sp.x) ev &= ~0ull << (sp.x - w);
            if (sp.y - w < 64u) ev &= (1ull << (sp.y - w)) - 1ull;
            while (ev && !bad) {
                const uint32_t j = (uint32_t)__builtin_ctzll(ev);
                ev &= ev - 1u;
                const uint32_t q = w + j;
                // word j / 4 of the step by a select tree on values (register-resident)
                const bool o1 = (j >> 2) & 1u, o2 = (j >> 3) & 1u;
                const uint32_t s0 = o2 ? (o1 ? v0.w : v0.z) : (o1 ? v0.y : v0.x);
                const uint32_t s1 = o2 ? (o1 ? v1.w : v1.z) : (o1 ? v1.y : v1.x);
                const uint32_t s2 = o2 ? (o1 ? v2.w : v2.z) : (o1 ? v2.y : v2.x);
                const uint32_t s3 = o2 ? (o1 ? v3.w : v3.z) : (o1 ? v3.y : v3.x);
                const uint32_t xw = (j & 32u) ? ((j & 16u) ? s3 : s2) : ((j & 16u) ? s1 : s0);
                const uint32_t b = (xw >> (8u * (j & 3u))) & 0xffu;
                if (in_str) {
                    if (q == esc_pos) continue;  // the escaped byte
                    if (b == '\\') { esc_pos = q + 1; kesc = true; vbs = true; }
                    else if (b == '"') { in_str = false; str_e = q; }
                    continue;
                }
                if (b == '\\') { vbs = true; continue; }  // outside strings a backslash is no event
                if (b == '"') {
                    if (depth == 0) bad = true;
                    in_str = true;
                    kesc = false;
                    str_s = q + 1;
                    esc_pos = JS_NONE;
                    continue;
                }
                if (done) { bad = true; continue; }
                if (b == '{' || b == '[') {
                    if (depth == 0) {
                        if (b != '{') bad = true;
                        open_pos = q;
                    }
                    ++depth;
                } else if (b == '}' || b == ']') {
                    if (depth == 0) { bad = true; continue; }
                    if (depth == 1) {
                        if (b != '}') bad = true;
                        if (cur_key >= 0) {
                            my[cur_key] = make_uint2(val_s, q);
                            escm = (escm & ~(1ull << cur_key)) | ((uint64_t)vbs << cur_key);
                        }
                        cur_key = -1;
                        done = true;
                        close_pos = q;
                    }
                    --depth;
                } else if (depth == 1) {
                    if (b == ':') {
                        const uint32_t kl = str_e - str_s;
                        const uint32_t c0 = kl ? (uint32_t)a.buf[str_s] : 0x100u;
                        const uint32_t id = kl | (c0 << 16);
                        cur_key = -1;
                        for (uint32_t k = 0; k < nk; ++k) {
                            bool eq;
                            if (kesc) {  // escaped key: compare its decoded form
                                JsKeyEq cmp{s_keys + s_koff[k], s_koff[k + 1] - s_koff[k]};
                                js_decode<true>(a.buf, str_s, str_e, cmp);
                                eq = cmp.eq();
                            } else {
                                if (s_kid[k] != id) continue;
                                eq = true;
                                for (uint32_t x = 1; x < kl && eq; ++x) eq = a.buf[str_s + x] == s_keys[s_koff[k] + x];
                            }
                            if (eq) { cur_key = (int)k; break; }
                        }
                        val_s = q + 1;
                        vbs = false;
                    } else {  // ','
                        if (cur_key >= 0) {
                            my[cur_key] = make_uint2(val_s, q);
                            escm = (escm & ~(1ull << cur_key)) | ((uint64_t)vbs << cur_key);
                        }
                        cur_key = -1;
                    }
                }
            }
        }
        // the line's first and last non-blank bytes (a JSON line starts with '{' and ends
        // with '}', so these loops stop at once)
        if (!bad) {
            for (uint32_t q = sp.x; q < sp.y; ++q)
                if (!js_ws(a.buf[q])) { first_nws = q; break; }
            for (uint32_t q = sp.y; q > sp.x; --q)
                if (!js_ws(a.buf[q - 1])) { last_nws = q - 1; break; }
        }
        const bool ok = !bad && !in_str && depth == 0 && done && first_nws == open_pos && last_nws == close_pos;
        for (uint32_t k = 0; k < nk; ++k) {
            uint4 d = make_uint4(0, 0, 0, 0);
            const uint2 vsp = my[k];
            if (ok && vsp.x != JS_NONE) {
                uint32_t vs = vsp.x, ve = vsp.y;
                while (vs < ve && js_ws(a.buf[vs])) ++vs;
                while (ve > vs && js_ws(a.buf[ve - 1])) --ve;
                // rows without a walk: a value with no backslash that is not an array is one
                // row of its raw text, or of the text between its quotes (js_value: a string
                // without escapes decodes to itself; "" gives no row)
                const uint8_t c0 = vs < ve ? a.buf[vs] : 0;
                const bool strv = c0 == '"' && ve - vs >= 2 && a.buf[ve - 1] == '"';
                if (vs >= ve) {
                    d = make_uint4(vs, ve, 0, 0);
                } else if (c0 != '[' && !((escm >> k) & 1u)) {
                    const uint32_t len = strv ? ve - vs - 2 : ve - vs;
                    d = make_uint4(vs, ve, len ? 1u : 0u, len ? len + 1u : 0u);
                } else if (c0 == '[' && !((escm >> k) & 1u)) {
                    uint32_t nr, nbt;
                    js_count_array_plain(a.buf, vs, ve, &nr, &nbt);
                    d = make_uint4(vs, ve, nr, nbt);
                } else {
                    JsCount cnt;
                    js_value(a.buf, vs, ve, cnt);
                    d = make_uint4(vs, ve, cnt.rows, cnt.bytes);
                }
            }
            a.desc[(size_t)r * nk + k] = d;
        }
    }
}

// packed (bytes << 32 | rows) per (record, key). Rows never outgrow the input: each
// value's rows are no longer than its raw text plus the delimiter that follows it, so
// the output total stays below the 4 GiB input limit and the fields never carry.
struct JsonLen {
    const uint4 *desc;
    __device__ uint64_t operator()(uint32_t i) const {
        const uint4 d = desc[i];
        return ((uint64_t)d.w << 32) | d.z;
    }
};

// A wave's 64 items write one contiguous output range (items in order, offsets from one
// scan): the rows are decoded into a per-wave LDS window at their offsets inside that range,
// then the wave stores the range with consecutive lanes on consecutive bytes — the direct
// version had each lane store its own rows one byte at a time (64 scattered bytes per store
// instruction). A wave whose range exceeds the window writes directly.
constexpr uint32_t JE_CAP = 4096;
struct JsWriteLds {
    uint8_t *win;  // the wave's window (or the output at the wave's range start); o relative to it
    uint32_t *row_rec, *row_key;
    uint32_t o, row, rec, key;
    __device__ void begin() {}
    __device__ void operator()(uint8_t ch) { win[o++] = ch; }
    __device__ void end() {
        win[o++] = '\n';
        row_rec[row] = rec;
        row_key[row] = key;
        ++row;
    }
};

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void k_json_emit(const uint8_t *__restrict__ buf, const uint4 *__restrict__ desc,
                                                   const uint64_t *__restrict__ offs, uint32_t nitems, uint32_t nkeys,
                                                   uint64_t total_bytes, uint8_t *__restrict__ out,
                                                   uint32_t *__restrict__ row_rec, uint32_t *__restrict__ row_key) {
    __shared__ uint8_t s_win[4][JE_CAP];
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t iw0 = i - lane;
    if (iw0 >= nitems) return;  // whole wave
    const uint64_t wb = offs[iw0] >> 32;
    const uint64_t we = iw0 + 64 < nitems ? offs[iw0 + 64] >> 32 : total_bytes;
    const bool staged = we - wb <= JE_CAP;
    if (i < nitems) {
        const uint4 d = desc[i];
        if (d.z != 0) {
            const uint64_t off = offs[i];
            // one writer for both cases (two instantiations of the walk cost registers): the
            // window, or the output at the wave's range start
            JsWriteLds w{staged ? s_win[wid] : out + wb, row_rec, row_key, (uint32_t)((off >> 32) - wb), (uint32_t)off,
                         i / nkeys, i % nkeys};
            if (buf[d.x] == '[' && js_no_backslash(buf, d.x, d.y)) {
                // an array whose strings decode to themselves: items from the 16-byte walk
                js_array_plain_items(buf, d.x, d.y, [&](uint32_t a, uint32_t b, bool q) {
                    if (q) {
                        if (b - a == 2u) return;
                        ++a;
                        --b;
                    }
                    for (uint32_t q = a; q < b; ++q) w(buf[q]);
                    w.end();
                });
            } else {
                js_value(buf, d.x, d.y, w);
            }
        }
    }
    if (!staged) return;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    const uint32_t len = (uint32_t)(we - wb);
    for (uint32_t k = lane; k < len; k += 64) out[wb + k] = s_win[wid][k];
}

int dev_json_fields(sg_ctx *c, const uint8_t *d_buf, uint64_t n, const uint8_t *keys, const uint32_t *key_offs,
                           uint32_t nkeys, sg_dev_rows *res) {
    *res = sg_dev_rows{};
    if (nkeys == 0 || nkeys > JS_MAXKEYS) { set_error("json fields: 1..%u keys", JS_MAXKEYS); return SG_E_INVAL; }
    if (key_offs[0] != 0 || key_offs[nkeys] > JS_KEYBYTES) { set_error("json fields: keys exceed %u bytes", JS_KEYBYTES); return SG_E_INVAL; }
    for (uint32_t k = 0; k < nkeys; ++k)
        if (key_offs[k + 1] < key_offs[k]) { set_error("json fields: bad key offsets"); return SG_E_INVAL; }
    Lines L;
    SG_TRY(run_lines(c, d_buf, n, FMT_SLOTS, &L, false));
    const uint32_t R = L.n_rec;
    res->in_records = R;
    if (R == 0) return SG_OK;
    const uint64_t items = (uint64_t)R * nkeys;
    if (items >= (1ull << 32)) { set_error("json fields: records x keys exceeds 2^32"); return SG_E_TOO_LARGE; }
    uint32_t *d_koff;
    uint8_t *d_keys;
    SG_TRY(slot(c, S_F_KEYS, JS_KEYBYTES + 4 * (JS_MAXKEYS + 1), &d_keys));
    d_koff = reinterpret_cast<uint32_t *>(d_keys + JS_KEYBYTES);
    SG_HIP(hipMemcpyAsync(d_keys, keys, key_offs[nkeys] ? key_offs[nkeys] : 1, hipMemcpyHostToDevice, c->stream));
    SG_HIP(hipMemcpyAsync(d_koff, key_offs, 4 * (nkeys + 1), hipMemcpyHostToDevice, c->stream));
    uint4 *desc;
    uint64_t *offs;
    SG_TRY(slot(c, S_F_DESC, items + 1, &desc));
    SG_TRY(slot(c, S_F_OFFS, items + 1, &offs));
    JsonArgs ja{d_buf, L.spans, R, d_keys, d_koff, nkeys, desc};
    const uint32_t grid = (uint32_t)std::min<uint64_t>((R + JT_BLOCK - 1) / JT_BLOCK, 256u * 16u);
    SG_LAUNCH_B(c, "json_scan", (double)n + 16.0 * items, k_json_scan_t, grid, JT_BLOCK,
                JT_BLOCK * nkeys * sizeof(uint2), ja);
    uint64_t total = 0;
    SG_TRY(run_scan64(c, "json_scan_len", JsonLen{desc}, (uint32_t)items, offs, &total));
    const uint64_t rows = total & 0xffffffffu, bytes = total >> 32;
    uint8_t *out;
    uint32_t *rrec, *rkey;
    SG_TRY(slot(c, S_F_OUT, bytes + 16, &out));
    SG_TRY(slot(c, S_F_REC, rows + 1, &rrec));
    SG_TRY(slot(c, S_F_KEY, rows + 1, &rkey));
    SG_LAUNCH_B(c, "json_emit", 2.0 * bytes + 8.0 * rows, k_json_emit, (uint32_t)((items + 255) / 256), 256, 0, d_buf,
                desc, offs, (uint32_t)items, nkeys, bytes, out, rrec, rkey);
    res->data = out;
    res->bytes = bytes;
    res->rows = rows;
    res->row_rec = rrec;
    res->row_key = rkey;
    return SG_OK;
}

}  // namespace sg

using namespace sg;

namespace {
struct Acq {
    sg_ctx *c = nullptr;
    ~Acq() { if (c) pool_release(c); }
};
int acquire_ctx(Acq *a) {
    int dev = 0;
    SG_TRY(pick_device(&dev));
    SG_TRY(pool_acquire(dev, &a->c));
    SG_HIP(hipSetDevice(dev));
    return SG_OK;
}
int upload_aligned(sg_ctx *c, const uint8_t *host, size_t n, uint8_t **d) {
    SG_TRY(slot(c, S_IN, n + 16, d));
    if (n) SG_HIP(hipMemcpyAsync(*d, host, n, hipMemcpyHostToDevice, c->stream));
    return SG_OK;
}
int dev_aligned(sg_ctx *c, const uint8_t *d, size_t n, const uint8_t **out) {
    if (((uintptr_t)d & 15) == 0) { *out = d; return SG_OK; }
    uint8_t *a;
    SG_TRY(slot(c, S_IN, n + 16, &a));
    if (n) SG_HIP(hipMemcpyAsync(a, d, n, hipMemcpyDeviceToDevice, c->stream));
    *out = a;
    return SG_OK;
}
}  // namespace

extern "C" {

int sg_dev_nmap_ports(sg_ctx *c, const uint8_t *d_buf, size_t n, sg_dev_text *res) {
    if (!c || !res || (!d_buf && n)) { set_error("sg_dev_nmap_ports: bad arguments"); return SG_E_INVAL; }
    if (n > MAX_BYTES) { set_error("input exceeds 4 GiB per call"); return SG_E_TOO_LARGE; }
    SG_HIP(hipSetDevice(c->device));
    const uint8_t *b;
    SG_TRY(dev_aligned(c, d_buf, n, &b));
    return dev_nmap_ports(c, b, n, res);
}

int sg_nmap_ports(const uint8_t *buf, size_t n, uint8_t *out, size_t cap, size_t *out_n) {
    if (!out_n || (!buf && n)) { set_error("sg_nmap_ports: bad arguments"); return SG_E_INVAL; }
    if (n > MAX_BYTES) { set_error("input exceeds 4 GiB per call"); return SG_E_TOO_LARGE; }
    Acq a;
    SG_TRY(acquire_ctx(&a));
    sg_ctx *c = a.c;
    uint8_t *d;
    SG_TRY(upload_aligned(c, buf, n, &d));
    sg_dev_text r;
    SG_TRY(dev_nmap_ports(c, d, n, &r));
    *out_n = r.bytes;
    if (r.bytes > cap) { SG_HIP(hipStreamSynchronize(c->stream)); set_error("output capacity too small"); return SG_E_CAP; }
    if (r.bytes) SG_HIP(hipMemcpyAsync(out, r.data, r.bytes, hipMemcpyDeviceToHost, c->stream));
    SG_HIP(hipStreamSynchronize(c->stream));
    return SG_OK;
}

int sg_dev_json_fields(sg_ctx *c, const uint8_t *d_buf, size_t n, const uint8_t *keys, const uint32_t *key_offs,
                       uint32_t n_keys, sg_dev_rows *res) {
    if (!c || !res || !key_offs || (!d_buf && n) || (!keys && n_keys)) {
        set_error("sg_dev_json_fields: bad arguments");
        return SG_E_INVAL;
    }
    if (n > MAX_BYTES) { set_error("input exceeds 4 GiB per call"); return SG_E_TOO_LARGE; }
    SG_HIP(hipSetDevice(c->device));
    const uint8_t *b;
    SG_TRY(dev_aligned(c, d_buf, n, &b));
    return dev_json_fields(c, b, n, keys, key_offs, n_keys, res);
}

int sg_json_fields(const uint8_t *buf, size_t n, const uint8_t *keys, const uint32_t *key_offs, uint32_t n_keys,
                   uint8_t *out, size_t cap, size_t *out_n, uint32_t *row_rec, uint32_t *row_key, size_t rows_cap,
                   size_t *n_rows) {
    if (!out_n || !n_rows || !key_offs || (!buf && n) || (!keys && n_keys)) {
        set_error("sg_json_fields: bad arguments");
        return SG_E_INVAL;
    }
    if (n > MAX_BYTES) { set_error("input exceeds 4 GiB per call"); return SG_E_TOO_LARGE; }
    Acq a;
    SG_TRY(acquire_ctx(&a));
    sg_ctx *c = a.c;
    uint8_t *d;
    SG_TRY(upload_aligned(c, buf, n, &d));
    sg_dev_rows r;
    SG_TRY(dev_json_fields(c, d, n, keys, key_offs, n_keys, &r));
    *out_n = r.bytes;
    *n_rows = r.rows;
    if (r.bytes > cap || r.rows > rows_cap) {
        SG_HIP(hipStreamSynchronize(c->stream));
        set_error("output capacity too small");
        return SG_E_CAP;
    }
    if (r.bytes) SG_HIP(hipMemcpyAsync(out, r.data, r.bytes, hipMemcpyDeviceToHost, c->stream));
    if (r.rows && row_rec) SG_HIP(hipMemcpyAsync(row_rec, r.row_rec, 4 * r.rows, hipMemcpyDeviceToHost, c->stream));
    if (r.rows && row_key) SG_HIP(hipMemcpyAsync(row_key, r.row_key, 4 * r.rows, hipMemcpyDeviceToHost, c->stream));
    SG_HIP(hipStreamSynchronize(c->stream));
    return SG_OK;
}

}  // extern "C"
