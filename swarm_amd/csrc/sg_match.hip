// sg_match.hip — A4 signature matching: Aho-Corasick for literal signatures (grep -F /
// `sig in line`) and multi-DFA for regex signatures (re.search existence), on records of
// an HBM-resident line buffer.
//
// Automata are built on the host (C++) into dense byte-class transition tables:
//   * byte classes: every byte that occurs in some pattern gets its own class, all other
//     bytes share class 0 (for Aho-Corasick class 0 always returns to the root); with
//     SG_NOCASE 'A'-'Z' share the class of 'a'-'z' (C-locale grep -i);
//   * states are numbered breadth-first, so the hot shallow states come first: the first
//     H rows (u16 entries) are staged in LDS, the rest are read from HBM/L2;
//   * a per-state "has output" bitmap (LDS when it fits) gates the output walk.
// Device: one thread per record walks its bytes (aligned 4-byte loads) through the table;
// every (record, signature) event is appended with an atomic slot; events are then
// radix-sorted and de-duplicated, so hits come out sorted by (record, signature) and the
// matched lines in input order (grep's output).
#include "sg_internal.hpp"
#include "sg_prims.hpp"

#include <algorithm>
#include <deque>
#include <map>
#include <string.h>

#include "sg_regex.hpp"

using namespace sg;

struct sg_matcher {
    int kind = 0;                 // 0 = Aho-Corasick, 1 = regex DFA set
    uint32_t n_pats = 0, flags = 0;
    // one or more automata (AC: exactly one)
    struct Table {
        uint32_t n_states = 0, n_classes = 0;
        uint8_t cls[256];
        std::vector<uint32_t> delta;    // n_states * n_classes
        std::vector<uint32_t> own_off;  // n_states + 1 (CSR of pattern ids accepted here)
        std::vector<uint32_t> own_ids;
        std::vector<uint32_t> dict;     // AC: next state on the suffix chain with output
        std::vector<uint32_t> outbits;  // (n_states + 31) / 32
        uint32_t anchored_eol = 0;      // DFA: class used for the end-of-record step (0 = none)
    };
    std::vector<Table> tables;
    uint64_t total_states = 0;
    // regex prefilter plan: factor Aho-Corasick + per-pattern verification DFAs
    bool has_pre = false;
    Table pre;
    std::vector<uint32_t> fac_off, fac_pids;
    std::vector<uint32_t> s_delta, s_off, s_C, s_eol, s_acc_off, single_of_pid;
    std::vector<uint8_t> s_cls, s_acc;
    uint32_t n_singles = 0;
    struct DevPlan {
        uint32_t *fac_off = nullptr, *fac_pids = nullptr, *s_delta = nullptr, *s_off = nullptr, *s_C = nullptr,
                 *s_eol = nullptr, *s_acc_off = nullptr, *single_of_pid = nullptr;
        uint8_t *s_cls = nullptr, *s_acc = nullptr;
    } dplan;
    // device copies (one device)
    int dev = -1;
    struct DevTable {
        uint32_t *delta = nullptr, *own_off = nullptr, *own_ids = nullptr, *dict = nullptr, *outbits = nullptr;
        uint16_t *hot = nullptr;  // first H rows as u16 (if n_states <= 65535)
        uint8_t *cls = nullptr;
        uint32_t H = 0;
    };
    std::vector<DevTable> dtabs;
    // hashed q-gram literal filter (used instead of the automaton when it does not fit LDS)
    struct Lit {
        bool on = false;
        bool nocase = false;
        uint32_t cls_mask = 0;           // bit L-1: some pattern has prefix class L (1..4)
        uint32_t bits[4] = {0, 0, 0, 0}; // log2 bitmap size per class
        uint32_t bm_off[4] = {0, 0, 0, 0}, bk_base[4] = {0, 0, 0, 0};
        std::vector<uint32_t> bitmap, bk_off, bk_ids, pat_off;
        std::vector<uint8_t> pat;
        uint32_t *d_bitmap = nullptr, *d_bk_off = nullptr, *d_bk_ids = nullptr, *d_pat_off = nullptr;
        uint8_t *d_pat = nullptr;
    };
    Lit lit;      // literal signatures
    Lit prelit;   // regex prefilter factors
    std::mutex mu;
};

namespace sg {

constexpr uint32_t NONE = 0xffffffffu;
constexpr uint32_t AC_HOT_BYTES = 64 * 1024;   // LDS budget for hot rows
constexpr uint32_t AC_BITS_BYTES = 16 * 1024;  // LDS budget for the output bitmap

static int build_ac(const uint8_t *pats, const uint32_t *offs, uint32_t n, uint32_t flags, sg_matcher::Table *T) {
    const bool nocase = flags & SG_NOCASE;
    auto fold = [&](uint8_t b) -> uint8_t { return (nocase && b >= 'A' && b <= 'Z') ? (uint8_t)(b + 32) : b; };
    // byte classes
    bool used[256] = {};
    for (uint32_t i = 0; i < n; ++i) {
        if (offs[i + 1] <= offs[i]) { set_error("signature %u is empty", i); return SG_E_INVAL; }
        for (uint32_t p = offs[i]; p < offs[i + 1]; ++p) {
            if (pats[p] == '\n') { set_error("signature %u contains a newline", i); return SG_E_INVAL; }
            used[fold(pats[p])] = true;
        }
    }
    uint32_t C = 1;
    uint8_t cls_of[256] = {};
    for (int b = 0; b < 256; ++b)
        if (used[b]) cls_of[b] = (uint8_t)C++;
    if (C > 256) { set_error("too many byte classes"); return SG_E_UNSUPPORTED; }
    for (int b = 0; b < 256; ++b) T->cls[b] = cls_of[fold((uint8_t)b)];
    // trie with map children, then BFS renumbering
    std::vector<std::map<uint8_t, uint32_t>> kids(1);
    std::vector<std::vector<uint32_t>> own(1);
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t s = 0;
        for (uint32_t p = offs[i]; p < offs[i + 1]; ++p) {
            const uint8_t c = cls_of[fold(pats[p])];
            auto it = kids[s].find(c);
            if (it == kids[s].end()) {
                kids.emplace_back();
                own.emplace_back();
                const uint32_t ns = (uint32_t)kids.size() - 1;
                kids[s][c] = ns;
                s = ns;
            } else {
                s = it->second;
            }
        }
        own[s].push_back(i);
    }
    const uint32_t S = (uint32_t)kids.size();
    std::vector<uint32_t> order, newid(S, NONE);
    order.reserve(S);
    order.push_back(0);
    newid[0] = 0;
    for (size_t q = 0; q < order.size(); ++q)
        for (auto &kv : kids[order[q]]) {
            newid[kv.second] = (uint32_t)order.size();
            order.push_back(kv.second);
        }
    T->n_states = S;
    T->n_classes = C;
    T->delta.assign((size_t)S * C, 0);
    std::vector<uint32_t> fail(S, 0);
    T->dict.assign(S, NONE);
    std::vector<bool> has_out(S, false);
    // BFS over new ids (order[] is already BFS)
    for (uint32_t q = 0; q < S; ++q) {
        const uint32_t old = order[q];
        const uint32_t s = q;
        has_out[s] = !own[old].empty();
        for (uint32_t c = 0; c < C; ++c) {
            auto it = kids[old].find((uint8_t)c);
            if (it != kids[old].end()) {
                const uint32_t t = newid[it->second];
                T->delta[(size_t)s * C + c] = t;
                fail[t] = (s == 0) ? 0 : T->delta[(size_t)fail[s] * C + c];
            } else {
                T->delta[(size_t)s * C + c] = (s == 0) ? 0 : T->delta[(size_t)fail[s] * C + c];
            }
        }
        if (s != 0) {
            const uint32_t f = fail[s];
            T->dict[s] = has_out[f] ? f : T->dict[f];
        }
    }
    T->delta[0] = 0;
    for (uint32_t s = 0; s < S; ++s) T->delta[(size_t)s * C + 0] = 0;  // class 0: no pattern byte
    T->own_off.assign(S + 1, 0);
    for (uint32_t q = 0; q < S; ++q) T->own_off[q + 1] = T->own_off[q] + (uint32_t)own[order[q]].size();
    T->own_ids.resize(T->own_off[S]);
    for (uint32_t q = 0; q < S; ++q)
        std::copy(own[order[q]].begin(), own[order[q]].end(), T->own_ids.begin() + T->own_off[q]);
    T->outbits.assign((S + 31) / 32, 0);
    for (uint32_t s = 0; s < S; ++s)
        if (has_out[s] || T->dict[s] != NONE) T->outbits[s / 32] |= 1u << (s % 32);
    return SG_OK;
}

// ------------------------------------------------------------------ hashed q-gram literal filter
// Prefix class L = min(len, 4). Classes 1 and 2 index exactly (256 / 65,536 buckets);
// classes 3 and 4 hash the prefix (multiplicative) into 2^bits buckets. A bitmap per
// class (LDS-resident) says which buckets hold patterns; a CSR per class lists them.
__host__ __device__ __forceinline__ uint32_t lit_h(uint32_t key, uint32_t L, uint32_t bits) {
    return (L <= 2) ? key : (uint32_t)((key * 0x9E3779B1u) >> (32u - bits));
}

static int build_lit(const uint8_t *pats, const uint32_t *offs, uint32_t n, uint32_t flags, sg_matcher::Lit *T) {
    const bool nocase = flags & SG_NOCASE;
    auto fold = [&](uint8_t b) -> uint8_t { return (nocase && b >= 'A' && b <= 'Z') ? (uint8_t)(b + 32) : b; };
    T->on = true;
    T->nocase = nocase;
    T->pat.clear();
    T->pat_off.assign(1, 0);
    uint32_t cnt[5] = {0, 0, 0, 0, 0};
    for (uint32_t i = 0; i < n; ++i) {
        if (offs[i + 1] <= offs[i]) { set_error("signature %u is empty", i); return SG_E_INVAL; }
        for (uint32_t p = offs[i]; p < offs[i + 1]; ++p) {
            if (pats[p] == '\n') { set_error("signature %u contains a newline", i); return SG_E_INVAL; }
            T->pat.push_back(fold(pats[p]));
        }
        T->pat_off.push_back((uint32_t)T->pat.size());
        cnt[std::min<uint32_t>(offs[i + 1] - offs[i], 4)]++;
    }
    uint32_t words = 0, buckets = 0;
    T->cls_mask = 0;
    for (uint32_t L = 1; L <= 4; ++L) {
        uint32_t b = 0;
        if (cnt[L]) {
            T->cls_mask |= 1u << (L - 1);
            if (L <= 2) {
                b = 8 * L;
            } else {
                b = 10;
                while (b < (L == 4 ? 18u : 16u) && (1ull << b) < 64ull * cnt[L]) ++b;
            }
        }
        T->bits[L - 1] = b;
        T->bm_off[L - 1] = words;
        T->bk_base[L - 1] = buckets;
        if (cnt[L]) {
            words += std::max<uint32_t>((1u << b) / 32, 1);
            buckets += (1u << b) + 1;
        }
    }
    T->bitmap.assign(words, 0);
    std::vector<uint32_t> count(buckets + 1, 0), hid(n);
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t len = T->pat_off[i + 1] - T->pat_off[i];
        const uint32_t L = std::min<uint32_t>(len, 4);
        uint32_t key = 0;
        for (uint32_t j = 0; j < L; ++j) key |= (uint32_t)T->pat[T->pat_off[i] + j] << (8 * j);
        const uint32_t h = lit_h(key, L, T->bits[L - 1]);
        T->bitmap[T->bm_off[L - 1] + (h >> 5)] |= 1u << (h & 31);
        hid[i] = T->bk_base[L - 1] + h;
        count[hid[i]]++;
    }
    T->bk_off.assign(buckets + 1, 0);
    for (uint32_t b = 0; b < buckets; ++b) T->bk_off[b + 1] = T->bk_off[b] + count[b];
    T->bk_ids.assign(n, 0);
    std::vector<uint32_t> fillp(T->bk_off.begin(), T->bk_off.end() - 1);
    for (uint32_t i = 0; i < n; ++i) T->bk_ids[fillp[hid[i]]++] = i;
    return SG_OK;
}

template <class T>
static int upload_vec(const std::vector<T> &v, T **d) {
    const size_t bytes = std::max<size_t>(v.size() * sizeof(T), 16);
    if (hipMalloc(d, bytes) != hipSuccess) { (void)hipGetLastError(); set_error("hipMalloc matcher table"); return SG_E_NOMEM; }
    if (!v.empty()) SG_HIP(hipMemcpy(*d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return SG_OK;
}

static void free_dev(sg_matcher *h) {
    for (auto &d : h->dtabs) {
        (void)hipFree(d.delta); (void)hipFree(d.own_off); (void)hipFree(d.own_ids); (void)hipFree(d.dict);
        (void)hipFree(d.outbits); (void)hipFree(d.hot); (void)hipFree(d.cls);
    }
    h->dtabs.clear();
    auto &p = h->dplan;
    for (void *q : {(void *)p.fac_off, (void *)p.fac_pids, (void *)p.s_delta, (void *)p.s_off, (void *)p.s_C,
                    (void *)p.s_eol, (void *)p.s_acc_off, (void *)p.single_of_pid, (void *)p.s_cls, (void *)p.s_acc})
        if (q) (void)hipFree(q);
    h->dplan = sg_matcher::DevPlan{};
    for (sg_matcher::Lit *L : {&h->lit, &h->prelit}) {
        for (void *q : {(void *)L->d_bitmap, (void *)L->d_bk_off, (void *)L->d_bk_ids, (void *)L->d_pat_off,
                        (void *)L->d_pat})
            if (q) (void)hipFree(q);
        L->d_bitmap = L->d_bk_off = L->d_bk_ids = L->d_pat_off = nullptr;
        L->d_pat = nullptr;
    }
    h->dev = -1;
}

static int ensure_device(sg_matcher *h, int dev) {
    std::lock_guard<std::mutex> g(h->mu);
    if (h->dev == dev) return SG_OK;
    if (h->dev >= 0) { (void)hipSetDevice(h->dev); free_dev(h); }
    SG_HIP(hipSetDevice(dev));
    if (h->has_pre) {
        auto &p = h->dplan;
        SG_TRY(upload_vec(h->fac_off, &p.fac_off));
        SG_TRY(upload_vec(h->fac_pids, &p.fac_pids));
        SG_TRY(upload_vec(h->s_delta, &p.s_delta));
        SG_TRY(upload_vec(h->s_off, &p.s_off));
        SG_TRY(upload_vec(h->s_C, &p.s_C));
        SG_TRY(upload_vec(h->s_eol, &p.s_eol));
        SG_TRY(upload_vec(h->s_acc_off, &p.s_acc_off));
        SG_TRY(upload_vec(h->single_of_pid, &p.single_of_pid));
        SG_TRY(upload_vec(h->s_cls, &p.s_cls));
        SG_TRY(upload_vec(h->s_acc, &p.s_acc));
    }
    for (sg_matcher::Lit *L : {&h->lit, &h->prelit}) {
        if (!L->on) continue;
        SG_TRY(upload_vec(L->bitmap, &L->d_bitmap));
        SG_TRY(upload_vec(L->bk_off, &L->d_bk_off));
        SG_TRY(upload_vec(L->bk_ids, &L->d_bk_ids));
        SG_TRY(upload_vec(L->pat_off, &L->d_pat_off));
        SG_TRY(upload_vec(L->pat, &L->d_pat));
    }
    // tables[]: the automata scanned over every record; the prefilter AC goes last
    std::vector<sg_matcher::Table *> all;
    for (auto &T : h->tables) all.push_back(&T);
    for (auto *Tp : all) {
        auto &T = *Tp;
        sg_matcher::DevTable d;
        SG_TRY(upload_vec(T.delta, &d.delta));
        SG_TRY(upload_vec(T.own_off, &d.own_off));
        SG_TRY(upload_vec(T.own_ids, &d.own_ids));
        SG_TRY(upload_vec(T.dict, &d.dict));
        SG_TRY(upload_vec(T.outbits, &d.outbits));
        std::vector<uint8_t> cls(T.cls, T.cls + 256);
        SG_TRY(upload_vec(cls, &d.cls));
        uint32_t H = 0;
        if (T.n_states <= 65535) {
            H = std::min<uint32_t>(T.n_states, AC_HOT_BYTES / (2 * T.n_classes));
            std::vector<uint16_t> hot((size_t)H * T.n_classes);
            for (size_t q = 0; q < hot.size(); ++q) hot[q] = (uint16_t)T.delta[q];
            SG_TRY(upload_vec(hot, &d.hot));
        }
        d.H = H;
        h->dtabs.push_back(d);
    }
    h->dev = dev;
    return SG_OK;
}

// ------------------------------------------------------------------ device: Aho-Corasick
struct ACArgs {
    const uint8_t *buf;
    const uint2 *spans;
    uint32_t R;
    const uint8_t *cls;
    const uint32_t *delta;
    const uint16_t *hot;
    uint32_t C, H, S;
    const uint32_t *outbits, *own_off, *own_ids, *dict;
    unsigned long long *hits;
    uint32_t *hit_count;
    uint32_t cap;
    uint32_t bits_in_lds;
    const uint32_t *fac_off, *fac_pids;  // prefilter: factor -> candidate patterns (else null)
};

__device__ __forceinline__ void emit_hit(const ACArgs &a, uint32_t rec, uint32_t sig, uint32_t *seen, uint32_t &nseen) {
    const uint32_t key = sig;
    for (uint32_t q = 0; q < nseen; ++q)
        if (seen[q] == key) return;
    if (nseen < 4) seen[nseen++] = key;
    if (a.fac_off) {  // prefilter: every pattern that needs this factor is a candidate
        for (uint32_t q = a.fac_off[sig]; q < a.fac_off[sig + 1]; ++q) {
            const uint32_t slot_i = atomicAdd(a.hit_count, 1u);
            if (slot_i < a.cap) a.hits[slot_i] = ((unsigned long long)rec << 32) | a.fac_pids[q];
        }
        return;
    }
    const uint32_t slot_i = atomicAdd(a.hit_count, 1u);
    if (slot_i < a.cap) a.hits[slot_i] = ((unsigned long long)rec << 32) | sig;
}

__global__ __launch_bounds__(512) void k_ac_match(ACArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    uint8_t *s_cls = lds;
    uint16_t *s_hot = reinterpret_cast<uint16_t *>(lds + 256);
    const uint32_t hot_n = a.H * a.C;
    uint32_t *s_bits = reinterpret_cast<uint32_t *>(lds + 256 + ((hot_n * 2 + 15) & ~15u));
    for (uint32_t q = threadIdx.x; q < 256; q += blockDim.x) s_cls[q] = a.cls[q];
    for (uint32_t q = threadIdx.x; q < hot_n; q += blockDim.x) s_hot[q] = a.hot[q];
    const uint32_t nbits = (a.S + 31) / 32;
    if (a.bits_in_lds)
        for (uint32_t q = threadIdx.x; q < nbits; q += blockDim.x) s_bits[q] = a.outbits[q];
    __syncthreads();
    const uint32_t *bits = a.bits_in_lds ? s_bits : a.outbits;
    for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < a.R; r += gridDim.x * blockDim.x) {
        const uint2 sp_ = a.spans[r];
        const uint32_t s = sp_.x, e = sp_.y;
        uint32_t st = 0;
        uint32_t seen[4];
        uint32_t nseen = 0;
        for (uint32_t w = s & ~3u; w < e; w += 4) {
            const uint32_t x = *reinterpret_cast<const uint32_t *>(a.buf + w);
#pragma unroll
            for (uint32_t b = 0; b < 4; ++b) {
                const uint32_t p = w + b;
                if (p < s || p >= e) continue;
                const uint32_t c = s_cls[(x >> (8 * b)) & 0xffu];
                st = (st < a.H) ? (uint32_t)s_hot[st * a.C + c] : a.delta[(size_t)st * a.C + c];
                if ((bits[st >> 5] >> (st & 31)) & 1u) {
                    for (uint32_t t = st; t != NONE; t = a.dict[t])
                        for (uint32_t q = a.own_off[t]; q < a.own_off[t + 1]; ++q) emit_hit(a, r, a.own_ids[q], seen, nseen);
                }
            }
        }
    }
}

// ------------------------------------------------------------------ device: literal filter
struct LitArgs {
    const uint8_t *buf;
    const uint2 *spans;
    uint32_t R;
    const uint32_t *bitmap;
    uint32_t bm_words, cls_mask, nocase;
    uint32_t bits[4], bm_off[4], bk_base[4];
    const uint32_t *bk_off, *bk_ids, *pat_off;
    const uint8_t *pat;
    unsigned long long *hits;
    uint32_t *hit_count;
    uint32_t cap;
    const uint32_t *fac_off, *fac_pids;  // regex prefilter expansion (else null)
};

__device__ __forceinline__ uint32_t fold4(uint32_t w) {
    // ASCII 'A'..'Z' -> 'a'..'z' in each byte (SWAR)
    const uint32_t h7 = w & 0x7f7f7f7fu;
    const uint32_t ge_a = h7 + 0x3f3f3f3fu;  // high bit: byte >= 'A'
    const uint32_t gt_z = h7 + 0x25252525u;  // high bit: byte > 'Z'
    const uint32_t up = ge_a & ~gt_z & ~w & 0x80808080u;
    return w | (up >> 2);
}

__device__ __forceinline__ void emit_pair(unsigned long long *hits, uint32_t *hit_count, uint32_t cap,
                                          const uint32_t *fac_off, const uint32_t *fac_pids, uint32_t rec,
                                          uint32_t sig, uint32_t *seen, uint32_t &nseen) {
    for (uint32_t q = 0; q < nseen; ++q)
        if (seen[q] == sig) return;
    if (nseen < 4) seen[nseen++] = sig;
    if (fac_off) {
        for (uint32_t q = fac_off[sig]; q < fac_off[sig + 1]; ++q) {
            const uint32_t slot_i = atomicAdd(hit_count, 1u);
            if (slot_i < cap) hits[slot_i] = ((unsigned long long)rec << 32) | fac_pids[q];
        }
        return;
    }
    const uint32_t slot_i = atomicAdd(hit_count, 1u);
    if (slot_i < cap) hits[slot_i] = ((unsigned long long)rec << 32) | sig;
}

// One thread per record. At every byte position p the next min(r, 4) bytes (r = bytes
// left in the record) form the prefix key of each present class; a set bit in that
// class's LDS bitmap triggers the byte compare of the patterns in the bucket.
__global__ __launch_bounds__(512) void k_lit_match(LitArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t s_bm[];
    for (uint32_t q = threadIdx.x; q < a.bm_words; q += blockDim.x) s_bm[q] = a.bitmap[q];
    __syncthreads();
    for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < a.R; r += gridDim.x * blockDim.x) {
        const uint2 sp = a.spans[r];
        const uint32_t s = sp.x, e = sp.y;
        uint32_t seen[4];
        uint32_t nseen = 0;
        const uint32_t a0 = s & ~3u;
        uint32_t w0 = *reinterpret_cast<const uint32_t *>(a.buf + a0);
        uint32_t w1 = (a0 + 4 < e) ? *reinterpret_cast<const uint32_t *>(a.buf + a0 + 4) : 0u;
        if (a.nocase) { w0 = fold4(w0); w1 = fold4(w1); }
        for (uint32_t q = a0; q < e; q += 4) {
            const uint64_t win = (uint64_t)w0 | ((uint64_t)w1 << 32);
#pragma unroll
            for (uint32_t b = 0; b < 4; ++b) {
                const uint32_t p = q + b;
                if (p < s || p >= e) continue;
                const uint32_t rem = e - p;
                const uint32_t key4 = (uint32_t)(win >> (8 * b));
#pragma unroll
                for (uint32_t L = 1; L <= 4; ++L) {
                    if (!((a.cls_mask >> (L - 1)) & 1u) || rem < L) continue;
                    const uint32_t key = (L == 4) ? key4 : (key4 & ((1u << (8 * L)) - 1u));
                    const uint32_t h = lit_h(key, L, a.bits[L - 1]);
                    if (!((s_bm[a.bm_off[L - 1] + (h >> 5)] >> (h & 31)) & 1u)) continue;
                    const uint32_t bk = a.bk_base[L - 1] + h;
                    for (uint32_t i = a.bk_off[bk]; i < a.bk_off[bk + 1]; ++i) {
                        const uint32_t pid = a.bk_ids[i];
                        const uint32_t ps = a.pat_off[pid], pl = a.pat_off[pid + 1] - ps;
                        if (pl > rem || (pl < 4) != (L < 4)) continue;
                        bool eq = true;
                        for (uint32_t j = 0; j < pl && eq; ++j) {
                            uint32_t c = a.buf[p + j];
                            if (a.nocase && c >= 'A' && c <= 'Z') c += 32;
                            eq = c == a.pat[ps + j];
                        }
                        if (eq) emit_pair(a.hits, a.hit_count, a.cap, a.fac_off, a.fac_pids, r, pid, seen, nseen);
                    }
                }
            }
            w0 = w1;
            w1 = (q + 8 < e) ? *reinterpret_cast<const uint32_t *>(a.buf + q + 8) : 0u;
            if (a.nocase) w1 = fold4(w1);
        }
    }
}

// ------------------------------------------------------------------ device: regex DFAs
struct DFAArgs {
    const uint8_t *buf;
    const uint2 *spans;
    uint32_t R;
    const uint8_t *cls;
    const uint32_t *delta;
    const uint16_t *hot;
    uint32_t C, H, S, eol;
    const uint32_t *outbits, *own_off, *own_ids;
    unsigned long long *hits;
    uint32_t *hit_count;
    uint32_t cap;
    uint32_t bits_in_lds;
};

// One DFA of a set. State 0 = dead (no pattern can still match), state 1 = start. A state
// with output accepts the listed patterns; accepted patterns are removed from the
// successor states at build time, so each pattern is reported once per record.
__global__ __launch_bounds__(512) void k_dfa_match(DFAArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    uint8_t *s_cls = lds;
    uint16_t *s_hot = reinterpret_cast<uint16_t *>(lds + 256);
    const uint32_t hot_n = a.H * a.C;
    uint32_t *s_bits = reinterpret_cast<uint32_t *>(lds + 256 + ((hot_n * 2 + 15) & ~15u));
    for (uint32_t q = threadIdx.x; q < 256; q += blockDim.x) s_cls[q] = a.cls[q];
    for (uint32_t q = threadIdx.x; q < hot_n; q += blockDim.x) s_hot[q] = a.hot[q];
    const uint32_t nbits = (a.S + 31) / 32;
    if (a.bits_in_lds)
        for (uint32_t q = threadIdx.x; q < nbits; q += blockDim.x) s_bits[q] = a.outbits[q];
    __syncthreads();
    const uint32_t *bits = a.bits_in_lds ? s_bits : a.outbits;
    auto step = [&](uint32_t st, uint32_t c) -> uint32_t {
        return (st < a.H) ? (uint32_t)s_hot[st * a.C + c] : a.delta[(size_t)st * a.C + c];
    };
    auto accept = [&](uint32_t r, uint32_t st) {
        if ((bits[st >> 5] >> (st & 31)) & 1u)
            for (uint32_t q = a.own_off[st]; q < a.own_off[st + 1]; ++q) {
                const uint32_t slot_i = atomicAdd(a.hit_count, 1u);
                if (slot_i < a.cap) a.hits[slot_i] = ((unsigned long long)r << 32) | a.own_ids[q];
            }
    };
    for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < a.R; r += gridDim.x * blockDim.x) {
        const uint2 sp_ = a.spans[r];
        const uint32_t s = sp_.x, e = sp_.y;
        uint32_t st = 1;
        accept(r, st);
        for (uint32_t w = s & ~3u; w < e && st != 0; w += 4) {
            const uint32_t x = *reinterpret_cast<const uint32_t *>(a.buf + w);
#pragma unroll
            for (uint32_t b = 0; b < 4; ++b) {
                const uint32_t p = w + b;
                if (p < s || p >= e || st == 0) continue;
                st = step(st, s_cls[(x >> (8 * b)) & 0xffu]);
                accept(r, st);
            }
        }
        if (st != 0 && a.eol) accept(r, step(st, a.eol));
    }
}

// Verify prefilter candidates: one thread per (record, pattern) runs that pattern's own
// DFA over the record (state 0 dead, 1 start, EOL column last) and appends a hit on the
// first accepting state.
struct VerifyArgs {
    const uint8_t *buf;
    const uint2 *spans;
    const unsigned long long *cand;
    uint32_t n_cand;
    const uint32_t *s_delta, *s_off, *s_C, *s_eol, *s_acc_off, *single_of_pid;
    const uint8_t *s_cls, *s_acc;
    unsigned long long *hits;
    uint32_t *hit_count;
    uint32_t cap;
};

__global__ __launch_bounds__(256) void k_verify(VerifyArgs a) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n_cand) return;
    const unsigned long long cd = a.cand[i];
    const uint32_t r = (uint32_t)(cd >> 32), pid = (uint32_t)cd;
    const uint32_t k = a.single_of_pid[pid];
    const uint32_t *D = a.s_delta + a.s_off[k];
    const uint8_t *cls = a.s_cls + 256u * k;
    const uint8_t *acc = a.s_acc + a.s_acc_off[k];
    const uint32_t C = a.s_C[k];
    const uint2 sp_ = a.spans[r];
        const uint32_t s = sp_.x, e = sp_.y;
    uint32_t st = 1;
    bool hit = acc[st] != 0;
    for (uint32_t w = s & ~3u; w < e && !hit && st != 0; w += 4) {
        const uint32_t x = *reinterpret_cast<const uint32_t *>(a.buf + w);
#pragma unroll
        for (uint32_t b = 0; b < 4; ++b) {
            const uint32_t p = w + b;
            if (p < s || p >= e || hit || st == 0) continue;
            st = D[st * C + cls[(x >> (8 * b)) & 0xffu]];
            hit = acc[st] != 0;
        }
    }
    if (!hit && st != 0) hit = acc[D[st * C + a.s_eol[k]]] != 0;
    if (hit) {
        const uint32_t slot_i = atomicAdd(a.hit_count, 1u);
        if (slot_i < a.cap) a.hits[slot_i] = cd;
    }
}

// ------------------------------------------------------------------ host driver
struct HitKeyPred {
    const unsigned long long *K;
    uint32_t n;
    __device__ uint32_t operator()(uint32_t i) const { return (i == 0 || K[i] != K[i - 1]) ? 1u : 0u; }
};
struct RecHeadPred {
    const unsigned long long *K;
    __device__ uint32_t operator()(uint32_t i) const { return (i == 0 || (K[i] >> 32) != (K[i - 1] >> 32)) ? 1u : 0u; }
};

__global__ void k_split_hits(const unsigned long long *K, const uint32_t *idx, uint32_t n, uint32_t *rec, uint32_t *sig) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const unsigned long long k = K[idx[i]];
    rec[i] = (uint32_t)(k >> 32);
    sig[i] = (uint32_t)k;
}

__global__ void k_rec_of(const unsigned long long *K, const uint32_t *idx, uint32_t n, uint32_t *rec) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) rec[i] = (uint32_t)(K[idx[i]] >> 32);
}

template <class Pred>
static int select_one(sg_ctx *c, const char *name, Pred pred, uint32_t n, uint32_t *out, uint32_t *count) {
    *count = 0;
    if (n == 0) return SG_OK;
    const uint32_t ntiles = (n + SEL_TILE - 1) / SEL_TILE;
    uint64_t *status;
    SG_TRY(slot(c, S_COUNT, (size_t)ntiles + 4, &status));
    uint32_t *counter = reinterpret_cast<uint32_t *>(status + ntiles);
    SG_HIP(hipMemsetAsync(status, 0, ((size_t)ntiles + 4) * 8, c->stream));
    SG_LAUNCH(c, name, k_select2<Pred>, ntiles, SEL_BLOCK, 0, pred, n, out, (uint32_t *)nullptr, status, counter, ntiles);
    uint32_t cnt[2];
    SG_TRY(ctx_readback(c, cnt, counter, 8));
    *count = cnt[1];
    return SG_OK;
}

static int dev_match(sg_ctx *c, sg_matcher *h, const uint8_t *d_buf, uint64_t n, sg_dev_hits *res) {
    *res = sg_dev_hits{};
    SG_TRY(ensure_device(h, c->device));
    Lines L;
    SG_TRY(run_lines(c, d_buf, n, CUR_SLOTS, &L));
    const uint32_t R = L.n_rec;
    res->in_records = R;
    uint32_t *cnt;
    SG_TRY(slot(c, S_M_CNT, 8, &cnt));
    uint64_t cap = std::max<uint64_t>(1u << 20, (uint64_t)R / 4);
    uint32_t total = 0;
    unsigned long long *hits = nullptr;
    auto geometry = [&](const sg_matcher::Table &T, const sg_matcher::DevTable &D, uint32_t *bits_in_lds,
                        uint32_t *lds, uint32_t *grid) {
        const uint32_t nbits = (T.n_states + 31) / 32;
        *bits_in_lds = nbits * 4 <= AC_BITS_BYTES ? 1u : 0u;
        *lds = 256 + ((D.H * T.n_classes * 2 + 15) & ~15u) + (*bits_in_lds ? nbits * 4 : 0);
        *grid = std::min<uint32_t>((R + 511) / 512, 256u * 8u);
    };
    // prefilter candidates (regex plans): factor AC -> (record, pattern) pairs
    unsigned long long *cand = nullptr;
    uint32_t n_cand = 0;
    auto lit_args = [&](const sg_matcher::Lit &Lt, unsigned long long *out, uint32_t *counter, uint32_t ocap,
                        const uint32_t *fo, const uint32_t *fp) {
        LitArgs a{};
        a.buf = d_buf; a.spans = L.spans; a.R = R;
        a.bitmap = Lt.d_bitmap; a.bm_words = (uint32_t)Lt.bitmap.size(); a.cls_mask = Lt.cls_mask;
        a.nocase = Lt.nocase ? 1u : 0u;
        for (int k = 0; k < 4; ++k) { a.bits[k] = Lt.bits[k]; a.bm_off[k] = Lt.bm_off[k]; a.bk_base[k] = Lt.bk_base[k]; }
        a.bk_off = Lt.d_bk_off; a.bk_ids = Lt.d_bk_ids; a.pat_off = Lt.d_pat_off; a.pat = Lt.d_pat;
        a.hits = out; a.hit_count = counter; a.cap = ocap; a.fac_off = fo; a.fac_pids = fp;
        return a;
    };
    const uint32_t lgrid = std::min<uint32_t>((R + 511) / 512, 256u * 8u);
    if (h->has_pre && R) {
        uint64_t ccap = std::max<uint64_t>(1u << 20, (uint64_t)R);
        for (int attempt = 0; attempt < 2; ++attempt) {
            SG_TRY(slot(c, S_PART, ccap, &cand));
            SG_HIP(hipMemsetAsync(cnt + 1, 0, 4, c->stream));
            LitArgs a = lit_args(h->prelit, cand, cnt + 1, (uint32_t)ccap, h->dplan.fac_off, h->dplan.fac_pids);
            SG_LAUNCH_B(c, "re_prefilter", (double)n + 8.0 * R, k_lit_match, lgrid, 512, a.bm_words * 4, a);
            SG_TRY(ctx_readback(c, &n_cand, cnt + 1, 4));
            if (n_cand <= ccap) break;
            ccap = (uint64_t)n_cand + 1024;
        }
        cap = std::max<uint64_t>(cap, (uint64_t)n_cand + 1024);
    }
    for (int attempt = 0; attempt < 2; ++attempt) {
        SG_TRY(slot(c, S_M_HITS, cap, &hits));
        SG_HIP(hipMemsetAsync(cnt, 0, 4, c->stream));
        if (R && h->lit.on) {
            LitArgs a = lit_args(h->lit, hits, cnt, (uint32_t)cap, nullptr, nullptr);
            SG_LAUNCH_B(c, "lit_match", (double)n + 8.0 * R, k_lit_match, lgrid, 512, a.bm_words * 4, a);
        }
        if (R) {
            for (size_t ti = 0; ti < h->tables.size(); ++ti) {
                const auto &T = h->tables[ti];
                const auto &D = h->dtabs[ti];
                uint32_t bits_in_lds, lds, grid;
                geometry(T, D, &bits_in_lds, &lds, &grid);
                if (h->kind == 0) {
                    ACArgs a{d_buf, L.spans, R, D.cls, D.delta, D.hot, T.n_classes, D.H, T.n_states,
                             D.outbits, D.own_off, D.own_ids, D.dict, hits, cnt, (uint32_t)cap, bits_in_lds,
                             nullptr, nullptr};
                    SG_LAUNCH_B(c, "ac_match", (double)n + 8.0 * R, k_ac_match, grid, 512, lds, a);
                } else {
                    DFAArgs a{d_buf, L.spans, R, D.cls, D.delta, D.hot, T.n_classes, D.H, T.n_states,
                              T.anchored_eol, D.outbits, D.own_off, D.own_ids, hits, cnt, (uint32_t)cap, bits_in_lds};
                    SG_LAUNCH_B(c, "dfa_match", (double)n + 8.0 * R, k_dfa_match, grid, 512, lds, a);
                }
            }
            if (n_cand) {
                const auto &p = h->dplan;
                VerifyArgs v{d_buf, L.spans, cand, n_cand, p.s_delta, p.s_off, p.s_C, p.s_eol,
                             p.s_acc_off, p.single_of_pid, p.s_cls, p.s_acc, hits, cnt, (uint32_t)cap};
                SG_LAUNCH_B(c, "re_verify", n_cand * (16.0 + (double)n / R), k_verify, (n_cand + 255) / 256, 256, 0, v);
            }
        }
        SG_TRY(ctx_readback(c, &total, cnt, 4));
        if (total <= cap) break;
        cap = (uint64_t)total + 1024;
    }
    // sort (rec << 32 | sig) and de-duplicate
    uint64_t *k2;
    uint32_t *v1, *v2;
    SG_TRY(slot(c, S_R_KEY2, (size_t)total + 1, &k2));
    SG_TRY(slot(c, S_R_VAL, (size_t)total + 1, &v1));
    SG_TRY(slot(c, S_R_VAL2, (size_t)total + 1, &v2));
    int rbits = 1;
    while (rbits < 32 && (1u << rbits) < R) ++rbits;
    uint64_t *K;
    uint32_t *V;
    SG_TRY(radix_sort(c, reinterpret_cast<uint64_t *>(hits), v1, k2, v2, total, 0, 32 + rbits, true, &K, &V, "rs_pass_hits"));
    const unsigned long long *KK = reinterpret_cast<const unsigned long long *>(K);
    uint32_t *sel;
    SG_TRY(slot(c, S_SEL, (size_t)total + 16, &sel));
    uint32_t H = 0;
    SG_TRY(select_one(c, "hits_unique", HitKeyPred{KK, total}, total, sel, &H));
    uint32_t *rec, *sig;
    SG_TRY(slot(c, S_M_SIG, (size_t)H + 1, &sig));
    SG_TRY(slot(c, S_R_GID, (size_t)H + 1, &rec));
    if (H) SG_LAUNCH(c, "split_hits", k_split_hits, (H + 255) / 256, 256, 0, KK, sel, H, rec, sig);
    res->rec_idx = rec;
    res->sig_id = sig;
    res->n_hits = H;
    // matched records (input order) -> grep output
    uint32_t M = 0;
    SG_TRY(select_one(c, "hits_recs", RecHeadPred{KK}, total, sel, &M));
    uint32_t *mrec;
    SG_TRY(slot(c, S_R_POS, (size_t)M + 1, &mrec));
    if (M) SG_LAUNCH(c, "rec_of", k_rec_of, (M + 255) / 256, 256, 0, KK, sel, M, mrec);
    uint8_t *lines;
    uint64_t lb = 0;
    SG_TRY(serialize(c, d_buf, L.spans, mrec, nullptr, M, S_M_LINES, &lines, &lb));
    res->lines = lines;
    res->lines_bytes = lb;
    res->matched_records = M;
    return SG_OK;
}

}  // namespace sg

extern "C" {

int sg_ac_compile(const uint8_t *pats, const uint32_t *pat_offs, uint32_t n_pats, uint32_t flags, sg_matcher **h) {
    if (!h || (n_pats && (!pats || !pat_offs))) { set_error("sg_ac_compile: bad arguments"); return SG_E_INVAL; }
    sg_matcher *m = new sg_matcher();
    m->kind = 0;
    m->n_pats = n_pats;
    m->flags = flags;
    m->tables.emplace_back();
    int rc = build_ac(pats, pat_offs, n_pats, flags, &m->tables[0]);
    if (rc != SG_OK) { delete m; return rc; }
    m->total_states = m->tables[0].n_states;
    // An automaton whose rows all fit the LDS hot table walks at LDS speed; a larger one
    // would chase dependent HBM/L2 rows on every byte, so it is replaced by the hashed
    // q-gram filter (independent per-position probes, byte compares on bitmap hits).
    const auto &T = m->tables[0];
    if ((uint64_t)T.n_states * T.n_classes * 2 > AC_HOT_BYTES || getenv("SG_FORCE_LITFILTER")) {
        rc = build_lit(pats, pat_offs, n_pats, flags, &m->lit);
        if (rc != SG_OK) { delete m; return rc; }
        m->tables.clear();
    }
    *h = m;
    return SG_OK;
}

int sg_dfa_compile(const uint8_t *pats, const uint32_t *pat_offs, uint32_t n_pats, uint32_t flags, sg_matcher **h) {
    if (!h || (n_pats && (!pats || !pat_offs))) { set_error("sg_dfa_compile: bad arguments"); return SG_E_INVAL; }
    RegexPlan plan;
    int rc = regex_build_plan(pats, pat_offs, n_pats, flags, &plan);
    if (rc != SG_OK) return rc;
    sg_matcher *m = new sg_matcher();
    m->kind = 1;
    m->n_pats = n_pats;
    m->flags = flags;
    if (!plan.singles.empty()) {
        // factor Aho-Corasick (case-insensitive: a superset of the exact-case occurrences)
        std::vector<uint8_t> blob;
        std::vector<uint32_t> offs(1, 0);
        for (auto &f : plan.factors) {
            blob.insert(blob.end(), f.begin(), f.end());
            offs.push_back((uint32_t)blob.size());
        }
        rc = build_lit(blob.data(), offs.data(), (uint32_t)plan.factors.size(), SG_NOCASE, &m->prelit);
        if (rc != SG_OK) { delete m; return rc; }
        m->has_pre = true;
        m->fac_off = plan.fac_off;
        m->fac_pids = plan.fac_pids;
        m->single_of_pid = plan.single_of_pid;
        for (auto &d : plan.singles) {
            m->s_off.push_back((uint32_t)m->s_delta.size());
            m->s_C.push_back(d.n_classes);
            m->s_eol.push_back(d.eol_class);
            m->s_delta.insert(m->s_delta.end(), d.delta.begin(), d.delta.end());
            m->s_cls.insert(m->s_cls.end(), d.cls, d.cls + 256);
            m->s_acc_off.push_back((uint32_t)m->s_acc.size());
            for (uint32_t s = 0; s < d.n_states; ++s) m->s_acc.push_back(d.acc_off[s + 1] > d.acc_off[s] ? 1 : 0);
            m->total_states += d.n_states;
        }
        m->n_singles = (uint32_t)plan.singles.size();
    }
    for (auto &d : plan.groups) {
        sg_matcher::Table T;
        T.n_states = d.n_states;
        T.n_classes = d.n_classes;
        memcpy(T.cls, d.cls, 256);
        T.delta = std::move(d.delta);
        T.own_off = std::move(d.acc_off);
        T.own_ids = std::move(d.acc_ids);
        T.anchored_eol = d.eol_class;
        T.outbits.assign((T.n_states + 31) / 32, 0);
        for (uint32_t s = 0; s < T.n_states; ++s)
            if (T.own_off[s + 1] > T.own_off[s]) T.outbits[s / 32] |= 1u << (s % 32);
        m->total_states += T.n_states;
        m->tables.push_back(std::move(T));
    }
    *h = m;
    return SG_OK;
}

int sg_matcher_info(const sg_matcher *h, uint64_t *states, uint32_t *groups, uint32_t *n_pats) {
    if (!h) return SG_E_INVAL;
    if (states) *states = h->total_states;
    if (groups) *groups = (uint32_t)h->tables.size();
    if (n_pats) *n_pats = h->n_pats;
    return SG_OK;
}

int sg_dev_match(sg_ctx *c, sg_matcher *h, const uint8_t *d_buf, size_t n, sg_dev_hits *res) {
    if (!c || !h || !res || (!d_buf && n)) { set_error("sg_dev_match: bad arguments"); return SG_E_INVAL; }
    SG_HIP(hipSetDevice(c->device));
    const uint8_t *b = d_buf;
    if (((uintptr_t)d_buf & 15) != 0) {
        uint8_t *a;
        SG_TRY(slot(c, S_IN, n + 16, &a));
        if (n) SG_HIP(hipMemcpyAsync(a, d_buf, n, hipMemcpyDeviceToDevice, c->stream));
        b = a;
    }
    return dev_match(c, h, b, n, res);
}

int sg_match(sg_matcher *h, const uint8_t *buf, size_t n, uint64_t *rec_idx, uint32_t *sig_id, size_t cap,
             size_t *n_hit) {
    if (!h || !n_hit || (!buf && n)) { set_error("sg_match: bad arguments"); return SG_E_INVAL; }
    if (n > MAX_BYTES) { set_error("input exceeds 4 GiB per call"); return SG_E_TOO_LARGE; }
    int dev = 0;
    SG_TRY(pick_device(&dev));
    sg_ctx *c = nullptr;
    SG_TRY(pool_acquire(dev, &c));
    struct Rel { sg_ctx *c; ~Rel() { pool_release(c); } } rel{c};
    SG_HIP(hipSetDevice(dev));
    uint8_t *d;
    SG_TRY(slot(c, S_IN, n + 16, &d));
    if (n) SG_HIP(hipMemcpyAsync(d, buf, n, hipMemcpyHostToDevice, c->stream));
    sg_dev_hits r;
    SG_TRY(dev_match(c, h, d, n, &r));
    *n_hit = r.n_hits;
    if (r.n_hits > cap) { set_error("hit capacity too small"); SG_HIP(hipStreamSynchronize(c->stream)); return SG_E_CAP; }
    std::vector<uint32_t> rr(r.n_hits);
    if (r.n_hits) {
        SG_HIP(hipMemcpyAsync(rr.data(), r.rec_idx, r.n_hits * 4, hipMemcpyDeviceToHost, c->stream));
        SG_HIP(hipMemcpyAsync(sig_id, r.sig_id, r.n_hits * 4, hipMemcpyDeviceToHost, c->stream));
    }
    SG_HIP(hipStreamSynchronize(c->stream));
    for (uint64_t i = 0; i < r.n_hits; ++i) rec_idx[i] = rr[i];
    return SG_OK;
}

int sg_match_lines(sg_matcher *h, const uint8_t *buf, size_t n, uint8_t *out, size_t cap, size_t *out_n) {
    if (!h || !out_n || (!buf && n)) { set_error("sg_match_lines: bad arguments"); return SG_E_INVAL; }
    if (n > MAX_BYTES) { set_error("input exceeds 4 GiB per call"); return SG_E_TOO_LARGE; }
    int dev = 0;
    SG_TRY(pick_device(&dev));
    sg_ctx *c = nullptr;
    SG_TRY(pool_acquire(dev, &c));
    struct Rel { sg_ctx *c; ~Rel() { pool_release(c); } } rel{c};
    SG_HIP(hipSetDevice(dev));
    uint8_t *d;
    SG_TRY(slot(c, S_IN, n + 16, &d));
    if (n) SG_HIP(hipMemcpyAsync(d, buf, n, hipMemcpyHostToDevice, c->stream));
    sg_dev_hits r;
    SG_TRY(dev_match(c, h, d, n, &r));
    *out_n = r.lines_bytes;
    if (r.lines_bytes > cap) { set_error("output capacity too small"); SG_HIP(hipStreamSynchronize(c->stream)); return SG_E_CAP; }
    if (r.lines_bytes) SG_HIP(hipMemcpyAsync(out, r.lines, r.lines_bytes, hipMemcpyDeviceToHost, c->stream));
    SG_HIP(hipStreamSynchronize(c->stream));
    return SG_OK;
}

void sg_free(void *p) {
    sg_matcher *h = (sg_matcher *)p;
    if (!h) return;
    if (h->dev >= 0) { (void)hipSetDevice(h->dev); free_dev(h); }
    delete h;
}

}  // extern "C"
