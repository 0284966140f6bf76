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
#include "sg_keystat.hpp"
#include "sg_switches.hpp"
#include "sg_prims_host.hpp"

#include <algorithm>
#include <atomic>
#include <type_traits>
#include <deque>
#include <map>
#include <unordered_map>
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
        std::vector<uint32_t> gpids;    // DFA: group-local pattern -> signature id (<= 64)
        std::vector<uint64_t> omask;    // DFA: per state, group-local patterns accepted on entry
    };
    std::vector<Table> tables;
    uint64_t total_states = 0;
    // regex prefilter plan: factor Aho-Corasick + per-pattern verification DFAs
    bool has_pre = false;
    Table pre;
    std::vector<uint32_t> fac_off, fac_pids;
    std::vector<uint16_t> s_delta;  // single-pattern DFAs have <= 65535 states
    std::vector<uint32_t> s_off, s_C, s_eol, s_acc_off, single_of_pid;
    std::vector<uint32_t> s_mid;  // anchored: mid-record start states (non-word | word << 16), else ~0
    std::vector<uint8_t> s_cls, s_acc;
    uint32_t n_singles = 0;
    struct DevPlan {
        uint16_t *s_delta = nullptr;
        uint32_t *fac_off = nullptr, *fac_pids = nullptr, *s_off = nullptr, *s_C = nullptr,
                 *s_eol = nullptr, *s_acc_off = nullptr, *single_of_pid = nullptr, *s_mid = nullptr;
        uint8_t *s_cls = nullptr, *s_acc = nullptr;
    } dplan;
    // device copies (one device)
    int dev = -1;
    struct DevTable {
        uint32_t *delta = nullptr, *own_off = nullptr, *own_ids = nullptr, *dict = nullptr, *outbits = nullptr;
        uint16_t *hot = nullptr;  // first H rows as u16 (if n_states <= 65535)
        uint8_t *cls = nullptr;
        uint64_t *omask = nullptr;
        uint32_t *gpids = nullptr;
        uint32_t H = 0;
    };
    std::vector<DevTable> dtabs;
    // DFA groups walked together by k_dfa_multi (LDS-resident tables, <= 4 per pack)
    struct DfaPack {
        uint32_t G = 0, tab[4] = {0, 0, 0, 0}, off[4] = {0, 0, 0, 0}, hot_n = 0;
        unsigned long long init[4] = {0, 0, 0, 0};
        uint32_t *d_cls4 = nullptr;
        uint16_t *d_hot = nullptr;
    };
    std::vector<DfaPack> packs;
    std::vector<uint8_t> packed;  // per table: walked by a pack
    // hashed q-gram literal filter (used instead of the automaton when it does not fit LDS)
    struct Lit {
        bool on = false;
        bool nocase = false;
        uint32_t cls_mask = 0;               // bit c: some pattern is filed in class c (LIT_CLASSES)
        uint32_t tmpl = 0;                   // class set the scan kernel is compiled for
        bool joint = false;                  // class scheme: {4-gram, 8-gram} (false) or joint (true)
        uint32_t bits[6] = {0, 0, 0, 0, 0, 0};  // log2 bitmap size per class
        uint32_t bm_off[6] = {0, 0, 0, 0, 0, 0};
        std::vector<uint32_t> bitmap;        // all classes, word-concatenated
        std::vector<uint16_t> rank;          // per bitmap word: set bits in earlier words of its class
        uint32_t rank_base[6] = {0, 0, 0, 0, 0, 0};  // entries (buckets) of all earlier classes
        std::vector<uint32_t> eoff;          // per non-empty bucket: entry range (CSR)
        std::vector<uint32_t> efp;           // per entry: gram fingerprint (the gram itself for L <= 4)
        std::vector<uint32_t> einfo;         // per entry: {pid, anchor, len, 16-B pattern row}
        std::vector<uint32_t> brec;          // per bucket: {fp, pid, len | anchor << 24, row | more << 31}
        uint32_t n_shared = 0;               // buckets holding more than one entry
        std::vector<uint32_t> pat_off;       // per pattern (n + 1), into pat
        std::vector<uint8_t> pat;            // folded pattern bytes
        std::vector<uint8_t> pat16;          // folded pattern bytes, each padded to 16 B rows
        uint32_t *d_bitmap = nullptr, *d_eoff = nullptr, *d_efp = nullptr, *d_einfo = nullptr, *d_brec = nullptr;
        uint16_t *d_rank = nullptr;
        uint8_t *d_pat16 = nullptr;
    };
    // Each filter is built in both class schemes; the first device call times both on the
    // caller's data and keeps the faster (mode: -1 undecided, 0 two-class, 1 joint).
    Lit lit, lit_j;        // literal signatures
    Lit prelit, prelit_j;  // regex prefilter factors
    std::atomic<int> lit_mode{-1}, prelit_mode{-1};
    std::mutex mu;
};

namespace sg {

constexpr uint32_t NONE = 0xffffffffu;
constexpr uint32_t AC_HOT_BYTES = 64 * 1024;   // LDS budget for hot rows
constexpr uint32_t AC_BITS_BYTES = 16 * 1024;  // LDS budget for the output bitmap
constexpr int DFM_BLOCK = 1024;                     // k_dfa_multi block
constexpr uint32_t DFM_LDS = 163840u - 1024u - 512u;  // hot-row budget of one DFA pack (bytes)

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
// Every pattern is filed under ONE gram. Two class schemes:
//   two-class: len 1, 2, 3 -> the whole pattern (classes 0 and 1 index exactly, 2 hashes);
//              len 4..7   -> class 3: one of its 4-byte grams (hashed);
//              len >= 8   -> class 4: one of its 8-byte grams (hashed);
//   joint:     len 1, 2, 3 as above; len >= 4 -> class 5: a 4-byte gram and the byte after it
//              in ONE bitmap: a 32-bit row per 4-gram hash bucket, a bit per value of the next
//              byte's low 5 bits (a 4-byte pattern sets its whole row).
// The probe pass reads a random LDS word per class per text position and is bound by those
// reads' bank conflicts: the joint scheme reads one where the two-class one reads two (C3
// 5.5 -> 4.4 ms), but its 5-byte anchors are less selective than 8-grams, which costs more
// than it saves on some texts (C4 banners 3.5 -> 6.6 ms, the fields JSON 8.1 -> 18.4 ms).
// So both are built, and the first device call times both on its data (sg_matcher::lit_mode).
// Patterns of 8 bytes and more keep an 8-gram fingerprint in both, checked before their
// bytes are. The anchor offset is chosen per pattern to balance the buckets and to avoid
// bytes that are frequent in banners (shared prefixes such as "https://" would otherwise pile
// up and be confirmed at every line). Device side: one LDS bitmap bit per (class, bucket);
// a set bit is confirmed against the bucket's entry fingerprints (rank + CSR), then the
// whole pattern is byte-compared.
constexpr uint32_t LIT_CLASSES = 6;
// Scheme choice (dev_match): the joint scheme must be at least 10 % faster on the trial.
constexpr float LIT_MARGIN = 0.9f;
constexpr uint32_t LIT_J = 5;  // the joint class
__host__ __device__ constexpr uint32_t lit_len(uint32_t c) { return c < 3 ? c + 1 : (c == 3 ? 4 : (c == 4 ? 8 : 5)); }
// class-set templates of k_lit_scan: two-class {4-7, 8+}, {3, 4-7, 8+}, all; joint {J},
// {3, J}, {1, 2, 3, J}
static uint32_t lit_template(uint32_t cls_mask, bool joint) {
    const uint32_t hi = joint ? 0x20u : 0x18u;
    if ((cls_mask & ~hi) == 0) return hi;
    if ((cls_mask & ~(hi | 0x04u)) == 0) return hi | 0x04u;
    return hi | 0x07u;
}

// Bucket of a gram: multiplicative hash (a shift-xor fold measured no faster on X1: more
// false candidates). The joint class's row is the 4-gram's hash (bits - 5 bits), its bit the
// next byte's low 5 bits.
constexpr uint32_t LIT_MUL = 0x9E3779B1u;
__host__ __device__ __forceinline__ uint32_t lit_h(uint32_t lo, uint32_t hi, uint32_t c, uint32_t bits) {
    if (c <= 1) return lo;
    if (c == 4) return ((lo ^ ((hi << 13) | (hi >> 19))) * LIT_MUL) >> (32u - bits);
    if (c == LIT_J) return (((lo * LIT_MUL) >> (37u - bits)) << 5) | (hi & 31u);
    return (lo * LIT_MUL) >> (32u - bits);
}
// Fingerprint for entries of 8 bytes and more (the 8-gram's); shorter entries use the gram.
__host__ __device__ __forceinline__ uint32_t lit_fp8(uint32_t lo, uint32_t hi) {
    return lo ^ ((hi << 13) | (hi >> 19)) ^ (hi * 0xC2B2AE35u);
}

static uint32_t gram_commonness(const uint8_t *g, uint32_t L) {
    // bytes that are frequent in banners / HTTP lines make poor anchors
    static const char *freq = " etaoinsrhldcu/.:-_=<>\"'0123456789";
    uint32_t s = 0;
    for (uint32_t j = 0; j < L; ++j)
        if (g[j] && strchr(freq, g[j])) ++s;
    return s;
}

// extra_bits: bitmap size over the 64-bits-per-pattern base, as a power of two (more bits:
// fewer false candidates, more LDS per block). joint: the class scheme.
static int build_lit(const uint8_t *pats, const uint32_t *offs, uint32_t n, uint32_t flags, sg_matcher::Lit *T,
                     uint32_t extra_bits, bool joint) {
    const bool nocase = flags & SG_NOCASE;
    auto fold = [&](uint8_t b) -> uint8_t { return (nocase && b >= 'A' && b <= 'Z') ? (uint8_t)(b + 32) : b; };
    T->on = true;
    T->joint = joint;
    T->nocase = nocase;
    T->pat.clear();
    T->pat_off.assign(1, 0);
    auto cls_of_len = [joint](uint32_t len) -> uint32_t {
        return len < 4 ? len - 1 : (joint ? LIT_J : (len < 8 ? 3u : 4u));
    };
    uint32_t cnt[LIT_CLASSES] = {};
    for (uint32_t i = 0; i < n; ++i) {
        if (offs[i + 1] <= offs[i]) { set_error("signature %u is empty", i); return SG_E_INVAL; }
        for (uint32_t p = offs[i]; p < offs[i + 1]; ++p) {
            if (pats[p] == '\n') { set_error("signature %u contains a newline", i); return SG_E_INVAL; }
            T->pat.push_back(fold(pats[p]));
        }
        T->pat_off.push_back((uint32_t)T->pat.size());
        cnt[cls_of_len(offs[i + 1] - offs[i])]++;
    }
    uint32_t words = 0;
    T->cls_mask = 0;
    for (uint32_t c = 0; c < LIT_CLASSES; ++c) {
        uint32_t b = 0;
        if (cnt[c]) {
            T->cls_mask |= 1u << c;
            if (c <= 1) {
                b = 8 * (c + 1);
            } else {
                b = 10;
                constexpr uint32_t cap = 18u;
                while (b < (c == 2 ? 15u : cap) && (1ull << b) < (64ull << extra_bits) * cnt[c]) ++b;
            }
        }
        T->bits[c] = b;
        T->bm_off[c] = words;
        if (cnt[c]) words += std::max<uint32_t>((1u << b) / 32, 1);
    }
    // The scan kernel is compiled for a superset of the present classes (lit_template);
    // a class of the superset with no pattern probes an all-zero region of its size.
    T->tmpl = lit_template(T->cls_mask, joint);
    for (uint32_t c = 0; c < LIT_CLASSES; ++c) {
        if (cnt[c] || !((T->tmpl >> c) & 1u)) continue;
        T->bits[c] = (c <= 1) ? 8 * (c + 1) : (c == LIT_J ? 10 : 5);
        T->bm_off[c] = words;
        words += std::max<uint32_t>((1u << T->bits[c]) / 32, 1);
    }
    T->bitmap.assign(words, 0);
    auto word_at = [&](uint32_t i, uint32_t o, uint32_t L) {
        uint32_t key = 0;
        for (uint32_t j = 0; j < L && j < 4; ++j) key |= (uint32_t)T->pat[T->pat_off[i] + o + j] << (8 * j);
        return key;
    };
    auto len_of = [&](uint32_t i) { return T->pat_off[i + 1] - T->pat_off[i]; };
    // anchors: shortest patterns (fewest choices) first, each on its least-loaded gram
    std::vector<uint32_t> order(n);
    for (uint32_t i = 0; i < n; ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) { return len_of(x) < len_of(y); });
    // How many patterns contain each anchor gram: a gram that many signatures share is a
    // common substring of the domain ("openssh_", "server: "), so text holds it far more often
    // than a gram unique to one signature (C4 factors: 8.7 confirmed grams per banner for 1
    // factor hit when anchors ignored this).
    std::unordered_map<uint64_t, uint32_t> share;
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t len = len_of(i);
        const uint32_t c = cls_of_len(len);
        if (c < 3 || (c == LIT_J && len < 5)) continue;
        const uint32_t L = lit_len(c);
        std::vector<uint64_t> mine;
        for (uint32_t o = 0; o + L <= len; ++o) {
            uint64_t g = 0;
            memcpy(&g, &T->pat[T->pat_off[i] + o], L);
            mine.push_back(g | ((uint64_t)L << 60));
        }
        std::sort(mine.begin(), mine.end());
        mine.erase(std::unique(mine.begin(), mine.end()), mine.end());
        for (uint64_t g : mine) share[g]++;
    }
    auto shared_by = [&](uint32_t i, uint32_t o, uint32_t L) -> uint32_t {
        uint64_t g = 0;
        memcpy(&g, &T->pat[T->pat_off[i] + o], L);
        auto it = share.find(g | ((uint64_t)L << 60));
        return it == share.end() ? 0u : it->second;
    };
    struct Ent {
        uint32_t pid, cls, anc, hb, fp;
    };
    std::vector<Ent> ents;
    ents.reserve(n + 32);
    std::vector<std::vector<uint32_t>> load(LIT_CLASSES);
    for (uint32_t c = 0; c < LIT_CLASSES; ++c) load[c].assign(cnt[c] ? (1u << T->bits[c]) : 1, 0);
    for (uint32_t i : order) {
        const uint32_t len = len_of(i);
        const uint32_t c = cls_of_len(len);
        if (c < 3) {
            const uint32_t lo = word_at(i, 0, len);
            const uint32_t h = lit_h(lo, 0u, c, T->bits[c]);
            ents.push_back(Ent{i, c, 0u, h, lo});
            load[c][h]++;
            continue;
        }
        if (c == LIT_J && len == 4) {  // no next byte: the whole row
            const uint32_t lo = word_at(i, 0, 4);
            const uint32_t h0 = lit_h(lo, 0u, c, T->bits[c]) & ~31u;
            for (uint32_t y = 0; y < 32; ++y) {
                ents.push_back(Ent{i, c, 0u, h0 | y, lo});
                load[c][h0 | y]++;
            }
            continue;
        }
        // anchor range: the gram inside the pattern, and for 8+ byte patterns the 8-gram
        // fingerprint too
        const uint32_t L = lit_len(c);
        const uint32_t last = (len >= 8) ? len - 8 : len - L;
        uint64_t best = ~0ull;
        uint32_t bo = 0, bh = 0;
        for (uint32_t o = 0; o <= last && o < 256; ++o) {  // anchor fits the bucket record's 8 bits
            const uint32_t lo = word_at(i, o, 4);
            const uint32_t hi = (c == 4) ? word_at(i, o + 4, 4) : (c == LIT_J ? (uint32_t)T->pat[T->pat_off[i] + o + 4] : 0u);
            const uint32_t h = lit_h(lo, hi, c, T->bits[c]);
            constexpr uint32_t w_share = 64u;  // cost of one more pattern sharing the gram
            // (a load weight of 256 instead of 16, fewer hash-shared buckets: C4 5.78 -> 5.87 ms)
            const uint64_t cost = (uint64_t)(std::max(shared_by(i, o, L), 1u) - 1) * w_share + (uint64_t)load[c][h] * 16 +
                                  gram_commonness(&T->pat[T->pat_off[i] + o], L);
            if (cost < best) { best = cost; bo = o; bh = h; }
        }
        const uint32_t lo = word_at(i, bo, 4);
        const uint32_t fp = len >= 8 ? lit_fp8(lo, word_at(i, bo + 4, 4)) : lo;
        ents.push_back(Ent{i, c, bo, bh, fp});
        load[c][bh]++;
    }
    // entries sorted by (class, bucket); the bitmap word order is the same
    const uint32_t ne = (uint32_t)ents.size();
    std::vector<uint32_t> ids(ne);
    for (uint32_t q = 0; q < ne; ++q) {
        ids[q] = q;
        T->bitmap[T->bm_off[ents[q].cls] + (ents[q].hb >> 5)] |= 1u << (ents[q].hb & 31);
    }
    std::stable_sort(ids.begin(), ids.end(), [&](uint32_t x, uint32_t y) {
        return ents[x].cls != ents[y].cls ? ents[x].cls < ents[y].cls : ents[x].hb < ents[y].hb;
    });
    T->rank.assign(words, 0);
    uint32_t acc = 0;
    for (uint32_t c = 0; c < LIT_CLASSES; ++c) {
        T->rank_base[c] = acc;
        if (!((T->tmpl >> c) & 1u) && !cnt[c]) continue;
        const uint32_t w0 = T->bm_off[c], w1 = w0 + std::max<uint32_t>((1u << T->bits[c]) / 32, 1);
        uint32_t in_cls = 0;
        for (uint32_t w = w0; w < w1; ++w) {
            T->rank[w] = (uint16_t)in_cls;
            in_cls += (uint32_t)__builtin_popcount(T->bitmap[w]);
        }
        if (in_cls > 65535) { set_error("build_lit: more than 65,535 buckets in one length class"); return SG_E_UNSUPPORTED; }
        acc += in_cls;
    }
    T->eoff.assign(1, 0);
    T->efp.clear();
    T->einfo.clear();
    T->pat16.clear();
    std::vector<uint32_t> row(n);
    for (uint32_t i = 0; i < n; ++i) {
        row[i] = (uint32_t)(T->pat16.size() / 16);
        T->pat16.insert(T->pat16.end(), T->pat.begin() + T->pat_off[i], T->pat.begin() + T->pat_off[i + 1]);
        T->pat16.resize((T->pat16.size() + 15) & ~(size_t)15, 0);
    }
    for (uint32_t q = 0; q < ne; ++q) {
        const Ent &e = ents[ids[q]];
        if (q > 0 && (ents[ids[q - 1]].cls != e.cls || ents[ids[q - 1]].hb != e.hb)) T->eoff.push_back(q);
        T->efp.push_back(e.fp);
        T->einfo.insert(T->einfo.end(), {e.pid, e.anc, len_of(e.pid), row[e.pid]});
    }
    if (ne) T->eoff.push_back(ne);
    T->n_shared = 0;
    for (size_t k = 0; k + 1 < T->eoff.size(); ++k) T->n_shared += (T->eoff[k + 1] - T->eoff[k] > 1) ? 1u : 0u;
    if (T->eoff.size() != (size_t)acc + 1) { set_error("build_lit: bucket bookkeeping mismatch"); return SG_E_INVAL; }
    // one 16-B record per bucket: its first entry, plus a flag when more entries follow
    T->brec.assign((size_t)acc * 4, 0);
    for (uint32_t k = 0; k < acc; ++k) {
        const uint32_t e = T->eoff[k];
        const uint32_t *inf = &T->einfo[(size_t)e * 4];
        if (inf[2] >= (1u << 24)) { set_error("signature %u longer than 16 MiB", inf[0]); return SG_E_INVAL; }
        T->brec[4 * k + 0] = T->efp[e];
        T->brec[4 * k + 1] = inf[0];
        T->brec[4 * k + 2] = inf[2] | (inf[1] << 24);
        T->brec[4 * k + 3] = inf[3] | ((T->eoff[k + 1] - e > 1) ? 0x80000000u : 0u);
    }
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
        (void)hipFree(d.omask); (void)hipFree(d.gpids);
    }
    h->dtabs.clear();
    for (auto &k : h->packs) { (void)hipFree(k.d_cls4); (void)hipFree(k.d_hot); }
    h->packs.clear();
    h->packed.clear();
    auto &p = h->dplan;
    for (void *q : {(void *)p.fac_off, (void *)p.fac_pids, (void *)p.s_delta, (void *)p.s_off, (void *)p.s_C,
                    (void *)p.s_eol, (void *)p.s_acc_off, (void *)p.single_of_pid, (void *)p.s_cls, (void *)p.s_acc,
                    (void *)p.s_mid})
        if (q) (void)hipFree(q);
    h->dplan = sg_matcher::DevPlan{};
    for (sg_matcher::Lit *L : {&h->lit, &h->lit_j, &h->prelit, &h->prelit_j}) {
        for (void *q : {(void *)L->d_bitmap, (void *)L->d_rank, (void *)L->d_eoff, (void *)L->d_efp,
                        (void *)L->d_einfo, (void *)L->d_pat16, (void *)L->d_brec})
            if (q) (void)hipFree(q);
        L->d_bitmap = L->d_eoff = L->d_efp = L->d_einfo = L->d_brec = nullptr;
        L->d_rank = nullptr;
        L->d_pat16 = nullptr;
    }
    h->dev = -1;
}

// Packs for k_dfa_multi: regex groups whose whole table fits LDS as u16 with a spare accept
// bit (< 32768 states), whose dead row stays dead, greedily in table order while the pack's
// rows fit one block's LDS.
static int build_packs(sg_matcher *h) {
    h->packed.assign(h->tables.size(), 0);
    if (h->kind != 1) return SG_OK;
    const uint32_t budget = DFM_LDS;
    sg_matcher::DfaPack cur;
    std::vector<uint32_t> cls4(256, 0);
    std::vector<uint16_t> hot;
    auto close = [&]() -> int {
        if (cur.G == 0) return SG_OK;
        hot.resize((hot.size() + 7) & ~(size_t)7, 0);
        cur.hot_n = (uint32_t)hot.size();
        SG_TRY(upload_vec(cls4, &cur.d_cls4));
        SG_TRY(upload_vec(hot, &cur.d_hot));
        h->packs.push_back(cur);
        cur = sg_matcher::DfaPack{};
        std::fill(cls4.begin(), cls4.end(), 0u);
        hot.clear();
        return SG_OK;
    };
    for (size_t ti = 0; ti < h->tables.size(); ++ti) {
        const auto &T = h->tables[ti];
        const uint64_t ents = (uint64_t)T.n_states * T.n_classes;
        auto outbit = [&](uint32_t q) { return (T.outbits[q >> 5] >> (q & 31)) & 1u; };
        bool ok = T.n_states >= 2 && T.n_states <= 32768 && T.n_classes <= 256 && ents * 2 <= budget &&
                  !outbit(0) && T.omask.size() == T.n_states;
        for (uint32_t c = 0; ok && c < T.n_classes; ++c) ok = T.delta[c] == 0;
        if (!ok) continue;
        if (cur.G == 4 || (hot.size() + ents) * 2 > budget) SG_TRY(close());
        const uint32_t g = cur.G++;
        cur.tab[g] = (uint32_t)ti;
        cur.off[g] = (uint32_t)hot.size();
        cur.init[g] = outbit(1) ? T.omask[1] : 0ull;
        for (uint32_t b = 0; b < 256; ++b) cls4[b] |= (uint32_t)T.cls[b] << (8 * g);
        for (uint64_t q = 0; q < ents; ++q)
            hot.push_back((uint16_t)(T.delta[q] | (outbit(T.delta[q]) << 15)));
        h->packed[ti] = 1;
    }
    return close();
}

static int ensure_device(sg_matcher *h, int dev) {
    std::lock_guard<std::mutex> g(h->mu);
    if (h->dev == dev) return SG_OK;
    if (h->dev >= 0) {
        // tables are read by calls in flight on their device: never freed under them
        set_error("matcher tables live on device %d; compile one matcher per device (asked for %d)", h->dev, dev);
        return SG_E_INVAL;
    }
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
        SG_TRY(upload_vec(h->s_mid, &p.s_mid));
        SG_TRY(upload_vec(h->s_cls, &p.s_cls));
        SG_TRY(upload_vec(h->s_acc, &p.s_acc));
    }
    for (sg_matcher::Lit *L : {&h->lit, &h->lit_j, &h->prelit, &h->prelit_j}) {
        if (!L->on) continue;
        SG_TRY(upload_vec(L->bitmap, &L->d_bitmap));
        SG_TRY(upload_vec(L->rank, &L->d_rank));
        SG_TRY(upload_vec(L->eoff, &L->d_eoff));
        SG_TRY(upload_vec(L->efp, &L->d_efp));
        SG_TRY(upload_vec(L->einfo, &L->d_einfo));
        SG_TRY(upload_vec(L->pat16, &L->d_pat16));
        SG_TRY(upload_vec(L->brec, &L->d_brec));
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
        if (!T.omask.empty()) {
            std::vector<uint32_t> gp(64, 0);
            std::copy(T.gpids.begin(), T.gpids.end(), gp.begin());
            SG_TRY(upload_vec(T.omask, &d.omask));
            SG_TRY(upload_vec(gp, &d.gpids));
        }
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
    SG_TRY(build_packs(h));
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

// Per-block LDS staging of (record << 32 | signature) events: an append is one LDS atomic;
// the block drains the buffer with ONE global atomic per flush. (One global atomic per
// event serialises every block on a single counter, which bounded the regex kernels at a
// few GB/s on hit-dense inputs.) A full buffer falls back to a direct global append.
constexpr uint32_t HS_CAP = 1024;
struct HitSink {
    unsigned long long *lds;  // HS_CAP entries
    uint32_t *n, *g;          // LDS counter, LDS broadcast slot
    unsigned long long *hits;
    uint32_t *count;
    uint32_t cap;
    __device__ __forceinline__ void push(unsigned long long v) const {
        const uint32_t i = atomicAdd(n, 1u);
        if (i < HS_CAP) {
            lds[i] = v;
        } else {
            const uint32_t q = atomicAdd(count, 1u);
            if (q < cap) hits[q] = v;
        }
    }
    // Whole block, uniform control flow. Drains when at least half full (or `force`).
    __device__ __forceinline__ void flush(bool force) const {
        __syncthreads();
        const uint32_t hn = min(*n, HS_CAP);
        if (!force && hn < HS_CAP / 2) return;
        if (threadIdx.x == 0) *g = hn ? atomicAdd(count, hn) : 0u;
        __syncthreads();
        const uint32_t base = *g;
        for (uint32_t i = threadIdx.x; i < hn; i += blockDim.x)
            if (base + i < cap) hits[base + i] = lds[i];
        __syncthreads();
        if (threadIdx.x == 0) *n = 0;
        __syncthreads();
    }
};

__device__ __forceinline__ void emit_hit(const ACArgs &a, const HitSink &sink, uint32_t rec, uint32_t sig,
                                         uint32_t *seen, uint32_t &nseen) {
    const uint32_t key = sig;
    for (uint32_t q = 0; q < nseen; ++q)
        if (seen[q] == key) return;
    if (nseen < 4) seen[nseen++] = key;
    if (a.fac_off) {  // prefilter: every pattern that needs this factor is a candidate
        for (uint32_t q = a.fac_off[sig]; q < a.fac_off[sig + 1]; ++q)
            sink.push(((unsigned long long)rec << 32) | a.fac_pids[q]);
        return;
    }
    sink.push(((unsigned long long)rec << 32) | sig);
}

// WIDE (mean record >= 128 B: JSON lines): 64-byte steps, four 16-B loads issued together,
// so a lane's cache line is requested twice rather than 32 times (4-byte steps); short
// records (banners) keep 4-byte steps that end at the record.
template <bool WIDE>
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
    __shared__ unsigned long long s_hb[HS_CAP];
    __shared__ uint32_t s_hn, s_hg;
    if (threadIdx.x == 0) s_hn = 0;
    __syncthreads();
    const HitSink sink{s_hb, &s_hn, &s_hg, a.hits, a.hit_count, a.cap};
    const uint32_t *bits = a.bits_in_lds ? s_bits : a.outbits;
    for (uint32_t r0 = blockIdx.x * blockDim.x; r0 < a.R; r0 += gridDim.x * blockDim.x, sink.flush(false)) {
        const uint32_t r = r0 + threadIdx.x;
        if (r >= a.R) continue;
        const uint2 sp_ = a.spans[r];
        const uint32_t s = sp_.x, e = sp_.y;
        uint32_t st = 0;
        uint32_t seen[4];
        uint32_t nseen = 0;
        auto step = [&](uint32_t p, uint32_t byte) {
            if (p < s || p >= e) return;
            const uint32_t c = s_cls[byte];
            st = (st < a.H) ? (uint32_t)s_hot[st * a.C + c] : a.delta[(size_t)st * a.C + c];
            if ((bits[st >> 5] >> (st & 31)) & 1u) {
                for (uint32_t t = st; t != NONE; t = a.dict[t])
                    for (uint32_t q = a.own_off[t]; q < a.own_off[t + 1]; ++q)
                        emit_hit(a, sink, r, a.own_ids[q], seen, nseen);
            }
        };
        if constexpr (WIDE) {
            for (uint32_t w = s & ~63u; w < e; w += 64) {
                uint4 q[4];
#pragma unroll
                for (uint32_t k = 0; k < 4; ++k) {
                    const uint32_t wk = w + 16u * k;
                    q[k] = (wk < e && wk + 16u > s) ? *reinterpret_cast<const uint4 *>(a.buf + wk) : make_uint4(0u, 0u, 0u, 0u);
                }
#pragma unroll 1
                for (uint32_t k = 0; k < 4; ++k) {
                    const uint32_t wk = w + 16u * k;
                    const uint4 v = q[0];  // (rotated down one register per pass, as in k_dfa_multi)
                    q[0] = q[1]; q[1] = q[2]; q[2] = q[3];
                    if (wk >= e || wk + 16u <= s) continue;
                    const uint32_t xs[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                    for (uint32_t b = 0; b < 16; ++b) step(wk + b, (xs[b >> 2] >> (8 * (b & 3))) & 0xffu);
                }
            }
        } else {
            for (uint32_t w = s & ~3u; w < e; w += 4) {
                const uint32_t x = *reinterpret_cast<const uint32_t *>(a.buf + w);
#pragma unroll
                for (uint32_t b = 0; b < 4; ++b) step(w + b, (x >> (8 * b)) & 0xffu);
            }
        }
    }
    sink.flush(true);
}

// ------------------------------------------------------------------ device: literal filter
struct LitArgs {
    const uint8_t *buf;
    uint64_t n;
    const uint64_t *tile_excl;    // the parse's exclusive packed (starts << 31 | ends) prefix per tile
    uint32_t n_tiles;
    const uint32_t *bitmap, *eoff, *efp;
    const uint16_t *rank;
    const uint4 *einfo;           // {pid, anchor, len, 16-B row}
    const uint4 *brec;            // per bucket {fp, pid, len | anchor << 24, row | more << 31}
    const uint4 *pat16;
    uint32_t bm_words, n_bk, n_ent, cls_mask, nocase;
    uint32_t bits[LIT_CLASSES], bm_off[LIT_CLASSES], rank_base[LIT_CLASSES];
    unsigned long long *hits;
    uint32_t *hit_count;
    uint32_t cap;
    const uint32_t *fac_off, *fac_pids;  // regex prefilter expansion (else null)
    uint2 *spans_out;                    // non-null: also write the parse's record spans (fused A3)
    uint8_t *rec_flag;                   // non-null: mark matched records here instead of listing hits
    uint64_t *keys_out, *raw7_out;       // non-null (with spans_out): every record's key0 and its bytes
                                         // 7..14 (little-endian), taken from the staged tile (X1)
    uint32_t rank_lds;                   // the bitmap words' ranks staged in LDS too (else read from L2)
    uint32_t mw_cap;                     // shared-bucket pair queue entries in dynamic LDS (0: walked in line)
    unsigned long long *diag;            // calibration (SG_LIT_TRIAL_LOG): queued, fingerprint-confirmed, verified
};

constexpr uint32_t LS_HB = 256;    // per-block LDS hit buffer (entries)
constexpr uint32_t LS_HALO = 64;   // text bytes staged on each side of the tile
constexpr uint32_t LS_Q = 512;     // per-block candidate queue (entries: pos:14 | class:3 | record:14)
constexpr int LS_BATCH = 4;        // candidates per lane whose global loads are issued together
constexpr uint32_t LS_MW = 256;    // per-block queue of (further entry, candidate) pairs of shared buckets (when it fits)

__device__ __forceinline__ uint32_t fold4(uint32_t w) {
    // ASCII 'A'..'Z' -> 'a'..'z' in each byte (SWAR)
    const uint32_t h7 = w & 0x7f7f7f7fu;
    const uint32_t ge_a = h7 + 0x3f3f3f3fu;  // high bit: byte >= 'A'
    const uint32_t gt_z = h7 + 0x25252525u;  // high bit: byte > 'Z'
    const uint32_t up = ge_a & ~gt_z & ~w & 0x80808080u;
    return w | (up >> 2);
}


// Byte-compare pattern `row` (len bytes, first 32 preloaded in w0/w1) with the text at
// p - anchor; text from the LDS tile (with halos) when it lies there, else from HBM.
// Grams of classes 1..3 are the whole pattern and already compared exactly.
template <class Args>
__device__ __forceinline__ bool lit_verify(const Args &a, const uint8_t *s_tile, uint64_t base, uint32_t tile,
                                           uint64_t p, uint32_t an, uint32_t len, uint32_t row, uint32_t c,
                                           uint4 w0, uint4 w1) {
    if (p < an) return false;
    const uint64_t ps = p - an;
    if (ps + len > a.n) return false;
    if (c <= 2) return true;
    const bool in_lds = ps + LS_HALO >= base && ps + len + 8 <= base + tile + LS_HALO;
    bool eq = true;
    if (in_lds) {
        // word compares: aligned LDS reads + alignbyte
        const int64_t off = (int64_t)(ps - base);          // >= -LS_HALO
        const uint8_t *tb = s_tile + (off & ~(int64_t)3);
        const uint32_t sh = (uint32_t)(off & 3);
        uint32_t prev = *reinterpret_cast<const uint32_t *>(tb);
        for (uint32_t j = 0; j < len && eq; j += 4) {
            const uint32_t nxt = *reinterpret_cast<const uint32_t *>(tb + j + 4);
            uint32_t tw = sh ? __builtin_amdgcn_alignbyte(nxt, prev, sh) : prev;
            prev = nxt;
            if (a.nocase) tw = fold4(tw);
            uint32_t pw;
            if (j < 32) {
                const uint32_t q = j >> 2;
                const uint32_t x0 = (q & 2) ? ((q & 1) ? w0.w : w0.z) : ((q & 1) ? w0.y : w0.x);
                const uint32_t x1 = (q & 2) ? ((q & 1) ? w1.w : w1.z) : ((q & 1) ? w1.y : w1.x);
                pw = (q & 4) ? x1 : x0;
            } else {
                pw = reinterpret_cast<const uint32_t *>(a.pat16 + row)[j >> 2];
            }
            const uint32_t rem = len - j;
            const uint32_t mask = rem >= 4 ? 0xffffffffu : ((1u << (8 * rem)) - 1u);
            eq = ((tw ^ pw) & mask) == 0;
        }
    } else {
        const uint8_t *pb = reinterpret_cast<const uint8_t *>(a.pat16 + row);
        for (uint32_t j = 0; j < len && eq; ++j) {
            uint32_t ch = a.buf[ps + j];
            if (a.nocase && ch >= 'A' && ch <= 'Z') ch += 32;
            eq = ch == pb[j];
        }
    }
    return eq;
}

template <class Args, class Push>
__device__ __forceinline__ void lit_emit(const Args &a, Push &push, uint32_t rec, uint32_t pid) {
    if (a.rec_flag) {  // idempotent byte store: the set of matched records, no list
        a.rec_flag[rec] = 1;
        return;
    }
    if (a.fac_off) {
        for (uint32_t z = a.fac_off[pid]; z < a.fac_off[pid + 1]; ++z) push(rec, a.fac_pids[z]);
    } else {
        push(rec, pid);
    }
}

// One block per tile of the parse (same tile size as k_lines, so the record index of any
// position is the tile's inclusive start count from the parse plus a block scan of the
// tile's own starts). Each thread owns BPT consecutive positions. Pass 1 tests the LDS
// bitmap of every class of the template CM at every position (unconditional ds_reads the
// compiler can keep in flight together) into candidate masks. The tile's candidates are
// then compacted into an LDS queue and pass 2 spreads them over all lanes: confirm against
// the bucket's entry fingerprints, then byte-compare the pattern (16-B rows from L2, text
// from the LDS tile). Hits go through a per-block LDS buffer flushed with one atomic.
template <int BLK, int BPT, uint32_t CM>
__device__ __forceinline__ void lit_scan_body(const LitArgs &a) {
    constexpr int TILE = BLK * BPT;
    constexpr int NW = BPT / 4;
    extern __shared__ __attribute__((aligned(16))) uint32_t s_dyn[];
    __shared__ __attribute__((aligned(16))) uint8_t s_t[LS_HALO + TILE + LS_HALO];
    __shared__ unsigned long long s_hits[LS_HB];
    __shared__ uint32_t s_q[LS_Q];
    __shared__ uint2 s_kf[LS_Q];  // per queued candidate: (bucket, 8-gram fingerprint)
    __shared__ uint32_t s_mn;
    __shared__ uint32_t s_red[BLK / 64];
    __shared__ uint32_t s_hn, s_g, s_base, s_ebase;
    uint32_t *s_bm = s_dyn;
    // The bitmap words' ranks (a candidate's bucket lookup) are staged after the bitmaps unless
    // leaving them in L2 gives the CU another block (their LDS is half the bitmaps': the fields
    // matcher's tables 68 -> 45 KB, 1 -> 2 blocks per CU, lit_match 8.2 -> 5.7 ms).
    uint16_t *s_rank = reinterpret_cast<uint16_t *>(s_dyn + a.bm_words);
    // {entry, 8-gram fingerprint, gram, queue word} of shared buckets: after the bitmaps (and
    // their ranks), 16-B aligned; a.mw_cap entries (0 when the filter has no shared bucket or
    // the queue would cost the CU a block)
    uint4 *s_mw = reinterpret_cast<uint4 *>(s_dyn + ((a.bm_words + (a.rank_lds ? (a.bm_words + 1) / 2 : 0) + 3) & ~3u));
    const uint32_t mwcap = a.mw_cap;
    for (uint32_t q = threadIdx.x; q < a.bm_words; q += BLK) {
        s_bm[q] = a.bitmap[q];
        if (a.rank_lds) s_rank[q] = a.rank[q];
    }
    if (threadIdx.x == 0) { s_hn = 0; s_mn = 0; }
    __syncthreads();
    const uint32_t t = threadIdx.x;
    const uint64_t n = a.n;
    uint8_t *s_tile = s_t + LS_HALO;

    auto push = [&](uint32_t rec, uint32_t sig) {
        const unsigned long long v = ((unsigned long long)rec << 32) | sig;
        const uint32_t i = atomicAdd(&s_hn, 1u);
        if (i < LS_HB) {
            s_hits[i] = v;
        } else {
            // overflow: one global atomic per wave (the lanes pushing now), not per event
            const uint64_t act = __ballot(1);
            const int lead = __ffsll((long long)act) - 1;
            uint32_t g0 = 0;
            if (lane_id() == lead) g0 = atomicAdd(a.hit_count, (uint32_t)__popcll(act));
            const uint32_t g = (uint32_t)__shfl((int)g0, lead) + (uint32_t)__popcll(act & ((1ull << lane_id()) - 1));
            if (g < a.cap) a.hits[g] = v;
        }
    };
    // drain the LDS hit buffer with one global atomic (block-uniform call sites only)
    auto flush = [&](bool force) {
        const uint32_t hn = min(s_hn, LS_HB);
        if (hn >= LS_HB / 2 || (force && hn)) {
            __syncthreads();
            if (t == 0) s_g = atomicAdd(a.hit_count, hn);
            __syncthreads();
            for (uint32_t i = t; i < hn; i += BLK) {
                const uint32_t g = s_g + i;
                if (g < a.cap) a.hits[g] = s_hits[i];
            }
            __syncthreads();
            if (t == 0) s_hn = 0;
            __syncthreads();
        }
    };

    // A tile's text (its BPT bytes per thread, the halo words, its parse counts) is loaded
    // into registers one tile ahead: the next tile's loads are issued after pass 1 and land
    // while pass 2 runs (LDS bounds these blocks' occupancy, so the registers are free).
    uint32_t w[NW];
    uint32_t hx = 0;
    uint64_t tex = 0;
    auto load_text = [&](uint32_t tl) {
        const uint64_t b0 = (uint64_t)tl * TILE;
        const uint64_t m0 = b0 + (uint64_t)t * BPT;
        if (b0 + TILE + LS_HALO <= n) {
            const uint4 *p = reinterpret_cast<const uint4 *>(a.buf + m0);
#pragma unroll
            for (int j = 0; j < NW / 4; ++j) {
                const uint4 v = p[j];
                w[4 * j] = v.x; w[4 * j + 1] = v.y; w[4 * j + 2] = v.z; w[4 * j + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int j = 0; j < NW; ++j) {
                uint32_t x = 0;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint64_t pos = m0 + 4 * j + k;
                    x |= (uint32_t)((pos < n) ? a.buf[pos] : 0x0au) << (8 * k);
                }
                w[j] = x;
            }
        }
        // halos: 16 lanes x 4 B on each side ('\n' outside the buffer)
        if (t < 2 * LS_HALO / 4) {
            const bool right = t >= LS_HALO / 4;
            const int64_t pos0 = right ? (int64_t)(b0 + TILE) + 4 * (t - LS_HALO / 4) : (int64_t)b0 - LS_HALO + 4 * t;
            uint32_t x = 0;
            if (pos0 >= 0 && (uint64_t)pos0 + 4 <= n) {
                x = *reinterpret_cast<const uint32_t *>(a.buf + pos0);
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int64_t pos = pos0 + k;
                    x |= (uint32_t)((pos >= 0 && (uint64_t)pos < n) ? a.buf[pos] : 0x0au) << (8 * k);
                }
            }
            hx = x;
        }
        if (t == 0) tex = a.tile_excl[tl];
    };
    if (blockIdx.x < a.n_tiles) load_text(blockIdx.x);

    for (uint32_t tile = blockIdx.x; tile < a.n_tiles; tile += gridDim.x) {
        const uint64_t base = (uint64_t)tile * TILE;
        const uint64_t my0 = base + (uint64_t)t * BPT;
        if (t < 2 * LS_HALO / 4) {
            const bool right = t >= LS_HALO / 4;
            *reinterpret_cast<uint32_t *>(right ? s_tile + TILE + 4 * (t - LS_HALO / 4) : s_t + 4 * t) = hx;
        }
#pragma unroll
        for (int j = 0; j < NW / 4; ++j)
            reinterpret_cast<uint4 *>(s_tile)[(NW / 4) * t + j] = make_uint4(w[4 * j], w[4 * j + 1], w[4 * j + 2], w[4 * j + 3]);
        if (t == 0) {
            s_base = (uint32_t)(tex >> 31);
            s_ebase = (uint32_t)(tex & 0x7fffffffu);
        }
        uint64_t m = 0;
#pragma unroll
        for (int j = 0; j < NW; ++j) {
            const uint32_t y = w[j] ^ 0x0a0a0a0au;
            const uint32_t r = ~(((y & 0x7f7f7f7fu) + 0x7f7f7f7fu) | y | 0x7f7f7f7fu);
            m |= (uint64_t)(((r >> 7) & 1u) | ((r >> 14) & 2u) | ((r >> 21) & 4u) | ((r >> 28) & 8u)) << (4 * j);
        }
        __syncthreads();
        const uint64_t cin = (s_tile[(int)(t * BPT) - 1] == 0x0a) || (base == 0 && t == 0);
        const uint64_t full = (BPT == 64) ? ~0ull : ((1ull << (BPT & 63)) - 1);
        const uint64_t sm = ~m & ((m << 1) | cin) & full;
        uint32_t tot;
        const uint32_t excl = block_excl_scan<BLK>((uint32_t)__popcll(sm), &tot, s_red);
        if (a.spans_out) {
            // the record spans of this tile, as k_lines writes them (k-th start / k-th end)
            const uint64_t em = m & ~((m << 1) | cin) & full;
            uint32_t etot;
            const uint32_t eexcl = block_excl_scan<BLK>((uint32_t)__popcll(em), &etot, s_red);
            uint32_t si = s_base + excl, ei = s_ebase + eexcl;
            if (a.keys_out) {
                // X1: each record's key0 (chunk_key at 0) and its bytes 7..14, read from the
                // staged tile at the record's start (the right halo holds 64 bytes past the
                // tile, '\n' past the buffer): the matched records' gather then reads 16 B per
                // record instead of each record's first line again
                for (uint64_t bits = sm; bits; bits &= bits - 1) {
                    const uint32_t o = t * BPT + (uint32_t)__ffsll((long long)bits) - 1u;  // tile offset
                    const uint32_t *dw = reinterpret_cast<const uint32_t *>(s_tile + (o & ~3u));
                    const uint32_t sh = o & 3u;
                    const uint32_t d0 = dw[0], d1 = dw[1], d2 = dw[2], d3 = dw[3], d4 = dw[4];
                    const uint32_t b0 = __builtin_amdgcn_alignbyte(d1, d0, sh), b1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
                    const uint32_t b2 = __builtin_amdgcn_alignbyte(d3, d2, sh), b3 = __builtin_amdgcn_alignbyte(d4, d3, sh);
                    const uint64_t v = (uint64_t)b0 | ((uint64_t)b1 << 32);  // bytes 0..7
                    // the record's length within its first 8 bytes: the first '\n' there
                    const uint64_t y = v ^ 0x0a0a0a0a0a0a0a0aull;
                    const uint64_t z = ~(((y & 0x7f7f7f7f7f7f7f7full) + 0x7f7f7f7f7f7f7f7full) | y | 0x7f7f7f7f7f7f7f7full);
                    const uint32_t len8 = z ? (uint32_t)__builtin_ctzll(z) >> 3 : 8u;
                    const uint32_t take = len8 < 7u ? len8 : 7u;
                    const uint64_t kv = v & ((1ull << (8u * take)) - 1ull);
                    a.keys_out[si] = len8 ? ((__builtin_bswap64(kv) & ~0xffull) | len8) : 0ull;
                    // bytes 7..14: byte 3 of b1 on, then b2, then b3's first 3
                    a.raw7_out[si] = (uint64_t)__builtin_amdgcn_alignbyte(b2, b1, 3u) |
                                     ((uint64_t)__builtin_amdgcn_alignbyte(b3, b2, 3u) << 32);
                    a.spans_out[si++].x = (uint32_t)(my0 + __ffsll((long long)bits) - 1);
                }
            } else {
                for (uint64_t bits = sm; bits; bits &= bits - 1) a.spans_out[si++].x = (uint32_t)(my0 + __ffsll((long long)bits) - 1);
            }
            for (uint64_t bits = em; bits; bits &= bits - 1) a.spans_out[ei++].y = (uint32_t)(my0 + __ffsll((long long)bits) - 1);
        }
        uint32_t wn0 = *reinterpret_cast<const uint32_t *>(s_tile + (t + 1) * BPT);
        uint32_t wn1 = *reinterpret_cast<const uint32_t *>(s_tile + (t + 1) * BPT + 4);
        if (a.nocase) {
#pragma unroll
            for (int j = 0; j < NW; ++j) w[j] = fold4(w[j]);
            wn0 = fold4(wn0);
            wn1 = fold4(wn1);
        }
        // pass 1: bitmap probes. g[b] = the 4-byte word at b times LIT_MUL (the joint class's
        // row hash); the byte at b + 4 picks the row's bit
        auto word_at = [&](int b) -> uint32_t {
            const int i0 = b >> 2;
            const uint32_t x0 = (i0 < NW) ? w[i0] : (i0 == NW ? wn0 : wn1);
            const uint32_t x1 = (i0 + 1 < NW) ? w[i0 + 1] : (i0 + 1 == NW ? wn0 : wn1);
            return (b & 3) ? __builtin_amdgcn_alignbyte(x1, x0, b & 3) : x0;
        };
        // candidate bit masks per class: 32-bit words when a thread holds <= 32 positions
        using CT = typename std::conditional<(BPT <= 32), uint32_t, uint64_t>::type;
        CT cand[LIT_CLASSES] = {};
        // g[b] = the 4-byte word at b times LIT_MUL (b = 0 .. BPT + 3): the 4-gram class's
        // bucket and the joint class's row
        uint32_t g[BPT + 4];
#pragma unroll
        for (int b = 0; b < 4; ++b) g[b] = word_at(b) * LIT_MUL;
#pragma unroll
        for (int b = 0; b < BPT; ++b) {
            const uint32_t lo = word_at(b);
            const uint32_t w4 = word_at(b + 4);
            g[b + 4] = w4 * LIT_MUL;
#pragma unroll
            for (uint32_t c = 0; c < LIT_CLASSES; ++c) {
                if (!((CM >> c) & 1u)) continue;
                if (c == LIT_J) {  // one read: the 4-gram's row, the next byte's bit
                    const uint32_t row = s_bm[a.bm_off[c] + (g[b] >> (37u - a.bits[c]))];
                    cand[c] |= (CT)((row >> (w4 & 31u)) & 1u) << b;
                    continue;
                }
                uint32_t h;
                if (c == 4) h = lit_h(lo, w4, 4u, a.bits[c]);
                else if (c == 3) h = g[b] >> (32u - a.bits[c]);
                else h = lit_h(lo & ((1u << (8 * (c + 1))) - 1u), 0u, c, a.bits[c]);
                cand[c] |= (CT)((s_bm[a.bm_off[c] + (h >> 5)] >> (h & 31)) & 1u) << b;
            }
        }
        if (my0 + BPT > n) {
            const uint64_t valid = (my0 >= n) ? 0ull : ((1ull << (n - my0)) - 1);
#pragma unroll
            for (uint32_t c = 0; c < LIT_CLASSES; ++c) cand[c] &= valid;
        }
        // pass 2: queue the tile's candidates, then confirm/verify them across all lanes
        uint32_t ncand = 0;
#pragma unroll
        for (uint32_t c = 0; c < LIT_CLASSES; ++c) ncand += (uint32_t)__popcll(cand[c]);
        uint32_t qtot;
        const uint32_t qex = block_excl_scan<BLK>(ncand, &qtot, s_red);
        if (a.diag && t == 0) atomicAdd(&a.diag[0], (unsigned long long)qtot);
        if (tile + gridDim.x < a.n_tiles) load_text(tile + gridDim.x);
        const uint32_t lrec0 = excl;  // tile-local index of this thread's first record start
        // one further entry e of a shared bucket against the candidate at p (fp8/fp4: its
        // 8-gram fingerprint and its gram)
        auto check_entry = [&](uint32_t e, uint32_t fp8v, uint32_t fp4v, uint32_t c, uint64_t p, uint32_t rec) {
            const uint4 inf = a.einfo[e];
            if (a.diag) atomicAdd(&a.diag[4], 1ull);
            if (a.efp[e] != (inf.z >= 8u ? fp8v : fp4v)) return;
            if (a.diag) atomicAdd(&a.diag[5], 1ull);
            const uint4 w0 = a.pat16[inf.w];
            const uint4 w1 = inf.z > 16 ? a.pat16[inf.w + 1] : make_uint4(0, 0, 0, 0);
            if (lit_verify(a, s_tile, base, TILE, p, inf.y, inf.z, inf.w, c, w0, w1)) lit_emit(a, push, rec, inf.x);
        };
        // the queued pairs, one per thread (block-uniform call sites; the tile's text must
        // still be in LDS)
        auto run_pairs = [&]() {
            const uint32_t mn = min(s_mn, mwcap);
            for (uint32_t j = t; j < mn; j += BLK) {
                const uint4 pr = s_mw[j];
                check_entry(pr.x, pr.y, pr.z, (pr.w >> 14) & 7u, base + (pr.w >> 17), s_base + (pr.w & 0x3fffu) - 1);
            }
            __syncthreads();
            if (t == 0) s_mn = 0;
        };
        for (uint32_t r0 = 0; r0 < qtot; r0 += LS_Q) {
            uint32_t qi = qex;
            if (qi < r0 + LS_Q && qi + ncand > r0) {
#pragma unroll
                for (uint32_t c = 0; c < LIT_CLASSES; ++c) {
                    uint64_t cm = cand[c];
                    while (cm) {
                        const int b = __ffsll((long long)cm) - 1;
                        cm &= cm - 1;
                        if (qi >= r0 && qi < r0 + LS_Q) {
                            // record containing p: starts at or before p, minus one (may be -1
                            // relative to the tile: the record began in an earlier tile)
                            const uint32_t lrec = lrec0 + (uint32_t)__popcll(sm & ((2ull << b) - 1));
                            s_q[qi - r0] = ((t * BPT + b) << 17) | (c << 14) | lrec;
                        }
                        ++qi;
                    }
                }
            }
            __syncthreads();
            const uint32_t qn = min(LS_Q, qtot - r0);
            // stage 1 (LDS only): gram -> bucket and fingerprint
            for (uint32_t i = t; i < qn; i += BLK) {
                const uint32_t ent = s_q[i];
                const int q = (int)(ent >> 17);
                const uint32_t c = (ent >> 14) & 7u;
                uint32_t lo = *reinterpret_cast<const uint32_t *>(s_tile + (q & ~3));
                uint32_t l1 = *reinterpret_cast<const uint32_t *>(s_tile + (q & ~3) + 4);
                uint32_t l2 = *reinterpret_cast<const uint32_t *>(s_tile + (q & ~3) + 8);
                if (a.nocase) { lo = fold4(lo); l1 = fold4(l1); l2 = fold4(l2); }
                const uint32_t sh = q & 3;
                const uint32_t k0 = sh ? __builtin_amdgcn_alignbyte(l1, lo, sh) : lo;
                const uint32_t k1 = sh ? __builtin_amdgcn_alignbyte(l2, l1, sh) : l1;
                const uint32_t key = (c >= 3) ? k0 : (k0 & ((1u << (8 * (c + 1))) - 1u));
                const uint32_t h = lit_h(key, k1, c, a.bits[c]);
                const uint32_t wi = a.bm_off[c] + (h >> 5);
                const uint32_t rk = a.rank_lds ? (uint32_t)s_rank[wi] : (uint32_t)a.rank[wi];
                const uint32_t k = a.rank_base[c] + rk + (uint32_t)__popc(s_bm[wi] & ((1u << (h & 31)) - 1u));
                // fingerprints: the gram itself (entries shorter than 8) and the 8-gram's
                s_kf[i] = make_uint2(k, lit_fp8(k0, k1));
            }
            // stage 2: LS_BATCH candidates per lane, their bucket records and first pattern
            // rows loaded together, then verified against the LDS text
            for (uint32_t i0 = t; i0 < qn; i0 += LS_BATCH * BLK) {
                uint4 br[LS_BATCH];
                uint32_t fp8[LS_BATCH], fp4[LS_BATCH];
#pragma unroll
                for (int u = 0; u < LS_BATCH; ++u) {
                    const uint32_t i = i0 + u * BLK;
                    br[u] = make_uint4(0, 0, 0, 0);
                    fp8[u] = 1;
                    fp4[u] = 1;
                    if (i < qn) {
                        const uint2 kf = s_kf[i];
                        br[u] = a.brec[kf.x];
                        fp8[u] = kf.y;
                        // the gram itself (fingerprint of entries shorter than 8), from the tile
                        const uint32_t ent = s_q[i];
                        const int q = (int)(ent >> 17);
                        const uint32_t c = (ent >> 14) & 7u;
                        uint32_t w0 = *reinterpret_cast<const uint32_t *>(s_tile + (q & ~3));
                        uint32_t w1 = *reinterpret_cast<const uint32_t *>(s_tile + (q & ~3) + 4);
                        if (a.nocase) { w0 = fold4(w0); w1 = fold4(w1); }
                        const uint32_t k0 = (q & 3) ? __builtin_amdgcn_alignbyte(w1, w0, q & 3) : w0;
                        fp4[u] = (c >= 3) ? k0 : (k0 & ((1u << (8 * (c + 1))) - 1u));
                    }
                }
                // the bucket's first entry: its fingerprint kind by its pattern length
                uint32_t fpv[LS_BATCH];
#pragma unroll
                for (int u = 0; u < LS_BATCH; ++u) fpv[u] = (br[u].z & 0xffffffu) >= 8u ? fp8[u] : fp4[u];
                uint4 r0w[LS_BATCH], r1w[LS_BATCH];
#pragma unroll
                for (int u = 0; u < LS_BATCH; ++u) {
                    const bool m = (i0 + u * BLK < qn) && br[u].x == fpv[u];
                    const uint32_t row = br[u].w & 0x7fffffffu;
                    const uint32_t len = br[u].z & 0xffffffu;
                    r0w[u] = m ? a.pat16[row] : make_uint4(0, 0, 0, 0);
                    r1w[u] = (m && len > 16) ? a.pat16[row + 1] : make_uint4(0, 0, 0, 0);
                }
#pragma unroll
                for (int u = 0; u < LS_BATCH; ++u) {
                    const uint32_t i = i0 + u * BLK;
                    if (i >= qn) continue;
                    const uint32_t ent = s_q[i];
                    const uint32_t q = ent >> 17;
                    const uint32_t c = (ent >> 14) & 7u;
                    const uint32_t rec = s_base + (ent & 0x3fffu) - 1;
                    const uint64_t p = base + q;
                    if (br[u].x == fpv[u]) {
                        const bool ok = lit_verify(a, s_tile, base, TILE, p, br[u].z >> 24, br[u].z & 0xffffffu,
                                                   br[u].w & 0x7fffffffu, c, r0w[u], r1w[u]);
                        if (ok) lit_emit(a, push, rec, br[u].y);
                        if (a.diag) {
                            atomicAdd(&a.diag[1], 1ull);
                            if (ok) atomicAdd(&a.diag[2], 1ull);
                        }
                    }
                    if (br[u].w >> 31) {
                        // more patterns share this bucket: its further entries are queued as
                        // (entry, candidate) pairs that the whole block checks once the queue is
                        // half full or the tile ends, one pair per thread, instead of this lane
                        // walking them one dependent load chain after another while its wave
                        // waits (C4: 3.7 % of candidates, half of the scan's time in line)
                        const uint32_t k = s_kf[i].x;
                        const uint32_t e0 = a.eoff[k] + 1, e1 = a.eoff[k + 1];
                        if (a.diag) atomicAdd(&a.diag[3], 1ull);
                        const uint32_t slot = atomicAdd(&s_mn, e1 - e0);
                        for (uint32_t e = e0; e < e1; ++e) {
                            if (slot + (e - e0) < mwcap) s_mw[slot + (e - e0)] = make_uint4(e, fp8[u], fp4[u], ent);
                            else check_entry(e, fp8[u], fp4[u], c, p, rec);  // queue full: in line
                        }
                    }
                }
            }
            __syncthreads();
            if (mwcap && s_mn >= mwcap / 2) run_pairs();
            // hit-dense inputs (regex prefilter fan-out): drain between queue batches, so the
            // buffer rarely overflows into per-wave global atomics
            flush(false);
        }
        __syncthreads();
        if (mwcap && s_mn) run_pairs();
        flush(tile + gridDim.x >= a.n_tiles);
    }
}

template <int BLK, int BPT, uint32_t CM>
__global__ __launch_bounds__(BLK) __attribute__((amdgpu_waves_per_eu(4))) void k_lit_scan(LitArgs a) {
    lit_scan_body<BLK, BPT, CM>(a);
}

// The class-scheme trial (the same scan over the first tiles, every output dropped): its own
// symbol, so kernel statistics and PMC passes of k_lit_scan hold the real scans only.
template <int BLK, int BPT, uint32_t CM>
__global__ __launch_bounds__(BLK) __attribute__((amdgpu_waves_per_eu(4))) void k_lit_trial(LitArgs a) {
    lit_scan_body<BLK, BPT, CM>(a);
}

// LDS bytes of k_lit_scan's dynamic tables for a filter: the bitmaps (u32), + their ranks (u16).
static uint32_t lit_lds_bytes(const sg_matcher::Lit &T, bool ranks = true) {
    const uint32_t bmw = (uint32_t)T.bitmap.size();
    return 4u * bmw + (ranks ? 4u * ((bmw + 1) / 2) : 0u);
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
    const uint32_t *outbits;
    const unsigned long long *omask;  // per state: group-local patterns accepted on entry
    const uint32_t *gpids;            // group-local pattern -> signature id (<= 64)
    unsigned long long *hits;
    uint32_t *hit_count;
    uint32_t cap;
    uint32_t bits_in_lds;
};

constexpr int DFA_BLOCK = 512;

// One DFA of a set (<= 64 patterns). State 0 = dead (no pattern can still match), state
// 1 = start. A state with output accepts a mask of group-local patterns; accepted
// patterns are removed from the successor states at build time. One thread walks one
// record, OR-ing the accept masks into a register; the block then appends all of its
// records' hits at once (block scan of the popcounts -> LDS staging buffer, one global
// atomic per drain), so generic signatures that fire on every banner cost no contended
// atomics at all.
__global__ __launch_bounds__(DFA_BLOCK) void k_dfa_match(DFAArgs a) {
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
    __shared__ unsigned long long s_hb[HS_CAP];
    __shared__ uint32_t s_gp[64];
    __shared__ uint32_t s_red[DFA_BLOCK / 64];
    __shared__ uint32_t s_hn, s_hg;
    if (threadIdx.x < 64) s_gp[threadIdx.x] = a.gpids[threadIdx.x];
    if (threadIdx.x == 0) s_hn = 0;
    __syncthreads();
    const HitSink sink{s_hb, &s_hn, &s_hg, a.hits, a.hit_count, a.cap};
    const uint32_t *bits = a.bits_in_lds ? s_bits : a.outbits;
    auto step = [&](uint32_t st, uint32_t c) -> uint32_t {
        return (st < a.H) ? (uint32_t)s_hot[st * a.C + c] : a.delta[(size_t)st * a.C + c];
    };
    unsigned long long acc = 0;
    auto accept = [&](uint32_t st) {
        if ((bits[st >> 5] >> (st & 31)) & 1u) acc |= a.omask[st];
    };
    for (uint32_t r0 = blockIdx.x * DFA_BLOCK; r0 < a.R; r0 += gridDim.x * DFA_BLOCK) {
        const uint32_t r = r0 + threadIdx.x;
        acc = 0;
        if (r < a.R) {
            const uint2 sp_ = a.spans[r];
            const uint32_t s = sp_.x, e = sp_.y;
            uint32_t st = 1;
            accept(st);
            // 16-B loads: lanes walk different records, so every load instruction touches
            // up to 64 cache lines; a quarter of the 4-B loads' instructions
            for (uint32_t w = s & ~15u; w < e && st != 0; w += 16) {
                const uint4 v = *reinterpret_cast<const uint4 *>(a.buf + w);
                const uint32_t xs[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (uint32_t b = 0; b < 16; ++b) {
                    const uint32_t p = w + b;
                    if (p < s || p >= e || st == 0) continue;
                    st = step(st, s_cls[(xs[b >> 2] >> (8 * (b & 3))) & 0xffu]);
                    accept(st);
                }
            }
            if (st != 0 && a.eol) accept(step(st, a.eol));
        }
        // block-uniform append of this round's hits
        uint32_t tot;
        const uint32_t ex = block_excl_scan<DFA_BLOCK>((uint32_t)__popcll(acc), &tot, s_red);
        if (tot == 0) continue;
        if (s_hn + tot > HS_CAP) sink.flush(true);
        unsigned long long *dst;
        if (tot > HS_CAP) {
            if (threadIdx.x == 0) s_hg = atomicAdd(a.hit_count, tot);
            __syncthreads();
            const uint32_t g = s_hg;
            for (unsigned long long m = acc, k = 0; m; m &= m - 1, ++k) {
                const uint32_t q = g + ex + (uint32_t)k;
                if (q < a.cap) a.hits[q] = ((unsigned long long)r << 32) | s_gp[__ffsll((long long)m) - 1];
            }
            __syncthreads();
            continue;
        }
        dst = s_hb + s_hn + ex;
        for (unsigned long long m = acc; m; m &= m - 1)
            *dst++ = ((unsigned long long)r << 32) | s_gp[__ffsll((long long)m) - 1];
        __syncthreads();
        if (threadIdx.x == 0) s_hn += tot;
        __syncthreads();
    }
    sink.flush(true);
}

// Several factor-less DFA groups walked together (a pack of G <= 4): one thread walks one
// record through all G automata at once, so the record's bytes are loaded, split and bounds-
// checked once, one LDS read gives the byte's class in every group (4 classes packed in a u32),
// and the G transition chains are independent (G loads in flight per byte). Each hot entry
// carries the target state's accept flag in bit 15, so accepting costs no outbits lookup.
// Every group of the pack is fully LDS-resident; the block's records' hits go out with one
// global atomic per round (no LDS staging: the tables use the LDS).
struct DFAMultiArgs {
    const uint8_t *buf;
    const uint2 *spans;
    uint32_t R;
    const uint32_t *cls4;    // per byte: class in group g at bits 8g..8g+7
    const uint16_t *hot;     // groups' rows back to back: next state | accept << 15
    uint32_t hot_n;          // entries (multiple of 8)
    uint32_t off[4], C[4], eol[4];
    unsigned long long init[4];              // accept mask of the start state
    const unsigned long long *omask[4];
    const uint32_t *gpids[4];
    unsigned long long *hits;
    uint32_t *hit_count;
    uint32_t cap;
};

// Lane refill: each wave owns a contiguous range of records and every lane takes the next
// record of the range the moment its own ends (ranks from a ballot, no atomics), so a wave
// no longer idles while its longest record finishes (banners: 31..105 B, mean 53). Bytes
// outside the lane's record leave its states unchanged (a select, not a branch), so lanes
// at a record's first or last chunk run the same instructions as lanes in its middle.
template <int G, int NQ>
__global__ __launch_bounds__(DFM_BLOCK) void k_dfa_multi(DFAMultiArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    uint32_t *s_cls = reinterpret_cast<uint32_t *>(lds);
    uint16_t *s_hot = reinterpret_cast<uint16_t *>(lds + 1024);
    if (threadIdx.x < 256) s_cls[threadIdx.x] = a.cls4[threadIdx.x];
    for (uint32_t q = threadIdx.x; q < a.hot_n / 8; q += DFM_BLOCK)
        reinterpret_cast<uint4 *>(s_hot)[q] = reinterpret_cast<const uint4 *>(a.hot)[q];
    __syncthreads();
    const uint32_t lane = (uint32_t)lane_id();
    const uint64_t lt = (1ull << lane) - 1ull;
    const uint32_t n_waves = gridDim.x * (DFM_BLOCK / 64);
    const uint32_t wv = blockIdx.x * (DFM_BLOCK / 64) + (threadIdx.x >> 6);
    const uint32_t per = (a.R + n_waves - 1) / n_waves;
    const uint32_t r_hi = min(a.R, (uint32_t)min<uint64_t>((uint64_t)(wv + 1) * per, 0xffffffffull));
    uint32_t nxt = min(a.R, (uint32_t)min<uint64_t>((uint64_t)wv * per, 0xffffffffull));  // wave-uniform
    unsigned long long acc[G];
    uint32_t st[G];
    uint32_t r = 0, w = 0, s = 0, e = 0;
    bool busy = false, done = false;
    while (true) {
        const uint64_t need = __ballot(!busy && !done);
        if (need) {
            if (!busy && !done) {
                const uint32_t rr = nxt + (uint32_t)__popcll(need & lt);
                if (rr < r_hi) {
                    r = rr;
                    const uint2 sp_ = a.spans[r];
                    s = sp_.x; e = sp_.y; w = s & ~(16u * NQ - 1u);
#pragma unroll
                    for (int g = 0; g < G; ++g) { st[g] = 1; acc[g] = a.init[g]; }
                    busy = true;
                } else {
                    done = true;
                }
            }
            nxt += (uint32_t)__popcll(need);
        }
        if (!__ballot(busy)) break;
        bool fin = false;
        if (busy) {
            // NQ x 16-byte steps. Long records (NQ = 4): the four 16-B loads issued together
            // (half a cache line per request: a line evicted between a lane's steps is fetched
            // 2x, not 8x; the fields step's dfa_match 9.9 -> 5.0 ms), walked 16 bytes at a
            // time. Short records (NQ = 1, banners of ~50 B) keep 16-B steps: a lane refills
            // sooner and walks fewer bytes outside its record (C4 1.0 vs 1.6 ms).
            uint4 vq[NQ];
#pragma unroll
            for (uint32_t k = 0; k < NQ; ++k) {
                const uint32_t wk = w + 16u * k;
                vq[k] = (wk < e && wk + 16u > s) ? *reinterpret_cast<const uint4 *>(a.buf + wk) : make_uint4(0u, 0u, 0u, 0u);
            }
#pragma unroll 1
            for (uint32_t k = 0; k < NQ; ++k) {
                const uint32_t wk = w + 16u * k;
                // chunk k is vq[0]: the chunks rotate down one register per pass (a select on k
                // would index them through scratch)
                const uint4 v = vq[0];
#pragma unroll
                for (int j = 0; j + 1 < NQ; ++j) vq[j] = vq[j + 1];
                const uint32_t xs[4] = {v.x, v.y, v.z, v.w};
                const uint32_t lo = s > wk ? min(s - wk, 16u) : 0u, hi = e > wk ? min(e - wk, 16u) : 0u;
                if (lo >= hi) continue;
                uint32_t cw[16];
#pragma unroll
                for (uint32_t b = 0; b < 16; ++b) cw[b] = s_cls[(xs[b >> 2] >> (8 * (b & 3))) & 0xffu];
#pragma unroll
                for (uint32_t b = 0; b < 16; ++b) {
                    const bool in = b >= lo && b < hi;
                    uint32_t vv[G], any = 0;
#pragma unroll
                    for (int g = 0; g < G; ++g)
                        vv[g] = s_hot[__umul24(st[g], a.C[g]) + a.off[g] + ((cw[b] >> (8 * g)) & 0xffu)];
#pragma unroll
                    for (int g = 0; g < G; ++g) {
                        vv[g] = in ? vv[g] : st[g];  // outside the record: state kept, no accept
                        st[g] = vv[g] & 0x7fffu;
                        any |= vv[g];
                    }
                    if (any & 0x8000u) {
#pragma unroll
                        for (int g = 0; g < G; ++g)
                            if (vv[g] & 0x8000u) acc[g] |= a.omask[g][st[g]];
                    }
                }
            }
            w += 16u * NQ;
            uint32_t alive = 0;
#pragma unroll
            for (int g = 0; g < G; ++g) alive |= st[g];
            if (w >= e || !alive) {  // every group dead: row 0 maps to 0, never accepting
#pragma unroll
                for (int g = 0; g < G; ++g)
                    if (a.eol[g] && st[g]) {
                        const uint32_t x = s_hot[__umul24(st[g], a.C[g]) + a.off[g] + a.eol[g]];
                        if (x & 0x8000u) acc[g] |= a.omask[g][x & 0x7fffu];
                    }
                fin = true;
            }
        }
        // finished lanes append their hits: one atomic per wave step that has any
        uint32_t cnt = 0;
        if (fin) {
#pragma unroll
            for (int g = 0; g < G; ++g) cnt += (uint32_t)__popcll(acc[g]);
        }
        if (__ballot(cnt != 0)) {
            const uint32_t inc = wave_incl_scan_shfl(cnt);
            const uint32_t tot = (uint32_t)__shfl((int)inc, 63, 64);
            uint32_t base = 0;
            if (lane == 0) base = atomicAdd(a.hit_count, tot);
            uint32_t q = (uint32_t)__shfl((int)base, 0, 64) + inc - cnt;
            if (cnt) {
#pragma unroll
                for (int g = 0; g < G; ++g)
                    for (unsigned long long m = acc[g]; m; m &= m - 1, ++q)
                        if (q < a.cap) a.hits[q] = ((unsigned long long)r << 32) | a.gpids[g][__ffsll((long long)m) - 1];
            }
        }
        if (fin) busy = false;
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
    const uint16_t *s_delta;
    const uint32_t *s_off, *s_C, *s_eol, *s_acc_off, *single_of_pid, *s_mid;
    const uint8_t *s_cls, *s_acc;
    unsigned long long *hits;
    uint32_t *hit_count;
    uint32_t cap;
    uint32_t n_singles, n_acc;  // automata count, total accept-table entries
};

constexpr int VF_PRE = 6;  // 16-B record chunks loaded before the walk (96 B: most banners)

// Walk automaton (D, cls, acc with C classes, eol column, anchored start states mid) over
// record [s, e): global tables, or the block's copy in LDS (the same code inlined with LDS
// pointers, so the lookups are ds_reads).
template <class DT, class CT, class AT>
__device__ __forceinline__ bool verify_walk(const uint8_t *__restrict__ buf, DT D, CT cls, AT acc, uint32_t C, uint32_t eol,
                                            uint32_t mid, uint32_t s, uint32_t e) {
    if (mid != 0xffffffffu) {
        // anchored DFA: a run from every start offset (most die on their first byte)
        bool hit = false;
        for (uint32_t p0 = s; p0 <= e && !hit; ++p0) {
            uint32_t st = 1;
            if (p0 > s) {
                const uint8_t pb = buf[p0 - 1];
                const bool pw = (pb >= '0' && pb <= '9') || ((pb | 0x20) >= 'a' && (pb | 0x20) <= 'z') || pb == '_';
                st = pw ? (mid >> 16) : (mid & 0xffffu);
            }
            hit = acc[st] != 0;
            for (uint32_t p = p0; p < e && !hit && st != 0; ++p) {
                st = D[st * C + cls[buf[p]]];
                hit = acc[st] != 0;
            }
            if (!hit && st != 0) hit = acc[D[st * C + eol]] != 0;
        }
        return hit;
    }
    uint32_t st = 1;
    bool hit = acc[st] != 0;
    auto walk16 = [&](uint32_t w, const uint4 &v) {
        const uint32_t xs[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (uint32_t b = 0; b < 16; ++b) {
            const uint32_t p = w + b;
            if (p < s || p >= e || hit || st == 0) continue;
            st = D[st * C + cls[(xs[b >> 2] >> (8 * (b & 3))) & 0xffu]];
            hit = acc[st] != 0;
        }
    };
    // the record's first VF_PRE 16-B chunks are loaded together before the walk: one line
    // fetch per record instead of a load per chunk spread over the walk, by which time the
    // line has left L2 (round 2 PMC: 6x over-fetch, 6 % L2 hits); the rest as the walk goes
    const uint32_t w0 = s & ~15u;
    uint4 pre[VF_PRE];
#pragma unroll
    for (int j = 0; j < VF_PRE; ++j)
        pre[j] = (w0 + 16u * j < e) ? *reinterpret_cast<const uint4 *>(buf + w0 + 16u * j) : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < VF_PRE; ++j)
        if (w0 + 16u * j < e && !hit && st != 0) walk16(w0 + 16u * j, pre[j]);
    // past them, four chunks' loads issued together per step (long records: JSON lines)
    for (uint32_t w = w0 + 16u * VF_PRE; w < e && !hit && st != 0; w += 64) {
        uint4 q[4];
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k)
            q[k] = (w + 16u * k < e) ? *reinterpret_cast<const uint4 *>(buf + w + 16u * k) : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k)
            if (w + 16u * k < e && !hit && st != 0) walk16(w + 16u * k, q[k]);
    }
    if (!hit && st != 0) hit = acc[D[st * C + eol]] != 0;
    return hit;
}

// Blocks are dispatched round-robin over the 8 XCDs (block b -> XCD b % 8), each with its own
// L2. Candidates are sorted by pattern, so giving XCD g the g-th contiguous eighth of them
// confines each XCD to ~1/8 of the verify automata: their rows stay in that XCD's L2 instead of
// every XCD streaming every automaton (MI355X_MICROARCH.md: XCD-aware block mapping).
__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t nb) {
    const uint32_t g = b & 7u, j = b >> 3, q = nb >> 3, r = nb & 7u;
    return g * q + (g < r ? g : r) + j;
}

// Candidates are sorted by pattern, so almost every block verifies one automaton: when the
// first and last candidate share it and it fits, the block copies that automaton (rows, byte classes, accept flags) into LDS once and
// every lane walks it there — the per-byte transitions were dependent L1/L2 loads.
// u16 transition entries staged per block. Round 6: 12,288 -> 6,144 (a block's LDS 28.7 ->
// 16.4 KB, 5 -> 8 blocks per CU, the wave limit): the walks are latency-bound and the waves
// hide more than the automata pushed to L2 walks cost (C4 re_verify 1.35 -> 1.22 ms, fields
// 3.63 -> 2.71 ms; 4,096 / 3,072 / 2,048 flat, 16,384 slower: profiles/r06/ab/ab10*, ab11*)
#ifndef SG_VF_D
#define SG_VF_D 6144
#endif
constexpr uint32_t VF_D = SG_VF_D;
constexpr uint32_t VF_ACC = 4096;  // accept flags staged per block

// A block whose candidates span two automata (its first and last candidate's: 18 % of C4's
// blocks, at the boundary between two patterns' runs) stages both when they fit together, so
// its threads do not walk an automaton from L2 one dependent transition after another.
__global__ __launch_bounds__(256) void k_verify(VerifyArgs a) {
    __shared__ uint16_t s_D[VF_D];
    __shared__ uint8_t s_cls[512];
    __shared__ uint8_t s_acc[VF_ACC];
    const uint32_t i0 = xcd_block(blockIdx.x, gridDim.x) * blockDim.x;
    const uint32_t i = i0 + threadIdx.x;
    const uint32_t il = min(i0 + blockDim.x, a.n_cand) - 1u;
    const uint32_t k0 = a.single_of_pid[(uint32_t)a.cand[i0]];
    const uint32_t kl = a.single_of_pid[(uint32_t)a.cand[il]];
    auto n_states = [&](uint32_t k) { return (k + 1u < a.n_singles ? a.s_acc_off[k + 1u] : a.n_acc) - a.s_acc_off[k]; };
    const uint32_t nst = n_states(k0), nd = nst * a.s_C[k0];
    const uint32_t nst2 = k0 != kl ? n_states(kl) : 0u, nd2 = k0 != kl ? nst2 * a.s_C[kl] : 0u;
    // block-uniform: the first automaton, and the last one too when both fit
    const bool staged = nd <= VF_D && nst <= VF_ACC;
    const bool staged2 = staged && k0 != kl && nd + nd2 <= VF_D && nst + nst2 <= VF_ACC;
    if (staged) {
        const uint16_t *D = a.s_delta + a.s_off[k0];
        for (uint32_t q = threadIdx.x; q < nd; q += blockDim.x) s_D[q] = D[q];
        const uint8_t *acc = a.s_acc + a.s_acc_off[k0];
        for (uint32_t q = threadIdx.x; q < nst; q += blockDim.x) s_acc[q] = acc[q];
        s_cls[threadIdx.x] = a.s_cls[256u * k0 + threadIdx.x];
        if (staged2) {
            const uint16_t *D2 = a.s_delta + a.s_off[kl];
            for (uint32_t q = threadIdx.x; q < nd2; q += blockDim.x) s_D[nd + q] = D2[q];
            const uint8_t *acc2 = a.s_acc + a.s_acc_off[kl];
            for (uint32_t q = threadIdx.x; q < nst2; q += blockDim.x) s_acc[nst + q] = acc2[q];
            s_cls[256u + threadIdx.x] = a.s_cls[256u * kl + threadIdx.x];
        }
        __syncthreads();
    }
    bool hit = false;
    unsigned long long cd = 0;
    if (i < a.n_cand) {
        cd = a.cand[i];
        const uint32_t r = (uint32_t)(cd >> 32), pid = (uint32_t)cd;
        const uint32_t k = a.single_of_pid[pid];
        const uint2 sp = a.spans[r];
        if (staged && k == k0) {  // pids of one automaton need not be contiguous
            hit = verify_walk(a.buf, s_D, s_cls, s_acc, a.s_C[k], a.s_eol[k], a.s_mid[k], sp.x, sp.y);
        } else if (staged2 && k == kl) {
            hit = verify_walk(a.buf, s_D + nd, s_cls + 256, s_acc + nst, a.s_C[k], a.s_eol[k], a.s_mid[k], sp.x, sp.y);
        } else {
            hit = verify_walk(a.buf, a.s_delta + a.s_off[k], a.s_cls + 256u * k, a.s_acc + a.s_acc_off[k], a.s_C[k],
                              a.s_eol[k], a.s_mid[k], sp.x, sp.y);
        }
    }
    // one global append per wave: ballot, lane 0 reserves, each hitting lane its slot
    const uint64_t m = __ballot(hit);
    if (!m) return;
    uint32_t base = 0;
    if (lane_id() == 0) base = atomicAdd(a.hit_count, (uint32_t)__popcll(m));
    base = (uint32_t)__shfl((int)base, 0, 64);
    if (hit) {
        const uint32_t slot_i = base + (uint32_t)__popcll(m & ((1ull << lane_id()) - 1ull));
        if (slot_i < a.cap) a.hits[slot_i] = cd;
    }
}

// ------------------------------------------------------------------ host driver
// The count pass's block-major counters read in bucket-major order (i = bucket * nblk + block).
struct HbCountT {
    const uint32_t *v;
    uint32_t nblk, nb;
    __device__ uint64_t operator()(uint32_t i) const { return v[(size_t)(i % nblk) * nb + i / nblk]; }
};

struct HitKeyPred {
    const unsigned long long *K;
    uint32_t n;
    __device__ uint32_t operator()(uint32_t i) const { return (i == 0 || K[i] != K[i - 1]) ? 1u : 0u; }
};
struct RecHeadPred {
    const unsigned long long *K;
    __device__ uint32_t operator()(uint32_t i) const { return (i == 0 || (K[i] >> 32) != (K[i - 1] >> 32)) ? 1u : 0u; }
};

// ------------------------------------------------------------------ hit sort by record buckets
// The (record << 32 | signature) hits come from the engines in arbitrary order (per-block
// flushes). Instead of an LSD radix sort over ~37 key bits (6 passes on C3's 33M hits), they
// are bucketed by record (HB_RB records per bucket): a count pass (per-block LDS histograms),
// a scan, a scatter pass (LDS ranks), then one block per bucket sorts its hits in LDS — a
// counting sort by record, then an insertion sort of each record's few signatures. A bucket
// over HB_CAP hits (one record holding thousands of hits) sets *err and the caller falls back
// to the radix sort of the original hits.
constexpr uint32_t HB_RBMAX = 12;     // log2 records per bucket, at most (LDS counters)
constexpr uint32_t HB_CAP = 6144;     // hits per bucket sorted in LDS
constexpr uint32_t HB_T = 1024;       // count/scatter/sort block
constexpr uint32_t HB_NBLK = 256;     // count/scatter blocks
constexpr uint32_t HB_NBMAX = 32768;  // buckets at most (their counters in one block's LDS)

__global__ __launch_bounds__(HB_T) void k_hb_count(const unsigned long long *__restrict__ hits, uint32_t n,
                                                    uint32_t nb, uint32_t rb, uint32_t *__restrict__ cnt) {
    extern __shared__ uint32_t s_h[];
    for (uint32_t x = threadIdx.x; x < nb; x += HB_T) s_h[x] = 0;
    __syncthreads();
    const uint32_t per = (n + gridDim.x - 1) / gridDim.x;
    const uint32_t a = blockIdx.x * per, e = min(n, a + per);
    for (uint32_t i = a + threadIdx.x; i < e; i += HB_T) atomicAdd(&s_h[(uint32_t)(hits[i] >> (32 + rb))], 1u);
    __syncthreads();
    // block-major (one contiguous row per block; the scan reads it bucket-major)
    for (uint32_t x = threadIdx.x; x < nb; x += HB_T) cnt[(size_t)blockIdx.x * nb + x] = s_h[x];
}

__global__ __launch_bounds__(HB_T) void k_hb_scatter(const unsigned long long *__restrict__ hits, uint32_t n,
                                                      uint32_t nb, uint32_t rb, const uint64_t *__restrict__ off,
                                                      unsigned long long *__restrict__ out) {
    extern __shared__ uint32_t s_h[];
    for (uint32_t x = threadIdx.x; x < nb; x += HB_T) s_h[x] = 0;
    __syncthreads();
    const uint32_t per = (n + gridDim.x - 1) / gridDim.x;
    const uint32_t a = blockIdx.x * per, e = min(n, a + per);
    for (uint32_t i = a + threadIdx.x; i < e; i += HB_T) {
        const unsigned long long k = hits[i];
        const uint32_t b = (uint32_t)(k >> (32 + rb));
        const uint32_t r = atomicAdd(&s_h[b], 1u);
        out[off[(size_t)b * gridDim.x + blockIdx.x] + r] = k;
    }
}

// One block per bucket: its hits (m <= HB_CAP) counting-sorted by record in LDS, each
// record's run insertion-sorted (by signature), written back in place.
__global__ __launch_bounds__(HB_T) void k_hb_sort(unsigned long long *__restrict__ keys, const uint64_t *__restrict__ off,
                                                   uint32_t nblk, uint32_t nb, uint32_t rb, uint32_t n,
                                                   uint32_t *__restrict__ err) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long s_k[];  // HB_CAP keys
    uint32_t *s_c = reinterpret_cast<uint32_t *>(s_k + HB_CAP);             // 2^rb counters
    __shared__ uint32_t s_red[HB_T / 64];
    constexpr uint32_t PER = (1u << HB_RBMAX) / HB_T;
    const uint32_t NR = 1u << rb;
    const uint32_t b = blockIdx.x, t = threadIdx.x;
    const uint64_t e0 = off[(size_t)b * nblk];
    const uint64_t e1 = (b + 1 < nb) ? off[(size_t)(b + 1) * nblk] : (uint64_t)n;
    const uint32_t m = (uint32_t)(e1 - e0);
    if (m > HB_CAP) {
        if (t == 0) *err = 1u;
        return;
    }
    if (m <= 1) return;
    for (uint32_t x = t; x < NR; x += HB_T) s_c[x] = 0;
    __syncthreads();
    for (uint32_t q = t; q < m; q += HB_T) atomicAdd(&s_c[(uint32_t)(keys[e0 + q] >> 32) & (NR - 1u)], 1u);
    __syncthreads();
    // exclusive scan of the NR counters: thread t owns counters PER*t .. PER*t + PER - 1
    uint32_t v[PER], sum = 0;
#pragma unroll
    for (uint32_t j = 0; j < PER; ++j) { v[j] = (PER * t + j < NR) ? s_c[PER * t + j] : 0u; sum += v[j]; }
    uint32_t tot;
    uint32_t run = block_excl_scan<HB_T>(sum, &tot, s_red);
#pragma unroll
    for (uint32_t j = 0; j < PER; ++j) { if (PER * t + j < NR) s_c[PER * t + j] = run; run += v[j]; }
    __syncthreads();
    for (uint32_t q = t; q < m; q += HB_T) {
        const unsigned long long k = keys[e0 + q];
        s_k[atomicAdd(&s_c[(uint32_t)(k >> 32) & (NR - 1u)], 1u)] = k;
    }
    __syncthreads();
    // s_c[r] = end of record r's run = start of r + 1. Each hit's place inside its record's
    // run is its rank there (hits ordered before it, ties by position), one thread per hit:
    // every thread works, where an insertion sort per record kept 2^rb of them busy (dense
    // hits, ~18 per record: the fields step's 73M-hit engine spent 1.6 ms here)
    for (uint32_t q = t; q < m; q += HB_T) {
        const unsigned long long k = s_k[q];
        const uint32_t r = (uint32_t)(k >> 32) & (NR - 1u);
        const uint32_t a = r ? s_c[r - 1] : 0u, e = s_c[r];
        uint32_t rank = a;
        for (uint32_t j = a; j < e; ++j) {
            const unsigned long long x = s_k[j];
            rank += (x < k || (x == k && j < q)) ? 1u : 0u;
        }
        keys[e0 + rank] = k;
    }
}

// Sorted hits: bit 0 = first of its (record, signature), bit 1 = first of its record.
struct HitHeadsPred {
    const unsigned long long *K;
    __device__ uint32_t operator()(uint32_t i) const {
        const unsigned long long k = K[i], p = i ? K[i - 1] : ~k;
        return (k != p ? 1u : 0u) | ((k >> 32) != (p >> 32) ? 2u : 0u);
    }
};

__global__ void k_split_hits(const unsigned long long *K, const uint32_t *idx, uint32_t n, uint32_t *rec, uint32_t *sig) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const unsigned long long k = K[idx[i]];
    rec[i] = (uint32_t)(k >> 32);
    sig[i] = (uint32_t)k;
}

// Matched records (input order) -> their spans and key0 from byte 0, and (block minimum, a
// guarded atomic per block) their common prefix with the first matched record — the dedup's
// common-prefix scan of these records, done while their first bytes are being read anyway.
// keysL (Ls >= 8, the context's last common prefix): also the keys at Ls and their KeyStatD
// partial per block (stL), for the records tying the first one on key0 (all of them when the
// common prefix comes out at Ls again).
// K0 / R7 (optional): every record's key0 and bytes 7..14 as the literal scan took them from
// its staged tiles: the matched records' keys and first prefix step come from them (16 B per
// record, in record order) instead of each record's first line (X1 gather 204 µs, 1.27 GB
// fetched for 10M httpx lines).
__global__ __launch_bounds__(256) void k_gather_matched(const uint8_t *__restrict__ buf, const uint2 *__restrict__ spans,
                                                        const uint32_t *__restrict__ mrec, uint32_t m, uint2 *__restrict__ sp,
                                                        uint64_t *__restrict__ keys, uint32_t *__restrict__ lcp_out,
                                                        uint64_t *__restrict__ keysL, uint32_t Ls, KeyStatD *__restrict__ stL,
                                                        const uint64_t *__restrict__ K0, const uint64_t *__restrict__ R7) {
    __shared__ uint32_t s_min[4];
    __shared__ KeyStatD s_st[4];
    KeyStatAcc accL;
    const uint32_t r0 = mrec[0];
    const uint2 r = spans[r0];
    const uint64_t kr = K0 ? K0[r0] : chunk_key(buf, r.x, r.y, 0);
    const uint64_t rr7 = R7 ? R7[r0] : 0ull;
    const uint32_t tr = (uint32_t)(kr & 0xffu);
    uint32_t best = 255;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) {
        const uint32_t ri = mrec[i];
        const uint2 x = spans[ri];
        sp[i] = x;
        const uint64_t k = K0 ? K0[ri] : chunk_key(buf, x.x, x.y, 0);
        const uint64_t x7 = R7 ? R7[ri] : 0ull;
        keys[i] = k;
        const uint64_t d0 = (k ^ kr) >> 8;
        const uint32_t tk = (uint32_t)(k & 0xffu);
        uint32_t l;
        if (d0) {
            l = min((uint32_t)__builtin_clzll(d0 << 8) >> 3, min(tk, tr));
        } else if (tk < 8u || tr < 8u) {
            l = min(tk, tr);
        } else {
            const uint32_t mm = min(min(x.y - x.x, r.y - r.x), best);
            l = 7;
            uint64_t raw7 = 0;  // bytes 7..14 when the first step loaded all 8
            bool have7 = false;
            while (l < mm) {
                const uint32_t t = (mm - l) < 8u ? (mm - l) : 8u;
                const uint64_t tm = t == 8u ? ~0ull : ((1ull << (8u * t)) - 1ull);
                const bool from7 = R7 && l == 7u;  // the first step from the scan's bytes 7..14
                const uint64_t xb = from7 ? (x7 & tm) : load_le(buf, x.x + l, t);
                if (l == 7u && t == 8u) { raw7 = xb; have7 = true; }
                const uint64_t d = xb ^ (from7 ? (rr7 & tm) : load_le(buf, r.x + l, t));
                if (d) { l += (uint32_t)__builtin_ctzll(d) >> 3; break; }
                l += t;
            }
            l = min(l, mm);
            if (keysL) {
                // at Ls = 8 the key's bytes 8..14 are the first step's load
                const uint32_t len = x.y - x.x, rem = len > Ls ? len - Ls : 0u, take = rem < 7u ? rem : 7u;
                const uint64_t kl = (Ls == 8u && have7)
                                        ? (rem ? ((__builtin_bswap64((raw7 >> 8) & ((1ull << (8u * take)) - 1ull)) & ~0xffull) |
                                                  (uint64_t)(rem < 8u ? rem : 8u))
                                               : 0ull)
                                        : chunk_key(buf, x.x, x.y, Ls);
                keysL[i] = kl;
                accL.add(kl);
            }
        }
        best = min(best, l);
    }
    if (stL) kstat_flush(accL, s_st, stL);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) best = min(best, (uint32_t)__shfl_xor((int)best, o, 64));
    if (lane_id() == 0) s_min[threadIdx.x >> 6] = best;
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t b = min(min(s_min[0], s_min[1]), min(s_min[2], s_min[3]));
        if (b < 255u && b < __hip_atomic_load(lcp_out, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMin(lcp_out, b);
    }
}

// The matched records' compaction and gather in one pass (X1): over the flag select's tiles
// (k_sel_count's ballots and the tile scan), each flagged record's span, key0 (K0) and bytes
// 7..14 (R7, both written by the literal scan) are read in record order and written at its
// position in the matched list, with the common-prefix scan of k_gather_matched: per block
// against the tile's first matched record (the set's common prefix is the minimum, over the
// set, of the prefix any one member shares with the others, so every block may use its own).
// Replaces select.apply + k_gather_matched (two dependent gathers through the record list).
struct MFlagPred {
    const uint8_t *f;
    __device__ uint32_t operator()(uint32_t i) const { return f[i] ? 1u : 0u; }
};
__global__ __launch_bounds__(SEL_BLOCK) void k_gather_flagged(uint32_t n, const uint64_t *__restrict__ mA,
                                                              const uint64_t *__restrict__ pre, const uint8_t *__restrict__ buf,
                                                              const uint2 *__restrict__ spans, const uint64_t *__restrict__ K0,
                                                              const uint64_t *__restrict__ R7, uint2 *__restrict__ sp,
                                                              uint64_t *__restrict__ keys, uint32_t *__restrict__ lcp_out,
                                                              uint64_t *__restrict__ keysL, uint32_t Ls,
                                                              KeyStatD *__restrict__ stL) {
    __shared__ uint32_t s_ca[SEL_MASKS];
    __shared__ uint64_t s_ma[SEL_MASKS];
    __shared__ uint32_t s_first;
    __shared__ uint32_t s_min[SEL_BLOCK / 64];
    __shared__ KeyStatD s_st[SEL_BLOCK / 64];
    const int t = threadIdx.x, lane = lane_id(), wid = t >> 6;
    const uint32_t base = blockIdx.x * SEL_TILE;
    const uint64_t *ma = mA + (uint64_t)blockIdx.x * SEL_MASKS;
    if (t < 64) {
        const uint64_t xa = ma[t];
        const uint32_t a = (uint32_t)__popcll(xa);
        s_ca[t] = wave_incl_scan(a) - a;
        s_ma[t] = xa;
        // the tile's first flagged item: mask t covers row t / 4, wave t % 4 (items base +
        // (t / 4) * 256 + (t % 4) * 64 + lane)
        const uint32_t f = xa ? (t >> 2) * SEL_BLOCK + (t & 3) * 64 + (uint32_t)(__ffsll((long long)xa) - 1) : 0xffffffffu;
        uint32_t m = f;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) m = min(m, (uint32_t)__shfl_xor((int)m, o, 64));
        if (t == 0) s_first = m;
    }
    __syncthreads();
    KeyStatAcc accL;
    uint32_t best = 255;
    if (s_first != 0xffffffffu) {
        const uint32_t ri = base + s_first;
        const uint2 r = spans[ri];
        const uint64_t kr = K0[ri], rr7 = R7[ri];
        const uint32_t tr = (uint32_t)(kr & 0xffu);
        const uint32_t preA = (uint32_t)(pre[blockIdx.x] >> 31);
        const uint64_t lt = (1ull << lane) - 1ull;
#pragma unroll 4
        for (int j = 0; j < SEL_ROWS; ++j) {
            const uint32_t i = base + j * SEL_BLOCK + t;
            const uint64_t xa = s_ma[j * 4 + wid];
            if (!((xa >> lane) & 1ull)) continue;
            const uint32_t pos = preA + s_ca[j * 4 + wid] + (uint32_t)__popcll(xa & lt);
            const uint2 x = spans[i];
            const uint64_t k = K0[i], x7 = R7[i];
            sp[pos] = x;
            keys[pos] = k;
            const uint64_t d0 = (k ^ kr) >> 8;
            const uint32_t tk = (uint32_t)(k & 0xffu);
            uint32_t l;
            if (d0) {
                l = min((uint32_t)__builtin_clzll(d0 << 8) >> 3, min(tk, tr));
            } else if (tk < 8u || tr < 8u) {
                l = min(tk, tr);
            } else {
                const uint32_t mm = min(min(x.y - x.x, r.y - r.x), best);
                l = 7;
                uint64_t raw7 = 0;
                bool have7 = false;
                while (l < mm) {
                    const uint32_t tt = (mm - l) < 8u ? (mm - l) : 8u;
                    const uint64_t tm = tt == 8u ? ~0ull : ((1ull << (8u * tt)) - 1ull);
                    const bool from7 = l == 7u;
                    const uint64_t xb = from7 ? (x7 & tm) : load_le(buf, x.x + l, tt);
                    if (from7 && tt == 8u) { raw7 = xb; have7 = true; }
                    const uint64_t d = xb ^ (from7 ? (rr7 & tm) : load_le(buf, r.x + l, tt));
                    if (d) { l += (uint32_t)__builtin_ctzll(d) >> 3; break; }
                    l += tt;
                }
                l = min(l, mm);
                if (keysL) {
                    const uint32_t len = x.y - x.x, rem = len > Ls ? len - Ls : 0u, take = rem < 7u ? rem : 7u;
                    uint64_t kl;
                    if (Ls == 8u && (have7 || len >= 15u)) {
                        const uint64_t b8 = have7 ? raw7 : x7;  // bytes 7..14: the key's are 8..14
                        kl = rem ? ((__builtin_bswap64((b8 >> 8) & ((1ull << (8u * take)) - 1ull)) & ~0xffull) |
                                    (uint64_t)(rem < 8u ? rem : 8u))
                                 : 0ull;
                    } else {
                        kl = chunk_key(buf, x.x, x.y, Ls);
                    }
                    keysL[pos] = kl;
                    accL.add(kl);
                }
            }
            best = min(best, l);
        }
    }
    if (stL) kstat_flush(accL, s_st, stL);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) best = min(best, (uint32_t)__shfl_xor((int)best, o, 64));
    if (lane == 0) s_min[wid] = best;
    __syncthreads();
    if (t == 0) {
        const uint32_t b = min(min(s_min[0], s_min[1]), min(s_min[2], s_min[3]));
        if (b < 255u && b < __hip_atomic_load(lcp_out, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMin(lcp_out, b);
    }
}

__global__ void k_rec_of(const unsigned long long *K, const uint32_t *idx, uint32_t n, uint32_t *rec) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) rec[i] = (uint32_t)(K[idx[i]] >> 32);
}

template <class Pred>
static int select_one(sg_ctx *c, const char *name, Pred pred, uint32_t n, uint32_t *out, uint32_t *count) {
    return run_select2(c, name, pred, n, out, (uint32_t *)nullptr, count, nullptr);
}

int dev_match(sg_ctx *c, sg_matcher *h, const uint8_t *d_buf, uint64_t n, sg_dev_hits *res, bool want_lines,
              MatchFlags *mf, Lines *reuse) {
    if (mf && !(h->lit.on && h->tables.empty() && !h->has_pre)) {
        set_error("dev_match: record flags need a literal-filter matcher");
        return SG_E_INVAL;
    }
    *res = sg_dev_hits{};
    SG_TRY(ensure_device(h, c->device));
    Lines L;
    // reuse: the parse of this same buffer by an earlier call (several engines over one input:
    // the template evaluation), its spans and tile prefixes still in the context's CUR slots;
    // filled with this call's parse otherwise
    const bool reused = reuse && reuse->spans && reuse->tile_excl;
    // When a literal scan runs first (literal filter or regex prefilter), it writes the
    // record spans itself from the same tiles, so the parse's second pass is skipped.
    const bool fuse_spans = !reused && (h->has_pre || h->lit.on);
    const char *span_writer = h->has_pre ? "re_prefilter" : "lit_match";
    if (reused) L = *reuse;
    else SG_TRY(run_lines(c, d_buf, n, CUR_SLOTS, &L, false, !fuse_spans));
    if (reuse && !reused) *reuse = L;  // (the spans are complete once this call's kernels have run)
    const uint32_t R = L.n_rec;
    res->in_records = R;
    uint32_t *cnt;
    SG_TRY(slot(c, S_M_CNT, 8, &cnt));
    // hit capacity: remembered from earlier calls through the slot size (no relaunch in
    // steady state), at least R / 4
    uint64_t cap = std::max<uint64_t>(1u << 20, (uint64_t)R / 4);
    cap = std::min<uint64_t>(std::max<uint64_t>(cap, slot_elems<uint64_t>(c, S_M_HITS)), 0xfffff000ull);
    uint32_t total = 0;
    unsigned long long *hits = nullptr;
    auto geometry = [&](const sg_matcher::Table &T, const sg_matcher::DevTable &D, uint32_t *bits_in_lds,
                        uint32_t *lds, uint32_t *grid) {
        const uint32_t nbits = (T.n_states + 31) / 32;
        *bits_in_lds = nbits * 4 <= AC_BITS_BYTES ? 1u : 0u;
        *lds = 256 + ((D.H * T.n_classes * 2 + 15) & ~15u) + (*bits_in_lds ? nbits * 4 : 0);
        *grid = std::min<uint32_t>((R + 511) / 512, 256u * 8u);
    };
    // prefilter candidates (regex plans): factor filter -> (record, pattern) pairs
    unsigned long long *cand = nullptr;
    uint32_t n_cand = 0;
    // trial_tiles > 0: a timing run over the first tiles only, every output dropped (no spans,
    // flags or hits: capacity 0)
    auto run_lit = [&](const char *name, const sg_matcher::Lit &Lt, unsigned long long *out, uint32_t *counter,
                       uint32_t ocap, const uint32_t *fo, const uint32_t *fp, uint32_t trial_tiles = 0) -> int {
        LitArgs a{};
        a.buf = d_buf; a.n = n; a.tile_excl = L.tile_excl; a.n_tiles = trial_tiles ? trial_tiles : L.n_tiles;
        a.bitmap = Lt.d_bitmap; a.rank = Lt.d_rank; a.eoff = Lt.d_eoff; a.efp = Lt.d_efp;
        a.brec = reinterpret_cast<const uint4 *>(Lt.d_brec);
        a.einfo = reinterpret_cast<const uint4 *>(Lt.d_einfo); a.pat16 = reinterpret_cast<const uint4 *>(Lt.d_pat16);
        a.bm_words = (uint32_t)Lt.bitmap.size(); a.n_bk = (uint32_t)Lt.eoff.size() - 1;
        a.n_ent = (uint32_t)Lt.efp.size(); a.cls_mask = Lt.cls_mask; a.nocase = Lt.nocase ? 1u : 0u;
        for (uint32_t k = 0; k < LIT_CLASSES; ++k) {
            a.bits[k] = Lt.bits[k]; a.bm_off[k] = Lt.bm_off[k]; a.rank_base[k] = Lt.rank_base[k];
        }
        a.hits = out; a.hit_count = counter; a.cap = ocap; a.fac_off = fo; a.fac_pids = fp;
        a.spans_out = (!trial_tiles && fuse_spans && strcmp(name, span_writer) == 0) ? L.spans : nullptr;
        a.rec_flag = (mf && !trial_tiles) ? mf->flags : nullptr;
        a.keys_out = (a.rec_flag && a.spans_out) ? mf->key0 : nullptr;
        a.raw7_out = a.keys_out ? mf->raw7 : nullptr;
        const uint32_t stat = L.tile_bytes + 2 * LS_HALO + LS_HB * 8 + LS_Q * 12 + 64;
        auto blocks_per_cu = [&](uint32_t dyn) {
            return std::max<uint32_t>(1u, std::min<uint32_t>(8u, (160u * 1024u) / (dyn + stat)));
        };
        // the shared-bucket pair queue (LS_MW entries of 16 B after the tables) when the filter
        // has shared buckets: it decides with the tables whether the ranks fit too (a static
        // queue in every filter's scan took X1's lit_match from 1.02 to 1.28-1.31 ms; C4's
        // prefilter, 847 shared buckets, runs 3.67 -> 2.57 ms with it)
        const uint32_t qb = Lt.n_shared ? LS_MW * 16u + 16u : 0u;
        const uint32_t dyn_r = lit_lds_bytes(Lt, true) + qb, dyn_n = lit_lds_bytes(Lt, false) + qb;
        a.rank_lds = blocks_per_cu(dyn_r) == blocks_per_cu(dyn_n) ? 1u : 0u;
        a.mw_cap = Lt.n_shared ? LS_MW : 0u;
        a.diag = nullptr;
        unsigned long long *diag = nullptr;
        if (sw_lit_trial_log() && !trial_tiles) {
            SG_TRY(slot(c, S_M_TMP2, 8, &diag));
            SG_HIP(hipMemsetAsync(diag, 0, 64, c->stream));
            a.diag = diag;
        }
        const uint32_t dyn = a.rank_lds ? dyn_r : dyn_n;
        const uint32_t bpc = blocks_per_cu(dyn);
        const uint32_t grid = std::min<uint32_t>(a.n_tiles, 256u * bpc);
        // Block size: when the tables leave room for only <= 2 blocks per CU (large factor
        // sets: the regex prefilter), 512-thread blocks double the waves that hide the
        // candidate stage's L2 latency (C4 prefilter 2.71 -> 1.84 ms per 4M banners); with
        // room for 3+ blocks, 256 threads x 64 positions probe faster (C3 1.35 vs 1.54 ms).
        const int ls_block = bpc <= 2 ? 512 : 256;
        if (sw_lit_trial_log() && !trial_tiles)
            fprintf(stderr, "sg %s: %u shared buckets, pair queue %u, ranks in LDS %u, %u B LDS + %u static, %u blocks/CU of %d\n",
                    name, Lt.n_shared, a.mw_cap, a.rank_lds, dyn, stat, bpc, ls_block);
        const int bpt = (int)(L.tile_bytes / ls_block);
        const double bytes = (double)n + 8.0 * R;
        auto launch = [&](auto kern, int blk) -> int {
            SG_HIP(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn));
            if (trial_tiles) hipLaunchKernelGGL(kern, dim3(grid), dim3(blk), dyn, c->stream, a);
            else SG_LAUNCH_B(c, name, bytes, kern, grid, blk, dyn, a);
            SG_HIP(hipGetLastError());
            return SG_OK;
        };
        // (block, positions per thread) pairs of one parse tile; the template picks the
        // class scheme and the length classes probed per position
        auto by_tmpl = [&](auto k18, auto k1c, auto k1f, auto k20, auto k24, auto k27, int blk) -> int {
            switch (Lt.tmpl) {
                case 0x18u: return launch(k18, blk);
                case 0x1Cu: return launch(k1c, blk);
                case 0x1Fu: return launch(k1f, blk);
                case 0x20u: return launch(k20, blk);
                case 0x24u: return launch(k24, blk);
                default: return launch(k27, blk);
            }
        };
#define SG_LIT_KERNELS(K, B, P) K<B, P, 0x18u>, K<B, P, 0x1Cu>, K<B, P, 0x1Fu>, K<B, P, 0x20u>, K<B, P, 0x24u>, \
                                K<B, P, 0x27u>
#define SG_LIT_GEOMS(K)                                                                             \
        if (ls_block == 512 && bpt == 16) SG_TRY(by_tmpl(SG_LIT_KERNELS(K, 512, 16), 512));         \
        else if (ls_block == 512 && bpt == 32) SG_TRY(by_tmpl(SG_LIT_KERNELS(K, 512, 32), 512));    \
        else if (ls_block == 256 && bpt == 32) SG_TRY(by_tmpl(SG_LIT_KERNELS(K, 256, 32), 256));    \
        else if (ls_block == 256 && bpt == 64) SG_TRY(by_tmpl(SG_LIT_KERNELS(K, 256, 64), 256));    \
        else { set_error("k_lit_scan: unsupported tile geometry"); return SG_E_INVAL; }
        if (trial_tiles) { SG_LIT_GEOMS(k_lit_trial) } else { SG_LIT_GEOMS(k_lit_scan) }
#undef SG_LIT_GEOMS
#undef SG_LIT_KERNELS
        if (diag) {
            unsigned long long dv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            SG_TRY(ctx_readback(c, dv, diag, 64));
            fprintf(stderr, "sg %s: %u records, %llu bitmap candidates, %llu fingerprint-confirmed, %llu verified "
                            "(first bucket entries; tmpl 0x%x, %s scheme); %llu candidates in shared buckets, "
                            "%llu further entries walked, %llu fingerprint-equal\n",
                    name, R, dv[0], dv[1], dv[2], Lt.tmpl, Lt.joint ? "joint" : "two", dv[3], dv[4], dv[5]);
            uint32_t nb = (uint32_t)Lt.eoff.size() - 1, multi = 0, mx = 0, in_multi = 0;
            for (uint32_t k = 0; k < nb; ++k) {
                const uint32_t e = Lt.eoff[k + 1] - Lt.eoff[k];
                if (e > 1) { ++multi; in_multi += e; }
                mx = std::max(mx, e);
            }
            fprintf(stderr, "sg %s: %u buckets, %u shared (%u entries), largest %u entries\n", name, nb, multi, in_multi, mx);
        }
        return SG_OK;
    };
    // The class scheme of a filter (two-class or joint, see build_lit): decided once per
    // matcher, on the first input large enough to tell (until then the two-class scheme runs):
    // both schemes scan the first tiles (k_lit_trial, outputs dropped), three times each after
    // a warm-up, and the joint scheme is kept only if its best time beats the two-class one's
    // by LIT_MARGIN — so near-ties always resolve to the two-class scheme, and a choice never
    // flips between runs on the measured inputs (C3/X1: joint 20-30 % faster; C4 banners and
    // the fields JSON: joint 1.9-2.2x slower, although it passes FEWER candidates there: the
    // candidate count does not predict the cost). SG_LIT_SCHEME=0/1 forces one.
    auto scheme = [&](const sg_matcher::Lit &two, const sg_matcher::Lit &joint, std::atomic<int> &mode,
                      const uint32_t *fo, const uint32_t *fp) -> const sg_matcher::Lit & {
        const int forced = sw_lit_scheme();
        if (forced >= 0) return forced ? joint : two;
        int m = mode.load();
        constexpr uint32_t TRIAL_TILES = 2048, MIN_TILES = 1024;
        if (m < 0 && L.n_tiles >= MIN_TILES) {
            const uint32_t tt = std::min<uint32_t>(L.n_tiles, TRIAL_TILES);
            hipEvent_t ev[2];
            for (auto &e : ev) (void)hipEventCreate(&e);
            float best[2] = {1e30f, 1e30f};
            bool ok = true;
            for (int rep = 0; rep < 4 && ok; ++rep) {  // rep 0 warms caches and code
                for (int sch = 0; sch < 2 && ok; ++sch) {
                    (void)hipEventRecord(ev[0], c->stream);
                    ok = run_lit("lit_trial", sch ? joint : two, nullptr, cnt + 4, 0u, fo, fp, tt) == SG_OK;
                    (void)hipEventRecord(ev[1], c->stream);
                    ok = ok && hipEventSynchronize(ev[1]) == hipSuccess;
                    float ms = 0.f;
                    if (ok && rep > 0 && hipEventElapsedTime(&ms, ev[0], ev[1]) == hipSuccess) best[sch] = std::min(best[sch], ms);
                }
            }
            for (auto &e : ev) (void)hipEventDestroy(e);
            if (ok) {
                m = best[1] < LIT_MARGIN * best[0] ? 1 : 0;
                mode.store(m);
                if (sw_lit_trial_log())
                    fprintf(stderr, "sg lit scheme: trial %u tiles, best two %.3f ms joint %.3f ms -> %s (tables: two %u B, joint %u B of LDS)\n",
                            tt, best[0], best[1], m ? "joint" : "two", lit_lds_bytes(two), lit_lds_bytes(joint));
            }
        }
        return m == 1 ? joint : two;
    };
    if (h->has_pre && R) {
        uint64_t ccap = std::min<uint64_t>(std::max<uint64_t>(std::max<uint64_t>(1u << 20, (uint64_t)R), slot_elems<uint64_t>(c, S_PART)),
                                           0xfffff000ull);
        for (int attempt = 0; attempt < 2; ++attempt) {
            SG_TRY(slot(c, S_PART, ccap, &cand));
            SG_HIP(hipMemsetAsync(cnt + 1, 0, 4, c->stream));
            SG_TRY(run_lit("re_prefilter", scheme(h->prelit, h->prelit_j, h->prelit_mode, h->dplan.fac_off, h->dplan.fac_pids),
                           cand, cnt + 1, (uint32_t)ccap, h->dplan.fac_off, h->dplan.fac_pids));
            SG_TRY(ctx_readback(c, &n_cand, cnt + 1, 4));
            if (n_cand <= ccap) break;
            ccap = std::min<uint64_t>((uint64_t)n_cand + (n_cand >> 3) + 1024, 0xfffff000ull);
        }
        cap = std::max<uint64_t>(cap, (uint64_t)n_cand + 1024);
    }
    // Verify candidates grouped by pattern (stable sort on the pattern bits): the lanes of
    // a wave then walk the same DFA, so its rows are shared in L1/L2 instead of every lane
    // pulling a different automaton's rows from HBM.
    const unsigned long long *vcand = cand;
    if (n_cand > 4096) {
        int pbits = 1;
        while (pbits < 32 && (1u << pbits) < h->n_pats) ++pbits;
        uint64_t *alt, *KC;
        uint32_t *w1, *w2, *WV;
        SG_TRY(slot(c, S_M_TMP, (size_t)n_cand + 1, &alt));
        SG_TRY(slot(c, S_R_VAL, (size_t)n_cand + 1, &w1));
        SG_TRY(slot(c, S_R_VAL2, (size_t)n_cand + 1, &w2));
        SG_TRY(radix_sort(c, reinterpret_cast<uint64_t *>(cand), w1, alt, w2, n_cand, 0, pbits, true, &KC, &WV, "rs_cand"));
        vcand = reinterpret_cast<const unsigned long long *>(KC);
        if (sw_lit_trial_log()) {
            // calibration: the verify's shape (candidates per record and per automaton, blocks
            // that can stage their automaton in LDS)
            std::vector<unsigned long long> hc(n_cand);
            SG_HIP(hipMemcpyAsync(hc.data(), vcand, 8ull * n_cand, hipMemcpyDeviceToHost, c->stream));
            SG_HIP(hipStreamSynchronize(c->stream));
            std::vector<uint32_t> per_rec(R, 0);
            for (auto x : hc) ++per_rec[(uint32_t)(x >> 32)];
            uint32_t recs_with = 0, maxc = 0;
            for (uint32_t v : per_rec) { recs_with += v ? 1u : 0u; maxc = std::max(maxc, v); }
            uint32_t blocks = 0, single = 0, stageable = 0, autos = 0, big_autos = 0;
            for (uint32_t k = 0; k < h->n_singles; ++k) {
                const uint32_t nst = (k + 1u < h->n_singles ? h->s_acc_off[k + 1u] : (uint32_t)h->s_acc.size()) - h->s_acc_off[k];
                ++autos;
                if (nst * h->s_C[k] > 12288u || nst > 4096u) ++big_autos;
            }
            for (uint32_t i0 = 0; i0 < n_cand; i0 += 256) {
                const uint32_t il = std::min(i0 + 256u, n_cand) - 1u;
                const uint32_t k0 = h->single_of_pid[(uint32_t)hc[i0]], kl = h->single_of_pid[(uint32_t)hc[il]];
                ++blocks;
                if (k0 == kl) {
                    ++single;
                    const uint32_t nst = (k0 + 1u < h->n_singles ? h->s_acc_off[k0 + 1u] : (uint32_t)h->s_acc.size()) -
                                         h->s_acc_off[k0];
                    if (nst * h->s_C[k0] <= 12288u && nst <= 4096u) ++stageable;
                }
            }
            fprintf(stderr, "sg verify: %u candidates over %u records (%u with any, max %u per record); %u verify "
                            "automata (%u too big for LDS); %u blocks, %u on one automaton, %u staged\n",
                    n_cand, R, recs_with, maxc, autos, big_autos, blocks, single, stageable);
        }
    }
    if (mf) {
        SG_TRY(slot(c, S_M_FLAG, (size_t)R + 16, &mf->flags));
        SG_HIP(hipMemsetAsync(mf->flags, 0, (size_t)R + 16, c->stream));
        if (fuse_spans) {  // (the scan writes the spans, so it also takes the keys there)
            SG_TRY(slot(c, S_M_K0, (size_t)R + 1, &mf->key0));
            SG_TRY(slot(c, S_M_R7, (size_t)R + 1, &mf->raw7));
        }
        if (R) SG_TRY(run_lit("lit_match", scheme(h->lit, h->lit_j, h->lit_mode, nullptr, nullptr), nullptr, cnt, 0u, nullptr, nullptr));
        mf->L = L;
        return SG_OK;
    }
    for (int attempt = 0; attempt < 2; ++attempt) {
        SG_TRY(slot(c, S_M_HITS, cap, &hits));
        SG_HIP(hipMemsetAsync(cnt, 0, 4, c->stream));
        if (R && h->lit.on)
            SG_TRY(run_lit("lit_match", scheme(h->lit, h->lit_j, h->lit_mode, nullptr, nullptr), hits, cnt, (uint32_t)cap, nullptr,
                           nullptr));
        if (R) {
            const bool multi = sw_dfa_multi();
            if (multi) {
                for (const auto &k : h->packs) {
                    DFAMultiArgs a{};
                    a.buf = d_buf; a.spans = L.spans; a.R = R; a.cls4 = k.d_cls4; a.hot = k.d_hot; a.hot_n = k.hot_n;
                    for (uint32_t g = 0; g < k.G; ++g) {
                        const auto &T = h->tables[k.tab[g]];
                        const auto &D = h->dtabs[k.tab[g]];
                        a.off[g] = k.off[g]; a.C[g] = T.n_classes; a.eol[g] = T.anchored_eol; a.init[g] = k.init[g];
                        a.omask[g] = reinterpret_cast<const unsigned long long *>(D.omask);
                        a.gpids[g] = D.gpids;
                    }
                    a.hits = hits; a.hit_count = cnt; a.cap = (uint32_t)cap;
                    const uint32_t lds = 1024 + k.hot_n * 2;
                    const uint32_t per_cu = std::max<uint32_t>(1u, 163840u / (lds + 128));
                    const uint32_t grid = std::min<uint32_t>((R + DFM_BLOCK - 1) / DFM_BLOCK, 256u * per_cu);
                    // 64-byte steps for long records (mean >= 128 B: JSON lines), else 16-byte
                    const bool wide = n >= 128ull * R;
#define SG_DFM_LAUNCH(G_)                                                                                   \
    do {                                                                                                    \
        if (wide) SG_LAUNCH_B(c, "dfa_match", (double)n + 8.0 * R, (k_dfa_multi<G_, 4>), grid, DFM_BLOCK, lds, a); \
        else SG_LAUNCH_B(c, "dfa_match", (double)n + 8.0 * R, (k_dfa_multi<G_, 1>), grid, DFM_BLOCK, lds, a);      \
    } while (0)
                    switch (k.G) {
                        case 1: SG_DFM_LAUNCH(1); break;
                        case 2: SG_DFM_LAUNCH(2); break;
                        case 3: SG_DFM_LAUNCH(3); break;
                        default: SG_DFM_LAUNCH(4); break;
                    }
#undef SG_DFM_LAUNCH
                }
            }
            for (size_t ti = 0; ti < h->tables.size(); ++ti) {
                if (multi && h->packed[ti]) continue;
                const auto &T = h->tables[ti];
                const auto &D = h->dtabs[ti];
                uint32_t bits_in_lds, lds, grid;
                geometry(T, D, &bits_in_lds, &lds, &grid);
                if (h->kind == 0) {
                    ACArgs a{d_buf, L.spans, R, D.cls, D.delta, D.hot, T.n_classes, D.H, T.n_states,
                             D.outbits, D.own_off, D.own_ids, D.dict, hits, cnt, (uint32_t)cap, bits_in_lds,
                             nullptr, nullptr};
                    if (n >= 128ull * R) SG_LAUNCH_B(c, "ac_match", (double)n + 8.0 * R, k_ac_match<true>, grid, 512, lds, a);
                    else SG_LAUNCH_B(c, "ac_match", (double)n + 8.0 * R, k_ac_match<false>, grid, 512, lds, a);
                } else {
                    DFAArgs a{d_buf, L.spans, R, D.cls, D.delta, D.hot, T.n_classes, D.H, T.n_states,
                              T.anchored_eol, D.outbits, reinterpret_cast<const unsigned long long *>(D.omask), D.gpids,
                              hits, cnt, (uint32_t)cap, bits_in_lds};
                    SG_LAUNCH_B(c, "dfa_match", (double)n + 8.0 * R, k_dfa_match, grid, DFA_BLOCK, lds, a);
                }
            }
            if (n_cand) {
                const auto &p = h->dplan;
                VerifyArgs v{d_buf, L.spans, vcand, n_cand, p.s_delta, p.s_off, p.s_C, p.s_eol,
                             p.s_acc_off, p.single_of_pid, p.s_mid, p.s_cls, p.s_acc, hits, cnt, (uint32_t)cap,
                             h->n_singles, (uint32_t)h->s_acc.size()};
                SG_LAUNCH_B(c, "re_verify", n_cand * (16.0 + (double)n / R), k_verify, (n_cand + 255) / 256, 256, 0, v);
            }
        }
        SG_TRY(ctx_readback(c, &total, cnt, 4));
        if (total <= cap) break;
        cap = std::min<uint64_t>((uint64_t)total + (total >> 3) + 1024, 0xfffff000ull);
    }
    // sort (rec << 32 | sig): record buckets sorted in LDS (the radix sort when a bucket
    // overflows, or with SG_HIT_RADIX=1)
    const unsigned long long *KK = hits;
    bool sorted = false;
    // bucket width: 4096 records, narrower when the hits are dense (about HB_CAP / 2 per bucket)
    uint32_t rb = HB_RBMAX;
    while (rb > 4 && (double)total * (1u << rb) / std::max<uint32_t>(R, 1u) > HB_CAP / 2) --rb;
    const uint32_t nb = (uint32_t)(((uint64_t)R + (1u << rb) - 1) >> rb);
    // (up to 32,768 buckets: the count and scatter blocks' LDS counters then take up to 128 KB,
    // one block per CU; the fields step's dense engine, 73M hits over 4M records, needs 31,250
    // buckets and went through a 5-pass radix sort of its hits: 2.9 ms)
    if (total > 1 && !sw_hit_radix() && nb <= HB_NBMAX) {
        const uint32_t nblk = std::max<uint32_t>(1u, std::min<uint32_t>(HB_NBLK, (total + 4095) / 4096));
        if (nb * 4u > 65536u) {
            SG_HIP(hipFuncSetAttribute((const void *)k_hb_count, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(nb * 4u)));
            SG_HIP(hipFuncSetAttribute((const void *)k_hb_scatter, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(nb * 4u)));
        }
        const size_t nc = (size_t)nb * nblk;
        uint32_t *hcnt, *herr;
        uint64_t *hoff;
        unsigned long long *hout;
        SG_TRY(slot(c, S_HB_CNT, nc, &hcnt));
        SG_TRY(slot(c, S_HB_OFF, nc, &hoff));
        SG_TRY(slot(c, S_HB_OUT, (size_t)total + 1, &hout));
        SG_TRY(slot(c, S_HB_ERR, 1, &herr));
        SG_HIP(hipMemsetAsync(herr, 0, 4, c->stream));
        SG_LAUNCH_B(c, "hit_count", 8.0 * total, k_hb_count, nblk, HB_T, nb * 4, hits, total, nb, rb, hcnt);
        const uint32_t nt = (uint32_t)((nc + SCAN_TILE - 1) / SCAN_TILE);
        uint64_t *tp;
        SG_TRY(slot(c, S_TILES, 2 * (size_t)nt + 4, &tp));
        SG_LAUNCH(c, "scan.count", k_scan64_count<HbCountT>, nt, SCAN_BLOCK, 0, HbCountT{hcnt, nblk, nb}, (uint32_t)nc, tp);
        SG_TRY(tile_scan(c, tp, nt, tp + nt, tp + 2 * (size_t)nt));
        SG_LAUNCH(c, "scan.apply", k_scan64_apply<HbCountT>, nt, SCAN_BLOCK, 0, HbCountT{hcnt, nblk, nb}, (uint32_t)nc, tp + nt, hoff);
        SG_LAUNCH_B(c, "hit_scatter", 16.0 * total, k_hb_scatter, nblk, HB_T, nb * 4, hits, total, nb, rb, hoff, hout);
        const uint32_t lds = HB_CAP * 8 + (4u << HB_RBMAX);
        SG_HIP(hipFuncSetAttribute((const void *)k_hb_sort, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        SG_LAUNCH_B(c, "hit_sort", 16.0 * total, k_hb_sort, nb, HB_T, lds, hout, hoff, nblk, nb, rb, total, herr);
        uint32_t ev = 0;
        SG_TRY(ctx_readback(c, &ev, herr, 4));
        if (!ev) {
            KK = hout;
            sorted = true;
        }
    }
    if (sw_lit_trial_log())
        fprintf(stderr, "sg hit sort: %u hits over %u records, rb %u, %u buckets: %s\n", total, R, rb, nb,
                sorted ? "bucket sort" : "radix sort");
    if (!sorted) {
        uint64_t *k2;
        uint32_t *v1, *v2;
        SG_TRY(slot(c, S_R_KEY2, (size_t)total + 1, &k2));
        SG_TRY(slot(c, S_R_VAL, (size_t)total + 1, &v1));
        SG_TRY(slot(c, S_R_VAL2, (size_t)total + 1, &v2));
        int rbits = 1;
        while (rbits < 32 && (1u << rbits) < R) ++rbits;
        uint64_t *K;
        uint32_t *V;
        SG_TRY(radix_sort(c, reinterpret_cast<uint64_t *>(hits), v1, k2, v2, total, 0, 32 + rbits, true, &K, &V,
                          "rs_pass_hits"));
        KK = reinterpret_cast<const unsigned long long *>(K);
    }
    // unique hits and matched records in one selection (one host sync for both counts)
    uint32_t *sel, *sel2;
    SG_TRY(slot(c, S_SEL, (size_t)total + 16, &sel));
    SG_TRY(slot(c, S_HB_SEL2, (size_t)total + 16, &sel2));
    uint32_t H = 0, M = 0;
    SG_TRY(run_select2(c, "hits_heads", HitHeadsPred{KK}, total, sel, sel2, &H, &M));
    uint32_t *rec, *sig;
    SG_TRY(slot(c, S_M_SIG, (size_t)H + 1, &sig));
    SG_TRY(slot(c, S_R_GID, (size_t)H + 1, &rec));
    if (H) SG_LAUNCH(c, "split_hits", k_split_hits, (H + 255) / 256, 256, 0, KK, sel, H, rec, sig);
    res->rec_idx = rec;
    res->sig_id = sig;
    res->n_hits = H;
    if (!want_lines) return SG_OK;
    // matched records (input order) -> grep output
    sel = sel2;
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
    if ((uint64_t)T.n_states * T.n_classes * 2 > AC_HOT_BYTES || sw_force_litfilter()) {
        // 128 bitmap bits per pattern: X1 candidates 37M -> 17M per 10M lines for 2 blocks/CU
        rc = build_lit(pats, pat_offs, n_pats, flags, &m->lit, 1u, false);
        if (rc == SG_OK) rc = build_lit(pats, pat_offs, n_pats, flags, &m->lit_j, 1u, true);
        if (rc == SG_E_UNSUPPORTED) {
            m->lit = sg_matcher::Lit{};  // too many patterns of one length class: keep the automaton
        } else if (rc != SG_OK) {
            delete m;
            return rc;
        } else {
            m->tables.clear();
        }
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
        // 128 bitmap bits per factor, as for literal sets (64: C4 prefilter 2.57 ms, fields'
        // 2.92; 128: 2.36 and 2.76; 256: 2.33 and 3.54, the fields table outgrowing its blocks)
        rc = build_lit(blob.data(), offs.data(), (uint32_t)plan.factors.size(), SG_NOCASE, &m->prelit, 1u, false);
        if (rc == SG_OK)
            rc = build_lit(blob.data(), offs.data(), (uint32_t)plan.factors.size(), SG_NOCASE, &m->prelit_j, 1u, true);
        if (rc != SG_OK) { delete m; return rc; }
        m->has_pre = true;
        m->fac_off = plan.fac_off;
        m->fac_pids = plan.fac_pids;
        m->single_of_pid = plan.single_of_pid;
        for (auto &d : plan.singles) {
            m->s_off.push_back((uint32_t)m->s_delta.size());
            m->s_C.push_back(d.n_classes);
            m->s_eol.push_back(d.eol_class);
            m->s_mid.push_back(d.anchored ? (d.mid_start[0] | (d.mid_start[1] << 16)) : 0xffffffffu);
            if (d.n_states > 65536) { delete m; set_error("regex signature DFA exceeds 65536 states"); return SG_E_STATES; }
            for (uint32_t x : d.delta) m->s_delta.push_back((uint16_t)x);
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
        // group-local pattern numbering for the per-thread accept mask
        std::map<uint32_t, uint32_t> local;
        for (uint32_t id : T.own_ids) local.emplace(id, 0u);
        if (local.size() > 64) { delete m; set_error("regex group holds more than 64 patterns"); return SG_E_STATES; }
        for (auto &kv : local) { kv.second = (uint32_t)T.gpids.size(); T.gpids.push_back(kv.first); }
        T.omask.assign(T.n_states, 0);
        for (uint32_t s = 0; s < T.n_states; ++s)
            for (uint32_t q = T.own_off[s]; q < T.own_off[s + 1]; ++q) T.omask[s] |= 1ull << local[T.own_ids[q]];
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
    return dev_match(c, h, b, n, res, true);
}

int sg_dev_match_dedup_diff(sg_ctx *c, sg_matcher *h, const uint8_t *d_buf, size_t n, const uint8_t *d_prior,
                            size_t n_prior, sg_dev_result *res, uint64_t *n_hits, uint64_t *matched_records) {
    if (!c || !h || !res || (!d_buf && n) || (!d_prior && n_prior)) {
        set_error("sg_dev_match_dedup_diff: bad arguments");
        return SG_E_INVAL;
    }
    SG_HIP(hipSetDevice(c->device));
    const uint8_t *b = d_buf, *p = d_prior;
    if (((uintptr_t)d_buf & 15) != 0) {
        uint8_t *a;
        SG_TRY(slot(c, S_IN, n + 16, &a));
        if (n) SG_HIP(hipMemcpyAsync(a, d_buf, n, hipMemcpyDeviceToDevice, c->stream));
        b = a;
    }
    if (n_prior && ((uintptr_t)d_prior & 15) != 0) {
        uint8_t *a;
        SG_TRY(slot(c, S_IN2, n_prior + 16, &a));
        SG_HIP(hipMemcpyAsync(a, d_prior, n_prior, hipMemcpyDeviceToDevice, c->stream));
        p = a;
    }
    if (!n_hits && h->lit.on && h->tables.empty() && !h->has_pre) {
        // literal matcher, hit count not asked: the scan flags matched records, and the
        // dedup runs on their spans in the input buffer (no hit list, no hit sort, no
        // grep-output copy and no second parse)
        sg_dev_hits hits;
        MatchFlags mf;
        SG_TRY(dev_match(c, h, b, n, &hits, false, &mf));
        const uint32_t R = mf.L.n_rec;
        uint32_t M = 0;
        Lines Lm;
        uint32_t *lcp;
        SG_TRY(slot(c, S_M_TMP, 4, &lcp));
        const uint32_t init = 255u;
        SG_HIP(hipMemcpyAsync(lcp, &init, 4, hipMemcpyHostToDevice, c->stream));
        if (R && mf.key0) {
            // the scan took every record's key0 and bytes 7..14: select and gather in one pass
            // (output slots sized for every record: the matched count is known after it)
            const uint32_t ntiles = (R + SEL_TILE - 1) / SEL_TILE;
            uint64_t *tp;  // tot | pre | total | masks A | masks B (unused: one predicate)
            SG_TRY(slot(c, S_COUNT, 2 * (size_t)ntiles + 4 + 2 * (size_t)ntiles * SEL_MASKS, &tp));
            uint64_t *tot = tp, *pre = tp + ntiles, *total = tp + 2 * (size_t)ntiles, *mA = total + 4;
            uint64_t *mB = mA + (size_t)ntiles * SEL_MASKS;
            SG_TRY(slot(c, S_M_SP2, (size_t)R + 1, &Lm.spans));
            SG_TRY(slot(c, S_M_K2, (size_t)R + 1, &Lm.keys));
            KeyStatD *gparts = nullptr;
            if (R >= 4096 && c->last_base >= 8u) {
                SG_TRY(slot(c, S_KEYSL, (size_t)R + 1, &Lm.spec_keys));
                SG_TRY(slot(c, S_SPEC_PARTS, (size_t)ntiles * sizeof(KeyStatD) / 8 + 1, &gparts));
                Lm.spec_off = c->last_base;
                Lm.spec_parts = gparts;
                Lm.spec_nparts = ntiles;
            }
            SG_LAUNCH(c, "select", k_sel_count<MFlagPred>, ntiles, SEL_BLOCK, 0, MFlagPred{mf.flags}, R, mA, mB, tot);
            SG_TRY(tile_scan(c, tot, ntiles, pre, total));
            // model: flag masks, then span + key0 + bytes 7..14 read and span + keys written per
            // matched record (the prefix scan's rare byte compares not credited)
            SG_LAUNCH(c, "gather_matched", k_gather_flagged, ntiles, SEL_BLOCK, 0, R, mA, pre, b, mf.L.spans,
                      (const uint64_t *)mf.key0, (const uint64_t *)mf.raw7, Lm.spans, Lm.keys, lcp, Lm.spec_keys,
                      Lm.spec_off, gparts);
            uint64_t tv = 0;
            SG_TRY(ctx_readback(c, &tv, total, 8));
            M = (uint32_t)(tv >> 31);
            if (c->profile) prof_bytes(c, "gather_matched", R / 8.0 + (Lm.spec_keys ? 48.0 : 40.0) * M);
        } else {
            uint32_t *mrec;
            SG_TRY(slot(c, S_R_POS, (size_t)R + 1, &mrec));
            if (R) SG_TRY(select_flags(c, mf.flags, R, mrec, &M));
            SG_TRY(slot(c, S_M_SP2, (size_t)M + 1, &Lm.spans));
            SG_TRY(slot(c, S_M_K2, (size_t)M + 1, &Lm.keys));
            const uint32_t gg = std::min<uint32_t>((M + 255) / 256, 2048u);
            // keys at the last call's common prefix too (see sg_dedup.hip: a re-key pass saved
            // when the matched records share that prefix again)
            KeyStatD *gparts = nullptr;
            if (M >= 4096 && c->last_base >= 8u) {
                SG_TRY(slot(c, S_KEYSL, (size_t)M + 1, &Lm.spec_keys));
                SG_TRY(slot(c, S_SPEC_PARTS, (size_t)gg * sizeof(KeyStatD) / 8 + 1, &gparts));
                Lm.spec_off = c->last_base;
                Lm.spec_parts = gparts;
                Lm.spec_nparts = gg;
            }
            if (M) SG_LAUNCH_B(c, "gather_matched", 24.0 * M, k_gather_matched, gg, 256, 0, b, mf.L.spans, mrec, M, Lm.spans,
                               Lm.keys, lcp, Lm.spec_keys, Lm.spec_off, gparts, (const uint64_t *)nullptr,
                               (const uint64_t *)nullptr);
        }
        Lm.n_rec = M;
        if (matched_records) *matched_records = M;
        SG_TRY(dev_dedup_diff_lines(c, b, n, Lm, n_prior ? p : nullptr, n_prior, res, M ? lcp : nullptr));
        res->in_records = R;
        return SG_OK;
    }
    // A3 + A4: the matched records in input order (grep output, context slot S_M_LINES)
    sg_dev_hits hits;
    SG_TRY(dev_match(c, h, b, n, &hits, true));
    if (n_hits) *n_hits = hits.n_hits;
    if (matched_records) *matched_records = hits.matched_records;
    // A7 + A8 on them: sort -u and the records new since the prior scan's matched set
    SG_TRY(dev_dedup_diff(c, hits.lines, hits.lines_bytes, n_prior ? p : nullptr, n_prior, true, res));
    res->in_records = hits.in_records;
    return SG_OK;
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
    SG_TRY(dev_match(c, h, d, n, &r, true));
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
    SG_TRY(dev_match(c, h, d, n, &r, true));
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
