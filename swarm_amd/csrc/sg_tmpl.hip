// sg_tmpl.hip — nuclei matcher semantics on the GPU.
//
// A template is a list of matchers joined by `matchers-condition` and/or
// (technologies/tech-detect.yaml:16); a matcher is a list of words or regexes joined by
// its `condition` and/or, optionally `negative` (file/audit/cisco/disable-ip-source-
// route.yaml:19-22) and `case-insensitive` (technologies/typo3-detect.yaml:23), and reads
// one `part`: the record itself (part 0) or a field of an httpx -json line (part k+1 =
// requested key k, e.g. title / webserver / tech; a word matches a field when it occurs in
// any of the field's rows). `encoding: hex` words arrive already decoded.
//
// Compile: every distinct (part, kind, case, pattern) is an "atom"; atoms are matched by
// the A4 engines (literal filter / Aho-Corasick, regex DFA plan), one engine per (stream,
// kind, case) where stream 0 is the record buffer and stream 1 the field rows of
// sg_json_fields. Evaluation is a sparse join done entirely with sort/select primitives:
//   hits (record, atom)  --sort, unique-->  expand over atom -> matchers
//   (record, matcher)    --sort-->          segments per (record, template)
//   one thread per segment walks the template's matchers (counts distinct words per
//   matcher for `and`), applies `negative`, joins with the template condition;
//   templates that hold on an empty record ("vacuous": e.g. a lone negative matcher)
//   are added for every record without a segment for them (binary search).
// Output: (record, template) pairs, sorted.
#include "sg_internal.hpp"
#include "sg_switches.hpp"
#include "sg_prims_host.hpp"

#include <algorithm>
#include <map>
#include <memory>
#include <string>
#include <tuple>

namespace sg {

struct TmRun {
    sg_matcher *m = nullptr;
    int stream = 0;
    std::vector<uint32_t> soff, satoms;  // signature -> atoms (CSR)
};

constexpr int TM_MAX_DEV = 64;

// Record-wave evaluation (one wave per record). LDS per block: the packed tables (atom ->
// occurrence offsets (16-bit), occurrences (matcher | template << 16), template (first
// matcher | count << 16 | and << 31), matcher (need | and | negative), vacuous bitmap), then
// per wave the matchers' 8-bit counters four to a word (a count never exceeds the matcher's
// distinct words, at most 255 here), the touched and true template bitmaps, the atoms seen and
// the list of templates to evaluate (16-bit ids). Twelve waves and at most 80 KB per block: 24 waves per CU.
constexpr uint32_t TMW_WAVES = 12;          // waves per block
constexpr uint32_t TMW_WORDS_MAX = 20480;   // 80 KB per block (two blocks per CU)
constexpr uint32_t TMW_NEED_AND = 1u << 16, TMW_NEED_NEG = 1u << 17;
// per wave: the matcher counters, touched + result template bitmaps, the seen-atom bitmap,
// and the touched-template list (its words also serve as the occurrence scratch: 128 words)
constexpr uint32_t tm_wave_words(uint32_t n_match, uint32_t n_tmpl, uint32_t n_atoms) {
    return (n_match + 3) / 4 + 2 * ((n_tmpl + 31) / 32) + (n_atoms + 31) / 32 +
           ((n_tmpl + 1) / 2 > 128u ? (n_tmpl + 1) / 2 : 128u);
}
constexpr uint64_t tm_block_words(uint32_t n_atoms, uint32_t n_occ, uint32_t n_match, uint32_t n_tmpl) {
    return (uint64_t)(n_atoms + 2) / 2 + n_occ + n_tmpl + n_match + (n_tmpl + 31) / 32 +
           (uint64_t)TMW_WAVES * tm_wave_words(n_match, n_tmpl, n_atoms);
}

}  // namespace sg

struct sg_templates {
    uint32_t n_tmpl = 0, n_match = 0, n_atoms = 0;
    std::vector<uint8_t> key_blob;
    std::vector<uint32_t> key_offs;
    std::vector<sg::TmRun> runs;
    std::vector<uint32_t> atom_part, occ_off, occ_m, m_tmpl, m_need, m_flags, t_first, t_count, t_flags, vac;
    std::vector<uint32_t> vacm;  // record-wave tables: vacuous bitmap, occurrence (m | t << 16),
    std::vector<uint32_t> occ_mt, tinfo, minfo, occ16;  // template (first, count | and << 31), matcher (need | flags)
    bool rec_wave = false;       // tables fit the record-wave evaluation (LDS counters, 16-bit counts)
    // Device tables, one set per device, uploaded on first use there and kept until
    // sg_tmpl_free: a call on another device never frees tables an eval may be using.
    struct Dev {
        bool ready = false;
        uint32_t *atom_part = nullptr, *occ_off = nullptr, *occ_m = nullptr, *m_tmpl = nullptr, *m_need = nullptr,
                 *m_flags = nullptr, *t_first = nullptr, *t_count = nullptr, *t_flags = nullptr, *vac = nullptr,
                 *vacm = nullptr, *occ_mt = nullptr, *tinfo = nullptr, *minfo = nullptr, *occ16 = nullptr;
        std::vector<uint32_t *> soff, satoms;  // per run
    } d[sg::TM_MAX_DEV];
    std::mutex mu;
};

namespace sg {

template <class T>
static int tm_upload(const std::vector<T> &v, T **d) {
    const size_t bytes = std::max<size_t>(v.size() * sizeof(T), 16);
    if (hipMalloc(d, bytes) != hipSuccess) { (void)hipGetLastError(); set_error("hipMalloc template table"); return SG_E_NOMEM; }
    if (!v.empty()) SG_HIP(hipMemcpy(*d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return SG_OK;
}

static void tm_free_dev(sg_templates::Dev &d) {
    for (void *p : {(void *)d.atom_part, (void *)d.occ_off, (void *)d.occ_m, (void *)d.m_tmpl, (void *)d.m_need,
                    (void *)d.m_flags, (void *)d.t_first, (void *)d.t_count, (void *)d.t_flags, (void *)d.vac,
                    (void *)d.vacm, (void *)d.occ_mt, (void *)d.tinfo, (void *)d.minfo, (void *)d.occ16})
        if (p) (void)hipFree(p);
    for (auto *p : d.soff) if (p) (void)hipFree(p);
    for (auto *p : d.satoms) if (p) (void)hipFree(p);
    d = sg_templates::Dev{};
}

static int tm_upload_all(sg_templates *h, sg_templates::Dev &d) {
    SG_TRY(tm_upload(h->atom_part, &d.atom_part));
    SG_TRY(tm_upload(h->occ_off, &d.occ_off));
    SG_TRY(tm_upload(h->occ_m, &d.occ_m));
    SG_TRY(tm_upload(h->m_tmpl, &d.m_tmpl));
    SG_TRY(tm_upload(h->m_need, &d.m_need));
    SG_TRY(tm_upload(h->m_flags, &d.m_flags));
    SG_TRY(tm_upload(h->t_first, &d.t_first));
    SG_TRY(tm_upload(h->t_count, &d.t_count));
    SG_TRY(tm_upload(h->t_flags, &d.t_flags));
    SG_TRY(tm_upload(h->vac, &d.vac));
    SG_TRY(tm_upload(h->vacm, &d.vacm));
    SG_TRY(tm_upload(h->occ_mt, &d.occ_mt));
    SG_TRY(tm_upload(h->tinfo, &d.tinfo));
    SG_TRY(tm_upload(h->minfo, &d.minfo));
    SG_TRY(tm_upload(h->occ16, &d.occ16));
    d.soff.assign(h->runs.size(), nullptr);
    d.satoms.assign(h->runs.size(), nullptr);
    for (size_t i = 0; i < h->runs.size(); ++i) {
        SG_TRY(tm_upload(h->runs[i].soff, &d.soff[i]));
        SG_TRY(tm_upload(h->runs[i].satoms, &d.satoms[i]));
    }
    return SG_OK;
}

// The tables on `dev` (uploaded once, under the handle's lock; a failed upload frees what
// it allocated and leaves the device not ready, so the next call retries cleanly).
static int tm_ensure_device(sg_templates *h, int dev, const sg_templates::Dev **out) {
    if (dev < 0 || dev >= TM_MAX_DEV) { set_error("device %d out of range", dev); return SG_E_INVAL; }
    std::lock_guard<std::mutex> g(h->mu);
    auto &d = h->d[dev];
    if (!d.ready) {
        SG_HIP(hipSetDevice(dev));
        const int rc = tm_upload_all(h, d);
        if (rc != SG_OK) { tm_free_dev(d); return rc; }
        d.ready = true;
    }
    *out = &d;
    return SG_OK;
}

// ------------------------------------------------------------------ device
constexpr uint32_t TM_NO_ATOM = ~0u;

// hits (record or row, signature) -> (record << 32 | atom); a field-row hit keeps the atom
// whose part is the row's field (none: atom TM_NO_ATOM, skipped by both evaluations). Each
// engine's hits arrive sorted by record (rows map to records monotonically), so every
// collect launch leaves one record-ordered segment.
__global__ __launch_bounds__(256) void k_tm_collect(const uint32_t *__restrict__ rec_idx, const uint32_t *__restrict__ sig,
                                                    uint32_t nh, const uint32_t *__restrict__ soff,
                                                    const uint32_t *__restrict__ satoms,
                                                    const uint32_t *__restrict__ apart,
                                                    const uint32_t *__restrict__ row_rec,
                                                    const uint32_t *__restrict__ row_key, uint64_t *__restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nh) return;
    const uint32_t r = rec_idx[i], s = sig[i];
    uint64_t key;
    if (!row_rec) {
        key = ((uint64_t)r << 32) | satoms[soff[s]];
    } else {
        const uint32_t want = row_key[r] + 1;
        key = ((uint64_t)row_rec[r] << 32) | TM_NO_ATOM;
        for (uint32_t q = soff[s]; q < soff[s + 1]; ++q)
            if (apart[satoms[q]] == want) { key = ((uint64_t)row_rec[r] << 32) | satoms[q]; break; }
    }
    out[i] = key;
}

struct TmUniqPred {
    const uint64_t *K;
    __device__ uint32_t operator()(uint32_t i) const {
        const uint64_t k = K[i];
        return ((uint32_t)k != TM_NO_ATOM && (i == 0 || k != K[i - 1])) ? 1u : 0u;
    }
};

struct TmOccLen {
    const uint64_t *K;
    const uint32_t *U, *occ_off;
    __device__ uint64_t operator()(uint32_t i) const {
        const uint32_t a = (uint32_t)K[U[i]];
        return occ_off[a + 1] - occ_off[a];
    }
};

__global__ __launch_bounds__(256) void k_tm_expand(const uint64_t *__restrict__ K, const uint32_t *__restrict__ U,
                                                   uint32_t nu, const uint64_t *__restrict__ offs,
                                                   const uint32_t *__restrict__ occ_off,
                                                   const uint32_t *__restrict__ occ_m, uint64_t *__restrict__ E) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nu) return;
    const uint64_t k = K[U[i]];
    const uint32_t a = (uint32_t)k;
    const uint64_t rec = k & 0xffffffff00000000ull;
    uint64_t o = offs[i];
    for (uint32_t q = occ_off[a]; q < occ_off[a + 1]; ++q) E[o++] = rec | occ_m[q];
}

struct TmSegPred {
    const uint64_t *E;
    const uint32_t *m_tmpl;
    __device__ uint32_t operator()(uint32_t i) const {
        if (i == 0) return 1u;
        const uint64_t a = E[i - 1], b = E[i];
        return ((a >> 32) != (b >> 32) || m_tmpl[(uint32_t)a] != m_tmpl[(uint32_t)b]) ? 1u : 0u;
    }
};

__global__ __launch_bounds__(256) void k_tm_eval(const uint64_t *__restrict__ E, uint32_t n2,
                                                 const uint32_t *__restrict__ seg, uint32_t ns,
                                                 const uint32_t *__restrict__ m_tmpl, const uint32_t *__restrict__ m_need,
                                                 const uint32_t *__restrict__ m_flags,
                                                 const uint32_t *__restrict__ t_first,
                                                 const uint32_t *__restrict__ t_count,
                                                 const uint32_t *__restrict__ t_flags, uint32_t *__restrict__ flag,
                                                 uint64_t *__restrict__ segkey) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= ns) return;
    const uint32_t e1 = (s + 1 < ns) ? seg[s + 1] : n2;
    uint32_t e = seg[s];
    const uint64_t k0 = E[e];
    const uint32_t t = m_tmpl[(uint32_t)k0];
    const bool and_t = t_flags[t] & SG_TM_AND;
    bool acc = and_t;
    const uint32_t m0 = t_first[t], m1 = m0 + t_count[t];
    for (uint32_t m = m0; m < m1; ++m) {
        uint32_t cnt = 0;
        while (e < e1 && (uint32_t)E[e] == m) { ++cnt; ++e; }
        const uint32_t f = m_flags[m];
        bool hit = (f & SG_TM_AND) ? cnt >= m_need[m] : cnt > 0;
        if (f & SG_TM_NEGATIVE) hit = !hit;
        acc = and_t ? (acc && hit) : (acc || hit);
    }
    flag[s] = acc ? 1u : 0u;
    segkey[s] = (k0 & 0xffffffff00000000ull) | t;
}

struct TmFlagPred {
    const uint32_t *flag;
    __device__ uint32_t operator()(uint32_t i) const { return flag[i]; }
};

// (record, vacuous template) pairs with no segment: the template holds there.
struct TmVacPred {
    const uint64_t *segkey;
    uint32_t ns;
    const uint32_t *vac;
    uint32_t nv;
    __device__ uint32_t operator()(uint32_t i) const {
        const uint32_t r = i / nv, t = vac[i % nv];
        const uint64_t key = ((uint64_t)r << 32) | t;
        uint32_t lo = 0, hi = ns;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (segkey[mid] < key) lo = mid + 1; else hi = mid;
        }
        return (lo < ns && segkey[lo] == key) ? 0u : 1u;
    }
};

__global__ __launch_bounds__(256) void k_tm_gather(const uint64_t *__restrict__ segkey, const uint32_t *__restrict__ sel,
                                                   uint32_t nt, const uint32_t *__restrict__ vsel, uint32_t nvac,
                                                   const uint32_t *__restrict__ vac, uint32_t nv,
                                                   uint64_t *__restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nt) {
        out[i] = segkey[sel[i]];
    } else if (i < nt + nvac) {
        const uint32_t x = vsel[i - nt];
        out[i] = ((uint64_t)(x / nv) << 32) | vac[x % nv];
    }
}

__global__ __launch_bounds__(256) void k_tm_split(const uint64_t *__restrict__ K, uint32_t n, uint32_t *__restrict__ rec,
                                                  uint32_t *__restrict__ tid) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t k = K[i];
    rec[i] = (uint32_t)(k >> 32);
    tid[i] = (uint32_t)k;
}

// ------------------------------------------------------------------ record-wave evaluation
// The default evaluation: no sort at all. Instead of sorting the (record, atom) hits,
// expanding them to (record, matcher) pairs, sorting those, evaluating segments, adding the
// vacuous templates by binary search and sorting the union, one wave takes one record's
// hits from every engine's record-ordered segment, drops repeated atoms with an LDS bitmap,
// counts them per matcher in LDS, evaluates every touched or vacuous template and writes the
// record's true templates as a bitmap; a scan of the per-record counts places each record's
// pairs, which the emit pass writes in (record, template) order — the sorted output.

// off[r] .. off[r + 1] = record r's entries of the segment K[0, n) (record-ordered), as
// absolute indices (+ start).
__global__ __launch_bounds__(256) void k_tm_rec_off(const uint64_t *__restrict__ K, uint32_t n, uint32_t R,
                                                    uint32_t start, uint32_t *__restrict__ off) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i > n) return;
    const uint32_t cur = i < n ? (uint32_t)min<uint64_t>(K[i] >> 32, R) : R;
    const uint32_t lo = i ? (uint32_t)min<uint64_t>(K[i - 1] >> 32, R) + 1 : 0u;
    for (uint32_t r = lo; r <= cur; ++r) off[r] = start + i;
}

__device__ __forceinline__ void tm_wave_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

__global__ __launch_bounds__(64 * TMW_WAVES) void k_tm_rec_eval(
    const uint64_t *__restrict__ K, const uint32_t *__restrict__ roff, uint32_t nseg, uint32_t R,
    const uint32_t *__restrict__ occ_off,
    const uint32_t *__restrict__ occ_mt, const uint32_t *__restrict__ tinfo, const uint32_t *__restrict__ minfo,
    const uint32_t *__restrict__ vacm, uint32_t n_atoms, uint32_t n_occ, uint32_t n_match, uint32_t n_tmpl,
    uint32_t *__restrict__ G,
    uint32_t *__restrict__ rcnt) {
    extern __shared__ uint32_t s_w[];
    const uint32_t ntw = (n_tmpl + 31) / 32, cw = (n_match + 3) / 4;
    uint32_t *s_occw = s_w, *s_mt = s_occw + (n_atoms + 2) / 2, *s_ti = s_mt + n_occ, *s_mi = s_ti + n_tmpl,
             *s_vac = s_mi + n_match;
    const uint16_t *s_occ = reinterpret_cast<const uint16_t *>(s_occw);
    const uint32_t wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint32_t *cnt = s_vac + ntw + wid * tm_wave_words(n_match, n_tmpl, n_atoms), *tch = cnt + cw, *res = tch + ntw;
    const uint32_t naw = (n_atoms + 31) / 32;
    uint32_t *seen = res + ntw;
    uint16_t *list = reinterpret_cast<uint16_t *>(seen + naw);
    for (uint32_t x = threadIdx.x; x < (n_atoms + 2) / 2; x += blockDim.x) s_occw[x] = occ_off[x];
    for (uint32_t x = threadIdx.x; x < n_occ; x += blockDim.x) s_mt[x] = occ_mt[x];
    for (uint32_t x = threadIdx.x; x < n_tmpl; x += blockDim.x) s_ti[x] = tinfo[x];
    for (uint32_t x = threadIdx.x; x < n_match; x += blockDim.x) s_mi[x] = minfo[x];
    for (uint32_t x = threadIdx.x; x < ntw; x += blockDim.x) s_vac[x] = vacm[x];
    __syncthreads();
    const uint32_t nw = gridDim.x * TMW_WAVES;
    for (uint32_t r = blockIdx.x * TMW_WAVES + wid; r < R; r += nw) {
        for (uint32_t x = lane; x < cw; x += 64) cnt[x] = 0;
        for (uint32_t x = lane; x < ntw; x += 64) { tch[x] = 0; res[x] = 0; }
        for (uint32_t x = lane; x < naw; x += 64) seen[x] = 0;
        // every segment's [start, end) of this record at once (lanes 2g, 2g + 1), not one
        // dependent pair of offset loads per segment (loading them one record ahead gained nothing)
        uint32_t myo = 0;
        if (nseg <= 32 && lane < 2 * nseg) myo = roff[(size_t)(lane >> 1) * (R + 1) + r + (lane & 1)];
        tm_wave_sync();
        // one atom per lane (TM_NO_ATOM: none; wave-uniform call): each atom counted once per
        // record, and the (matcher, template) occurrences of the wave's new atoms spread over
        // all 64 lanes (lane k's run at its prefix in scratch), instead of each lane walking
        // its own atom's list while the wave waits for the longest (an atom can sit in dozens
        // of matchers)
        uint32_t *sc_inc = reinterpret_cast<uint32_t *>(list), *sc_q0 = sc_inc + 64;
        auto count_atoms = [&](uint32_t at) {
            uint32_t q0 = 0, c = 0;
            if (at != TM_NO_ATOM) {
                const uint32_t bit = 1u << (at & 31);
                if (!(atomicOr(&seen[at >> 5], bit) & bit)) {
                    q0 = s_occ[at];
                    c = (uint32_t)s_occ[at + 1] - q0;
                }
            }
            const uint32_t inc = wave_incl_scan_shfl(c);
            const uint32_t T = (uint32_t)__shfl((int)inc, 63, 64);
            if (T == 0u) return;
            sc_inc[lane] = inc;
            sc_q0[lane] = q0;
            tm_wave_sync();
            for (uint32_t o = lane; o < T; o += 64) {
                uint32_t lo = 0, hi = 63;  // the first lane whose inclusive prefix exceeds o
                while (lo < hi) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (sc_inc[mid] > o) hi = mid; else lo = mid + 1;
                }
                const uint32_t q = sc_q0[lo] + o - (lo ? sc_inc[lo - 1] : 0u);
                const uint32_t mt = s_mt[q], m = mt & 0xffffu, t = mt >> 16;
                atomicAdd(&cnt[m >> 2], 1u << (8 * (m & 3)));
                atomicOr(&tch[t >> 5], 1u << (t & 31));
            }
            tm_wave_sync();  // scratch reused by the next batch
        };
        if (nseg <= 32) {
            // the record's hits of all segments as one list: lane j loads hit j, so the
            // segments' loads are issued together instead of one round trip per segment
            uint32_t tot = 0;
            for (uint32_t sg = 0; sg < nseg; ++sg)
                tot += (uint32_t)__shfl((int)myo, (int)(2 * sg + 1), 64) - (uint32_t)__shfl((int)myo, (int)(2 * sg), 64);
            for (uint32_t j0 = 0; j0 < tot; j0 += 64) {
                const uint32_t j = j0 + lane;
                uint32_t idx = 0xffffffffu, base = 0;
                for (uint32_t sg = 0; sg < nseg; ++sg) {
                    const uint32_t sa = (uint32_t)__shfl((int)myo, (int)(2 * sg), 64);
                    const uint32_t c = (uint32_t)__shfl((int)myo, (int)(2 * sg + 1), 64) - sa;
                    if (j >= base && j < base + c) idx = sa + (j - base);
                    base += c;
                }
                count_atoms(idx != 0xffffffffu ? (uint32_t)K[idx] : TM_NO_ATOM);
            }
        } else {
            for (uint32_t sg = 0; sg < nseg; ++sg) {
                const uint32_t *ro = roff + (size_t)sg * (R + 1);
                const uint32_t a0 = ro[r], a1 = ro[r + 1];  // (wave-uniform: one record per wave)
                for (uint32_t i0 = a0; i0 < a1; i0 += 64)
                    count_atoms(i0 + lane < a1 ? (uint32_t)K[i0 + lane] : TM_NO_ATOM);
            }
        }
        tm_wave_sync();
        // the templates to evaluate: the touched ones. An untouched template sees every count
        // 0, so it holds iff it is vacuous: those start true.
        uint32_t nl = 0;
        for (uint32_t w0 = 0; w0 < ntw; w0 += 64) {
            const uint32_t w = w0 + lane;
            uint32_t bits = w < ntw ? tch[w] : 0u;
            if (w < ntw) res[w] = s_vac[w] & ~bits;
            const uint32_t c = (uint32_t)__popc(bits), inc = wave_incl_scan_shfl(c);
            uint32_t p = nl + inc - c;
            while (bits) {
                list[p++] = (uint16_t)(32 * w + (uint32_t)__builtin_ctz(bits));
                bits &= bits - 1;
            }
            nl += __shfl(inc, 63, 64);
        }
        tm_wave_sync();
        for (uint32_t j = lane; j < nl; j += 64) {
            const uint32_t t = list[j], ti = s_ti[t], m0 = ti & 0xffffu;
            const bool and_t = ti >> 31;
            bool acc = and_t;
            for (uint32_t m = m0, me = m0 + ((ti >> 16) & 0x7fffu); m < me; ++m) {
                const uint32_t c = (cnt[m >> 2] >> (8 * (m & 3))) & 0xffu, mi = s_mi[m];
                bool hit = (mi & TMW_NEED_AND) ? c >= (mi & 0xffffu) : c > 0;
                if (mi & TMW_NEED_NEG) hit = !hit;
                acc = and_t ? (acc && hit) : (acc || hit);
                if (acc != and_t) break;  // and: a false matcher decides; or: a true one
            }
            if (acc) atomicOr(&res[t >> 5], 1u << (t & 31));
        }
        tm_wave_sync();
        uint32_t tot = 0;
        for (uint32_t w = lane; w < ntw; w += 64) {
            const uint32_t tr = res[w];
            G[(size_t)r * ntw + w] = tr;
            tot += (uint32_t)__popc(tr);
        }
        tot = wave_sum_shfl(tot);
        if (lane == 0) rcnt[r] = tot;
        tm_wave_sync();
    }
}

struct TmRecCnt {
    const uint32_t *rcnt;
    __device__ uint64_t operator()(uint32_t i) const { return rcnt[i]; }
};

// Each record's (record, template) pairs go through a per-wave LDS buffer: the lanes (one per
// bitmap word) scatter their template ids there, then the wave writes the record's run with
// consecutive lanes on consecutive slots (the direct version had every lane store its own run
// one pair at a time: 64 runs per store instruction). Runs longer than the buffer are written
// directly.
constexpr uint32_t TE_CAP = 1024;
__global__ __launch_bounds__(256) void k_tm_rec_emit(const uint32_t *__restrict__ G, const uint64_t *__restrict__ off,
                                                     const uint32_t *__restrict__ rcnt, uint32_t R, uint32_t ntw,
                                                     uint32_t *__restrict__ rec, uint32_t *__restrict__ tid) {
    __shared__ uint32_t s_t[4][TE_CAP];
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t *buf = s_t[wid];
    // each wave a contiguous range of records, so its runs follow each other in the output
    // and a cache line is filled by one wave within a few records, not by waves of other
    // blocks at other times (partially written lines were fetched back: 0.9 GB per launch)
    const uint32_t nw = gridDim.x * (blockDim.x >> 6), gw = blockIdx.x * (blockDim.x >> 6) + wid;
    const uint32_t per = (R + nw - 1) / nw;
    const uint32_t ra = min(R, gw * per), rz = min(R, ra + per);
    for (uint32_t r = ra; r < rz; ++r) {
        const uint64_t base = off[r];
        const uint32_t n = rcnt[r];
        const bool staged = n <= TE_CAP;
        uint32_t lp = 0;  // pairs of the words before this lane's, within the record
        for (uint32_t w0 = 0; w0 < ntw; w0 += 64) {
            const uint32_t w = w0 + lane;
            uint32_t bits = w < ntw ? G[(size_t)r * ntw + w] : 0u;
            const uint32_t c = (uint32_t)__popc(bits);
            const uint32_t inc = wave_incl_scan_shfl(c);
            uint32_t p = lp + inc - c;
            while (bits) {
                const uint32_t t = 32 * w + (uint32_t)__builtin_ctz(bits);
                bits &= bits - 1;
                if (staged) buf[p] = t;
                else { rec[base + p] = r; tid[base + p] = t; }
                ++p;
            }
            lp += (uint32_t)__shfl((int)inc, 63, 64);
        }
        if (staged) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            for (uint32_t j = lane; j < n; j += 64) {
                rec[base + j] = r;
                tid[base + j] = buf[j];
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        }
    }
}

struct TmAccum {
    int slot_id = S_T_HITS;
    uint64_t *p = nullptr;
    uint64_t n = 0, cap = 0;
};

static int tm_grow(sg_ctx *c, TmAccum *a, uint64_t need) {
    if (need <= a->cap) return SG_OK;
    const int other = a->slot_id == S_T_HITS ? S_T_EXP : S_T_HITS;
    const uint64_t cap = std::max<uint64_t>(std::max<uint64_t>(need, 2 * a->cap), 1u << 16);
    uint64_t *np;
    SG_TRY(slot(c, other, cap, &np));
    if (a->n) SG_HIP(hipMemcpyAsync(np, a->p, a->n * 8, hipMemcpyDeviceToDevice, c->stream));
    a->slot_id = other;
    a->p = np;
    a->cap = cap;
    return SG_OK;
}

// The record-wave evaluation of the collected hits K: segs = each collect launch's (start,
// count), record-ordered within (see k_tm_rec_eval).
static int tm_rec_wave(sg_ctx *c, const sg_templates *h, const sg_templates::Dev &D, const uint64_t *K,
                       const std::vector<std::pair<uint32_t, uint32_t>> &segs, uint64_t R, sg_dev_tmatches *res) {
    const uint32_t ntw = (h->n_tmpl + 31) / 32;
    if (R * ntw >= (1ull << 40)) { set_error("template eval: records x templates too large"); return SG_E_TOO_LARGE; }
    uint32_t *roff, *G, *rcnt;
    uint64_t *off;
    const uint32_t nseg = (uint32_t)segs.size();
    SG_TRY(slot(c, S_T_SEG, (R + 1) * nseg + 16, &roff));
    SG_TRY(slot(c, S_T_E, R * ntw + 16, &G));
    SG_TRY(slot(c, S_T_FLAG, R + 16, &rcnt));
    SG_TRY(slot(c, S_T_O, R + 16, &off));
    const uint32_t Ru = (uint32_t)R;
    for (uint32_t g = 0; g < nseg; ++g)
        SG_LAUNCH(c, "tm_rec_off", k_tm_rec_off, (segs[g].second + 1 + 255) / 256, 256, 0, K + segs[g].first,
                  segs[g].second, Ru, segs[g].first, roff + (size_t)g * (R + 1));
    const uint32_t n_occ = (uint32_t)h->occ_m.size();
    const size_t lds = (size_t)tm_block_words(h->n_atoms, n_occ, h->n_match, h->n_tmpl) * 4;
    const uint32_t blocks = (uint32_t)std::min<uint64_t>((R + TMW_WAVES - 1) / TMW_WAVES, 8192);
    if (lds > 65536)
        SG_HIP(hipFuncSetAttribute((const void *)k_tm_rec_eval, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    if (sw_lit_trial_log())
        fprintf(stderr, "sg tm_rec_eval: %u records, %u hit segments, %u matchers, %u atoms, %u templates, %zu B LDS per block\n",
                Ru, nseg, h->n_match, h->n_atoms, h->n_tmpl, lds);
    SG_LAUNCH(c, "tm_rec_eval", k_tm_rec_eval, blocks, 64 * TMW_WAVES, lds, K, roff, nseg, Ru, D.occ16, D.occ_mt, D.tinfo,
              D.minfo, D.vacm, h->n_atoms, n_occ, h->n_match, h->n_tmpl, G, rcnt);
    uint64_t nout = 0;
    SG_TRY(run_scan64(c, "tm_rec_scan", TmRecCnt{rcnt}, Ru, off, &nout));
    res->n = nout;
    if (nout == 0) return SG_OK;
    uint32_t *rec, *tid;
    SG_TRY(slot(c, S_T_REC, nout + 1, &rec));
    SG_TRY(slot(c, S_T_TID, nout + 1, &tid));
    const uint32_t eblocks = (uint32_t)std::min<uint64_t>((R + 3) / 4, 16384);
    SG_LAUNCH_B(c, "tm_rec_emit", 8.0 * nout + 4.0 * R * ntw, k_tm_rec_emit, eblocks, 256, 0, G, off, rcnt, Ru, ntw, rec,
                tid);
    res->rec_idx = rec;
    res->tmpl_id = tid;
    return SG_OK;
}

// given_rows: the field rows of d_buf for the handle's keys, from the caller's own
// sg_dev_json_fields call on this context (the fields step parses the JSON once); null: the
// rows are built here.
static int dev_tmpl_eval(sg_ctx *c, sg_templates *h, const uint8_t *d_buf, uint64_t n, sg_dev_tmatches *res,
                         const sg_dev_rows *given_rows = nullptr) {
    *res = sg_dev_tmatches{};
    const sg_templates::Dev *pd = nullptr;
    SG_TRY(tm_ensure_device(h, c->device, &pd));
    const auto &D = *pd;
    TmAccum acc;
    std::vector<std::pair<uint32_t, uint32_t>> segs;  // each collect launch's hits in acc
    uint64_t R = 0;
    bool have_R = false;
    // stream 0: the records themselves (one parse shared by every engine's run: the parse
    // of a 2.4 GB JSON body was redone per engine)
    Lines parse0;
    for (size_t ri = 0; ri < h->runs.size(); ++ri) {
        auto &run = h->runs[ri];
        if (run.stream != 0) continue;
        sg_dev_hits r;
        SG_TRY(dev_match(c, run.m, d_buf, n, &r, false, nullptr, &parse0));
        R = r.in_records;
        have_R = true;
        if (!r.n_hits) continue;
        SG_TRY(tm_grow(c, &acc, acc.n + r.n_hits));
        SG_LAUNCH(c, "tm_collect", k_tm_collect, (uint32_t)((r.n_hits + 255) / 256), 256, 0, r.rec_idx, r.sig_id,
                  (uint32_t)r.n_hits, D.soff[ri], D.satoms[ri], D.atom_part, (const uint32_t *)nullptr,
                  (const uint32_t *)nullptr, acc.p + acc.n);
        segs.emplace_back((uint32_t)acc.n, (uint32_t)r.n_hits);
        acc.n += r.n_hits;
    }
    // stream 1: httpx -json field rows
    bool any1 = false;
    for (auto &run : h->runs) any1 |= run.stream == 1;
    if (any1) {
        sg_dev_rows rows;
        if (given_rows) rows = *given_rows;
        else SG_TRY(dev_json_fields(c, d_buf, n, h->key_blob.data(), h->key_offs.data(), (uint32_t)h->key_offs.size() - 1,
                                    &rows));
        R = rows.in_records;
        have_R = true;
        Lines parse1;  // the rows' parse, shared the same way
        for (size_t ri = 0; ri < h->runs.size(); ++ri) {
            auto &run = h->runs[ri];
            if (run.stream != 1 || rows.bytes == 0) continue;
            sg_dev_hits r;
            SG_TRY(dev_match(c, run.m, rows.data, rows.bytes, &r, false, nullptr, &parse1));
            if (!r.n_hits) continue;
            SG_TRY(tm_grow(c, &acc, acc.n + r.n_hits));
            SG_LAUNCH(c, "tm_collect", k_tm_collect, (uint32_t)((r.n_hits + 255) / 256), 256, 0, r.rec_idx, r.sig_id,
                      (uint32_t)r.n_hits, D.soff[ri], D.satoms[ri], D.atom_part, rows.row_rec, rows.row_key,
                      acc.p + acc.n);
            segs.emplace_back((uint32_t)acc.n, (uint32_t)r.n_hits);
            acc.n += r.n_hits;
        }
    }
    if (!have_R) {
        Lines L;
        SG_TRY(run_lines(c, d_buf, n, CUR_SLOTS, &L, false));
        R = L.n_rec;
    }
    res->in_records = R;
    if (acc.n >= (1ull << 32)) { set_error("template eval: more than 2^32 atom hits"); return SG_E_TOO_LARGE; }
    int rbits = 1;
    while (rbits < 32 && (1ull << rbits) < R) ++rbits;
    const int kbits = 32 + rbits;
    // (record, atom): sort + unique
    uint32_t nu = 0, ns = 0, nt = 0;
    uint64_t *E = nullptr;
    uint64_t n2 = 0;
    uint32_t *seg = nullptr, *flag = nullptr, *sel = nullptr;
    uint64_t *segkey = nullptr;
    static const bool tm_sort = sw_tm_sort();  // test switch: the sort-based evaluation below
    if (acc.n && h->rec_wave && !tm_sort) return tm_rec_wave(c, h, D, acc.p, segs, R, res);
    if (acc.n) {
        const uint32_t n1 = (uint32_t)acc.n;
        uint64_t *k2, *K;
        uint32_t *v1, *v2, *V;
        SG_TRY(slot(c, S_T_K2, (size_t)n1 + 1, &k2));
        SG_TRY(slot(c, S_T_V1, (size_t)n1 + 1, &v1));
        SG_TRY(slot(c, S_T_V2, (size_t)n1 + 1, &v2));
        SG_TRY(radix_sort(c, acc.p, v1, k2, v2, n1, 0, kbits, true, &K, &V, "tm_rs_atoms"));
        SG_TRY(slot(c, S_T_SEL, (size_t)n1 + 16, &sel));
        SG_TRY(run_select2(c, "tm_unique", TmUniqPred{K}, n1, sel, (uint32_t *)nullptr, &nu, nullptr, 16.0));
        if (nu) {
            uint64_t *offs;
            SG_TRY(slot(c, S_T_OUT, (size_t)nu + 1, &offs));
            SG_TRY(run_scan64(c, "tm_occ_scan", TmOccLen{K, sel, D.occ_off}, nu, offs, &n2));
            if (n2 >= (1ull << 32)) { set_error("template eval: more than 2^32 matcher hits"); return SG_E_TOO_LARGE; }
            if (n2) {
                uint64_t *e1, *e2;
                SG_TRY(slot(c, S_T_E, n2 + 1, &e1));
                SG_TRY(slot(c, S_T_E2, n2 + 1, &e2));
                SG_LAUNCH(c, "tm_expand", k_tm_expand, (nu + 255) / 256, 256, 0, K, sel, nu, offs, D.occ_off, D.occ_m, e1);
                uint32_t *w1, *w2, *WV;
                SG_TRY(slot(c, S_T_V1, n2 + 1, &w1));
                SG_TRY(slot(c, S_T_V2, n2 + 1, &w2));
                SG_TRY(radix_sort(c, e1, w1, e2, w2, (uint32_t)n2, 0, kbits, true, &E, &WV, "tm_rs_matchers"));
                SG_TRY(slot(c, S_T_SEG, n2 + 16, &seg));
                SG_TRY(run_select2(c, "tm_segments", TmSegPred{E, D.m_tmpl}, (uint32_t)n2, seg, (uint32_t *)nullptr, &ns,
                                   nullptr, 24.0));
                SG_TRY(slot(c, S_T_FLAG, (size_t)ns + 16, &flag));
                SG_TRY(slot(c, S_T_O, (size_t)ns + 16, &segkey));
                SG_LAUNCH(c, "tm_eval", k_tm_eval, (ns + 255) / 256, 256, 0, E, (uint32_t)n2, seg, ns, D.m_tmpl, D.m_need,
                          D.m_flags, D.t_first, D.t_count, D.t_flags, flag, segkey);
                SG_TRY(slot(c, S_T_SEL, (size_t)ns + 16, &sel));  // segments may outnumber the atom hits
                SG_TRY(run_select2(c, "tm_true", TmFlagPred{flag}, ns, sel, (uint32_t *)nullptr, &nt, nullptr, 4.0));
            }
        }
    }
    // vacuous templates on records without a segment for them
    const uint32_t nv = (uint32_t)h->vac.size();
    uint32_t nvac = 0;
    uint32_t *vsel = nullptr;
    if (nv && R) {
        const uint64_t items = R * nv;
        if (items >= (1ull << 32)) { set_error("template eval: records x vacuous templates exceeds 2^32"); return SG_E_TOO_LARGE; }
        SG_TRY(slot(c, S_T_HITS, items + 16, &vsel));
        uint64_t *sk = segkey;
        if (!sk) SG_TRY(slot(c, S_T_O, 16, &sk));
        SG_TRY(run_select2(c, "tm_vacuous", TmVacPred{sk, ns, D.vac, nv}, (uint32_t)items, vsel, (uint32_t *)nullptr, &nvac,
                           nullptr, 8.0));
    }
    const uint64_t nout = (uint64_t)nt + nvac;
    res->n = nout;
    if (nout == 0) return SG_OK;
    uint64_t *o1, *o2, *OK;
    uint32_t *u1, *u2, *UV;
    SG_TRY(slot(c, S_T_OUT, nout + 1, &o1));
    SG_TRY(slot(c, S_T_K2, nout + 1, &o2));
    SG_TRY(slot(c, S_T_V1, nout + 1, &u1));
    SG_TRY(slot(c, S_T_V2, nout + 1, &u2));
    SG_LAUNCH(c, "tm_gather", k_tm_gather, (uint32_t)((nout + 255) / 256), 256, 0, segkey, sel, nt, vsel, nvac, D.vac,
              nv ? nv : 1u, o1);
    if (nvac && nt) SG_TRY(radix_sort(c, o1, u1, o2, u2, (uint32_t)nout, 0, kbits, true, &OK, &UV, "tm_rs_out"));
    else OK = o1;  // one sorted source: segment keys or the (record, vacuous) grid order
    uint32_t *rec, *tid;
    SG_TRY(slot(c, S_T_REC, nout + 1, &rec));
    SG_TRY(slot(c, S_T_TID, nout + 1, &tid));
    SG_LAUNCH(c, "tm_split", k_tm_split, (uint32_t)((nout + 255) / 256), 256, 0, OK, (uint32_t)nout, rec, tid);
    res->rec_idx = rec;
    res->tmpl_id = tid;
    return SG_OK;
}

}  // namespace sg

using namespace sg;

extern "C" {

int sg_tmpl_compile(const uint8_t *pats, const uint32_t *pat_offs, uint32_t n_pats, const sg_tm_matcher *ms,
                    uint32_t n_matchers, const uint32_t *tmpl_flags, uint32_t n_templates, const uint8_t *keys,
                    const uint32_t *key_offs, uint32_t n_keys, sg_templates **out) {
    if (!out || (n_pats && (!pats || !pat_offs)) || (n_matchers && !ms) || (n_templates && !tmpl_flags) ||
        (n_keys && (!keys || !key_offs))) {
        set_error("sg_tmpl_compile: bad arguments");
        return SG_E_INVAL;
    }
    if (n_keys > 64) { set_error("sg_tmpl_compile: at most 64 field keys"); return SG_E_INVAL; }
    std::unique_ptr<sg_templates> h(new sg_templates());
    h->n_tmpl = n_templates;
    h->n_match = n_matchers;
    h->key_offs.assign(1, 0);
    for (uint32_t k = 0; k < n_keys; ++k) {
        h->key_blob.insert(h->key_blob.end(), keys + key_offs[k], keys + key_offs[k + 1]);
        h->key_offs.push_back((uint32_t)h->key_blob.size());
    }
    if (h->key_blob.empty()) h->key_blob.push_back(0);
    h->t_first.assign(n_templates, 0);
    h->t_count.assign(n_templates, 0);
    h->t_flags.assign(tmpl_flags, tmpl_flags + n_templates);
    // atoms: (part, kind, nocase, bytes)
    std::map<std::tuple<uint32_t, uint32_t, uint32_t, std::string>, uint32_t> atoms;
    std::vector<std::vector<uint32_t>> m_atoms(n_matchers);
    std::vector<std::tuple<uint32_t, uint32_t, uint32_t, std::string>> atom_key;
    for (uint32_t i = 0; i < n_matchers; ++i) {
        const sg_tm_matcher &m = ms[i];
        if (m.tmpl >= n_templates || (i && m.tmpl < ms[i - 1].tmpl)) {
            set_error("matcher %u: template ids must be < n_templates and non-decreasing", i);
            return SG_E_INVAL;
        }
        if (m.kind > SG_TM_REGEX || m.part > n_keys || m.count == 0 || (uint64_t)m.first + m.count > n_pats) {
            set_error("matcher %u: bad kind/part/pattern range", i);
            return SG_E_INVAL;
        }
        if (h->t_count[m.tmpl] == 0) h->t_first[m.tmpl] = i;
        h->t_count[m.tmpl]++;
        // case-insensitive applies to words (nuclei lowercases words and part); regexes use (?i)
        const uint32_t nc = ((m.flags & SG_TM_NOCASE) && m.kind == SG_TM_WORD) ? 1u : 0u;
        for (uint32_t q = m.first; q < m.first + m.count; ++q) {
            std::string s((const char *)pats + pat_offs[q], pat_offs[q + 1] - pat_offs[q]);
            if (s.empty()) { set_error("matcher %u: empty pattern", i); return SG_E_INVAL; }
            if (nc && m.kind == SG_TM_WORD)
                for (auto &ch : s) if (ch >= 'A' && ch <= 'Z') ch = (char)(ch + 32);
            auto key = std::make_tuple(m.part, m.kind, nc, s);
            auto it = atoms.find(key);
            uint32_t a;
            if (it == atoms.end()) {
                a = (uint32_t)atom_key.size();
                atoms.emplace(key, a);
                atom_key.push_back(key);
            } else {
                a = it->second;
            }
            m_atoms[i].push_back(a);
        }
        std::sort(m_atoms[i].begin(), m_atoms[i].end());
        m_atoms[i].erase(std::unique(m_atoms[i].begin(), m_atoms[i].end()), m_atoms[i].end());
        h->m_tmpl.push_back(m.tmpl);
        h->m_need.push_back((uint32_t)m_atoms[i].size());
        h->m_flags.push_back(m.flags);
    }
    for (uint32_t t = 0; t < n_templates; ++t)
        if (h->t_count[t] == 0) { set_error("template %u has no matchers", t); return SG_E_INVAL; }
    h->n_atoms = (uint32_t)atom_key.size();
    // atom -> matchers (CSR)
    std::vector<std::vector<uint32_t>> occ(h->n_atoms);
    for (uint32_t i = 0; i < n_matchers; ++i)
        for (uint32_t a : m_atoms[i]) occ[a].push_back(i);
    h->occ_off.assign(1, 0);
    for (auto &v : occ) {
        h->occ_m.insert(h->occ_m.end(), v.begin(), v.end());
        h->occ_off.push_back((uint32_t)h->occ_m.size());
    }
    h->atom_part.resize(h->n_atoms);
    // engines: (stream, kind, nocase) over the distinct pattern bytes of that group
    std::map<std::tuple<int, uint32_t, uint32_t>, std::map<std::string, std::vector<uint32_t>>> groups;
    for (uint32_t a = 0; a < h->n_atoms; ++a) {
        const auto &k = atom_key[a];
        h->atom_part[a] = std::get<0>(k);
        const std::string &s = std::get<3>(k);
        // a word holding '\n' can never occur inside a record or a row: it never hits
        if (std::get<1>(k) == SG_TM_WORD && s.find('\n') != std::string::npos) continue;
        const int stream = std::get<0>(k) == 0 ? 0 : 1;
        groups[std::make_tuple(stream, std::get<1>(k), std::get<2>(k))][s].push_back(a);
    }
    for (auto &g : groups) {
        TmRun run;
        run.stream = std::get<0>(g.first);
        const uint32_t kind = std::get<1>(g.first), nc = std::get<2>(g.first);
        std::vector<uint8_t> blob;
        std::vector<uint32_t> offs(1, 0);
        run.soff.assign(1, 0);
        for (auto &kv : g.second) {
            blob.insert(blob.end(), kv.first.begin(), kv.first.end());
            offs.push_back((uint32_t)blob.size());
            run.satoms.insert(run.satoms.end(), kv.second.begin(), kv.second.end());
            run.soff.push_back((uint32_t)run.satoms.size());
        }
        const uint32_t flags = nc ? SG_NOCASE : 0u;
        int rc = kind == SG_TM_WORD
                     ? sg_ac_compile(blob.data(), offs.data(), (uint32_t)(offs.size() - 1), flags, &run.m)
                     : sg_dfa_compile(blob.data(), offs.data(), (uint32_t)(offs.size() - 1), flags, &run.m);
        if (rc != SG_OK) {
            for (auto &r : h->runs) sg_free(r.m);
            return rc;
        }
        h->runs.push_back(std::move(run));
    }
    // vacuous templates: true with no evidence at all (every matcher count 0)
    for (uint32_t t = 0; t < n_templates; ++t) {
        const bool and_t = h->t_flags[t] & SG_TM_AND;
        bool acc = and_t;
        for (uint32_t m = h->t_first[t]; m < h->t_first[t] + h->t_count[t]; ++m) {
            const bool hit = (h->m_flags[m] & SG_TM_NEGATIVE) != 0;
            acc = and_t ? (acc && hit) : (acc || hit);
        }
        if (acc) h->vac.push_back(t);
    }
    h->vacm.assign((n_templates + 31) / 32, 0);
    for (uint32_t t : h->vac) h->vacm[t >> 5] |= 1u << (t & 31);
    uint32_t max_need = 0;
    for (uint32_t v : h->m_need) max_need = std::max(max_need, v);
    h->rec_wave = max_need <= 0xffu && n_matchers <= 0x7fffu && n_templates <= 0xffffu && h->occ_m.size() <= 0xffffu &&
                  tm_block_words(h->n_atoms, (uint32_t)h->occ_m.size(), n_matchers, n_templates) <= TMW_WORDS_MAX;
    if (h->rec_wave) {
        for (uint32_t m : h->occ_m) h->occ_mt.push_back(m | (h->m_tmpl[m] << 16));
        for (uint32_t t = 0; t < n_templates; ++t)
            h->tinfo.push_back(h->t_first[t] | (h->t_count[t] << 16) | ((h->t_flags[t] & SG_TM_AND) ? 1u << 31 : 0u));
        for (uint32_t a = 0; a <= h->n_atoms; a += 2)
            h->occ16.push_back(h->occ_off[a] | (a + 1 <= h->n_atoms ? h->occ_off[a + 1] << 16 : 0u));
        for (uint32_t m = 0; m < n_matchers; ++m)
            h->minfo.push_back(h->m_need[m] | ((h->m_flags[m] & SG_TM_AND) ? TMW_NEED_AND : 0u) |
                               ((h->m_flags[m] & SG_TM_NEGATIVE) ? TMW_NEED_NEG : 0u));
    }
    *out = h.release();
    return SG_OK;
}

int sg_tmpl_info(const sg_templates *h, uint32_t *n_atoms, uint32_t *n_engines, uint32_t *n_vacuous) {
    if (!h) return SG_E_INVAL;
    if (n_atoms) *n_atoms = h->n_atoms;
    if (n_engines) *n_engines = (uint32_t)h->runs.size();
    if (n_vacuous) *n_vacuous = (uint32_t)h->vac.size();
    return SG_OK;
}

int sg_dev_tmpl_eval_rows(sg_ctx *c, sg_templates *h, const uint8_t *d_buf, size_t n, const sg_dev_rows *rows,
                          sg_dev_tmatches *res) {
    if (!c || !h || !res || !rows || (!d_buf && n)) { set_error("sg_dev_tmpl_eval_rows: bad arguments"); return SG_E_INVAL; }
    if (n > MAX_BYTES) { set_error("input exceeds 4 GiB per call"); return SG_E_TOO_LARGE; }
    if (((uintptr_t)d_buf & 15) != 0) { set_error("sg_dev_tmpl_eval_rows: d_buf must be 16-byte aligned"); return SG_E_INVAL; }
    SG_HIP(hipSetDevice(c->device));
    return dev_tmpl_eval(c, h, d_buf, n, res, rows);
}

int sg_dev_tmpl_eval(sg_ctx *c, sg_templates *h, const uint8_t *d_buf, size_t n, sg_dev_tmatches *res) {
    if (!c || !h || !res || (!d_buf && n)) { set_error("sg_dev_tmpl_eval: bad arguments"); return SG_E_INVAL; }
    if (n > MAX_BYTES) { set_error("input exceeds 4 GiB per call"); return SG_E_TOO_LARGE; }
    SG_HIP(hipSetDevice(c->device));
    const uint8_t *b = d_buf;
    if (((uintptr_t)d_buf & 15) != 0) {
        uint8_t *a;
        SG_TRY(slot(c, S_IN, n + 16, &a));
        if (n) SG_HIP(hipMemcpyAsync(a, d_buf, n, hipMemcpyDeviceToDevice, c->stream));
        b = a;
    }
    return dev_tmpl_eval(c, h, b, n, res);
}

int sg_tmpl_eval(sg_templates *h, const uint8_t *buf, size_t n, uint32_t *rec_idx, uint32_t *tmpl_id, size_t cap,
                 size_t *n_out) {
    if (!h || !n_out || (!buf && n)) { set_error("sg_tmpl_eval: bad arguments"); return SG_E_INVAL; }
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
    sg_dev_tmatches r;
    SG_TRY(dev_tmpl_eval(c, h, d, n, &r));
    *n_out = r.n;
    if (r.n > cap) { SG_HIP(hipStreamSynchronize(c->stream)); set_error("output capacity too small"); return SG_E_CAP; }
    if (r.n) {
        SG_HIP(hipMemcpyAsync(rec_idx, r.rec_idx, 4 * r.n, hipMemcpyDeviceToHost, c->stream));
        SG_HIP(hipMemcpyAsync(tmpl_id, r.tmpl_id, 4 * r.n, hipMemcpyDeviceToHost, c->stream));
    }
    SG_HIP(hipStreamSynchronize(c->stream));
    return SG_OK;
}

void sg_tmpl_free(sg_templates *h) {
    if (!h) return;
    for (int dv = 0; dv < TM_MAX_DEV; ++dv)
        if (h->d[dv].ready) { (void)hipSetDevice(dv); tm_free_dev(h->d[dv]); }
    for (auto &r : h->runs) sg_free(r.m);
    delete h;
}

}  // extern "C"
