// sg_internal.hpp — host-side internal API shared by the libswarmgpu translation units.
#pragma once
#include "sg_common.hpp"

namespace sg {

int pool_acquire(int device, sg_ctx **out);
void pool_release(sg_ctx *c);
int pick_device(int *dev);

// Exclusive scan of nt per-tile u64 aggregates into pre; the sum into *total (device).
// pre[t] = init + exclusive prefix of tot (packed (count << 32 | bytes) aggregates: init
// shifts the byte offsets, e.g. to a destination that starts mid-word); total excludes init.
int tile_scan(sg_ctx *c, const uint64_t *tot, uint32_t nt, uint64_t *pre, uint64_t *total, uint64_t init = 0);

// Slot sets let the cur and prior buffers be parsed/sorted without sharing buffers.
struct SlotSet {
    int starts, ends, keys, keys2, vals, vals2, uniq, lb;
};
extern const SlotSet CUR_SLOTS;
extern const SlotSet PRIOR_SLOTS;

// A3 parse result (device arrays, n_rec records).
struct Lines {
    uint2 *spans = nullptr;     // (start, end) per record, interleaved: one 8-B load per record
    uint64_t *keys = nullptr;   // chunk_key(rec, 0) (null when not requested)
    uint32_t n_rec = 0;
    // Exclusive packed (starts << 31 | ends) record-boundary counts before tile t (tiles of
    // tile_bytes bytes): the tile prefixes of the parse's reduce-then-scan.
    const uint64_t *tile_excl = nullptr;
    uint32_t tile_bytes = 0, n_tiles = 0;
    // Keys at offset spec_off (the context's last common prefix, >= 8) written by whoever
    // gathered the records (X1's matched records), with their per-block KeyStatD partials:
    // used when the common prefix comes out at spec_off again (sg_dedup.hip).
    uint64_t *spec_keys = nullptr;
    const struct KeyStatD *spec_parts = nullptr;
    uint32_t spec_off = 0, spec_nparts = 0;
    // A parse handed over by another call (sg_dev_dedup_diff_spans_into): checked by the
    // dedup's prefix scan before anything indexes the bytes with it (records tile the buffer,
    // sum of span_mix terms == chk_sum, sampled records end at a '\n' and match their keys).
    bool chk = false;
    uint64_t chk_sum = 0;
};
// Split d_buf (16-byte aligned device pointer, n bytes) into non-empty records.
// apply = false: count and allocate only; the spans are then written by a consumer that
// re-reads the same tiles anyway (k_lit_scan with LitArgs::spans_out).
int run_lines2(sg_ctx *c, const uint8_t *a, uint64_t na, const SlotSet &sa, Lines *la, const uint8_t *b, uint64_t nb,
               const SlotSet &sb, Lines *lb);
int run_lines(sg_ctx *c, const uint8_t *d_buf, uint64_t n, const SlotSet &ss, Lines *out, bool want_keys = true,
              bool apply = true);
// The piece partition's parse with routing (sg_lines.hip): count + tile scan into tp (2 x
// lines_tiles(n) + 4 words; packed record count at tp[2 x nt]), then spans + part bytes.
uint32_t lines_tiles(uint64_t n);
int lines_count_scan(sg_ctx *c, const uint8_t *d_buf, uint64_t n, uint64_t *tp);
int lines_route_apply(sg_ctx *c, const uint8_t *d_buf, uint64_t n, const uint64_t *tp, uint32_t R, uint2 *spans,
                      const uint64_t *split_w, const uint32_t *split_len, uint32_t ns, uint8_t *parts);

// LSD radix sort of (u64 key, u32 val) pairs on bits [begin_bit, end_bit), stable.
// Ping-pongs between (keys, vals) and (keys_alt, vals_alt); returns the final arrays.
// iota_vals: vals[i] = i is implied on input (vals need not be initialised).
// What the caller already knows about the keys of a sort over bits [0, 64):
//   vary   : OR ^ AND over every key — the bits that differ between two keys (exact; a digit
//            position with no varying bit is a trivial pass, skipped);
//   hist   : host copy of the 8 digit histograms of a SAMPLE of hist_n keys (key_sample_hist),
//            used only to plan (never as offsets).
struct KeyStats {
    uint64_t vary = ~0ull;
    const uint32_t *hist = nullptr;
    uint32_t hist_n = 0;
};
// Device form of the keys' varying bits and tag range (per-block partials, then combined).
struct KeyStatD {
    unsigned long long o, a;  // OR, AND over the keys
    uint32_t tmin, tmax;      // the tag byte's range
};
// Stable sort of (key, span) pairs: the spans themselves are the payload (no id gather after).
int radix_sort_spans(sg_ctx *c, uint64_t *keys, uint2 *spans, uint64_t *keys_alt, uint2 *spans_alt, uint32_t n,
                     int begin_bit, int end_bit, uint64_t **keys_out, uint2 **spans_out,
                     const char *pass_name = "rs_pass", const KeyStats *ks = nullptr,
                     uint32_t narrow_kw = 0, uint32_t **lsort_err = nullptr, uint32_t *err_at = nullptr);
// lsort_err (with ks->hist): allows the hybrid sort (global passes over the top digits, the
// rest per group in one block's LDS). The tiles one window cannot hold are redone right behind
// the local sort, in the same stream (k_rs_lsort_fix over the listed tiles); *lsort_err is then
// the device word counting the groups too large for any window ("big groups": the pairs there
// are a valid permutation but not sorted), and the caller that reads it nonzero must run
// lsort_fixup_big (null when the plain LSD sort ran). err_at: the device words to use (2: the
// big-group count, then the count of tiles redone), e.g. beside the caller's other counters.
// The hybrid sort's big groups (listed by its fix-up pass) sorted from the local sort's input
// (Kin, Vin: the pairs after the global passes) into (Ko, Vo) by one stable radix sort of
// their members on (group, local digits). Uses the ctx's last hybrid plan (c->ls_last).
int lsort_fixup_big(sg_ctx *c, const uint64_t *Kin, const uint2 *Vin, uint64_t *Ko, uint2 *Vo, uint32_t n, uint32_t B);
// Queue the digit histograms of a row sample of the keys into dev_hist (8 x 256 u32, zeroed
// by the caller); *sample_n = the keys counted. With parts: the nparts per-block KeyStatD
// partials of an earlier kernel are combined into *st in the same launch.
int key_sample_hist(sg_ctx *c, const uint64_t *keys, uint32_t n, uint32_t *dev_hist, uint32_t *sample_n,
                    const KeyStatD *parts = nullptr, uint32_t nparts = 0, KeyStatD *st = nullptr);
int radix_sort(sg_ctx *c, uint64_t *keys, uint32_t *vals, uint64_t *keys_alt, uint32_t *vals_alt,
               uint32_t n, int begin_bit, int end_bit, bool iota_vals,
               uint64_t **keys_out, uint32_t **vals_out, const char *pass_name = "rs_pass");

// Compaction: indices i < n with flag[i] != 0, in order. Returns count.
int select_flags(sg_ctx *c, const uint8_t *flags, uint32_t n, uint32_t *out_idx, uint32_t *count);

// Serialize records (ids into starts/ends, in list order) as '\n'-terminated bytes.
// rec_of: list[i] is a position into `map` (if map != null) giving the record id.
int serialize(sg_ctx *c, const uint8_t *d_buf, const uint2 *spans,
              const uint32_t *list, const uint32_t *map, uint32_t count, int out_slot,
              uint8_t **d_out, uint64_t *bytes);
// Same, into a caller buffer of dst_cap bytes (SG_E_CAP if too small).
int emit_into(sg_ctx *c, const uint8_t *d_buf, const uint2 *spans, const uint32_t *recs, uint32_t count,
              uint8_t *dst_base, uint32_t shift);
int dev_dedup_diff_into(sg_ctx *c, const uint8_t *d_cur, uint64_t n_cur, const uint8_t *d_prior, uint64_t n_prior,
                        uint8_t *d_uniq, size_t uniq_cap, uint8_t *d_fresh, size_t fresh_cap, sg_dev_result *res);
int serialize_into(sg_ctx *c, const uint8_t *d_buf, const uint2 *spans,
                   const uint32_t *recs, uint32_t count, uint8_t *dst, size_t dst_cap, uint64_t *bytes);

// A7+A8 on device buffers (sg_dedup.hip): the radix pipeline.
int dev_dedup_diff(sg_ctx *c, const uint8_t *d_cur, uint64_t n_cur, const uint8_t *d_prior, uint64_t n_prior,
                   bool want_fresh, sg_dev_result *res);

// A4 matching of a device line buffer (sg_match.hip); want_lines = false skips the grep
// output (hits only).
// Literal-only matchers, fused step: the scan marks matched records in a per-record flag
// array (no (record, signature) list, no hit sort); the parse's spans come back with it.
struct MatchFlags {
    Lines L;
    uint8_t *flags = nullptr;
    uint64_t *key0 = nullptr, *raw7 = nullptr;  // every record's key0 and bytes 7..14 (from the scan)
};
int dev_match(sg_ctx *c, sg_matcher *h, const uint8_t *d_buf, uint64_t n, sg_dev_hits *res, bool want_lines,
              MatchFlags *mf = nullptr, Lines *reuse = nullptr);
// dev_dedup_diff (radix pipeline) for a current scan given as already parsed records of
// d_cur (spans + key0 from byte 0), e.g. the matched subset of a larger buffer.
// dev_dedup_diff_into with cur's records already parsed (spans + byte-0 keys).
int dev_dedup_diff_into_lines(sg_ctx *c, const uint8_t *d_cur, uint64_t n_cur, const Lines &cur, const uint8_t *d_prior,
                              uint64_t n_prior, uint8_t *d_uniq, size_t uniq_cap, uint8_t *d_fresh, size_t fresh_cap,
                              sg_dev_result *res);
int dev_dedup_diff_lines(sg_ctx *c, const uint8_t *d_cur, uint64_t n_cur, const Lines &cur, const uint8_t *d_prior,
                         uint64_t n_prior, sg_dev_result *res, const uint32_t *cur_lcp = nullptr);
// httpx -json field rows (sg_formats.hip).
int dev_json_fields(sg_ctx *c, const uint8_t *d_buf, uint64_t n, const uint8_t *keys, const uint32_t *key_offs,
                    uint32_t nkeys, sg_dev_rows *res);

}  // namespace sg
