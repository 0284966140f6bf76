/*
 * swarmgpu.h — C-ABI of libswarmgpu.so, the MI355X (gfx950) scan-result hot path.
 *
 * The reference (Jec00/swarm) has no native code and no FFI: its hot path is Python
 * (server/server.py, worker/worker.py) around third-party scanners. Each entry point
 * below replaces one reference step; the citation says which. Python binds these with
 * ctypes (swarm_amd/_abi.py); INTEGRATION.md shows the binding a maintainer would add to
 * the reference's worker.py / server.py.
 *
 * Conventions
 *   - Every function returns an int status: SG_OK (0) or an SG_E_* code. No exception
 *     crosses the ABI. sg_last_error() returns a thread-local message for the last error.
 *   - Host-buffer entry points (no `_dev` suffix) take host pointers owned by the caller;
 *     the library copies to HBM, computes, and copies back. If `cap` is too small they
 *     return SG_E_CAP and store the required size in the *_n out-parameter.
 *   - Device entry points (`sg_dev_*`) take device pointers on the context's device and
 *     enqueue on the context's stream; their outputs are device buffers owned by the
 *     context, valid until the next call on that context.
 *   - Re-entrant: the host API draws a context from a mutex-guarded per-device pool, so
 *     concurrent Flask request threads (flask/app.py threaded=True) may call it. A
 *     single sg_ctx must not be used by two threads at once.
 *   - Record = maximal run of non-'\n' bytes; empty records are dropped; '\r' is kept
 *     (SURVEY.md §8(a) A3). Ordering is bytewise (memcmp, shorter-prefix first), i.e.
 *     Python bytes order == LC_ALL=C sort.
 *   - Buffers are < 4 GiB per call (32-bit record offsets); larger inputs are split by
 *     the caller or sharded over GPUs (sg_dev_partition).
 */
#ifndef SWARMGPU_H
#define SWARMGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SG_OK 0
#define SG_E_INVAL 1        /* bad argument */
#define SG_E_CAP 2          /* output capacity too small; required size returned */
#define SG_E_HIP 3          /* HIP runtime error */
#define SG_E_NOMEM 4        /* device or host allocation failed */
#define SG_E_TOO_LARGE 5    /* buffer >= 4 GiB */
#define SG_E_UNSUPPORTED 6  /* regex construct outside the supported subset */
#define SG_E_STATES 7       /* automaton exceeds its state budget */
#define SG_E_NODEV 8        /* no HIP device */
#define SG_E_CORRUPT 9      /* a handed-over parse does not match its bytes (sg_dev_dedup_diff_spans_into) */

/* matcher flags */
#define SG_NOCASE 1u        /* ASCII case-insensitive (nuclei `case-insensitive: true`, grep -i) */

const char *sg_last_error(void);
int sg_version(void);
int sg_device_count(int *n);

/* ------------------------------------------------------------------ contexts */
typedef struct sg_ctx sg_ctx;
/* stream: a hipStream_t on `device` (e.g. torch.cuda.current_stream().cuda_stream),
 * SG_NULL_STREAM for the device's null (legacy default) stream — the one torch uses unless
 * told otherwise, whose handle reads as 0 — or NULL for a context-owned non-blocking
 * stream (which does not order against the null stream: the caller synchronises). */
#define SG_NULL_STREAM ((void *)-1)
int sg_ctx_create(int device, void *stream, sg_ctx **out);
int sg_ctx_destroy(sg_ctx *ctx);
int sg_ctx_sync(sg_ctx *ctx);
/* Per-kernel HIP-event timing, recorded on the context's stream while enabled. */
int sg_ctx_profile(sg_ctx *ctx, int enable);
/* Restrict event timing to launches named `name` (NULL or "": all launches). */
int sg_ctx_profile_only(sg_ctx *ctx, const char *name);
/* Kernel stats by index: name (static string), launches, total device ms and the total
 * algorithmic bytes those launches moved (0 where not modelled). Returns SG_E_INVAL past
 * the last index. */
int sg_ctx_kernel_stat(sg_ctx *ctx, int idx, const char **name, uint64_t *launches, double *total_ms,
                       double *total_bytes);
int sg_ctx_reset_stats(sg_ctx *ctx);
/* Synchronous copy on the context's stream (any direction: hipMemcpyDefault). */
int sg_ctx_memcpy(sg_ctx *ctx, void *dst, const void *src, size_t n);
/* Which dedup/diff pipeline served the context's last sg_dev_dedup_diff: *path = 0, the radix
 * pipeline — since round 3 the only one in the library (the bucket sample sort and the probe
 * path, both measured slower, live in tools/experiments/); *flags: bit 0 (SG_SORT_HYBRID) the
 * current scan's sort ran its top digits globally and finished each group in LDS, bit 1
 * (SG_SORT_RESORTED) the plain LSD sort ran again, bit 2 (SG_SORT_FIXUP) a group outgrew the
 * local sort's LDS and its tiles were sorted again, bit 3 (SG_SEG_ALL) the all-segments mode
 * (every segment of 2+ records ranked by the segment sorts, no adjacent byte compare). For
 * tests/benchmarks. */
#define SG_SORT_HYBRID 1u
#define SG_SORT_RESORTED 2u
#define SG_SORT_FIXUP 4u
#define SG_SEG_ALL 8u
#define SG_PATH_RADIX 0
int sg_ctx_last_path(sg_ctx *ctx, int *path, uint32_t *flags);
/* Sort-key width (bytes after the common prefix, 5..7) the last radix dedup chose from the
 * keys' byte entropies. For tests and benchmarks. */
int sg_ctx_last_key_width(sg_ctx *ctx, uint32_t *kw);

/* ------------------------------------------------------------------ A3: parse
 * Replaces: nothing in the reference parses module output; it is uploaded verbatim at
 * worker/worker.py:96-98. Output: spans[2k] = start, spans[2k+1] = end (exclusive) of the
 * k-th non-empty record. cap counts records. */
int sg_lines(const uint8_t *buf, size_t n, uint64_t *spans, size_t cap, size_t *n_rec);

/* ------------------------------------------------------------------ A5+A7: merge + dedup
 * sort -u of the concatenation of `k` chunk bodies taken in the given order (the caller
 * supplies server/server.py:403-404's key order; concatenation without separator is
 * :407-410). Output is the unique records in byte order, each '\n'-terminated.
 * Replaces the planned dedup of README.md:11 (semantics: BASELINE.json north_star). */
int sg_dedup(const uint8_t *buf, size_t n, uint8_t *out, size_t cap, size_t *out_n);
int sg_dedup_chunks(const uint8_t *const *chunks, const size_t *lens, size_t k,
                    uint8_t *out, size_t cap, size_t *out_n);

/* ------------------------------------------------------------------ A8: new-record diff
 * sorted(set(cur) - set(prior)) == LC_ALL=C comm -13 (README.md:11 "alerting ... new
 * subdomains"; prior scan resolved from asm.scans, server/server.py:277-294). `prior` is
 * normally the previous scan's sort -u output; unsorted/duplicated priors are accepted
 * (they are sorted on the GPU first). */
int sg_diff(const uint8_t *cur, size_t n_cur, const uint8_t *prior, size_t n_prior,
            uint8_t *out, size_t cap, size_t *out_n);
/* Both at once (the scan-completion hook, server/server.py:274-294). */
int sg_dedup_diff(const uint8_t *cur, size_t n_cur, const uint8_t *prior, size_t n_prior,
                  uint8_t *uniq, size_t uniq_cap, size_t *uniq_n,
                  uint8_t *fresh, size_t fresh_cap, size_t *fresh_n);

/* ------------------------------------------------------------------ device-resident path */
typedef struct sg_dev_result {
    const uint8_t *uniq;      /* device: sort -u output */
    uint64_t uniq_bytes;
    uint64_t uniq_records;
    const uint8_t *fresh;     /* device: new records (cur - prior), sorted */
    uint64_t fresh_bytes;
    uint64_t fresh_records;
    uint64_t in_records;      /* non-empty records in cur */
    uint64_t prior_records;   /* non-empty records in prior */
} sg_dev_result;
/* d_prior may be NULL with n_prior 0 (then fresh == uniq). */
int sg_dev_dedup_diff(sg_ctx *ctx, const uint8_t *d_cur, size_t n_cur,
                      const uint8_t *d_prior, size_t n_prior, sg_dev_result *res);
/* sg_dev_dedup_diff writing its two outputs into caller device memory at any byte address
 * (capacities >= n_cur + 1 each): res->uniq = d_uniq, res->fresh = d_fresh (d_fresh may be NULL:
 * then res->fresh aliases d_uniq when there is no prior, and new records go to a context
 * buffer otherwise). Consecutive calls can append part outputs to one result buffer without a
 * copy (swarm_amd.sharded). */
int sg_dev_dedup_diff_into(sg_ctx *ctx, const uint8_t *d_cur, size_t n_cur, const uint8_t *d_prior,
                           size_t n_prior, uint8_t *d_uniq, size_t uniq_cap, uint8_t *d_fresh,
                           size_t fresh_cap, sg_dev_result *res);
/* sg_dev_dedup_diff_into for a 16-byte aligned d_cur already parsed by
 * sg_dev_partition_bytes_pieces_spans / _rounds_spans (a part's, or an exchange round's,
 * n_rec spans and keys): no second parse. The handed-over parse is checked before any kernel
 * reads a byte through it, in the pass that already reads every key (the common-prefix
 * scan), and a mismatch returns SG_E_CORRUPT with nothing written:
 *   - the records tile d_cur in order: record 0 starts at 0, record i + 1 starts right after
 *     record i's '\n' (end + 1), every record is non-empty, the last '\n' is byte n_cur - 1
 *     (so every span lies inside the buffer whatever arrived);
 *   - sg_span_sum(spans, keys) == span_sum, the producer's checksum (part_sums of the
 *     partition calls, summed over the sources of an exchange round): a changed key or length
 *     is caught;
 *   - every 256th record ends at a '\n' of d_cur and its key equals its own bytes' key.
 * n_rec == 0 requires n_cur == 0 and span_sum == 0. d_spans and d_keys are consumed: the
 * sort works in them (their contents are unspecified afterwards). */
int sg_dev_dedup_diff_spans_into(sg_ctx *ctx, const uint8_t *d_cur, size_t n_cur, uint32_t *d_spans,
                                 uint64_t *d_keys, size_t n_rec, uint64_t span_sum, const uint8_t *d_prior,
                                 size_t n_prior, uint8_t *d_uniq, size_t uniq_cap, uint8_t *d_fresh, size_t fresh_cap,
                                 sg_dev_result *res);
/* The handover checksum of n_rec records (host arrays: spans as 2 x uint32 start, end;
 * first-chunk keys): the sum mod 2^64 over records of mix(end - start, key), with
 *   h = (k + l * 0x9E3779B97F4A7C15) * 0xBF58476D1CE4E5B9 (mod 2^64); mix = h ^ h >> 31.
 * Order-free, so producers sum it per tile and receivers per call. It detects transport
 * damage (any one changed key or length; stale, truncated or shifted runs), not a deliberate
 * exchange of two equal-length records' keys. */
uint64_t sg_span_sum(const uint32_t *spans, const uint64_t *keys, size_t n_rec);

/* Multi-GPU: route every record of d_buf to partition
 * part(hash64(record), n_parts), n_parts <= 256. Writes '\n'-terminated records grouped by
 * partition (input order kept inside a partition) into the caller's device buffer d_out
 * (capacity out_cap >= n + 1) and the per-partition byte and record counts (host arrays
 * of n_parts), ready for an all-to-all. */
int sg_dev_partition(sg_ctx *ctx, const uint8_t *d_buf, size_t n, uint32_t n_parts,
                     uint8_t *d_out, size_t out_cap, uint64_t *part_bytes, uint64_t *part_records);
/* Range routing: part(record) = number of splitters <= key0(record), where key0 = the
 * record's first 7 bytes big-endian << 8 | min(len, 8) (a key0 order is a
 * byte order). splitters: n_parts - 1 non-decreasing host values. Part p's records all sort
 * below part p+1's, so per-part sort -u outputs concatenated in part order are the global
 * sort -u output: the way a shard larger than one 4 GiB call, or a global byte order
 * across GPUs, is processed. Same output layout as sg_dev_partition. */
int sg_dev_partition_range(sg_ctx *ctx, const uint8_t *d_buf, size_t n, const uint64_t *splitters,
                           uint32_t n_parts, uint8_t *d_out, size_t out_cap, uint64_t *part_bytes,
                           uint64_t *part_records);
/* m evenly spaced records' key0 values (host array; ~0 when the buffer has no records), for
 * choosing splitters; *n_rec = the buffer's record count. */
int sg_dev_key_sample(sg_ctx *ctx, const uint8_t *d_buf, size_t n, uint32_t m, uint64_t *keys,
                      uint64_t *n_rec);
/* Range routing by byte-string splitters: part(record) = number of splitters <= record in
 * bytewise order (a shorter string that is a prefix of a longer one sorts first, as in sort).
 * Splitter q is splitters[split_offs[q] .. split_offs[q+1]) (n_parts entries in split_offs),
 * cut to its first SG_SPLIT_BYTES bytes; the cut splitters must be non-decreasing. Equal
 * records share a part and every record of part p sorts below every record of part p+1, so
 * the per-part sort -u outputs concatenated in part order are the global sort -u output;
 * unlike key0 splitters, byte splitters divide runs of records sharing their first 7 bytes
 * (https://..., 10.0.x.y:port). Same output layout as sg_dev_partition. */
#define SG_SPLIT_BYTES 64
int sg_dev_partition_bytes(sg_ctx *ctx, const uint8_t *d_buf, size_t n, const uint8_t *splitters,
                           const uint32_t *split_offs, uint32_t n_parts, uint8_t *d_out, size_t out_cap,
                           uint64_t *part_bytes, uint64_t *part_records);
/* Range routing of k pieces (each < 4 GiB, ending at a record boundary) into ONE device
 * buffer d_out (capacity >= the pieces' bytes + 1 each), part-contiguous across pieces: part
 * p = the part-p records of piece 0, then of piece 1, ... (input order kept inside a piece),
 * so every part is one contiguous range ready for a dedup call (replaces per-piece routing
 * followed by a concatenation). part_bytes / part_records: totals over the pieces. */
int sg_dev_partition_bytes_pieces(sg_ctx *ctx, const uint8_t *const *d_pieces, const size_t *lens, size_t k,
                                  const uint8_t *splitters, const uint32_t *split_offs, uint32_t n_parts,
                                  uint8_t *d_out, size_t out_cap, uint64_t *part_bytes, uint64_t *part_records);
/* Same, with part p starting at the 16-byte aligned offset after part p - 1's bytes (d_out
 * 16-byte aligned; capacity >= the pieces' bytes + 1 each + 16 per part): every part is a
 * dedup-ready aligned buffer, used in place with no staging copy. */
int sg_dev_partition_bytes_pieces_a16(sg_ctx *ctx, const uint8_t *const *d_pieces, const size_t *lens, size_t k,
                                      const uint8_t *splitters, const uint32_t *split_offs, uint32_t n_parts,
                                      uint8_t *d_out, size_t out_cap, uint64_t *part_bytes, uint64_t *part_records);
/* The _a16 routing that also hands over every part's parse: *d_spans (context-owned, valid
 * until the next _spans call on ctx) holds 2 x uint32 (start, end of the record before its
 * '\n', relative to its part's start) per record and *d_keys its first-chunk sort key,
 * part p's records at [sum of part_records[< p], + part_records[p]), in part order.
 * part_sums (host array of n_parts, may be NULL): part p's handover checksum (sg_span_sum of
 * its records' spans and keys), for sg_dev_dedup_diff_spans_into; computed in the copy pass,
 * so with part_sums the call returns after that pass instead of queueing it. */
int sg_dev_partition_bytes_pieces_spans(sg_ctx *ctx, const uint8_t *const *d_pieces, const size_t *lens,
                                        size_t k, const uint8_t *splitters, const uint32_t *split_offs,
                                        uint32_t n_parts, uint8_t *d_out, size_t out_cap, uint64_t *part_bytes,
                                        uint64_t *part_records, const uint32_t **d_spans, const uint64_t **d_keys,
                                        uint64_t *part_sums);
/* Range routing for a multi-GPU exchange in rounds (swarm_amd.distributed.dedup_diff_rounds_step):
 * n_parts = G x rounds byte-range parts, part q = g * rounds + p being local range p of rank g
 * (so rank g owns parts g * rounds .. g * rounds + rounds - 1, in byte order). The parts are
 * laid out ROUND-major in d_out: round p = parts (0, p), (1, p), ..., (G - 1, p) back to back,
 * each round starting at a 16-byte aligned offset, so one round is one contiguous
 * all-to-all send buffer whose split sizes are part_bytes[g * rounds + p]; the receiver's
 * buffer for round p is then its local range p, whole. Capacity >= the pieces' bytes + 1 each
 * + 16 per round. part_bytes / part_records in part order. Replaces the per-piece routing +
 * exchange + local re-routing of the round-2 path (server/server.py:185-187's chunk
 * parallelism, across GPUs). */
int sg_dev_partition_bytes_pieces_rounds(sg_ctx *ctx, const uint8_t *const *d_pieces, const size_t *lens, size_t k,
                                         const uint8_t *splitters, const uint32_t *split_offs, uint32_t n_parts,
                                         uint32_t rounds, uint8_t *d_out, size_t out_cap, uint64_t *part_bytes,
                                         uint64_t *part_records);
/* Pass 0 of a piece partition on its own: *n_records = the pieces' total record count, so a
 * caller can size the span buffers of sg_dev_partition_bytes_pieces_rounds_spans; the counts
 * are kept in ctx and reused by the next partition call on the same pieces. */
int sg_dev_partition_pieces_count(sg_ctx *ctx, const uint8_t *const *d_pieces, const size_t *lens, size_t k,
                                  uint64_t *n_records);
/* sg_dev_partition_bytes_pieces_rounds that also hands over every record's parse, for the
 * receivers of the exchange (no second parse of the received parts): d_spans (2 x uint32 per
 * record: start, end before its '\n', relative to its part's start) and d_keys (first-chunk
 * sort key), records in the round-major part order of the bytes; capacity rec_cap records.
 * part_sums (host, n_parts, may be NULL): each part's handover checksum, as in
 * sg_dev_partition_bytes_pieces_spans; it travels with the part's size and record count, and
 * a receiver passes the sum over its sources to sg_dev_dedup_diff_spans_into. */
int sg_dev_partition_bytes_pieces_rounds_spans(sg_ctx *ctx, const uint8_t *const *d_pieces, const size_t *lens,
                                               size_t k, const uint8_t *splitters, const uint32_t *split_offs,
                                               uint32_t n_parts, uint32_t rounds, uint8_t *d_out, size_t out_cap,
                                               uint64_t *part_bytes, uint64_t *part_records, uint32_t *d_spans,
                                               uint64_t *d_keys, size_t rec_cap, uint64_t *part_sums);
/* Received spans of nseg sources made relative to the receive buffer d_buf: records
 * [seg_first[s], seg_first[s + 1]) get + seg_off[s] (host arrays, seg_first[0] == 0; one
 * launch per SG_REBASE_SEGS sources). *bad = how many of each source's first and last 256
 * records do not end right before a '\n' of d_buf afterwards (0 for an intact transfer; a
 * short or stale message is caught at its tail; sg_dev_dedup_diff_spans_into then checks
 * every record). */
#define SG_REBASE_SEGS 64
int sg_dev_rebase_spans(sg_ctx *ctx, const uint8_t *d_buf, size_t n, uint32_t *d_spans, size_t n_rec,
                        const uint64_t *seg_first, const uint64_t *seg_off, uint32_t nseg, uint64_t *bad);
/* m evenly spaced records' first SG_SPLIT_BYTES bytes (heads: m x SG_SPLIT_BYTES host bytes,
 * zero-filled) and min(len, SG_SPLIT_BYTES) (lens), for choosing byte splitters; nothing is
 * written when the buffer has no records; *n_rec = the buffer's record count. */
int sg_dev_record_sample(sg_ctx *ctx, const uint8_t *d_buf, size_t n, uint32_t m, uint8_t *heads,
                         uint32_t *lens, uint64_t *n_rec);
/* The record hash used by sg_dev_partition, on one host record (for tests/oracles). */
uint64_t sg_hash64(const uint8_t *rec, size_t len);

/* ------------------------------------------------------------------ A4: signature matching
 * Patterns are concatenated in `pats`; pattern i is pats[pat_offs[i] .. pat_offs[i+1]).
 * Match output: (record index, signature id) for every signature that occurs in a record,
 * sorted by record then signature; record indices follow A3 order. Replaces the matcher
 * arithmetic of the absent nuclei/httpx/nmap binaries (worker/modules/nuclei.json:2,
 * httpx.json:2, nmap.json:2) with grep -F / re.search semantics. */
typedef struct sg_matcher sg_matcher;
int sg_ac_compile(const uint8_t *pats, const uint32_t *pat_offs, uint32_t n_pats,
                  uint32_t flags, sg_matcher **h);
int sg_dfa_compile(const uint8_t *pats, const uint32_t *pat_offs, uint32_t n_pats,
                   uint32_t flags, sg_matcher **h);
/* Compiled-automaton facts: states and groups (DFA count; 1 for Aho-Corasick). */
int sg_matcher_info(const sg_matcher *h, uint64_t *states, uint32_t *groups, uint32_t *n_pats);
int sg_match(sg_matcher *h, const uint8_t *buf, size_t n, uint64_t *rec_idx, uint32_t *sig_id,
             size_t cap, size_t *n_hit);
/* grep output: the matched records in input order, each '\n'-terminated. */
int sg_match_lines(sg_matcher *h, const uint8_t *buf, size_t n, uint8_t *out, size_t cap,
                   size_t *out_n);
/* Device form: hits stay in HBM (context-owned), plus the matched lines serialized in
 * input order (grep output). */
typedef struct sg_dev_hits {
    const uint32_t *rec_idx;  /* device */
    const uint32_t *sig_id;   /* device */
    uint64_t n_hits;
    const uint8_t *lines;     /* device: matched records, '\n'-terminated, input order */
    uint64_t lines_bytes;
    uint64_t matched_records;
    uint64_t in_records;
} sg_dev_hits;
int sg_dev_match(sg_ctx *ctx, sg_matcher *h, const uint8_t *d_buf, size_t n, sg_dev_hits *res);
/* The metric's fused step (BASELINE.json "match+dedup+diff"), device-resident end to end: raw
 * module output (worker/worker.py:83-98 uploads it verbatim) -> A3 parse -> A4 signature match
 * -> A7 sort -u of the MATCHED records (the /raw merge + dedup, server/server.py:399-412) ->
 * A8 the matched records new since the prior scan's matched set (README.md:11 alerting).
 * res: as sg_dev_dedup_diff over the matched records, with in_records = the input's records;
 * *n_hits = (record, signature) hits, *matched_records = records with at least one hit. The
 * hit arrays themselves are not returned (sg_dev_match gives them). d_prior may be NULL.
 * n_hits may be NULL: a literal matcher then only flags the matched records (no hit list or
 * hit sort), and the dedup runs on their spans in d_buf (no grep-output copy). */
int sg_dev_match_dedup_diff(sg_ctx *ctx, sg_matcher *h, const uint8_t *d_buf, size_t n, const uint8_t *d_prior,
                            size_t n_prior, sg_dev_result *res, uint64_t *n_hits, uint64_t *matched_records);
void sg_free(void *h);  /* frees an sg_matcher */

/* ------------------------------------------------------------------ module-output formats
 * the worker's module outputs (worker/modules/<name>.json:2) turned
 * into records on the GPU before matching (A4) and dedup (A7). */
typedef struct sg_dev_text {
    const uint8_t *data;      /* device: '\n'-terminated records (context-owned) */
    uint64_t bytes;
    uint64_t records;
    uint64_t in_records;      /* non-empty input lines */
} sg_dev_text;
/* nmap -oN (worker/modules/nmap.json:2) -> "host:port" records, one per open port, in
 * input order. Host = the text after "Nmap scan report for " up to the first space (the
 * name when nmap prints "NAME (IP)", else the address); an open-port line matches
 * [0-9]{1,5}/(tcp|udp|sctp)[ \t]+open([ \t]|$) at the start of a line; port lines before
 * any report line are dropped. */
int sg_nmap_ports(const uint8_t *buf, size_t n, uint8_t *out, size_t cap, size_t *out_n);
int sg_dev_nmap_ports(sg_ctx *ctx, const uint8_t *d_buf, size_t n, sg_dev_text *res);

typedef struct sg_dev_rows {
    const uint8_t *data;      /* device: rows, each '\n'-terminated (a line buffer) */
    uint64_t bytes;
    uint64_t rows;
    const uint32_t *row_rec;  /* device: input record of each row */
    const uint32_t *row_key;  /* device: requested-key index of each row */
    uint64_t in_records;
} sg_dev_rows;
/* httpx -json (worker/modules/http2.json:2, web.json:2) -> field rows. For every input
 * line that is one JSON object, and for each requested top-level key present (last
 * duplicate wins, as json.loads): a string value is one row of its decoded bytes (UTF-8;
 * a decoded newline is written as the two bytes '\' 'n'); an array value is one row per
 * element (strings decoded, other elements as their raw text); any other value is its raw
 * text. Empty rows are dropped. Rows are ordered by record, then key index, then element.
 * Lines that are not a single JSON object produce no rows. keys: n_keys (<= 64) names,
 * key i = keys[key_offs[i] .. key_offs[i+1]), total <= 4096 bytes, given in decoded
 * UTF-8 form: a member key written with escapes ("title", "ti\"tle") is decoded
 * before the comparison, as json.loads does. */
int sg_json_fields(const uint8_t *buf, size_t n, const uint8_t *keys, const uint32_t *key_offs,
                   uint32_t n_keys, uint8_t *out, size_t cap, size_t *out_n,
                   uint32_t *row_rec, uint32_t *row_key, size_t rows_cap, size_t *n_rows);
int sg_dev_json_fields(sg_ctx *ctx, const uint8_t *d_buf, size_t n, const uint8_t *keys,
                       const uint32_t *key_offs, uint32_t n_keys, sg_dev_rows *res);

/* ------------------------------------------------------------------ nuclei matcher logic
 * SURVEY.md §8(f) row 3. A template = matchers joined by `matchers-condition`
 * (technologies/tech-detect.yaml:16); a matcher = words or regexes joined by its
 * `condition`, optionally `negative` (file/audit/cisco/disable-ip-source-route.yaml:19-22)
 * and `case-insensitive` (technologies/typo3-detect.yaml:23), reading one part: 0 = the
 * record, k+1 = field key k of an httpx -json line (sg_json_fields rows; a pattern hits a
 * field when it occurs in any of its rows). `encoding: hex` words are passed decoded.
 * Semantics per part text: word = substring (case-insensitive: ASCII-folded), regex =
 * re.search; condition or = any, and = all; negative inverts the matcher; the template
 * joins its matchers with and/or. `dsl`, `status`, `size` matchers are out of scope. */
#define SG_TM_WORD 0u
#define SG_TM_REGEX 1u
#define SG_TM_AND 1u        /* condition: and (default: or); also the template flag */
#define SG_TM_NEGATIVE 2u
#define SG_TM_NOCASE 4u     /* case-insensitive words (regexes use (?i)) */
typedef struct sg_tm_matcher {
    uint32_t kind;          /* SG_TM_WORD | SG_TM_REGEX */
    uint32_t part;          /* 0 = record, k + 1 = field key k */
    uint32_t flags;         /* SG_TM_AND | SG_TM_NEGATIVE | SG_TM_NOCASE */
    uint32_t tmpl;          /* owning template (non-decreasing over the matcher array) */
    uint32_t first, count;  /* its patterns: pats[pat_offs[first] ..], count >= 1 */
} sg_tm_matcher;
typedef struct sg_templates sg_templates;
/* tmpl_flags[t]: SG_TM_AND for matchers-condition and. keys: field names for parts >= 1
 * (as sg_json_fields). */
int sg_tmpl_compile(const uint8_t *pats, const uint32_t *pat_offs, uint32_t n_pats,
                    const sg_tm_matcher *matchers, uint32_t n_matchers,
                    const uint32_t *tmpl_flags, uint32_t n_templates,
                    const uint8_t *keys, const uint32_t *key_offs, uint32_t n_keys,
                    sg_templates **h);
/* distinct atoms (part, kind, case, pattern), engines, templates true on empty evidence */
int sg_tmpl_info(const sg_templates *h, uint32_t *n_atoms, uint32_t *n_engines, uint32_t *n_vacuous);
typedef struct sg_dev_tmatches {
    const uint32_t *rec_idx;  /* device: record (A3 order) */
    const uint32_t *tmpl_id;  /* device: template */
    uint64_t n;               /* (record, template) pairs, sorted */
    uint64_t in_records;
} sg_dev_tmatches;
int sg_dev_tmpl_eval(sg_ctx *ctx, sg_templates *h, const uint8_t *d_buf, size_t n, sg_dev_tmatches *res);
/* sg_dev_tmpl_eval with the field rows already built: `rows` is the result of the caller's
 * own sg_dev_json_fields call on the same ctx, d_buf (16-byte aligned) and n, with the keys
 * the handle was compiled with, in the same order — the httpx -json fields step then parses
 * every line once for its rows and its template evaluation together. */
int sg_dev_tmpl_eval_rows(sg_ctx *ctx, sg_templates *h, const uint8_t *d_buf, size_t n, const sg_dev_rows *rows,
                          sg_dev_tmatches *res);
int sg_tmpl_eval(sg_templates *h, const uint8_t *buf, size_t n, uint32_t *rec_idx, uint32_t *tmpl_id,
                 size_t cap, size_t *n_out);
void sg_tmpl_free(sg_templates *h);

/* ------------------------------------------------------------------ streamed merge ingestion
 * instead of building the /raw body with `str +=`
 * (server/server.py:407-410), the server appends every chunk body — or each piece of one
 * as it streams from S3 — in the A5 key order (server/server.py:403-404). Pieces go
 * through two pinned staging buffers with async H2D copies on the context's stream, so
 * the merged body (concatenation, no separator, byte-identical to A5) is resident in HBM
 * when the last body ends. sg_ingest_finish returns the device buffer (owned by the
 * ingest handle, valid until sg_ingest_close) for sg_dev_dedup_diff / sg_dev_match. */
typedef struct sg_ingest sg_ingest;
int sg_ingest_open(sg_ctx *ctx, size_t size_hint, sg_ingest **out);
int sg_ingest_append(sg_ingest *s, const uint8_t *data, size_t n);
int sg_ingest_finish(sg_ingest *s, const uint8_t **d_buf, uint64_t *n);
int sg_ingest_close(sg_ingest *s);

#ifdef __cplusplus
}
#endif
#endif /* SWARMGPU_H */
