// sg_prims_host.hpp — host launchers for the reduce-then-scan primitives of sg_prims.hpp.
#pragma once
#include "sg_internal.hpp"
#include "sg_prims.hpp"

namespace sg {

// Order-preserving compaction of up to two predicates (one host sync for the counts).
// `bytes_per_item`: algorithmic bytes of one predicate evaluation (roofline accounting).
template <class Pred>
static int run_select2(sg_ctx *c, const char *name, Pred pred, uint32_t n, uint32_t *outA, uint32_t *outB,
                       uint32_t *cntA, uint32_t *cntB, double bytes_per_item = 8.0) {
    *cntA = 0;
    if (cntB) *cntB = 0;
    if (n == 0) return SG_OK;
    const uint32_t ntiles = (n + SEL_TILE - 1) / SEL_TILE;
    uint64_t *tp;  // tot | pre | total | maskA | maskB
    SG_TRY(slot(c, S_COUNT, 2 * (size_t)ntiles + 4 + 2 * (size_t)ntiles * SEL_MASKS, &tp));
    uint64_t *tot = tp, *pre = tp + ntiles, *total = tp + 2 * (size_t)ntiles;
    uint64_t *mA = tp + 2 * (size_t)ntiles + 4, *mB = mA + (size_t)ntiles * SEL_MASKS;
    SG_LAUNCH(c, name, k_sel_count<Pred>, ntiles, SEL_BLOCK, 0, pred, n, mA, mB, tot);
    SG_TRY(tile_scan(c, tot, ntiles, pre, total));
    SG_LAUNCH(c, "select.apply", k_sel_apply, ntiles, SEL_BLOCK, 0, n, mA, mB, pre, outA, outB);
    uint64_t tv = 0;
    SG_TRY(ctx_readback(c, &tv, total, 8));
    *cntA = (uint32_t)(tv >> 31);
    if (cntB) *cntB = (uint32_t)(tv & 0x7fffffffu);
    prof_bytes(c, name, bytes_per_item * n);
    prof_bytes(c, "select.apply", n / 4.0 + 4.0 * (*cntA + (cntB ? *cntB : 0)));
    return SG_OK;
}

// run_select2 without the host sync: returns the device word (countA << 31 | countB) in the
// given status slot, for the caller to read back together with other counts.
template <class Pred>
static int run_select2_nb(sg_ctx *c, const char *name, Pred pred, uint32_t n, uint32_t *outA, uint32_t *outB,
                          int status_slot, uint64_t **total_out, uint64_t *total_at = nullptr) {
    const uint32_t ntiles = (n + SEL_TILE - 1) / SEL_TILE;
    uint64_t *tp;  // tot | pre | total | maskA | maskB
    SG_TRY(slot(c, status_slot, 2 * (size_t)std::max<uint32_t>(ntiles, 1) + 4 + 2 * (size_t)ntiles * SEL_MASKS, &tp));
    uint64_t *tot = tp, *pre = tp + ntiles, *total = total_at ? total_at : tp + 2 * (size_t)ntiles;
    *total_out = total;
    if (n == 0) {
        SG_HIP(hipMemsetAsync(total, 0, 8, c->stream));
        return SG_OK;
    }
    uint64_t *mA = tp + 2 * (size_t)ntiles + 4, *mB = mA + (size_t)ntiles * SEL_MASKS;
    SG_LAUNCH(c, name, k_sel_count<Pred>, ntiles, SEL_BLOCK, 0, pred, n, mA, mB, tot);
    SG_TRY(tile_scan(c, tot, ntiles, pre, total));
    SG_LAUNCH(c, "select.apply", k_sel_apply, ntiles, SEL_BLOCK, 0, n, mA, mB, pre, outA, outB);
    return SG_OK;
}

// Exclusive scan of fn(i) into out; *total = the sum (one host sync).
template <class Fn>
static int run_scan64(sg_ctx *c, const char *name, Fn fn, uint32_t n, uint64_t *out, uint64_t *total_h) {
    *total_h = 0;
    if (n == 0) return SG_OK;
    const uint32_t ntiles = (n + SCAN_TILE - 1) / SCAN_TILE;
    uint64_t *tp;
    SG_TRY(slot(c, S_TILES, 2 * (size_t)ntiles + 4, &tp));
    uint64_t *tot = tp, *pre = tp + ntiles, *total = tp + 2 * (size_t)ntiles;
    SG_LAUNCH(c, "scan.count", k_scan64_count<Fn>, ntiles, SCAN_BLOCK, 0, fn, n, tot);
    SG_TRY(tile_scan(c, tot, ntiles, pre, total));
    SG_LAUNCH_B(c, name, 12.0 * n, k_scan64_apply<Fn>, ntiles, SCAN_BLOCK, 0, fn, n, pre, out);
    SG_TRY(ctx_readback(c, total_h, total, 8));
    return SG_OK;
}

}  // namespace sg
