"""How much of C2's step is the post-sort gathers' lack of locality? The same 10M records
in three physical orders: as drawn (the bench), bucketed by their first k bytes (random
order inside a bucket: what a byte-bucketing pass before the sort would produce), and fully
sorted. Outputs are identical (sort -u / comm -13 do not depend on input order); the
per-kernel times show what locality buys the adjacent compare, segment sorts, unique emit
and diff. Timing only (python tools/locality_probe.py [n_lines] [k ...])."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import swarm_amd  # noqa: E402
from swarm_amd import corpus  # noqa: E402


def lines_of(buf):
    nl = np.flatnonzero(buf == 10)
    st = np.concatenate([[0], nl[:-1] + 1])
    return st, nl + 1


def reorder(buf, order, st, en):
    ln = en - st
    ln_o = ln[order]
    out_st = np.concatenate([[0], np.cumsum(ln_o)[:-1]])
    idx = np.repeat(st[order] - out_st, ln_o) + np.arange(ln_o.sum())
    return buf[idx]


def bucket_order(buf, st, en, k, rng):
    """Records ordered by their first k bytes (bytes past the record's end as 0), random
    order inside a bucket; k >= the longest record: fully sorted."""
    cols = []
    for j in range(k):
        p = st + j
        cols.append(np.where(p < en - 1, buf[np.minimum(p, len(buf) - 1)], 0))
    tie = rng.permutation(len(st))
    return np.lexsort([tie] + cols[::-1])


def run(ctx, d_cur, d_pri, reps=10):
    for _ in range(3):
        r = ctx.dedup_diff(d_cur.data_ptr(), d_cur.numel(), d_pri.data_ptr(), d_pri.numel())
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        r = ctx.dedup_diff(d_cur.data_ptr(), d_cur.numel(), d_pri.data_ptr(), d_pri.numel())
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / reps
    ctx.reset_stats()
    ctx.profile(True)
    for _ in range(3):
        r = ctx.dedup_diff(d_cur.data_ptr(), d_cur.numel(), d_pri.data_ptr(), d_pri.numel())
    torch.cuda.synchronize()
    ctx.profile(False)
    st = ctx.kernel_stats()
    return el, st, r


def main():
    n_lines = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    ks = [int(x) for x in sys.argv[2:]] or [1, 2, 3]
    buf, ids = corpus.subdomains(n_lines, seed=1234)
    prior = corpus.prior_of(ids)
    st, en = lines_of(buf)
    rng = np.random.default_rng(7)
    d_pri = torch.from_numpy(prior).cuda()
    ctx = swarm_amd.Context(0, torch.cuda.current_stream().cuda_stream)
    variants = [("drawn", None)] + [("bucket%d" % k, k) for k in ks] + [("sorted", 99)]
    ref = None
    for name, k in variants:
        if k is None:
            b = buf
        elif k == 99:
            b = reorder(buf, bucket_order(buf, st, en, 40, rng), st, en)
        else:
            b = reorder(buf, bucket_order(buf, st, en, k, rng), st, en)
        d_cur = torch.from_numpy(np.ascontiguousarray(b)).cuda()
        el, stats, r = run(ctx, d_cur, d_pri)
        sig = (r.uniq_records, r.fresh_records, r.uniq_bytes, r.fresh_bytes)
        if ref is None:
            ref = sig
        out = {"order": name, "ms_step": round(el * 1e3, 3), "same_counts": sig == ref,
               "kernels_us": {kk: round(v[1] / v[0] * 1e3, 1) for kk, v in sorted(stats.items(), key=lambda kv: -kv[1][1])[:14]}}
        print(json.dumps(out), flush=True)
        del d_cur
    ctx.close()


if __name__ == "__main__":
    main()
