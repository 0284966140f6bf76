"""Probe path vs radix pipeline on the bench inputs (C2 and X1), device-resident: outputs
compared byte for byte; on a mismatch the differing records are printed with where they
occur (cur / prior). Timing of each path per call as well.
  python3 tools/probe_check.py [x1_lines]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
import swarm_amd  # noqa: E402
from swarm_amd import corpus  # noqa: E402


def both(ctx, call):
    out = {}
    for mode in ("1", "0"):
        os.environ["SG_PROBE"] = mode
        r = call()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            r = call()
        torch.cuda.synchronize()
        out[mode] = (ctx.to_bytes(r.uniq, r.uniq_bytes), ctx.to_bytes(r.fresh, r.fresh_bytes), ctx.last_path()[0],
                     (time.perf_counter() - t0) / 3 * 1e3, int(r.uniq_records), int(r.fresh_records))
    return out


def report(name, out, cur=None, prior=None):
    a, b = out["1"], out["0"]
    res = {"leg": name, "probe": {"path": a[2], "ms": round(a[3], 3), "uniq": a[4], "fresh": a[5]},
           "radix": {"path": b[2], "ms": round(b[3], 3), "uniq": b[4], "fresh": b[5]},
           "uniq_equal": a[0] == b[0], "fresh_equal": a[1] == b[1]}
    print(json.dumps(res), flush=True)
    if a[0] != b[0]:
        sa, sb = set(a[0].split(b"\n")), set(b[0].split(b"\n"))
        only_r, only_p = sorted(sb - sa)[:5], sorted(sa - sb)[:5]
        pset = set(prior.split(b"\n")) if prior is not None else set()
        for rec in only_r:
            print("  radix only:", rec[:120], "in prior:", rec in pset, "count in cur:",
                  cur.count(b"\n" + rec + b"\n") if cur is not None else None, flush=True)
        for rec in only_p:
            print("  probe only:", rec[:120], flush=True)
        # first differing byte and the records around it
        import numpy as np
        L = min(len(a[0]), len(b[0]))
        d = int(np.flatnonzero(np.frombuffer(a[0], np.uint8)[:L] != np.frombuffer(b[0], np.uint8)[:L])[0])
        lo = a[0].rfind(b"\n", 0, max(0, d - 200)) + 1
        print("  first diff at byte", d, "of", len(a[0]), flush=True)
        print("  probe:", a[0][lo:d + 300], flush=True)
        print("  radix:", b[0][lo:d + 300], flush=True)
        # order check of the probe output
        recs = a[0].split(b"\n")[:-1]
        bad = sum(1 for i in range(1, len(recs)) if recs[i - 1] >= recs[i])
        print("  probe output order violations:", bad, "records", len(recs), flush=True)


def main():
    ctx = swarm_amd.Context(0, torch.cuda.current_stream().cuda_stream)
    buf, ids = corpus.subdomains(10_000_000, seed=1234)
    prior = corpus.prior_of(ids)
    dc, dp = torch.from_numpy(buf).cuda(), torch.from_numpy(prior).cuda()
    report("c2", both(ctx, lambda: ctx.dedup_diff(dc.data_ptr(), dc.numel(), dp.data_ptr(), dp.numel())))
    del dc, dp

    n_lines = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    sigs = bench.c3_signatures()
    tails = corpus.httpx_tails(sigs)
    buf, ids = corpus.httpx_hosts(n_lines, tails, seed=1234)
    d = torch.from_numpy(buf).cuda()
    m = swarm_amd.Matcher(sigs, "literal")
    pbuf = corpus.httpx_rows(corpus.prior_ids(ids), tails)
    dp_in = torch.from_numpy(pbuf).cuda()
    r0, _, _ = m.dev_match_dedup_diff(ctx, dp_in.data_ptr(), dp_in.numel())
    n_prior = int(r0.uniq_bytes)
    d_prior = torch.empty(max(n_prior, 1), dtype=torch.uint8, device="cuda")
    ctx.memcpy(d_prior.data_ptr(), r0.uniq, n_prior)
    prior_host = ctx.to_bytes(d_prior.data_ptr(), n_prior)
    out = both(ctx, lambda: m.dev_match_dedup_diff(ctx, d.data_ptr(), d.numel(), d_prior.data_ptr(), n_prior,
                                                  count_hits=False)[0])
    report("x1", out, b"\n" + buf.tobytes(), prior_host)
    ctx.close()


if __name__ == "__main__":
    main()
