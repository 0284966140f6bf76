"""C5 at the size of one dedup part: does the order of the part's bytes matter? One part's
worth of host:port records (about 1/19 of the 1B-record step, with the step's duplication)
deduped in its drawn order, then with the same records grouped into G byte ranges (each a
contiguous run of the part, random order inside: what a finer routing pass would write),
then fully sorted. Outputs are identical; the per-kernel times show what locality buys the
segment sorts, the adjacent compare and the unique emit. Timing only.
python tools/c5_locality_probe.py [records] [G ...]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import swarm_amd  # noqa: E402
from swarm_amd import corpus  # noqa: E402


def rows_of(n, n_hosts, seed=100, dev="cuda"):
    """(rows (n, W) uint8 zero-padded, lengths) of n host:port records drawn as bench c5 does."""
    pool = corpus.host_pool_torch(n_hosts, seed=5, device=dev)
    K = 4
    # boolean-mask indexing past 2^31 elements fails in torch: pieces of 16M records
    pieces = corpus.hostport_pieces(pool, n, 0, n_hosts * K, seed, per_piece=1 << 24, ports_per_host=K)
    buf = torch.cat(pieces)
    nl = torch.nonzero(buf == 10).flatten()
    st = torch.cat([torch.zeros(1, dtype=nl.dtype, device=nl.device), nl[:-1] + 1])
    ln = nl + 1 - st
    W = int(ln.max())
    cols = torch.arange(W, device=buf.device)
    rows = torch.zeros((st.numel(), W), dtype=torch.uint8, device=buf.device)
    for a in range(0, st.numel(), 1 << 24):
        s_, l_ = st[a:a + (1 << 24)], ln[a:a + (1 << 24)]
        idx = s_[:, None] + cols[None, :]
        msk = cols[None, :] < l_[:, None]
        rows[a:a + (1 << 24)] = torch.where(msk, buf[idx.clamp(max=buf.numel() - 1)],
                                            torch.zeros((), dtype=torch.uint8, device=buf.device))
    return rows, ln


def sorted_order(rows):
    order = torch.arange(rows.shape[0], device=rows.device)
    for j in range(rows.shape[1] - 1, -1, -1):
        o = torch.sort(rows[order, j], stable=True).indices
        order = order[o]
    return order


def flatten(rows, ln, order):
    out = []
    for a in range(0, order.numel(), 1 << 24):
        o = order[a:a + (1 << 24)]
        r, l = rows[o], ln[o]
        msk = torch.arange(r.shape[1], device=r.device)[None, :] < l[:, None]
        out.append(r[msk])
    return torch.cat(out).contiguous()


def run(ctx, d, reps=5):
    for _ in range(2):
        r = ctx.dedup_diff(d.data_ptr(), d.numel(), 0, 0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        r = ctx.dedup_diff(d.data_ptr(), d.numel(), 0, 0)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / reps
    ctx.reset_stats()
    ctx.profile(True)
    for _ in range(2):
        r = ctx.dedup_diff(d.data_ptr(), d.numel(), 0, 0)
    torch.cuda.synchronize()
    ctx.profile(False)
    return el, ctx.kernel_stats(), (r.uniq_records, r.uniq_bytes)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 52_600_000
    Gs = [int(x) for x in sys.argv[2:]] or [13, 64, 256]
    n_hosts = max(1, 64_000_000 * n // 1_000_000_000)
    rows, ln = rows_of(n, n_hosts)
    srt = sorted_order(rows)
    ctx = swarm_amd.Context(0, torch.cuda.current_stream().cuda_stream)
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    ref = None
    variants = [("drawn", None)] + [("G%d" % G, G) for G in Gs] + [("sorted", 0)]
    for name, G in variants:
        if G is None:
            order = torch.arange(n, device=rows.device)
        elif G == 0:
            order = srt
        else:
            # position p of the sorted order -> range p * G // n; random order inside a range
            rng_of = torch.empty(n, dtype=torch.int64, device=rows.device)
            rng_of[srt] = torch.arange(n, device=rows.device) * G // n
            key = rng_of * (1 << 32) + torch.randint(0, 1 << 31, (n,), generator=g, device=rows.device)
            order = torch.sort(key).indices
        d = flatten(rows, ln, order)
        el, st, sig = run(ctx, d)
        if ref is None:
            ref = sig
        print(json.dumps({"order": name, "records": n, "bytes": d.numel(), "ms": round(el * 1e3, 3), "same": sig == ref,
                          "uniq": sig[0],
                          "kernels_us": {k: round(v[1] / v[0] * 1e3, 1)
                                         for k, v in sorted(st.items(), key=lambda kv: -kv[1][1])[:12]}}), flush=True)
        del d
    ctx.close()


if __name__ == "__main__":
    main()
