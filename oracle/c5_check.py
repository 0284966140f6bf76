"""Full-size check of the C5 step (BASELINE.json configs[4]: 1B host:port records) — TEST
INFRASTRUCTURE, like the rest of oracle/: imported only by tests/ and bench.py's
cpu_baseline leg, never by the product path.

The C5 records are rendered from combo ids (swarm_amd.corpus.hostport_pieces: host c // k,
port hostport_port(c)), so the expected sort -u / comm -13 results of a 1B-record step can be
computed from the ids without sorting any record bytes on the CPU:

* record identity = (canonical host, port), where the canonical host of a host id is the
  smallest id rendering the same name (host names are random strings, so a few thousand of
  64M collide; the host rows are sorted exactly, by their bytes, to find them);
* expected unique set U = distinct identities over the step's combo ids; expected new set =
  U minus the identities of the prior scan's ids (the prior is the sort -u of its own draw);
* the library's outputs are parsed back into records and checked three ways: the record
  counts, an order-independent checksum of the record bytes (the sum of a 64-bit mix of every
  record's zero-padded 40 bytes) against the same sum over U's rendered records, and strict
  byte order (adjacent records compared as big-endian words).
Counts + set checksum + strict order pin the output set and its order (a missing and an
extra record would have to cancel in the 64-bit sum). The semantics are those of the
reference path: server/server.py:399-412 merge, README.md:11 new-record alerting, sort -u.

Everything runs as torch ops on the GPU that holds the data (this is a checker: it never
calls the library)."""
from __future__ import annotations

W = 40  # bytes per padded record (host names <= 32 bytes + ':' + a port of <= 5 digits)


def _tmix(x):
    from swarm_amd.corpus import _tmix as t
    return t(x)


def _be_words(rows):
    """(m, W) uint8 -> (m, W/8) int64 big-endian words with the sign bit flipped, so signed
    comparison orders them like unsigned bytes."""
    import torch
    m = rows.shape[0]
    w = rows.view(m, W // 8, 8).flip(-1).contiguous().view(torch.int64).view(m, W // 8)
    return w ^ torch.tensor(-(1 << 63), dtype=torch.int64, device=rows.device)


def _fp(rows):
    """64-bit mix of each zero-padded row (records hold no NUL byte, so padding is unambiguous)."""
    import torch
    m = rows.shape[0]
    w = rows.contiguous().view(torch.int64).view(m, W // 8)
    h = _tmix(w[:, 0] + 0x51ED27)
    for j in range(1, W // 8):
        h = _tmix(h ^ w[:, j])
    return h


def canonical_hosts(pool):
    """Host id -> the smallest host id rendering the same name (exact: rows sorted by bytes)."""
    import torch
    mat, lens = pool
    H, Wm = mat.shape
    dev = mat.device
    cols = torch.arange(Wm, device=dev)
    rows = torch.zeros((H, W), dtype=torch.uint8, device=dev)
    rows[:, :Wm] = mat * (cols[None, :] < lens[:, None].to(torch.int64))
    words = _be_words(rows)
    order = torch.arange(H, device=dev)
    for j in reversed(range(W // 8)):  # LSD by word: stable sorts
        k = words[order, j]
        order = order[torch.sort(k, stable=True).indices]
    sw = words[order]
    same = torch.ones(H, dtype=torch.bool, device=dev)
    same[0] = False
    same[1:] = (sw[1:] == sw[:-1]).all(dim=1)
    # run heads: the smallest id of each run of equal names (ids inside a run are ascending:
    # every sort was stable over arange)
    head = torch.cummax(torch.where(same, torch.zeros_like(order), torch.arange(H, device=dev)), 0).values
    canon = torch.empty(H, dtype=torch.int64, device=dev)
    canon[order] = order[head]
    return canon


def identities(ids_iter, canon, K: int, ports_per_host):
    """Distinct (canonical host, port) identities over the combo ids, sorted (int64 keys)."""
    import torch
    from swarm_amd.corpus import hostport_port
    parts = []
    for c in ids_iter:
        key = canon[c // K] * 64 + hostport_port(c, ports_per_host)
        parts.append(torch.unique(key))
        del c, key
    return torch.unique(torch.cat(parts)) if parts else None


def render_keys(keys, pool, chunk: int = 1 << 23):
    """Yield (m, W) zero-padded record rows of identity keys (host name + ':' + port)."""
    import torch
    from swarm_amd.corpus import PORTS
    mat, lens = pool
    dev = mat.device
    Wm = mat.shape[1]
    pm = torch.zeros((len(PORTS), 8), dtype=torch.uint8)
    pl = torch.zeros(len(PORTS), dtype=torch.int64)
    for i, p in enumerate(PORTS):
        b = b":" + p
        pm[i, :len(b)] = torch.frombuffer(bytearray(b), dtype=torch.uint8)
        pl[i] = len(b)
    pm, pl = pm.to(dev), pl.to(dev)
    cols = torch.arange(W, device=dev)
    for s in range(0, keys.numel(), chunk):
        k = keys[s:s + chunk]
        h, p = k // 64, k % 64
        rows = torch.zeros((k.numel(), W + 8), dtype=torch.uint8, device=dev)
        rows[:, :Wm] = mat[h]
        hl = lens[h].to(torch.int64)
        rows.scatter_(1, hl[:, None] + torch.arange(8, device=dev)[None, :], pm[p])
        yield rows[:, :W] * (cols[None, :] < (hl + pl[p])[:, None])


def parse_rows(buf, chunk: int = 1 << 23):
    """Yield (m, W) zero-padded rows of the '\\n'-terminated records of a device byte buffer
    (empty records skipped; a record longer than W raises)."""
    import torch
    n = buf.numel()
    if n == 0:
        return
    # torch.nonzero counts in 32 bits on this build: find the newlines 1 GiB at a time
    step = 1 << 30
    ends = torch.cat([torch.nonzero(buf[o:o + step] == 10).flatten() + o for o in range(0, n, step)])
    starts = torch.cat([torch.zeros(1, dtype=torch.int64, device=buf.device), ends[:-1] + 1])
    lens = ends - starts
    keep = lens > 0
    starts, lens = starts[keep], lens[keep]
    if lens.numel() and int(lens.max()) > W:
        raise ValueError("record longer than %d bytes" % W)
    cols = torch.arange(W, device=buf.device)
    for s in range(0, starts.numel(), chunk):
        st, ln = starts[s:s + chunk], lens[s:s + chunk]
        idx = (st[:, None] + cols[None, :]).clamp_(max=n - 1)
        yield buf[idx] * (cols[None, :] < ln[:, None])


def summarize(rows_iter):
    """(records, sum of fingerprints, strictly increasing?) over a stream of row chunks."""
    import torch
    n, tot, inc, prev = 0, None, True, None
    for rows in rows_iter:
        if rows.shape[0] == 0:
            continue
        f = _fp(rows).sum()
        tot = f if tot is None else tot + f
        w = _be_words(rows)
        if prev is not None:
            w = torch.cat([prev, w])
        a, b = w[:-1], w[1:]
        # a < b lexicographically: the first differing word decides
        diff = a != b
        first = torch.where(diff.any(1), diff.int().argmax(1), torch.full((a.shape[0],), W // 8 - 1, device=a.device))
        lt = a.gather(1, first[:, None]).squeeze(1) < b.gather(1, first[:, None]).squeeze(1)
        inc = inc and bool(lt.all())
        prev = w[-1:]
        n += rows.shape[0]
    return n, (int(tot) if tot is not None else 0), inc


def expected(pool, K, ports_per_host, cur_ids, prior_ids):
    """(U summary, new-set summary) for the step's combo ids and the prior's."""
    import torch
    canon = canonical_hosts(pool)
    U = identities(cur_ids, canon, K, ports_per_host)
    P = identities(prior_ids, canon, K, ports_per_host) if prior_ids is not None else None
    del canon
    Fk = U[~torch.isin(U, P)] if P is not None else U
    su = summarize(render_keys(U, pool))
    sf = summarize(render_keys(Fk, pool))
    return su, sf


def check_step(pool, K, ports_per_host, cur_ids, prior_ids, uniq_buf, fresh_buf):
    """Compare a C5 step's device outputs with the id-level expectation. Returns a dict with
    the counts on both sides and full_size_bit_exact."""
    (nu, su, _), (nf, sf, _) = expected(pool, K, ports_per_host, cur_ids, prior_ids)
    gu, gsu, gincu = summarize(parse_rows(uniq_buf))
    gf, gsf, gincf = summarize(parse_rows(fresh_buf))
    ok = (nu == gu and su == gsu and gincu and nf == gf and sf == gsf and gincf)
    return {"expected_unique": nu, "expected_new": nf, "gpu_unique": gu, "gpu_new": gf,
            "set_checksum_equal": su == gsu and sf == gsf, "strictly_increasing": gincu and gincf,
            "full_size_bit_exact": bool(ok)}
