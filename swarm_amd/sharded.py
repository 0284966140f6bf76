"""Shards larger than one 4 GiB call (SURVEY.md §8(a) A7 at C5 sizes: 1B host:port
records, ~30 GB per scan) on one GPU, with the global sort -u byte order kept.

One call of the library handles < 4 GiB (32-bit record offsets). A bigger shard arrives in
pieces anyway (chunk files, S3 bodies); each piece is routed on the GPU into P parts by
key0 splitters (sg_dev_partition_range): part p holds only records that sort below every
record of part p+1, and equal records always share a part. Each part (< 4 GiB) is then
deduped and diffed against the same part of the prior scan, and the part outputs
concatenated in part order ARE the global sort -u / comm -13 output — no merge step.
Splitters are quantiles of key0 samples taken from every piece (sg_dev_key_sample).

All buffers are torch uint8 tensors on the context's device; pieces must end at a record
boundary (split_at_newlines cuts a long buffer that way).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np

PART_LIMIT = 0xFFFF0000  # bytes per library call (include/swarmgpu.h)
RECORD_LIMIT = 1 << 30   # records per library call (sg_dedup.hip build_unique)


def part_overflow_message(splitters: np.ndarray, b: int, cur_bytes: int, prior_bytes: int) -> str:
    """Why range part b is over the per-call limit, and whether more parts can help: a part
    whose two bounding splitters are equal is one key0 value (records sharing their first 7
    bytes), which no number of parts can divide."""
    lo = int(splitters[b - 1]) if b > 0 else None
    hi = int(splitters[b]) if b < splitters.size else None
    one_key = lo is not None and hi is not None and lo == hi
    msg = "key0 range part %d holds %d cur / %d prior bytes (per-call limit %d bytes, %d records)" % (
        b, cur_bytes, prior_bytes, PART_LIMIT, RECORD_LIMIT)
    if one_key or (lo is not None and b + 1 < splitters.size and int(splitters[b + 1]) == lo):
        return msg + ": its records share one key0 value %#x (first 7 bytes), which range routing cannot split" % lo
    return msg + ": use more parts (smaller part_bytes)"


def split_at_newlines(buf, max_bytes: int = 3 << 30, window: int = 1 << 20) -> List:
    """Cut a device byte tensor into views of <= max_bytes ending just after a '\\n' (the
    last piece may end without one). A window of `window` bytes before each cut must hold
    a newline."""
    import torch
    n = buf.numel()
    out, s = [], 0
    while n - s > max_bytes:
        t = s + max_bytes
        lo = max(s, t - window)
        nl = torch.nonzero(buf[lo:t] == 10)
        if nl.numel() == 0:
            raise ValueError("no record boundary within %d bytes before offset %d" % (window, t))
        cut = lo + int(nl[-1].item()) + 1
        out.append(buf[s:cut])
        s = cut
    if n > s:
        out.append(buf[s:n])
    return out


def choose_splitters(samples: np.ndarray, parts: int) -> np.ndarray:
    """parts - 1 non-decreasing key0 quantiles of the samples (sentinels ~0 ignored)."""
    s = np.sort(np.asarray(samples, dtype=np.uint64))
    s = s[s != np.uint64(0xFFFFFFFFFFFFFFFF)]
    if parts <= 1 or s.size == 0:
        return np.zeros(0, dtype=np.uint64)
    idx = (np.arange(1, parts, dtype=np.int64) * s.size) // parts
    return s[idx]


def route(ctx, pieces: Sequence, splitters: np.ndarray) -> List:
    """Route every piece into len(splitters) + 1 parts; returns one device tensor per part
    (the part's records from all pieces, in piece order)."""
    import torch
    parts = splitters.size + 1
    lists: List[list] = [[] for _ in range(parts)]
    keep = []
    for p in pieces:
        n = p.numel()
        if n == 0:
            continue
        out = torch.empty(n + 16, dtype=torch.uint8, device=p.device)
        ctx.fence_in()  # `out` may be a block torch's stream is still reading
        pb, _ = ctx.partition_range(p.data_ptr(), n, splitters, out.data_ptr(), out.numel())
        off = 0
        for b in range(parts):
            if pb[b]:
                lists[b].append(out[off:off + pb[b]])
            off += pb[b]
        keep.append(out)
    res = []
    for b in range(parts):
        if not lists[b]:
            res.append(None)
        elif len(lists[b]) == 1:
            res.append(lists[b][0])
        else:
            res.append(torch.cat(lists[b]))
    del keep
    return res


def _take(ctx, dptr: int, n: int, device):
    import torch
    t = torch.empty(max(n, 1), dtype=torch.uint8, device=device)
    if n:
        ctx.fence_in()
        ctx.memcpy(t.data_ptr(), dptr, n)
    return t[:n]


def plan_parts(cur_pieces: Sequence, prior_pieces: Sequence, part_bytes: int) -> int:
    big = max(sum(p.numel() for p in cur_pieces), sum(p.numel() for p in prior_pieces))
    return int(min(256, max(1, -(-int(big * 1.25) // part_bytes))))


def dedup_diff_large(ctx, cur_pieces: Sequence, prior_pieces: Sequence = (), part_bytes: int = 2 << 30,
                     samples_per_piece: int = 1 << 14, splitters: np.ndarray | None = None):
    """(sort -u of all cur records, new records vs prior, stats) as device tensors, each in
    global byte order, for shards of any size. `prior_pieces` is the prior scan (sorted
    unique or not). `splitters` may be given (e.g. agreed across ranks); otherwise they are
    chosen from key0 samples of every piece."""
    import torch
    cur_pieces = [p for p in cur_pieces if p.numel()]
    prior_pieces = [p for p in prior_pieces if p.numel()]
    dev = cur_pieces[0].device if cur_pieces else torch.device("cuda", ctx.device)
    if splitters is None:
        parts = plan_parts(cur_pieces, prior_pieces, part_bytes)
        samples = [ctx.key_sample(p.data_ptr(), p.numel(), samples_per_piece)[0] for p in cur_pieces + prior_pieces]
        splitters = choose_splitters(np.concatenate(samples) if samples else np.zeros(0, np.uint64), parts)
    cur_parts = route(ctx, cur_pieces, splitters)
    prior_parts = route(ctx, prior_pieces, splitters) if prior_pieces else [None] * (splitters.size + 1)
    uniq, fresh = [], []
    st = {"parts": splitters.size + 1, "in_records": 0, "uniq_records": 0, "fresh_records": 0,
          "max_part_bytes": 0}
    for b, (c, p) in enumerate(zip(cur_parts, prior_parts)):
        if c is None:
            continue
        if c.numel() > PART_LIMIT or (p is not None and p.numel() > PART_LIMIT):
            raise ValueError(part_overflow_message(splitters, b, c.numel(), p.numel() if p is not None else 0))
        st["max_part_bytes"] = max(st["max_part_bytes"], c.numel())
        ctx.fence_in()
        try:
            r = ctx.dedup_diff(c.data_ptr(), c.numel(), p.data_ptr() if p is not None else 0,
                               p.numel() if p is not None else 0)
        except Exception as e:
            raise type(e)(e.rc, "%s (part of %d bytes at %#x, prior %s)" % (
                e, c.numel(), c.data_ptr(), None if p is None else p.numel())) if hasattr(e, "rc") else e
        uniq.append(_take(ctx, r.uniq, r.uniq_bytes, dev))
        fresh.append(_take(ctx, r.fresh, r.fresh_bytes, dev) if p is not None else uniq[-1])
        st["in_records"] += int(r.in_records)
        st["uniq_records"] += int(r.uniq_records)
        st["fresh_records"] += int(r.fresh_records) if p is not None else int(r.uniq_records)
    empty = torch.empty(0, dtype=torch.uint8, device=dev)
    return (torch.cat(uniq) if uniq else empty), (torch.cat(fresh) if fresh else empty), st


def pieces_bytes(pieces) -> Tuple[int, int]:
    return sum(p.numel() for p in pieces), len(pieces)
