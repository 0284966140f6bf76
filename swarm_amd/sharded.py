"""Shards larger than one 4 GiB call (SURVEY.md §8(a) A7 at C5 sizes: 1B host:port
records, ~30 GB per scan) on one GPU, with the global sort -u byte order kept.

One call of the library handles < 4 GiB (32-bit record offsets). A bigger shard arrives in
pieces anyway (chunk files, S3 bodies); each piece is routed on the GPU into P parts by
byte-string splitters (sg_dev_partition_bytes): part p holds only records that sort below
every record of part p+1, and equal records always share a part. Each part (< 4 GiB) is
then deduped and diffed against the same part of the prior scan, and the part outputs
concatenated in part order ARE the global sort -u / comm -13 output — no merge step.
Splitters are byte quantiles of records sampled from every piece (sg_dev_record_sample,
first 64 bytes), so runs of records sharing a long prefix (https://..., 10.0.x.y:port) are
divided too; a part that still ends up over the per-call limit is routed again with
splitters sampled from that part alone.

All buffers are torch uint8 tensors on the context's device; pieces must end at a record
boundary (split_at_newlines cuts a long buffer that way).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np

from .api import part_offsets

PART_LIMIT = 0xFFFF0000  # bytes per library call (include/swarmgpu.h)
RECORD_LIMIT = 1 << 30   # records per library call (sg_dedup.hip build_unique)
SPLIT_BYTES = 64         # bytes of a splitter compared (include/swarmgpu.h SG_SPLIT_BYTES)


def part_overflow_message(splitters, b: int, cur_bytes: int, prior_bytes: int) -> str:
    """Why range part b is over the per-call limit after re-routing: its records share their
    first SPLIT_BYTES bytes (every sampled splitter inside it is the same string), which no
    number of parts can divide."""
    return ("range part %d holds %d cur / %d prior bytes (per-call limit %d bytes, %d records) and its "
            "records share their first %d bytes, which range routing cannot split"
            % (b, cur_bytes, prior_bytes, PART_LIMIT, RECORD_LIMIT, SPLIT_BYTES))


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


def choose_splitters(samples, parts: int):
    """parts - 1 non-decreasing quantiles of the samples: byte strings (a list of bytes,
    from sample_records) -> byte splitters; key0 values (uint64 array, sentinels ~0
    ignored) -> key0 splitters."""
    if isinstance(samples, (list, tuple)):
        s = sorted(samples)
        if parts <= 1 or not s:
            return []
        return [s[(k * len(s)) // parts] for k in range(1, parts)]
    s = np.sort(np.asarray(samples, dtype=np.uint64))
    s = s[s != np.uint64(0xFFFFFFFFFFFFFFFF)]
    if parts <= 1 or s.size == 0:
        return np.zeros(0, dtype=np.uint64)
    idx = (np.arange(1, parts, dtype=np.int64) * s.size) // parts
    return s[idx]


def sample_records(ctx, pieces: Sequence, per_piece: int = 1 << 12) -> List[bytes]:
    """First SPLIT_BYTES bytes of per_piece evenly spaced records of every piece."""
    out: List[bytes] = []
    for p in pieces:
        if p is not None and p.numel():
            out += ctx.record_sample(p.data_ptr(), p.numel(), per_piece)[0]
    return out


def n_splitters(splitters) -> int:
    return len(splitters) if isinstance(splitters, (list, tuple)) else int(np.asarray(splitters).size)


def route_piece(ctx, p, splitters, out_ptr: int, out_cap: int):
    """Route one piece into out (parts contiguous); returns bytes per part."""
    if isinstance(splitters, (list, tuple)):
        pb, _ = ctx.partition_bytes(p.data_ptr(), p.numel(), splitters, out_ptr, out_cap)
    else:
        pb, _ = ctx.partition_range(p.data_ptr(), p.numel(), splitters, out_ptr, out_cap)
    return pb


def route(ctx, pieces: Sequence, splitters) -> List:
    """Route every piece into n_splitters + 1 parts; returns one device tensor per part (the
    part's records from all pieces, in piece order; None for an empty part). Byte splitters:
    one sg_dev_partition_bytes_pieces call writes every part contiguously into one buffer
    (the part tensors are views of it). Key0 splitters: per piece, then joined."""
    import torch
    parts = n_splitters(splitters) + 1
    live = [p for p in pieces if p is not None and p.numel()]
    if isinstance(splitters, (list, tuple)):
        if not live:
            return [None] * parts
        total = sum(p.numel() for p in live)
        out = torch.empty(total + len(live) + 16 * (parts + 1), dtype=torch.uint8, device=live[0].device)
        ctx.fence_in()  # `out` may be a block torch's stream is still reading
        # parts at 16-byte aligned offsets: each dedup call then reads its part in place
        pb, _ = ctx.partition_bytes_pieces([(p.data_ptr(), p.numel()) for p in live], splitters, out.data_ptr(),
                                           out.numel(), align16=True)
        offs = part_offsets(pb, align16=True)
        return [out[o:o + n] if n else None for o, n in zip(offs, pb)]
    lists: List[list] = [[] for _ in range(parts)]
    keep = []
    for p in live:
        n = p.numel()
        out = torch.empty(n + 16, dtype=torch.uint8, device=p.device)
        ctx.fence_in()
        pb = route_piece(ctx, p, splitters, out.data_ptr(), out.numel())
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


def route_spans(ctx, pieces: Sequence, splitters):
    """route() with byte splitters that also returns every part's parse from the routing
    pass: (parts, [(device spans, device keys, records, handover checksum) or None per part]).
    The parse lives in context buffers until the next route_spans call on ctx; the dedup checks
    it against the part's bytes and the checksum before using it."""
    import torch
    parts = n_splitters(splitters) + 1
    live = [p for p in pieces if p is not None and p.numel()]
    if not live:
        return [None] * parts, [None] * parts
    total = sum(p.numel() for p in live)
    out = torch.empty(total + len(live) + 16 * (parts + 1), dtype=torch.uint8, device=live[0].device)
    ctx.fence_in()
    pb, pr, sp, kp, ps = ctx.partition_bytes_pieces_spans([(p.data_ptr(), p.numel()) for p in live], splitters,
                                                          out.data_ptr(), out.numel())
    res, parse, r0 = [], [], 0
    for o, n, nr, s in zip(part_offsets(pb, align16=True), pb, pr, ps):
        res.append(out[o:o + n] if n else None)
        parse.append((sp + 8 * r0, kp + 8 * r0, nr, s) if n else None)
        r0 += nr
    return res, parse


class _Results:
    """The unique and new-record outputs of all parts, appended in part order into two
    preallocated device buffers (each part's dedup call writes there directly).
    align16: every top-level part's unique output starts at a 16-byte aligned offset (the
    gap filled with '\n', i.e. empty records, which no consumer sees): a stored prior kept
    this way is read in place, part by part, with no copy into an aligned slot."""

    def __init__(self, cap: int, device, want_fresh: bool, align16: bool = False):
        import torch
        self.align16 = align16
        cap += 16 * 257 if align16 else 0
        self.u = torch.empty(cap, dtype=torch.uint8, device=device)
        self.f = torch.empty(cap, dtype=torch.uint8, device=device) if want_fresh else None
        self.uo = 0
        self.fo = 0

    def begin_part(self) -> int:
        """Start of the next top-level part's unique output."""
        if self.align16 and self.uo & 15:
            a = (self.uo + 15) & ~15
            self.u[self.uo:a].fill_(10)
            self.uo = a
        return self.uo


def plan_parts(cur_pieces: Sequence, prior_pieces: Sequence, part_bytes: int) -> int:
    big = max(sum(p.numel() for p in cur_pieces), sum(p.numel() for p in prior_pieces))
    return int(min(256, max(1, -(-int(big * 1.25) // part_bytes))))


def new_stats(parts: int) -> dict:
    return {"parts": parts, "in_records": 0, "uniq_records": 0, "fresh_records": 0, "max_part_bytes": 0,
            "rerouted_parts": 0, "part_bytes": [], "uniq_part_bytes": [], "uniq_part_offs": []}


def stored_parts(u, st) -> List:
    """The per-part views of a unique output (st from dedup_diff_large / a rounds step): a
    stored prior kept this way is handed back as prior_parts, never routed again."""
    return [u[o:o + n] if n else None for o, n in zip(st["uniq_part_offs"], st["uniq_part_bytes"])]


def dedup_diff_large(ctx, cur_pieces: Sequence, prior_pieces: Sequence = (), part_bytes: int = 2 << 30,
                     samples_per_piece: int = 1 << 12, splitters=None, prior_parts: Sequence | None = None,
                     align_parts: bool = False):
    """(sort -u of all cur records, new records vs prior, stats) as device tensors, each in
    global byte order, for shards of any size. `prior_pieces` is the prior scan (sorted
    unique or not). `splitters` may be given (byte strings or key0 values, e.g. agreed
    across ranks); otherwise byte splitters are chosen from records sampled from every
    piece. `prior_parts` (with `splitters`): the prior already split by those splitters — the
    stored prior scan is this function's own part-ordered output, so it need not be routed
    again (stored_parts(u, st) gives the part views). align_parts: every part's unique output
    starts 16-byte aligned ('\n' padding between parts, so u is a line buffer holding the
    sort -u records but not byte-identical to the sort -u output): for storing a prior."""
    import torch
    cur_pieces = [p for p in cur_pieces if p.numel()]
    prior_pieces = [p for p in prior_pieces if p.numel()]
    dev = cur_pieces[0].device if cur_pieces else torch.device("cuda", ctx.device)
    if splitters is None:
        parts = plan_parts(cur_pieces, prior_pieces, part_bytes)
        splitters = choose_splitters(sample_records(ctx, cur_pieces + prior_pieces, samples_per_piece), parts)
    have_prior = bool(prior_pieces) or (prior_parts is not None and any(p is not None and p.numel()
                                                                        for p in prior_parts))
    st = new_stats(n_splitters(splitters) + 1)
    out = _Results(sum(p.numel() for p in cur_pieces) + 4096, dev, have_prior, align16=align_parts)
    _dedup_parts(ctx, cur_pieces, prior_pieces, splitters, out, st, samples_per_piece, prior_parts=prior_parts)
    u = out.u[:out.uo]
    return u, (out.f[:out.fo] if have_prior else u), st


def _dedup_parts(ctx, cur_pieces, prior_pieces, splitters, out, st, samples_per_piece, depth: int = 0,
                 prior_parts=None):
    if prior_parts is None and prior_pieces:
        prior_parts = route(ctx, prior_pieces, splitters)
    # byte splitters at the top level: the routing pass hands each part's parse to its dedup
    # (a rerouted part's recursion routes without it, so this parse stays valid)
    parse = None
    if depth == 0 and isinstance(splitters, (list, tuple)):
        cur_parts, parse = route_spans(ctx, cur_pieces, splitters)
    else:
        cur_parts = route(ctx, cur_pieces, splitters)
    if prior_parts is None:
        prior_parts = [None] * len(cur_parts)
    if len(prior_parts) != len(cur_parts):
        raise ValueError("prior_parts has %d entries for %d parts" % (len(prior_parts), len(cur_parts)))
    for b, (c, p) in enumerate(zip(cur_parts, prior_parts)):
        dedup_part(ctx, c, p, out, st, samples_per_piece, depth, parse[b] if parse is not None else None,
                   label=(splitters, b))


def dedup_part(ctx, c, p, out, st, samples_per_piece: int = 1 << 12, depth: int = 0, parse=None, label=None):
    """sort -u + diff of one range part `c` (device tensor or None) against the prior's same
    part `p`, appended to `out`; a part over the per-call limit is routed again with
    splitters sampled from it alone. depth 0 = a top-level part (its unique output's offset
    and size are recorded in st for stored_parts)."""
    if depth == 0:
        st["uniq_part_offs"].append(out.begin_part())
        st["uniq_part_bytes"].append(0)
        u_start = out.uo
    if c is None or not c.numel():
        return
    pn = p.numel() if p is not None else 0
    if c.numel() > PART_LIMIT or pn > PART_LIMIT:
        big = max(c.numel(), pn)
        sub_parts = int(min(256, max(2, -(-int(big * 1.25) // (PART_LIMIT // 2)))))
        sub = choose_splitters(sample_records(ctx, [c] + ([p] if pn else []), samples_per_piece), sub_parts)
        if depth >= 3 or not sub:
            sp, b = label if label else ([], 0)
            raise ValueError(part_overflow_message(sp, b, c.numel(), pn))
        st["rerouted_parts"] += 1
        _dedup_parts(ctx, [c], [p] if pn else [], sub, out, st, samples_per_piece, depth + 1)
        if depth == 0:
            st["uniq_part_bytes"][-1] = out.uo - u_start
        return
    st["max_part_bytes"] = max(st["max_part_bytes"], c.numel())
    st["part_bytes"].append(int(c.numel()))
    ctx.fence_in()
    try:
        outs = (out.u.data_ptr() + out.uo, out.u.numel() - out.uo,
                (out.f.data_ptr() + out.fo) if out.f is not None else 0,
                (out.f.numel() - out.fo) if out.f is not None else 0)
        if parse is not None:
            sp, kp, nr, ssum = parse
            r = ctx.dedup_diff_spans_into(c.data_ptr(), c.numel(), sp, kp, nr, ssum, p.data_ptr() if pn else 0, pn,
                                          *outs)
        else:
            r = ctx.dedup_diff_into(c.data_ptr(), c.numel(), p.data_ptr() if pn else 0, pn, *outs)
    except Exception as e:
        raise type(e)(e.rc, "%s (part of %d bytes at %#x, prior %s)" % (
            e, c.numel(), c.data_ptr(), None if p is None else pn)) if hasattr(e, "rc") else e
    out.uo += int(r.uniq_bytes)
    if depth == 0:
        st["uniq_part_bytes"][-1] = out.uo - u_start
    if out.f is not None:
        out.fo += int(r.fresh_bytes)
    st["in_records"] += int(r.in_records)
    st["uniq_records"] += int(r.uniq_records)
    st["fresh_records"] += int(r.fresh_records)


def split_parts(buf, part_bytes: Sequence[int]) -> List:
    """Views of a part-ordered buffer (e.g. dedup_diff_large's unique output with
    st["uniq_part_bytes"]): one per part, None where empty."""
    res, off = [], 0
    for n in part_bytes:
        res.append(buf[off:off + n] if n else None)
        off += n
    return res


def pieces_bytes(pieces) -> Tuple[int, int]:
    return sum(p.numel() for p in pieces), len(pieces)
