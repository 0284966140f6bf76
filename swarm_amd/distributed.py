"""Multi-GPU dedup+diff: one process per GPU, torch.distributed with the
"nccl" backend (RCCL over xGMI on ROCm). The reference's only parallelism is chunked data
parallelism (server/server.py:185-187 splits the target list, :414-461 queues the chunks);
here the records themselves are sharded, by byte range, so the global sort -u survives.

C5 step on every rank (dedup_diff_rounds_step, BASELINE configs[4]):
  1. ONE partition call routes all of the rank's pieces into world x R byte ranges (byte
     splitters agreed across ranks at setup) laid out round-major: round p = range p of
     rank 0, of rank 1, ... back to back (sg_dev_partition_bytes_pieces_rounds);
  2. ONE all-to-all of the world x R part sizes (host ints);
  3. R all-to-alls of bytes queued at once on RCCL's stream, straight from the partition
     output; round p's receive buffer IS the rank's local range p;
  4. part p is deduped and diffed against the rank's stored prior part p as soon as round p
     has arrived (work.wait() orders the compute stream after it), while rounds p+1.. are
     still on the xGMI links: the exchange hides behind the dedup.
Rank r ends with byte range r, so the ranks' outputs concatenated in rank order are the
global sort -u / comm -13 output: no merge exists because none is needed.

The gloo backend (CPU tests, several ranks rehearsing on one GPU) runs the same code; only
the transport differs (host staging in all_to_all_bytes / exchange_counts).

Also here: hash routing (sg_dev_partition by hash64, dedup_diff_step) and the single-call C2
shard path (dedup_diff_range_shard); matching (match_step) needs no record exchange:
replicated automata, contiguous input shards, summed counts.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import torch
import torch.distributed as dist

from . import _abi

_U64 = (1 << 64) - 1


def _i64(v: int) -> int:
    """A uint64 (a handover checksum) as the int64 with the same bits, for an int64 tensor."""
    v = int(v) & _U64
    return v - (1 << 64) if v >> 63 else v


def host_staged(group=None) -> bool:
    """gloo rehearsals (several ranks sharing one GPU, or CPU tests): the collectives take host
    tensors. This is the only place the gloo and nccl (RCCL) paths differ: the transport."""
    return dist.get_backend(group) == "gloo"


def _coll_device(group=None):
    return torch.device("cpu") if host_staged(group) else torch.device("cuda", torch.cuda.current_device())


def all_max_float(x: float, group=None) -> float:
    """max over ranks of a host float (the bench's elapsed time)."""
    t = torch.tensor([float(x)], dtype=torch.float64, device=_coll_device(group))
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def all_max_int(x: int, group=None) -> int:
    t = torch.tensor([int(x)], dtype=torch.int64, device=_coll_device(group))
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return int(t.item())


def exchange_counts(counts: Sequence[int], group=None) -> List[int]:
    """All-to-all of host integers: `counts` holds world x m values (m for each peer, in rank
    order); returns the world x m values the peers sent to this rank (source-rank order)."""
    t = torch.tensor([int(x) for x in counts], dtype=torch.int64, device=_coll_device(group))
    o = torch.empty_like(t)
    dist.all_to_all_single(o, t, group=group)
    return [int(x) for x in o.tolist()]


# Largest per-peer message of one RCCL all-to-all. The RCCL in this image (2.26.6, torch's
# wheel) returns wrong bytes for 1-rank all_to_all_single messages of 1,536 MB where 1,024 MB
# ones are exact (tools/rccl_probe.py): larger exchanges go as point-to-point
# pieces of at most this many bytes.
A2A_CHUNK = 512 << 20


def a2a_pieces(size: int, chunk: int) -> List[Tuple[int, int]]:
    """(start, end) pieces of one message of `size` bytes, each at most `chunk` long. Both
    ends of a message know its size, so sender and receiver cut it the same way."""
    return [(a, min(a + chunk, size)) for a in range(0, size, chunk)]


def _offsets(splits: Sequence[int]) -> List[int]:
    o, a = [], 0
    for x in splits:
        o.append(a)
        a += x
    return o


class _Works:
    """wait() of several async operations (the pieces of one chunked exchange)."""

    def __init__(self, works):
        self.works = works

    def wait(self):
        for w in self.works:
            w.wait()
        return True


_SIDE = {}


def _side_stream(device) -> "torch.cuda.Stream":
    s = _SIDE.get(device)
    if s is None:
        s = _SIDE[device] = torch.cuda.Stream(device=device)
    return s


class _EventWork:
    """wait() of a copy queued on a side stream: the caller's stream waits for its event."""

    def __init__(self, ev):
        self.ev = ev

    def wait(self):
        torch.cuda.current_stream().wait_event(self.ev)
        return True


def all_to_all_bytes(recv: torch.Tensor, send: torch.Tensor, out_splits: Sequence[int], in_splits: Sequence[int],
                     group=None, async_op: bool = False, global_max: int = None):
    """All-to-all of byte buffers with host split sizes (sum(in_splits) == send.numel(),
    sum(out_splits) == recv.numel()). RCCL: straight between the device buffers, optionally
    async (the returned work's wait() orders the caller's stream after it). gloo with device
    buffers: staged through host copies, synchronously (returns None).

    Every rank takes the same path: one all_to_all_single when the largest message of the
    whole exchange (global_max, the max over ranks of their largest split; agreed here by one
    max all-reduce when the caller has not) is at most A2A_CHUNK, else every message goes
    as point-to-point pieces of at most A2A_CHUNK bytes (one batched isend/irecv list; a
    rank's message to itself is a local copy). So no rank issues a collective its peers do
    not."""
    out_splits, in_splits = [int(x) for x in out_splits], [int(x) for x in in_splits]
    if host_staged(group) and (send.is_cuda or recv.is_cuda):
        h = torch.empty(recv.numel(), dtype=torch.uint8)
        dist.all_to_all_single(h, send.cpu(), output_split_sizes=out_splits, input_split_sizes=in_splits,
                               group=group)
        recv.copy_(h)
        return None
    if global_max is None:
        global_max = all_max_int(max(out_splits + in_splits + [0]), group)
    if global_max <= A2A_CHUNK:
        return dist.all_to_all_single(recv, send, output_split_sizes=out_splits, input_split_sizes=in_splits,
                                      group=group, async_op=async_op)
    me = dist.get_rank(group) if group is not None else dist.get_rank()
    io, oo = _offsets(in_splits), _offsets(out_splits)
    ops = []
    self_work = None
    for g in range(len(in_splits)):
        peer = dist.get_global_rank(group, g) if group is not None else g
        if g == me:
            if in_splits[g] != out_splits[g]:
                raise ValueError("self message: %d bytes sent, %d expected" % (in_splits[g], out_splits[g]))
            dst, src = recv[oo[g]:oo[g] + out_splits[g]], send[io[g]:io[g] + in_splits[g]]
            if async_op and recv.is_cuda and out_splits[g]:
                # on a side stream, as RCCL's own copies run: it overlaps the caller's work on
                # the earlier rounds instead of queueing ahead of it
                side = _side_stream(recv.device)
                side.wait_stream(torch.cuda.current_stream(recv.device))
                with torch.cuda.stream(side):
                    dst.copy_(src)
                recv.record_stream(side)
                send.record_stream(side)
                ev = torch.cuda.Event()
                ev.record(side)
                self_work = _EventWork(ev)
            else:
                dst.copy_(src)
            continue
        for a, b in a2a_pieces(in_splits[g], A2A_CHUNK):
            ops.append(dist.P2POp(dist.isend, send[io[g] + a:io[g] + b], peer, group))
        for a, b in a2a_pieces(out_splits[g], A2A_CHUNK):
            ops.append(dist.P2POp(dist.irecv, recv[oo[g] + a:oo[g] + b], peer, group))
    works = dist.batch_isend_irecv(ops) if ops else []
    if self_work is not None:
        works = list(works) + [self_work]
    if async_op:
        return _Works(works)
    for w in works:
        w.wait()
    return None


def exchange_records(send: torch.Tensor, part_bytes: Sequence[int], group=None) -> torch.Tensor:
    """All-to-all of a partitioned byte buffer: `send` holds part 0's bytes, then part 1's,
    ... (part_bytes[i] each). Returns the bytes all ranks sent to this rank, in rank order."""
    world = dist.get_world_size(group)
    if len(part_bytes) != world:
        raise ValueError("part_bytes has %d entries for world size %d" % (len(part_bytes), world))
    out_list = exchange_counts(part_bytes, group)
    recv = torch.empty(sum(out_list), dtype=torch.uint8, device=send.device)
    all_to_all_bytes(recv, send[: int(sum(part_bytes))], out_list, part_bytes, group)
    return recv


def partition_exchange(ctx, buf: torch.Tensor, n: int, group=None) -> torch.Tensor:
    """GPU partition of `buf[:n]` by record hash, then the all-to-all exchange."""
    world = dist.get_world_size(group)
    send = torch.empty(n + 1, dtype=torch.uint8, device=buf.device)
    ctx.fence_in()
    pbytes, _ = ctx.partition(buf.data_ptr(), n, world, send.data_ptr(), send.numel())
    ctx.fence_out()  # the partition's copy pass is queued on the ctx stream; the collective reads send
    return exchange_records(send, pbytes, group)


def dedup_diff_step(ctx, cur: torch.Tensor, prior_part: torch.Tensor, group=None):
    """One distributed dedup+diff step. Returns (device result, received byte count)."""
    recv = partition_exchange(ctx, cur, cur.numel(), group)
    ctx.fence_in()
    r = ctx.dedup_diff(recv.data_ptr(), recv.numel(), prior_part.data_ptr() if prior_part.numel() else 0,
                       prior_part.numel())
    return r, recv


def build_prior_partition(ctx, candidates: torch.Tensor, group=None) -> torch.Tensor:
    """Setup (untimed): route this rank's prior candidate records to their owners and sort -u
    them there, giving the rank's resident prior partition."""
    recv = partition_exchange(ctx, candidates, candidates.numel(), group)
    ctx.fence_in()
    r = ctx.dedup_diff(recv.data_ptr(), recv.numel(), 0, 0)
    out = torch.empty(max(int(r.uniq_bytes), 1), dtype=torch.uint8, device=candidates.device)
    if r.uniq_bytes:
        ctx.fence_in()
        ctx.memcpy(out.data_ptr(), r.uniq, int(r.uniq_bytes))
    return out[: int(r.uniq_bytes)]


# ------------------------------------------------------------------ C5: range-partitioned shards
def agree_splitters(ctx, pieces: Sequence[torch.Tensor], parts: int, samples_per_piece: int = 1 << 12,
                    group=None):
    """parts - 1 byte splitters, quantiles of records sampled from every rank's pieces (their
    first SPLIT_BYTES bytes), identical on every rank."""
    from . import sharded
    local = sharded.sample_records(ctx, pieces, samples_per_piece)
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        allv = [None] * dist.get_world_size(group)
        dist.all_gather_object(allv, local, group=group)
        local = [x for v in allv for x in v]
    return sharded.choose_splitters(local, parts)


def range_exchange(ctx, pieces: Sequence[torch.Tensor], gsplit, group=None, piece_bytes: int = 3 << 30):
    """Route every piece into world key ranges and exchange, one all-to-all per piece straight
    from the partition output (parts are contiguous in it, so nothing is concatenated first);
    returns this rank's range as pieces of < piece_bytes ending at record boundaries, in
    (piece, source rank) order. Ranks may hold different numbers of pieces."""
    from . import sharded
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if world == 1:
        return [q for p in pieces if p.numel() for q in sharded.split_at_newlines(p, piece_bytes)]
    dev = pieces[0].device if len(pieces) else ctx.torch_device
    npieces = exchange_counts([len(pieces)] * world, group)
    out_pieces = []
    for i in range(max(npieces)):
        p = pieces[i] if i < len(pieces) else torch.empty(0, dtype=torch.uint8, device=dev)
        n = int(p.numel())
        send = torch.empty(n + 16, dtype=torch.uint8, device=dev)
        if n:
            ctx.fence_in()
            pb = sharded.route_piece(ctx, p, gsplit, send.data_ptr(), send.numel())
            ctx.fence_out()  # the routing copy is queued on the ctx stream; the collective reads send
        else:
            pb = [0] * world
        recv = exchange_records(send, pb, group)
        del send
        if recv.numel():
            out_pieces += sharded.split_at_newlines(recv, piece_bytes)
    return out_pieces


# ------------------------------------------------------------------ exchange in rounds (C5)
def plan_rounds(bytes_per_rank: int, world: int, part_bytes: int = 2 << 30, min_rounds: int = 4) -> int:
    """Local range parts per rank: enough that each stays well under one library call
    (part_bytes, with 25 % headroom for imbalance), and at least min_rounds when there is an
    exchange to hide (round p + 1 travels while round p is deduped); G x rounds <= 256."""
    r = max(1, -(-int(bytes_per_rank * 1.25) // part_bytes))
    if world > 1:
        r = max(r, min_rounds)
    return int(max(1, min(r, 256 // max(world, 1))))


def exchange_rounds(ctx, pieces: Sequence[torch.Tensor], splitters, rounds: int, group=None,
                    force_exchange: bool = False, spans: bool = True):
    """Route this rank's pieces into world x rounds byte ranges with ONE partition call (the
    parts laid out round-major, sg_dev_partition_bytes_pieces_rounds), exchange every part's
    size and record count with ONE all-to-all, then queue one all-to-all per round, all at once
    (async on RCCL's stream). Returns ([(work or None, receive tensor, records the sources
    routed into it) per round], send buffer): the receive tensor of round p is this rank's
    local range p (every source's records of it, in source rank order), and work.wait()
    orders the caller's stream after its arrival. The send buffer must stay referenced until
    every round has been waited for.
    spans: every record's parse travels with its bytes (its span, relative to its source's
    bytes, and its first-chunk key: 16 B per record, written by the routing pass itself), so
    the receiver dedups the round without parsing it again; the 4th element of a round is
    then (spans, keys, [first record, byte offset] per source, handover checksum) — the
    segments for rebase_spans, the checksum (the sources' part sums, which travel with the
    sizes) for dedup_diff_spans_into, which checks the parse against it — else None.
    force_exchange: issue the size exchange and the per-round all-to-alls even at world size 1
    (a 1-rank RCCL group on one GPU runs the device-tensor collective path of the N-rank step;
    without it a single rank skips the collectives)."""
    from .api import round_offsets
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    live = [p for p in pieces if p is not None and p.numel()]
    dev = pieces[0].device if len(pieces) else ctx.torch_device
    nparts = world * rounds
    if len(splitters) != nparts - 1:
        raise ValueError("%d splitters for %d ranks x %d rounds" % (len(splitters), world, rounds))
    total = sum(int(p.numel()) for p in live)
    send = torch.empty(total + len(live) + 16 * (rounds + 1), dtype=torch.uint8, device=dev)
    ssp = skey = None
    if live:
        ctx.fence_in()
        plist = [(p.data_ptr(), p.numel()) for p in live]
        if spans:
            nrec = ctx.partition_pieces_count(plist)
            ssp = torch.empty(2 * max(nrec, 1), dtype=torch.int32, device=dev)
            skey = torch.empty(max(nrec, 1), dtype=torch.int64, device=dev)
            pb, pr, ps = ctx.partition_bytes_pieces_rounds_spans(plist, splitters, rounds, send.data_ptr(),
                                                                 send.numel(), ssp.data_ptr(), skey.data_ptr(), nrec)
        else:
            pb, pr = ctx.partition_bytes_pieces_rounds(plist, splitters, rounds, send.data_ptr(), send.numel())
            ps = [0] * nparts
        # the partition's copy pass is queued on the ctx stream and the call returns after the
        # size read-back only: drain it before a collective (on another stream) reads send
        ctx.fence_out()
    else:
        pb, pr, ps = [0] * nparts, [0] * nparts, [0] * nparts
        if spans:
            ssp = torch.empty(2, dtype=torch.int32, device=dev)
            skey = torch.empty(1, dtype=torch.int64, device=dev)
    R = rounds
    # records of round p start at rround[p] in the span outputs (round-major, like the bytes)
    rround, acc = [], 0
    for p in range(R):
        rround.append(acc)
        acc += sum(int(pr[g * R + p]) for g in range(world))
    if world == 1 and not (force_exchange and dist.is_initialized()):
        offs = round_offsets(pb, rounds)
        out = []
        for p in range(rounds):
            par = None
            if spans:
                r0, nr = rround[p], int(pr[p])
                par = (ssp[2 * r0:2 * (r0 + nr)], skey[r0:r0 + nr], [[0, 0]], int(ps[p]))
            out.append((None, send[offs[p]:offs[p] + pb[p]], int(pr[p]), par))
        return out, (send, ssp, skey)
    # per peer g: the bytes, the records and the handover checksums of its rounds parts
    # g * rounds .. + rounds - 1 (contiguous in pb / pr / ps); back: rc2[s * 3R + p] bytes,
    # rc2[s * 3R + R + p] records and rc2[s * 3R + 2R + p] the checksum that source s sends this
    # rank in round p (checksums as int64 two's complement)
    R = rounds
    cnt = []
    for g in range(world):
        cnt += [int(x) for x in pb[g * R:(g + 1) * R]] + [int(x) for x in pr[g * R:(g + 1) * R]]
        cnt += [_i64(x) for x in ps[g * R:(g + 1) * R]]
    rc2 = exchange_counts(cnt, group)
    rc = [rc2[s * 3 * R + p] for s in range(world) for p in range(R)]
    rcr = [rc2[s * 3 * R + R + p] for s in range(world) for p in range(R)]
    rcs = [rc2[s * 3 * R + 2 * R + p] & _U64 for s in range(world) for p in range(R)]
    rrec = [sum(rcr[s * R + p] for s in range(world)) for p in range(R)]
    offs = round_offsets(pb, rounds)
    # the largest message of any round on any rank (bytes, and 8 B per record for the spans
    # and keys): every rank picks the same transport
    gmax = all_max_int(max(list(pb) + list(rc) + [8 * int(x) for x in list(pr) + rcr] + [0]), group)
    out = []
    for p in range(rounds):
        ins = [pb[g * rounds + p] for g in range(world)]
        outs = [rc[s * rounds + p] for s in range(world)]
        recv = torch.empty(sum(outs), dtype=torch.uint8, device=dev)
        w = all_to_all_bytes(recv, send[offs[p]:offs[p] + sum(ins)], outs, ins, group, async_op=True,
                             global_max=gmax)
        par = None
        if spans:
            ins_r = [int(pr[g * rounds + p]) for g in range(world)]
            outs_r = [rcr[s * rounds + p] for s in range(world)]
            r0, nin, nout = rround[p], sum(ins_r), sum(outs_r)
            rsp = torch.empty(2 * max(nout, 1), dtype=torch.int32, device=dev)
            rk = torch.empty(max(nout, 1), dtype=torch.int64, device=dev)
            ws = [w]
            for src, dst in ((ssp[2 * r0:2 * (r0 + nin)], rsp[:2 * nout]), (skey[r0:r0 + nin], rk[:nout])):
                ws.append(all_to_all_bytes(dst.view(torch.uint8), src.view(torch.uint8), [8 * x for x in outs_r],
                                           [8 * x for x in ins_r], group, async_op=True, global_max=gmax))
            w = _Works([x for x in ws if x is not None])
            segs, fr, fo = [], 0, 0
            for s_ in range(world):
                segs.append([fr, fo])
                fr += outs_r[s_]
                fo += outs[s_]
            par = (rsp[:2 * nout], rk[:nout], segs, sum(rcs[s_ * rounds + p] for s_ in range(world)) & _U64)
        out.append((w, recv, rrec[p], par))
    return out, (send, ssp, skey)


def dedup_diff_rounds_step(ctx, cur_pieces, prior_parts, splitters, rounds: int, group=None, align_parts=False,
                           force_exchange: bool = False):
    """One multi-GPU dedup+diff step in exchange rounds: rank r ends with byte range r split
    into `rounds` local parts; each part is deduped and diffed against the rank's stored prior
    part as soon as its round has arrived, while the later rounds are still on the wire. The
    ranks' outputs concatenated in rank order are the global sort -u / comm -13 output.
    prior_parts: this rank's stored prior, one tensor (or None) per local part (None: no
    prior). Returns (unique, new, stats) device tensors (new is unique without a prior).
    force_exchange: run the collectives at world size 1 too (exchange_rounds)."""
    from . import sharded
    recvd, send = exchange_rounds(ctx, cur_pieces, splitters, rounds, group, force_exchange)
    have_prior = prior_parts is not None and any(p is not None and p.numel() for p in prior_parts)
    if prior_parts is not None and len(prior_parts) != rounds:
        raise ValueError("prior_parts has %d entries for %d rounds" % (len(prior_parts), rounds))
    dev = recvd[0][1].device
    st = sharded.new_stats(rounds)
    st["recv_bytes"] = [int(r.numel()) for _, r, _, _ in recvd]
    out = sharded._Results(sum(st["recv_bytes"]) + 4096, dev, have_prior, align16=align_parts)
    for p, (w, recv, want, par) in enumerate(recvd):
        if w is not None:
            w.wait()
        before = st["in_records"]
        parse = None
        if par is not None and (want or recv.numel()):
            rsp, rk, segs, ssum = par
            # the spans arrive relative to each source's bytes: rebased to this buffer, and each
            # source's first and last records checked to end before a '\n' (a short or stale
            # message is reported here, at its tail)
            if want and (w is not None or len(segs) > 1 or segs[0][1]):
                ctx.fence_in()
                bad = ctx.rebase_spans(recv.data_ptr(), recv.numel(), rsp.data_ptr(), want, [x[0] for x in segs],
                                       [x[1] for x in segs])
                if bad:
                    raise RuntimeError("exchange round %d: %d of %d records do not end at a newline of the %d "
                                       "received bytes: the transfer is corrupt" % (p, bad, want, recv.numel()))
            # every record's span and key is then checked by the dedup itself before any kernel
            # reads a byte through them (records tile the buffer, the senders' checksum, sampled
            # newlines and keys; include/swarmgpu.h sg_dev_dedup_diff_spans_into)
            parse = (rsp.data_ptr(), rk.data_ptr(), want, ssum)
        try:
            sharded.dedup_part(ctx, recv if recv.numel() else None, prior_parts[p] if have_prior else None, out, st,
                               parse=parse)
        except _abi.SGError as e:
            if e.rc != _abi.SG_E_CORRUPT:
                raise
            raise RuntimeError("exchange round %d: the parse handed over with %d records / %d bytes does not match "
                               "them: the transfer is corrupt (%s)" % (p, want, recv.numel(), e)) from e
        # without the parse handed over, the dedup parsed the bytes itself: its record count
        # must be the one the senders routed (round 4: this image's RCCL left half of a 1.5 GB
        # message unwritten; a transfer that delivered other bytes fails here)
        if parse is None and st["in_records"] - before != want:
            raise RuntimeError("exchange round %d: %d records arrived, the senders routed %d (%d bytes): the "
                               "transfer is corrupt" % (p, st["in_records"] - before, want, recv.numel()))
    del send, recvd
    u = out.u[:out.uo]
    return u, (out.f[:out.fo] if have_prior else u), st


def build_prior_rounds(ctx, prior_pieces, splitters, rounds: int, group=None, force_exchange: bool = False):
    """Setup (untimed): route the rank's share of the prior scan's records to their owners
    with the same splitters and sort -u them there: returns the rank's stored prior, one
    16-byte aligned tensor per local part (read in place by every later step), and the
    stored bytes."""
    from . import sharded
    u, _, st = dedup_diff_rounds_step(ctx, prior_pieces, None, splitters, rounds, group, align_parts=True,
                                      force_exchange=force_exchange)
    return sharded.stored_parts(u, st), u


def build_prior_range(ctx, candidates: torch.Tensor, gsplit, group=None) -> torch.Tensor:
    """Setup (untimed): route this rank's prior candidate records to the rank owning their key
    range and sort -u them there: the rank's resident slice of the prior scan, in byte order."""
    mine = range_exchange(ctx, [candidates], gsplit, group)
    dev = candidates.device
    if not mine:
        return torch.empty(0, dtype=torch.uint8, device=dev)
    buf = mine[0] if len(mine) == 1 else torch.cat(mine)
    ctx.fence_in()
    r = ctx.dedup_diff(buf.data_ptr(), buf.numel(), 0, 0)
    out = torch.empty(max(int(r.uniq_bytes), 1), dtype=torch.uint8, device=dev)
    if r.uniq_bytes:
        ctx.fence_in()
        ctx.memcpy(out.data_ptr(), r.uniq, int(r.uniq_bytes))
    return out[: int(r.uniq_bytes)]


def dedup_diff_range_shard(ctx, cur: torch.Tensor, prior_slice: torch.Tensor, gsplit, group=None):
    """One multi-GPU dedup+diff step for a shard that fits one library call (C2 per GPU):
    key0-range all-to-all, then sort -u + diff against the rank's prior slice. Rank r ends
    with the records of key range r, so the ranks' outputs concatenated in rank order are the
    global sort -u / comm -13 output (no merge). Returns (device result, received bytes)."""
    mine = range_exchange(ctx, [cur], gsplit, group)
    buf = (mine[0] if len(mine) == 1 else torch.cat(mine)) if mine else torch.empty(0, dtype=torch.uint8,
                                                                                     device=cur.device)
    ctx.fence_in()
    r = ctx.dedup_diff(buf.data_ptr() if buf.numel() else 0, buf.numel(),
                       prior_slice.data_ptr() if prior_slice.numel() else 0, prior_slice.numel())
    return r, buf


# ------------------------------------------------------------------ A4 matching across GPUs
def shard_bounds(buf, world: int) -> List[int]:
    """world + 1 cut points of a '\n'-separated byte buffer (numpy uint8 or bytes) at record
    boundaries, near equal byte counts: rank r matches buf[cuts[r]:cuts[r+1]]."""
    import numpy as np
    a = np.frombuffer(memoryview(buf), dtype=np.uint8) if not isinstance(buf, np.ndarray) else buf
    n = a.size
    nl = np.flatnonzero(a == 0x0A)
    cuts = [0]
    for k in range(1, world):
        j = np.searchsorted(nl, n * k // world)
        cuts.append(int(nl[j]) + 1 if j < nl.size else n)
    cuts.append(n)
    for k in range(1, len(cuts)):
        cuts[k] = max(cuts[k], cuts[k - 1])
    return cuts


def match_step(ctx, matcher, shard: torch.Tensor, group=None):
    """Multi-GPU signature matching: the automata are replicated (each rank
    compiled the same signatures), every rank matches its own contiguous shard of the input,
    and the only exchange is the count reduction. Returns (this rank's DevHits, global
    (records, hits, matched records)). The global grep output is the ranks' matched lines
    concatenated in rank order (gather_lines)."""
    r = matcher.dev_match(ctx, shard.data_ptr() if shard.numel() else 0, shard.numel())
    vals = [int(r.in_records), int(r.n_hits), int(r.matched_records)]
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        t = torch.tensor(vals, dtype=torch.int64, device=_coll_device(group))
        dist.all_reduce(t, group=group)
        vals = [int(x) for x in t.tolist()]
    return r, tuple(vals)


def gather_lines(local: bytes, group=None) -> bytes:
    """The ranks' byte outputs concatenated in rank order, on every rank (tests / small
    outputs; a writer would stream them instead)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return local
    allv = [None] * dist.get_world_size(group)
    dist.all_gather_object(allv, local, group=group)
    return b"".join(allv)


def dedup_diff_range_step(ctx, cur_pieces, prior_local, gsplit, lsplit, group=None, prior_parts=None):
    """One C5 step on this rank: range exchange (world > 1), then local range parts
    (sharded.dedup_diff_large with the rank's fixed local splitters). prior_parts: the
    rank's stored prior already split by lsplit (then prior_local is not routed again)."""
    from . import sharded
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    mine = range_exchange(ctx, cur_pieces, gsplit, group) if world > 1 else list(cur_pieces)
    if prior_parts is not None:
        return sharded.dedup_diff_large(ctx, mine, (), splitters=lsplit, prior_parts=prior_parts)
    return sharded.dedup_diff_large(ctx, mine, prior_local, splitters=lsplit)
