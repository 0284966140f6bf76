"""Multi-GPU dedup+diff: one process per GPU, torch.distributed with the
"nccl" backend (RCCL over xGMI on ROCm).

Per step and rank:
  1. sg_dev_partition routes each record of the rank's shard to part(hash64(record), G),
     grouped by destination, '\\n'-terminated (the wire format IS the line format, so the
     received buffer feeds dedup directly);
  2. all_to_all_single of the G byte counts, then one all_to_all_single of the records —
     every peer pair on its own xGMI link;
  3. local sort -u + diff against the rank's partition of the prior scan (partitioned by
     the same hash once, and kept resident).
The union of the ranks' outputs is the global result; rank r owns the records that hash
to r. (A byte-ordered global file is a k-way merge of the G sorted outputs, done where the
file is written, outside this path.)

Range routing (sg_dev_partition_bytes with byte splitters agreed across ranks) keeps the
global byte order instead: rank r owns key range r, so the ranks' outputs concatenated in rank order
are the global sort -u output with no merge. The bench's C2 multi-GPU step uses it
(dedup_diff_range_shard); the C5 path (1B host:port records, shards larger than one 4 GiB
call) adds local range parts of < 4 GiB per rank (swarm_amd.sharded). Matching (match_step)
needs no record exchange: replicated automata, contiguous input shards, summed counts.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import torch
import torch.distributed as dist


def exchange_records(send: torch.Tensor, part_bytes: Sequence[int], group=None) -> torch.Tensor:
    """All-to-all of a partitioned byte buffer: `send` holds part 0's bytes, then part 1's,
    ... (part_bytes[i] each). Returns the bytes all ranks sent to this rank, in rank order."""
    world = dist.get_world_size(group)
    if len(part_bytes) != world:
        raise ValueError("part_bytes has %d entries for world size %d" % (len(part_bytes), world))
    if send.is_cuda and dist.get_backend(group) == "gloo":
        # rehearsal mode (several ranks sharing one GPU): the collective runs on host copies
        return exchange_records(send.cpu(), part_bytes, group).to(send.device)
    dev = send.device
    in_splits = torch.tensor(list(part_bytes), dtype=torch.int64, device=dev)
    out_splits = torch.empty_like(in_splits)
    dist.all_to_all_single(out_splits, in_splits, group=group)
    out_list: List[int] = [int(x) for x in out_splits.tolist()]
    total_in = int(sum(part_bytes))
    recv = torch.empty(sum(out_list), dtype=torch.uint8, device=dev)
    dist.all_to_all_single(recv, send[:total_in], output_split_sizes=out_list,
                           input_split_sizes=[int(x) for x in part_bytes], group=group)
    return recv


def partition_exchange(ctx, buf: torch.Tensor, n: int, group=None) -> torch.Tensor:
    """GPU partition of `buf[:n]` by record hash, then the all-to-all exchange."""
    world = dist.get_world_size(group)
    send = torch.empty(n + 1, dtype=torch.uint8, device=buf.device)
    ctx.fence_in()
    pbytes, _ = ctx.partition(buf.data_ptr(), n, world, send.data_ptr(), send.numel())
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
    dev = pieces[0].device if len(pieces) else torch.device("cuda", ctx.device)
    npieces = torch.tensor([len(pieces)], dtype=torch.int64, device=dev if dist.get_backend(group) != "gloo" else "cpu")
    dist.all_reduce(npieces, op=dist.ReduceOp.MAX, group=group)
    out_pieces = []
    for i in range(int(npieces.item())):
        p = pieces[i] if i < len(pieces) else torch.empty(0, dtype=torch.uint8, device=dev)
        n = int(p.numel())
        send = torch.empty(n + 16, dtype=torch.uint8, device=dev)
        if n:
            ctx.fence_in()
            pb = sharded.route_piece(ctx, p, gsplit, send.data_ptr(), send.numel())
        else:
            pb = [0] * world
        recv = exchange_records(send, pb, group)
        del send
        if recv.numel():
            out_pieces += sharded.split_at_newlines(recv, piece_bytes)
    return out_pieces


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
    t = torch.tensor([int(r.in_records), int(r.n_hits), int(r.matched_records)], dtype=torch.int64)
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        if dist.get_backend(group) != "gloo":
            t = t.to(shard.device)
        dist.all_reduce(t, group=group)
    return r, tuple(int(x) for x in t.tolist())


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
