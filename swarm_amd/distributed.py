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

The C5 path (1B host:port records, shards larger than one 4 GiB call) routes by key0 RANGE
instead (sg_dev_partition_range with splitters agreed across ranks): rank r owns key range
r, so the ranks' outputs concatenated in rank order are the global sort -u output, and each
rank processes its range with swarm_amd.sharded (local range parts of < 4 GiB).
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
def agree_splitters(ctx, pieces: Sequence[torch.Tensor], parts: int, samples_per_piece: int = 1 << 14,
                    group=None):
    """Splitters (parts - 1 key0 quantiles) from key0 samples of every rank's pieces."""
    import numpy as np
    from . import sharded
    local = [ctx.key_sample(p.data_ptr(), p.numel(), samples_per_piece)[0] for p in pieces if p.numel()]
    local = np.concatenate(local) if local else np.zeros(0, dtype=np.uint64)
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        allv = [None] * dist.get_world_size(group)
        dist.all_gather_object(allv, local, group=group)
        local = np.concatenate(allv)
    return sharded.choose_splitters(local, parts)


def range_exchange(ctx, pieces: Sequence[torch.Tensor], gsplit, group=None, piece_bytes: int = 3 << 30):
    """Route every piece into world key ranges, exchange, return this rank's range as
    pieces of < piece_bytes ending at record boundaries."""
    from . import sharded
    parts = sharded.route(ctx, pieces, gsplit)
    dev = pieces[0].device if len(pieces) else torch.device("cuda", ctx.device)
    pb = [int(p.numel()) if p is not None else 0 for p in parts]
    send = torch.cat([p for p in parts if p is not None]) if any(pb) else torch.empty(0, dtype=torch.uint8, device=dev)
    del parts
    recv = exchange_records(send, pb, group)
    del send
    return sharded.split_at_newlines(recv, piece_bytes) if recv.numel() else []


def dedup_diff_range_step(ctx, cur_pieces, prior_local, gsplit, lsplit, group=None):
    """One C5 step on this rank: range exchange (world > 1), then local range parts
    (sharded.dedup_diff_large with the rank's fixed local splitters)."""
    from . import sharded
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    mine = range_exchange(ctx, cur_pieces, gsplit, group) if world > 1 else list(cur_pieces)
    return sharded.dedup_diff_large(ctx, mine, prior_local, splitters=lsplit)
