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
    pbytes, _ = ctx.partition(buf.data_ptr(), n, world, send.data_ptr(), send.numel())
    return exchange_records(send, pbytes, group)


def dedup_diff_step(ctx, cur: torch.Tensor, prior_part: torch.Tensor, group=None):
    """One distributed dedup+diff step. Returns (device result, received byte count)."""
    recv = partition_exchange(ctx, cur, cur.numel(), group)
    r = ctx.dedup_diff(recv.data_ptr(), recv.numel(), prior_part.data_ptr() if prior_part.numel() else 0,
                       prior_part.numel())
    return r, recv


def build_prior_partition(ctx, candidates: torch.Tensor, group=None) -> torch.Tensor:
    """Setup (untimed): route this rank's prior candidate records to their owners and sort -u
    them there, giving the rank's resident prior partition."""
    recv = partition_exchange(ctx, candidates, candidates.numel(), group)
    r = ctx.dedup_diff(recv.data_ptr(), recv.numel(), 0, 0)
    out = torch.empty(max(int(r.uniq_bytes), 1), dtype=torch.uint8, device=candidates.device)
    if r.uniq_bytes:
        ctx.memcpy(out.data_ptr(), r.uniq, int(r.uniq_bytes))
    return out[: int(r.uniq_bytes)]
