"""The N>1 path on CPU: world_size 2 (and 3) over gloo. Each rank partitions its shard
with the hash restatement (the GPU partition's own parity is tested in test_gpu_dedup),
exchanges through swarm_amd.distributed.exchange_records (the same function the bench
uses over RCCL), dedups+diffs its partition with the oracle, and the union of the ranks'
outputs must equal the single-process result."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from hash_oracle import hash64, part_of
from oracle import semantics as S


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def shard(rank, world):
    import random
    rng = random.Random(77)
    recs = [b"h%d.target%d.com" % (rng.randrange(3000), rng.randrange(8)) for _ in range(6000)]
    recs += [b"", b"x\r", b"\x00\xff"]
    per = len(recs) // world
    mine = recs[rank * per:(rank + 1) * per] if rank < world - 1 else recs[rank * per:]
    return b"\n".join(mine) + b"\n", recs


def prior_all():
    return b"".join(b"h%d.target%d.com\n" % (i, j) for i in range(0, 3000, 3) for j in range(8))


def worker(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from swarm_amd.distributed import exchange_records
    buf, _ = shard(rank, world)
    parts = [[] for _ in range(world)]
    for r in S.parse_records(buf):
        parts[part_of(hash64(r), world)].append(r + b"\n")
    send = b"".join(b"".join(p) for p in parts)
    pbytes = [sum(len(x) for x in p) for p in parts]
    t = torch.frombuffer(bytearray(send + b"\0"), dtype=torch.uint8)
    recv = exchange_records(t, pbytes)
    got = bytes(recv.numpy().tobytes())
    # every received record belongs to this rank
    assert all(part_of(hash64(r), world) == rank for r in S.parse_records(got))
    prior_part = b"".join(r + b"\n" for r in S.parse_records(prior_all()) if part_of(hash64(r), world) == rank)
    u, f = S.dedup_diff(got, prior_part)
    out_q.put((rank, u, f))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_exchange_dedup_diff_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    _, allrecs = shard(0, world)
    full = b"\n".join(allrecs) + b"\n"
    eu, ef = S.dedup_diff(full, prior_all())
    u = sorted(r for _, x, _ in res for r in S.parse_records(x))
    f = sorted(r for _, _, x in res for r in S.parse_records(x))
    assert S.serialize(u) == eu and S.serialize(f) == ef
    # partitions are disjoint
    assert len(u) == len(set(u))
