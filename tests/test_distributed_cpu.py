"""The N>1 path on CPU: world_size 2 (and 3) over gloo. Each rank partitions its shard
with the hash restatement (the GPU partition's own parity is tested in test_gpu_dedup),
exchanges through swarm_amd.distributed.exchange_records (the same function the bench
uses over RCCL), dedups+diffs its partition with the oracle, and the union of the ranks'
outputs must equal the single-process result. The byte-range path (agree_splitters,
range_exchange: the C2/C5 multi-GPU routing) and match_step run through the real
swarm_amd.distributed code with the routing / matching restated on the host (FakeCtx):
rank outputs concatenated in rank order must equal the global oracle output."""
import os
import socket

import numpy as np
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


def url_shard(rank, world):
    import random
    rng = random.Random(900 + rank)
    recs = [b"https://h%d.example.com/%s" % (rng.randrange(4000), b"x" * rng.randrange(3)) for _ in range(3000)]
    recs += [b"", b"10.0.0.%d:443" % rank, b"\xff"]
    prior = [b"https://h%d.example.com/" % i for i in range(0, 4000, 3)]
    return b"\n".join(recs) + b"\n", S.serialize(prior[rank::world])


def range_worker(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from route_oracle import FakeCtx
    from swarm_amd import distributed as D
    ctx = FakeCtx()
    cur, prior = url_shard(rank, world)
    t = lambda b: torch.frombuffer(bytearray(b + b"\0"), dtype=torch.uint8)[: len(b)]  # noqa: E731
    gsplit = D.agree_splitters(ctx, [t(prior)], world, samples_per_piece=256)
    assert len(gsplit) == world - 1
    mine_p = D.range_exchange(ctx, [t(prior)], gsplit)
    # this rank sent a second (empty) piece: ranks with fewer pieces still join every exchange
    pieces = [t(cur[: len(cur) // 2 + cur[len(cur) // 2:].index(b"\n") + 1]),
              t(cur[len(cur) // 2 + cur[len(cur) // 2:].index(b"\n") + 1:])] if rank == 0 else [t(cur)]
    mine_c = D.range_exchange(ctx, pieces, gsplit, piece_bytes=4096)
    got_c = b"".join(bytes(p.numpy().tobytes()) for p in mine_c)
    got_p = b"".join(bytes(p.numpy().tobytes()) for p in mine_p)
    u, f = S.dedup_diff(got_c, S.dedup(got_p))
    out_q.put((rank, u, f, cur, prior, max(p.numel() for p in mine_c)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_range_exchange_global_order_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=range_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    cur_all = b"".join(r[3] for r in res)
    prior_all = S.dedup(b"".join(r[4] for r in res))
    eu, ef = S.dedup_diff(cur_all, prior_all)
    assert b"".join(r[1] for r in res) == eu
    assert b"".join(r[2] for r in res) == ef
    assert all(r[5] <= 4096 for r in res)  # received ranges re-cut at record boundaries


def rounds_shard(rank, world):
    """Unequal pieces per rank: rank 0 three pieces (one empty), rank 1 none at all (an empty
    rank), the others one; records share long prefixes (URLs) and include CR / 0xff bytes."""
    import random
    rng = random.Random(500 + rank)
    recs = [b"https://h%d.example.com/%s" % (rng.randrange(2500), b"x" * rng.randrange(3)) for _ in range(1500)]
    recs += [b"10.0.%d.%d:443" % (rank, rng.randrange(9)) for _ in range(50)] + [b"\xff", b"x\r", b""]
    cur = b"\n".join(recs) + b"\n"
    if rank == 1:
        return []
    if rank == 0:
        cut = cur.index(b"\n", len(cur) // 3) + 1
        return [cur[:cut], b"", cur[cut:]]
    return [cur]


def rounds_worker(rank, world, rounds, port, out_q, chunk=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from route_oracle import FakeCtx
    from swarm_amd import distributed as D
    if chunk:
        D.A2A_CHUNK = chunk  # every exchange in point-to-point pieces of at most this many bytes
    ctx = FakeCtx()
    t = lambda b: torch.frombuffer(bytearray(b + b"\0"), dtype=torch.uint8)[: len(b)]  # noqa: E731
    prior_raw = [b"https://h%d.example.com/\n" % i for i in range(rank, 2500, 2 * world)]
    prior_raw = b"".join(prior_raw) + (b"10.0.0.1:443\n" if rank == world - 1 else b"")
    split = D.agree_splitters(ctx, [t(prior_raw)], world * rounds, samples_per_piece=64)
    assert len(split) == world * rounds - 1
    prior_parts, stored = D.build_prior_rounds(ctx, [t(prior_raw)], split, rounds)
    assert len(prior_parts) == rounds
    cur = rounds_shard(rank, world)
    u, f, st = D.dedup_diff_rounds_step(ctx, [t(c) for c in cur], prior_parts, split, rounds)
    # every partition's copy is fenced before the collective that reads its output (ADVICE r3:
    # a ctx off torch's stream must not hand a half-written send buffer to the all-to-all)
    assert all(ctx.log[i + 1] == "fence_out" for i, x in enumerate(ctx.log) if x == "partition"), ctx.log
    # the received rounds are deduped with the parse the routing handed over (no second parse)
    assert "spans_into" in ctx.log, ctx.log
    out_q.put((rank, bytes(u.numpy().tobytes()), bytes(f.numpy().tobytes()), b"".join(cur), prior_raw,
               bytes(stored.numpy().tobytes()), st["parts"]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,rounds,chunk", [(2, 3, None), (3, 2, None), (2, 1, None), (2, 3, 37), (3, 2, 1000)])
def test_rounds_step_global_order_gloo(world, rounds, chunk):
    """dedup_diff_rounds_step (the C5 multi-GPU step: one partition into world x rounds ranges,
    one size exchange, one all-to-all per round, each part deduped as its round arrives): the
    ranks' outputs concatenated in rank order equal the global oracle output, with unequal
    piece counts, an empty piece and a rank holding nothing. chunk: messages capped at that
    many bytes (the point-to-point pieces path, ranks with uneven message sizes)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=rounds_worker, args=(r, world, rounds, port, q, chunk)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    cur_all = b"".join(r[3] for r in res)
    prior_all = b"".join(r[4] for r in res)
    eu, ef = S.dedup_diff(cur_all, prior_all)
    assert b"".join(r[1] for r in res) == eu
    assert b"".join(r[2] for r in res) == ef
    # the stored prior: 16-byte aligned parts padded with empty lines = the prior's sort -u
    assert S.serialize(S.parse_records(b"".join(r[5] for r in res))) == S.dedup(prior_all)
    assert all(r[6] == rounds for r in res)


def single_rank_worker(port, out_q):
    """A 1-rank group with force_exchange: the size exchange and the per-round all-to-alls run
    at world size 1 (the code path a 1-rank RCCL group exercises on one GPU)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=0, world_size=1)
    from route_oracle import FakeCtx
    from swarm_amd import distributed as D
    ctx = FakeCtx()
    t = lambda b: torch.frombuffer(bytearray(b + b"\0"), dtype=torch.uint8)[: len(b)]  # noqa: E731
    prior_raw = b"".join(b"https://h%d.example.com/\n" % i for i in range(0, 2500, 3))
    split = D.agree_splitters(ctx, [t(prior_raw)], 3, samples_per_piece=64)
    prior_parts, _ = D.build_prior_rounds(ctx, [t(prior_raw)], split, 3, force_exchange=True)
    cur = rounds_shard(0, 1)
    recvd, send = D.exchange_rounds(ctx, [t(c) for c in cur], split, 3, force_exchange=True)
    exchanged = [w for w, _, _, _ in recvd]
    u, f, st = D.dedup_diff_rounds_step(ctx, [t(c) for c in cur], prior_parts, split, 3, force_exchange=True)
    out_q.put((bytes(u.numpy().tobytes()), bytes(f.numpy().tobytes()), b"".join(cur), prior_raw, len(exchanged)))
    dist.destroy_process_group()


def test_rounds_step_force_exchange_single_rank():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=single_rank_worker, args=(free_port(), q))
    p.start()
    u, f, cur, prior, nround = q.get(timeout=120)
    p.join(timeout=60)
    assert p.exitcode == 0
    eu, ef = S.dedup_diff(cur, prior)
    assert u == eu and f == ef
    assert nround == 3


def test_a2a_pieces_cover_each_message_once():
    """A message of `size` bytes in pieces of at most `chunk`: in order, covering it once
    (sender and receiver cut a message the same way, both knowing its size)."""
    from swarm_amd.distributed import a2a_pieces
    rng = np.random.default_rng(5)
    for _ in range(200):
        size, chunk = int(rng.integers(0, 5000)), int(rng.integers(1, 700))
        pcs = a2a_pieces(size, chunk)
        assert len(pcs) == -(-size // chunk)
        pos = 0
        for a, b in pcs:
            assert a == pos and 0 < b - a <= chunk
            pos = b
        assert pos == size
    assert a2a_pieces(0, 16) == []


def a2a_worker(rank, world, port, chunk, out_q):
    """all_to_all_bytes with uneven splits: rank 0's messages all fit one piece, the others'
    do not. Every rank must take the same transport and deliver exact bytes."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from swarm_amd import distributed as D
    D.A2A_CHUNK = chunk
    rng = np.random.default_rng(100 + rank)
    ins = [int(rng.integers(0, chunk + 1)) if rank == 0 else int(rng.integers(0, 4 * chunk)) for _ in range(world)]
    ins[(rank + 1) % world] = 0  # an empty message
    outs = D.exchange_counts(ins)
    send = torch.cat([torch.full((n,), 16 * rank + g, dtype=torch.uint8) for g, n in enumerate(ins)])
    recv = torch.empty(sum(outs), dtype=torch.uint8)
    w = D.all_to_all_bytes(recv, send, outs, ins, async_op=True)
    if w is not None:
        w.wait()
    exp = torch.cat([torch.full((n,), 16 * s + rank, dtype=torch.uint8) for s, n in enumerate(outs)])
    out_q.put((rank, bool(torch.equal(recv, exp)), max(ins + outs)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_all_to_all_bytes_pieces_uneven_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=a2a_worker, args=(r, world, port, 64, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok, _ in res)
    assert max(m for _, _, m in res) > 64  # the pieces path ran


def test_plan_rounds():
    from swarm_amd.distributed import plan_rounds
    assert plan_rounds(1 << 20, 1) == 1
    assert plan_rounds(31_500_000_000, 1) == 19
    assert plan_rounds(4_000_000_000, 8) == 4          # at least 4 rounds to hide the exchange
    assert plan_rounds(16_000_000_000, 2) == 10
    assert plan_rounds(10 ** 12, 8) == 32              # world x rounds <= 256


class _Hits:
    def __init__(self, data, sigs):
        hits = S.literal_hits(data, sigs)
        self.in_records = len(S.parse_records(data))
        self.n_hits = len(hits)
        self.matched_records = len(S.parse_records(S.matched_lines(data, hits)))
        self.lines = S.matched_lines(data, hits)


class _FakeMatcher:
    def __init__(self, sigs):
        self.sigs = sigs

    def dev_match(self, ctx, ptr, n):
        import ctypes
        return _Hits(ctypes.string_at(ptr, n) if n else b"", self.sigs)


SIGS = [b"target1", b"h7", b".com\r"]


def match_worker(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import numpy as np
    from swarm_amd import distributed as D
    data, _ = shard(0, 1)
    data = data + b"h7.com\r\nlast-no-newline-target1"
    cuts = D.shard_bounds(np.frombuffer(data, dtype=np.uint8), world)
    assert cuts[0] == 0 and cuts[-1] == len(data)
    assert all(data[c - 1:c] == b"\n" for c in cuts[1:-1] if 0 < c < len(data))
    part = data[cuts[rank]:cuts[rank + 1]]
    t = torch.frombuffer(bytearray(part + b"\0"), dtype=torch.uint8)[: len(part)]
    r, tot = D.match_step(None, _FakeMatcher(SIGS), t)
    out_q.put((rank, tot, D.gather_lines(r.lines), data))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_match_step_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=match_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    data = res[0][3]
    hits = S.literal_hits(data, SIGS)
    want = (len(S.parse_records(data)), len(hits), len(S.parse_records(S.matched_lines(data, hits))))
    for _, tot, lines, _ in res:
        assert tot == want
        assert lines == S.matched_lines(data, hits)


def corrupt_worker(port, out_q, mode="half"):
    """A transfer that arrives damaged: "half" leaves the upper half of a round's receive
    buffer unwritten (what this image's RCCL does with a 1.5 GB message, tools/rccl_probe.py
    detail); "key" changes one record's key and "span" one record's end in the middle of a
    round (outside the records the rebase samples); "tail" drops the last record's span. The
    rounds step must raise, not dedup what arrived."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=0, world_size=1)
    from route_oracle import FakeCtx
    from swarm_amd import distributed as D
    ctx = FakeCtx()
    t = lambda b: torch.frombuffer(bytearray(b + b"\0"), dtype=torch.uint8)[: len(b)]  # noqa: E731
    prior_raw = b"".join(b"https://h%d.example.com/\n" % i for i in range(0, 2500, 3))
    split = D.agree_splitters(ctx, [t(prior_raw)], 2, samples_per_piece=64)
    real = D.all_to_all_bytes
    calls = [0]

    def damaged(recv, send, outs, ins, group=None, async_op=False, global_max=None):
        w = real(recv, send, outs, ins, group, async_op, global_max)
        if w is not None:
            w.wait()
        k = calls[0]  # per round: the bytes, then the spans, then the keys
        calls[0] += 1
        if mode == "half" and k % 3 == 0:
            recv[recv.numel() // 2:] = 0
        elif mode == "key" and k == 2:
            kk = recv.view(torch.int64)
            kk[kk.numel() // 2] ^= 1 << 20
        elif mode == "span" and k == 1:
            sp = recv.view(torch.int32)
            sp[2 * (sp.numel() // 4) + 1] += 1
        elif mode == "tail" and k == 1:
            sp = recv.view(torch.int32)
            sp[-1] -= 1
        return None

    D.all_to_all_bytes = damaged
    try:
        D.dedup_diff_rounds_step(ctx, [t(c) for c in rounds_shard(0, 1)], None, split, 2, force_exchange=True)
        out_q.put("no error")
    except RuntimeError as e:
        out_q.put(str(e))
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["half", "key", "span", "tail"])
def test_rounds_step_detects_corrupt_transfer(mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=corrupt_worker, args=(free_port(), q, mode))
    p.start()
    msg = q.get(timeout=120)
    p.join(timeout=60)
    assert "transfer is corrupt" in msg, msg
