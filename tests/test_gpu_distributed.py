"""Multi-rank rehearsal on one GPU: 2 ranks share cuda:0, exchange over gloo (host copies),
and run the real GPU partition (sg_dev_partition), the exchange
(swarm_amd.distributed.exchange_records) and the per-rank dedup+diff. The union of the
ranks' outputs must equal the oracle on the concatenated input, and every rank may only
hold records that hash to it."""
import os
import socket

import pytest

from hash_oracle import hash64, part_of
from oracle import semantics as S

pytestmark = pytest.mark.gpu


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def inputs(world):
    from swarm_amd import corpus
    shards = [corpus.subdomains(40_000, seed=500 + r, universe=40_000 * world) for r in range(world)]
    return shards


def worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import numpy as np
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import swarm_amd
    from swarm_amd import corpus
    from swarm_amd import distributed as D
    shards = inputs(world)
    buf, ids = shards[rank]
    ctx = swarm_amd.Context(0, torch.cuda.current_stream().cuda_stream)
    u = np.unique(ids)
    cand = corpus._flatten(*corpus.render_names(u[(u % np.uint64(10)) != 0]))
    prior = D.build_prior_partition(ctx, torch.from_numpy(cand).cuda())
    cur = torch.from_numpy(buf).cuda()
    r, recv = D.dedup_diff_step(ctx, cur, prior)
    torch.cuda.synchronize()
    q.put((rank, ctx.to_bytes(r.uniq, r.uniq_bytes), ctx.to_bytes(r.fresh, r.fresh_bytes),
           bytes(prior.cpu().numpy().tobytes())))
    dist.barrier()
    ctx.close()
    dist.destroy_process_group()


def test_two_ranks_on_one_gpu():
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    import numpy as np
    from swarm_amd import corpus
    shards = inputs(world)
    full = b"".join(b.tobytes() for b, _ in shards)
    all_ids = np.concatenate([i for _, i in shards])
    prior_full = corpus.prior_of(all_ids).tobytes()
    eu, ef = S.dedup_diff(full, prior_full)
    for rank, u, f, p in res:
        for rec in S.parse_records(u) + S.parse_records(p):
            assert part_of(hash64(rec), world) == rank
    u_all = sorted(rec for _, u, _, _ in res for rec in S.parse_records(u))
    f_all = sorted(rec for _, _, f, _ in res for rec in S.parse_records(f))
    assert S.serialize(u_all) == eu
    assert S.serialize(f_all) == ef


def range_worker(rank, world, port, q):
    """C5 path: byte-range exchange + local range parts; rank outputs in rank order must be
    the global sort -u / comm -13 output."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import swarm_amd
    from swarm_amd import corpus, sharded
    from swarm_amd import distributed as D
    ctx = swarm_amd.Context(0, torch.cuda.current_stream().cuda_stream)
    pool = corpus.host_pool_gpu(20_000, seed=5)
    U = 20_000 * len(corpus.PORTS)
    prior_raw = corpus.hostport_pieces(pool, 150_000, U // 10, U, seed=900 + rank, per_piece=40_000)
    cur = corpus.hostport_pieces(pool, 200_000, 0, U, seed=100 + rank, per_piece=60_000)
    gsplit = D.agree_splitters(ctx, prior_raw, world)
    mine = D.range_exchange(ctx, prior_raw, gsplit, piece_bytes=1 << 20)
    lsplit = sharded.choose_splitters(sharded.sample_records(ctx, mine, 512), 3)
    pu, _, _ = sharded.dedup_diff_large(ctx, mine, (), splitters=lsplit)
    u, f, st = D.dedup_diff_range_step(ctx, cur, sharded.split_at_newlines(pu, 1 << 20), gsplit, lsplit)
    torch.cuda.synchronize()
    q.put((rank, u.cpu().numpy().tobytes(), f.cpu().numpy().tobytes(),
           b"".join(p.cpu().numpy().tobytes() for p in cur), b"".join(p.cpu().numpy().tobytes() for p in prior_raw)))
    dist.barrier()
    ctx.close()
    dist.destroy_process_group()


def test_two_ranks_range_sharded_global_order():
    import torch.multiprocessing as mp
    world = 2
    mctx = mp.get_context("spawn")
    q = mctx.Queue()
    port = free_port()
    procs = [mctx.Process(target=range_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    cur_all = b"".join(r[3] for r in res)
    prior_all = S.dedup(b"".join(r[4] for r in res))
    eu, ef = S.dedup_diff(cur_all, prior_all)
    assert b"".join(r[1] for r in res) == eu
    assert b"".join(r[2] for r in res) == ef


def rounds_worker(rank, world, port, q, rounds):
    """The C5 multi-GPU step (bench.py --gpus N): one partition into world x rounds ranges,
    one size exchange, one all-to-all per round, each part deduped as its round arrives,
    against the stored prior built the same way; rank 1 holds an empty piece besides its
    records. Rank outputs concatenated in rank order = the global sort -u / comm -13."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import swarm_amd
    from swarm_amd import corpus
    from swarm_amd import distributed as D
    ctx = swarm_amd.Context(0, torch.cuda.current_stream().cuda_stream)
    pool = corpus.host_pool_gpu(20_000, seed=5)
    U = 20_000 * len(corpus.PORTS)
    prior_raw = corpus.hostport_pieces(pool, 150_000, U // 10, U, seed=900 + rank, per_piece=40_000)
    cur = corpus.hostport_pieces(pool, 200_000 + 30_000 * rank, 0, U, seed=100 + rank, per_piece=60_000)
    if rank == 1:
        cur = cur[:1] + [torch.empty(0, dtype=torch.uint8, device="cuda")] + cur[1:]
    split = D.agree_splitters(ctx, prior_raw, world * rounds)
    prior_parts, stored = D.build_prior_rounds(ctx, prior_raw, split, rounds)
    assert all(p is None or p.data_ptr() % 16 == 0 for p in prior_parts)
    u, f, st = D.dedup_diff_rounds_step(ctx, cur, prior_parts, split, rounds)
    torch.cuda.synchronize()
    q.put((rank, u.cpu().numpy().tobytes(), f.cpu().numpy().tobytes(),
           b"".join(p.cpu().numpy().tobytes() for p in cur), b"".join(p.cpu().numpy().tobytes() for p in prior_raw),
           st["parts"]))
    dist.barrier()
    ctx.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("rounds", [1, 3])
def test_two_ranks_rounds_step_global_order(rounds):
    res = spawn(rounds_worker, 2, rounds)
    cur_all = b"".join(r[3] for r in res)
    prior_all = S.dedup(b"".join(r[4] for r in res))
    eu, ef = S.dedup_diff(cur_all, prior_all)
    assert b"".join(r[1] for r in res) == eu
    assert b"".join(r[2] for r in res) == ef
    assert all(r[5] == rounds for r in res)


def spawn(target, world, *extra):
    import torch.multiprocessing as mp
    mctx = mp.get_context("spawn")
    q = mctx.Queue()
    port = free_port()
    procs = [mctx.Process(target=target, args=(r, world, port, q) + extra) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return res


def c2_range_worker(rank, world, port, q, kind):
    """The bench's C2 N>1 step: prior candidates routed by agreed byte splitters and deduped
    at their owner (build_prior_range), then one range-routed dedup+diff step."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import numpy as np
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import swarm_amd
    from swarm_amd import corpus
    from swarm_amd import distributed as D
    ctx = swarm_amd.Context(0, torch.cuda.current_stream().cuda_stream)
    if kind == "subdomains":
        buf, ids = inputs(world)[rank]
        u = np.unique(ids)
        cand = corpus._flatten(*corpus.render_names(u[(u % np.uint64(10)) != 0]))
    else:  # URL records: every record shares 'https://' (one key0 for the whole run)
        import random
        from oracle import semantics as S
        rng = random.Random(40 + rank)
        recs = [b"https://h%d.example.com/%s" % (rng.randrange(20_000), b"p" * rng.randrange(3)) for _ in range(30_000)]
        buf = np.frombuffer(b"\n".join(recs) + b"\n", dtype=np.uint8)
        cand = np.frombuffer(S.serialize(recs[::4]), dtype=np.uint8)
    cand_t = torch.from_numpy(cand.copy()).cuda()
    gsplit = D.agree_splitters(ctx, [cand_t], world)
    prior = D.build_prior_range(ctx, cand_t, gsplit)
    cur = torch.from_numpy(buf.copy()).cuda()
    r, recv = D.dedup_diff_range_shard(ctx, cur, prior, gsplit)
    torch.cuda.synchronize()
    q.put((rank, ctx.to_bytes(r.uniq, r.uniq_bytes), ctx.to_bytes(r.fresh, r.fresh_bytes),
           buf.tobytes(), cand.tobytes(), int(recv.numel())))
    dist.barrier()
    ctx.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["subdomains", "urls"])
def test_two_ranks_c2_range_global_order(kind):
    """Rank outputs concatenated in rank order are the oracle's byte-ordered global output
    (no merge), and the byte splitters keep the ranks' shares balanced on URL data."""
    res = spawn(c2_range_worker, 2, kind)
    cur_all = b"".join(r[3] for r in res)
    prior_all = S.dedup(b"".join(r[4] for r in res))
    eu, ef = S.dedup_diff(cur_all, prior_all)
    assert b"".join(r[1] for r in res) == eu
    assert b"".join(r[2] for r in res) == ef
    recv = [r[5] for r in res]
    assert min(recv) > 0.5 * max(recv)


def match_worker(rank, world, port, q):
    """distributed.match_step: contiguous newline-aligned shards, replicated matcher, count
    all-reduce; matched lines gathered in rank order."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import numpy as np
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import swarm_amd
    from swarm_amd import corpus
    from swarm_amd import distributed as D
    ctx = swarm_amd.Context(0, torch.cuda.current_stream().cuda_stream)
    pats = corpus.nmap_signatures(n_products=30)
    data = corpus.lines_from_pool(corpus.banner_pool(n_products=30, pool=500, match_frac=0.3, seed=3), 9_000, seed=4)
    cuts = D.shard_bounds(data, world)
    shard = torch.from_numpy(data[cuts[rank]:cuts[rank + 1]].copy()).cuda()
    m = swarm_amd.Matcher(pats, "regex")
    r, tot = D.match_step(ctx, m, shard)
    torch.cuda.synchronize()
    lines = D.gather_lines(ctx.to_bytes(r.lines, r.lines_bytes))
    q.put((rank, tot, lines, data.tobytes() if rank == 0 else b""))
    dist.barrier()
    ctx.close()
    dist.destroy_process_group()


def test_two_ranks_match_step():
    from swarm_amd import corpus
    res = spawn(match_worker, 2)
    data = res[0][3]
    pats = corpus.nmap_signatures(n_products=30)
    hits = S.regex_hits(data, pats)
    matched = S.matched_lines(data, hits)
    for _, tot, lines, _ in res:
        assert tot == (len(S.parse_records(data)), len(hits), len(S.parse_records(matched)))
        assert lines == matched
