"""The device-tensor collective path of the multi-GPU step on the one GPU a box has: a
1-rank process group on the "nccl" backend (= RCCL on ROCm), started in a fresh process
before it touches the GPU. It runs what every N-rank step runs on RCCL and what the gloo
rehearsals never reach (they stage through host copies):

* all_to_all_bytes(..., async_op=True) on device tensors + work.wait();
* exchange_counts / all_max_int / all_max_float on device tensors;
* the round-pipelined C5 step (dedup_diff_rounds_step) with force_exchange, so its size
  exchange and its per-round all_to_all_single calls are issued at world size 1, checked
  bit for bit against the oracle.

Reference: the parallelism being replaced is chunked data parallelism (server/server.py:
185-187 slices the target list, :414-461 queues one job per chunk)."""
import os
import socket

import pytest

from oracle import semantics as S

pytestmark = pytest.mark.gpu


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def rccl_worker(port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    import torch
    import torch.distributed as dist
    out = {}
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1)
        import swarm_amd
        from swarm_amd import corpus
        from swarm_amd import distributed as D
        out["backend"] = dist.get_backend()
        out["world"] = dist.get_world_size()
        out["host_staged"] = D.host_staged()
        # 1. async byte all-to-all between device buffers
        g = torch.Generator(device="cuda")
        g.manual_seed(3)
        n = (1 << 20) + 3
        send = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda", generator=g)
        recv = torch.empty(n, dtype=torch.uint8, device="cuda")
        w = D.all_to_all_bytes(recv, send, [n], [n], async_op=True)
        out["work_is_async"] = w is not None
        if w is not None:
            w.wait()
        torch.cuda.synchronize()
        out["a2a_equal"] = bool(torch.equal(recv, send))
        # 1b. the same message over the pieces path (a rank's message to itself: a local copy)
        D.A2A_CHUNK = 1 << 18
        recv2 = torch.empty(n, dtype=torch.uint8, device="cuda")
        w2 = D.all_to_all_bytes(recv2, send, [n], [n], async_op=True)
        out["chunked_pieces"] = len(w2.works) if hasattr(w2, "works") else 0
        w2.wait()
        torch.cuda.synchronize()
        out["chunked_equal"] = bool(torch.equal(recv2, send))
        # 2. the small collectives on device tensors
        out["counts"] = D.exchange_counts([5, 6, 7])
        out["max_int"] = D.all_max_int(42)
        out["max_float"] = D.all_max_float(1.5)
        # 3. the C5 rounds step with its collectives issued at world size 1
        ctx = swarm_amd.Context(0, torch.cuda.current_stream().cuda_stream)
        pool = corpus.host_pool_gpu(20_000, seed=5)
        U = 20_000 * len(corpus.PORTS)
        prior_raw = corpus.hostport_pieces(pool, 150_000, U // 10, U, seed=900, per_piece=40_000)
        cur = corpus.hostport_pieces(pool, 200_000, 0, U, seed=100, per_piece=60_000)
        rounds = 3
        D.A2A_CHUNK = 1 << 16  # the rounds' exchanges in pieces too
        split = D.agree_splitters(ctx, prior_raw, rounds)
        prior_parts, _ = D.build_prior_rounds(ctx, prior_raw, split, rounds, force_exchange=True)
        recvd, _send = D.exchange_rounds(ctx, cur, split, rounds, force_exchange=True)
        out["round_works"] = sum(1 for wk, _, _, _ in recvd if wk is not None)
        for wk, _, _, _ in recvd:
            if wk is not None:
                wk.wait()
        del recvd, _send
        u, f, st = D.dedup_diff_rounds_step(ctx, cur, prior_parts, split, rounds, force_exchange=True)
        torch.cuda.synchronize()
        out["u"] = u.cpu().numpy().tobytes()
        out["f"] = f.cpu().numpy().tobytes()
        out["cur"] = b"".join(p.cpu().numpy().tobytes() for p in cur)
        out["prior"] = b"".join(p.cpu().numpy().tobytes() for p in prior_raw)
        out["parts"] = st["parts"]
        ctx.close()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001 - reported to the parent
        import traceback
        out["error"] = "%s: %s\n%s" % (type(e).__name__, e, traceback.format_exc())
    q.put(out)


def test_one_rank_rccl_collectives_and_rounds_step():
    import torch.multiprocessing as mp
    mctx = mp.get_context("spawn")
    q = mctx.Queue()
    p = mctx.Process(target=rccl_worker, args=(free_port(), q))
    p.start()
    out = q.get(timeout=300)
    p.join(timeout=120)
    assert "error" not in out, out.get("error")
    assert p.exitcode == 0
    assert out["backend"] == "nccl" and out["world"] == 1 and out["host_staged"] is False
    assert out["work_is_async"] and out["a2a_equal"]
    assert out["chunked_pieces"] == 1 and out["chunked_equal"]  # the self message: one side-stream copy
    assert out["counts"] == [5, 6, 7]
    assert out["max_int"] == 42 and out["max_float"] == 1.5
    assert out["round_works"] == 3  # one async all-to-all per round, on RCCL
    eu, ef = S.dedup_diff(out["cur"], S.dedup(out["prior"]))
    assert out["u"] == eu
    assert out["f"] == ef
    assert out["parts"] == 3
