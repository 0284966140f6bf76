"""Replays bench_c5's setup step by step (C5 debugging aid)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import swarm_amd  # noqa: E402
from swarm_amd import corpus, sharded  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
n_hosts = 1_000_000
U = n_hosts * 32
pool = corpus.host_pool_gpu(n_hosts + n_hosts // 10 + 1, seed=5, device=dev)
ctx = swarm_amd.Context(0, torch.cuda.current_stream(dev).cuda_stream)
per = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
prior_raw = corpus.hostport_pieces(pool, per, U // 10, U + U // 10, seed=900)
for i, p in enumerate(prior_raw):
    print("piece", i, p.numel(), p.data_ptr() % 512, flush=True)
parts = sharded.plan_parts(prior_raw, [], 2 << 30)
ks = [ctx.key_sample(p.data_ptr(), p.numel(), 1 << 14) for p in prior_raw]
print("samples", [k[1] for k in ks], flush=True)
lsplit = sharded.choose_splitters(np.concatenate([k[0] for k in ks]), parts)
print("parts", parts, lsplit, flush=True)
routed = sharded.route(ctx, prior_raw, lsplit)
for b, c in enumerate(routed):
    print("part", b, c.numel(), int((c == 10).sum()), c.data_ptr() % 512, flush=True)
pu, _, st = sharded.dedup_diff_large(ctx, prior_raw, (), splitters=lsplit)
print("ok", st, flush=True)
