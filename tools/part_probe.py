"""Time the per-rank compute of a multi-GPU C2 step on one GPU: the hash partition into G
parts (sg_dev_partition) and the local dedup+diff, without the exchange."""
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: E402

import swarm_amd  # noqa: E402
from swarm_amd import corpus  # noqa: E402

cur_np, ids = corpus.subdomains(10_000_000, seed=1234, universe=80_000_000)
cur = torch.from_numpy(cur_np).cuda()
prior = torch.from_numpy(corpus.prior_of(ids)).cuda()
ctx = swarm_amd.Context(0, torch.cuda.current_stream().cuda_stream)
send = torch.empty(cur.numel() + 1, dtype=torch.uint8, device="cuda")
for G in (2, 8):
    for _ in range(3):
        ctx.partition(cur.data_ptr(), cur.numel(), G, send.data_ptr(), send.numel())
    torch.cuda.synchronize()
    ctx.reset_stats()
    ctx.profile(True)
    t = time.perf_counter()
    for _ in range(10):
        pb, _ = ctx.partition(cur.data_ptr(), cur.numel(), G, send.data_ptr(), send.numel())
    torch.cuda.synchronize()
    t = (time.perf_counter() - t) / 10
    ctx.profile(False)
    st = ctx.kernel_stats()
    print("G=%d partition %.3f ms/call (wall, incl. host sync); kernels:" % (G, t * 1e3),
          {k: round(v[1] / 10, 4) for k, v in st.items()}, flush=True)
for _ in range(3):
    ctx.dedup_diff(cur.data_ptr(), cur.numel(), prior.data_ptr(), prior.numel())
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(10):
    ctx.dedup_diff(cur.data_ptr(), cur.numel(), prior.data_ptr(), prior.numel())
torch.cuda.synchronize()
print("dedup_diff %.3f ms/call" % ((time.perf_counter() - t) * 100), flush=True)
