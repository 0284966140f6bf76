"""Time the C2 dedup+diff pipeline per kernel (device-resident), for kernel experiments.
Env switches (timing only, outputs wrong): SG_EMIT_DEBUG=1 no copy, 2 no look-back;
SG_LINES_DEBUG likewise for k_lines."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import swarm_amd  # noqa: E402
from swarm_amd import corpus  # noqa: E402

n_lines = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
buf, ids = corpus.subdomains(n_lines, seed=1234)
prior = corpus.prior_of(ids)
d_cur = torch.from_numpy(buf).cuda()
d_pri = torch.from_numpy(prior).cuda()
ctx = swarm_amd.Context(0, torch.cuda.current_stream().cuda_stream)
for _ in range(2):
    r = ctx.dedup_diff(d_cur.data_ptr(), d_cur.numel(), d_pri.data_ptr(), d_pri.numel())
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(5):
    r = ctx.dedup_diff(d_cur.data_ptr(), d_cur.numel(), d_pri.data_ptr(), d_pri.numel())
torch.cuda.synchronize()
el_noprof = (time.perf_counter() - t0) / 5
ctx.reset_stats()
ctx.profile(True)
t0 = time.perf_counter()
for _ in range(5):
    r = ctx.dedup_diff(d_cur.data_ptr(), d_cur.numel(), d_pri.data_ptr(), d_pri.numel())
torch.cuda.synchronize()
el = (time.perf_counter() - t0) / 5
ctx.profile(False)
st = ctx.kernel_stats()
out = {"mode": {k: v for k, v in os.environ.items() if k.startswith("SG_")}, "ms_step": round(el * 1e3, 3), "ms_step_noprof": round(el_noprof * 1e3, 3),
       "kernel_sum_ms": round(sum(v[1] for v in st.values()) / 5, 3),
       "kernels_us": {k: round(v[1] / v[0] * 1e3, 1) for k, v in sorted(st.items(), key=lambda kv: -kv[1][1])}}
print(json.dumps(out), flush=True)
ctx.close()
