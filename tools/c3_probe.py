"""Time the literal matcher on a C3 slice (device-resident), for kernel experiments:
SG_LIT_DEBUG=<mode> selects the debug counters / skipped passes inside k_lit_scan."""
import base64
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import swarm_amd  # noqa: E402
from swarm_amd import corpus  # noqa: E402

n_lines = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sig = json.load(open(os.path.join(root, "tests", "golden", "signatures.json")))
words = [base64.b64decode(w) for w in sig["words"]]
sigs = random.Random(0).sample([w for w in words if len(w) >= 4], 2000)
pool = corpus.httpx_pool(sigs, 1 << 16, 0.01, seed=0)
buf = corpus.lines_from_pool(pool, n_lines, seed=1)
d = torch.from_numpy(buf).cuda()
ctx = swarm_amd.Context(0, torch.cuda.current_stream().cuda_stream)
m = swarm_amd.Matcher(sigs, "literal")
r = m.dev_match(ctx, d.data_ptr(), d.numel())
torch.cuda.synchronize()
ctx.reset_stats()
ctx.profile(True)
t0 = time.perf_counter()
for _ in range(3):
    r = m.dev_match(ctx, d.data_ptr(), d.numel())
torch.cuda.synchronize()
el = (time.perf_counter() - t0) / 3
ctx.profile(False)
st = ctx.kernel_stats()
lm = st.get("lit_match")
print(json.dumps({"mode": os.environ.get("SG_LIT_DEBUG"), "bytes": int(d.numel()), "ms_step": round(el * 1e3, 3),
                  "lit_ms": round(lm[1] / lm[0], 3) if lm else None,
                  "lit_gbps": round(d.numel() / (lm[1] / lm[0] * 1e-3) / 1e9, 1) if lm else None,
                  "hits": int(r.n_hits)}), flush=True)
ctx.close()
