"""Time the regex matcher on a C4 slice (device-resident). SG_LIT_DEBUG=8 prints the
prefilter's candidate / fingerprint / hit counts."""
import base64
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import swarm_amd  # noqa: E402
from swarm_amd import corpus  # noqa: E402

n_lines = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
which = sys.argv[2] if len(sys.argv) > 2 else "all"
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sig = json.load(open(os.path.join(root, "tests", "golden", "signatures.json")))
nuc = [base64.b64decode(r["p"]) for r in sig["regexes"]]
syn = corpus.nmap_signatures()
pats = {"all": nuc + syn, "nuclei": nuc, "nmap": syn, "bench": None}[which]
if pats is None:  # the bench's C4 set (generic extractor regexes left out)
    pats, _ = corpus.c4_signatures(nuc)
buf = corpus.lines_from_pool(corpus.banner_pool(), n_lines, seed=3)
d = torch.from_numpy(buf).cuda()
ctx = swarm_amd.Context(0, torch.cuda.current_stream().cuda_stream)
m = swarm_amd.Matcher(pats, "regex")
r = m.dev_match(ctx, d.data_ptr(), d.numel())
torch.cuda.synchronize()
ctx.reset_stats()
ctx.profile(True)
t0 = time.perf_counter()
r = m.dev_match(ctx, d.data_ptr(), d.numel())
torch.cuda.synchronize()
el = time.perf_counter() - t0
ctx.profile(False)
st = ctx.kernel_stats()
print(json.dumps({"which": which, "n_pats": len(pats), "lines": n_lines, "ms": round(el * 1e3, 2), "info": m.info(),
                  "hits": int(r.n_hits),
                  "kernels_ms": {k: round(v[1], 3) for k, v in sorted(st.items(), key=lambda kv: -kv[1][1])[:8]}}),
      flush=True)
ctx.close()
