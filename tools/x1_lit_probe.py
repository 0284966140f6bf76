"""Time the literal matcher on the X1 input (httpx lines with per-URL tails, C3's 2,000
signatures), device-resident, once per SG_LIT_DEBUG mode given on the command line:
-1 normal, 1 skip pass 2 (verify), 2 skip pass 1 probes, 3 both (load + parse only),
8 count candidates / fingerprint matches / hits (printed from the library's stderr)."""
import json
import os
import subprocess
import sys

if len(sys.argv) > 1 and sys.argv[1] == "--child":
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import time
    import torch
    import swarm_amd
    from swarm_amd import corpus
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    n_lines = int(sys.argv[2])
    sigs = bench.c3_signatures()
    tails = corpus.httpx_tails(sigs)
    buf, _ = corpus.httpx_hosts(n_lines, tails, seed=1234)
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
    print(json.dumps({"mode": os.environ.get("SG_LIT_DEBUG", "-1"), "bytes": int(d.numel()), "ms_step": round(el * 1e3, 3),
                      "lit_ms": round(lm[1] / lm[0], 3) if lm else None,
                      "lit_gbps": round(d.numel() / (lm[1] / lm[0] * 1e-3) / 1e9, 1) if lm else None,
                      "hits": int(r.n_hits), "matched": int(r.matched_records),
                      "top": sorted(((k, round(v[1] / v[0], 3)) for k, v in st.items()), key=lambda kv: -kv[1])[:6]}),
          flush=True)
    ctx.close()
    sys.exit(0)

n_lines = os.environ.get("X1_LINES", "10000000")
for mode in (sys.argv[1:] or ["-1"]):
    env = dict(os.environ)
    if mode != "-1":
        env["SG_LIT_DEBUG"] = mode
    rc = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", n_lines], env=env, timeout=300).returncode
    if rc != 0:
        sys.exit(rc)
