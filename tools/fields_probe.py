"""Wall-clock phases of the §8(f) fields leg (device-resident input): json_fields alone,
template evaluation alone, and the per-kernel table of one profiled template pass."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import swarm_amd  # noqa: E402
from swarm_amd import corpus  # noqa: E402
import bench  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4_000_000
buf = corpus.lines_from_pool(corpus.httpx_json_pool(1 << 14, seed=5), n, seed=6)
d = torch.from_numpy(buf).cuda()
ctx = swarm_amd.Context(0, torch.cuda.current_stream().cuda_stream)
keys = [b"url", b"title", b"webserver", b"tech"]
tm = swarm_amd.Templates(bench.field_templates(), keys)


def wall(f, k=3):
    f()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(k):
        r = f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / k * 1e3, r


ms_j, rows = wall(lambda: ctx.json_fields(d.data_ptr(), d.numel(), keys))
ms_t, r = wall(lambda: tm.dev_match(ctx, d.data_ptr(), d.numel()))
ctx.reset_stats()
ctx.profile(True)
tm.dev_match(ctx, d.data_ptr(), d.numel())
torch.cuda.synchronize()
ctx.profile(False)
st = ctx.kernel_stats()
ksum = sum(v[1] for v in st.values())
print(json.dumps({"lines": n, "bytes": int(d.numel()), "json_fields_ms": round(ms_j, 2), "rows": int(rows.rows),
                  "templates_ms": round(ms_t, 2), "matches": int(r.n), "kernel_sum_ms": round(ksum, 2),
                  "top": {k: round(v[1], 3) for k, v in sorted(st.items(), key=lambda kv: -kv[1][1])[:12]}}), flush=True)
ctx.close()
