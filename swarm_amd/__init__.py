"""swarm_amd — MI355X-native scan-result hot path for Swarm (parse, match, merge, dedup,
diff), hand-written HIP for gfx950 behind a ctypes C-ABI (include/swarmgpu.h).

Importing the package loads libswarmgpu.so and raises if it is missing: there is no CPU
fallback on the product path.
"""
from .api import (Context, Matcher, dedup, dedup_chunks, dedup_diff, device_count, diff, hash64,
                  Ingest, Templates, json_fields, lines, nmap_ports, records)

__all__ = ["Context", "Matcher", "dedup", "dedup_chunks", "dedup_diff", "device_count", "diff",
           "hash64", "json_fields", "lines", "nmap_ports", "records", "Templates", "Ingest"]
