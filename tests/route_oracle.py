"""Restatement of the byte-range routing (include/swarmgpu.h sg_dev_partition_bytes,
sg_dev_record_sample) for tests: part = number of splitters, cut to 64 bytes, <= record in
sort's byte order (Python's bytes order); input order kept inside a part. FakeCtx runs the
host-side multi-rank logic (swarm_amd.distributed) on CPU tensors with these semantics."""
import bisect
import ctypes

from oracle import semantics as S

SPLIT_BYTES = 64


def route_parts(data: bytes, splitters):
    cut = [x[:SPLIT_BYTES] for x in splitters]
    parts = [[] for _ in range(len(cut) + 1)]
    for r in S.parse_records(data):
        parts[bisect.bisect_right(cut, r)].append(r + b"\n")
    return [b"".join(p) for p in parts]


def sample_heads(data: bytes, m: int):
    R = S.parse_records(data)
    if not R:
        return [], 0
    return [R[(k * len(R)) // m][:SPLIT_BYTES] for k in range(m)], len(R)


class FakeCtx:
    """The Context methods swarm_amd.distributed / sharded call for routing, on host memory."""
    device = 0

    def fence_in(self):
        pass

    def record_sample(self, ptr, n, m):
        return sample_heads(ctypes.string_at(ptr, n) if n else b"", m)

    def partition_bytes(self, ptr, n, splitters, out_ptr, cap):
        parts = route_parts(ctypes.string_at(ptr, n) if n else b"", splitters)
        blob = b"".join(parts)
        assert len(blob) <= cap
        ctypes.memmove(out_ptr, blob, len(blob))
        return [len(p) for p in parts], [len(S.parse_records(p)) for p in parts]
