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


class _Res:
    def __init__(self, ub, fb, nin, nu, nf):
        self.uniq_bytes, self.fresh_bytes, self.in_records, self.uniq_records, self.fresh_records = ub, fb, nin, nu, nf


class FakeCtx:
    """The Context methods swarm_amd.distributed / sharded call for routing, on host memory.
    `log` records the routing calls and the stream fences in call order (a test checks that
    every partition's output is fenced before a collective may read it)."""
    device = 0

    def __init__(self):
        self.log = []

    @property
    def torch_device(self):
        import torch
        return torch.device("cpu")

    def fence_in(self):
        pass

    def fence_out(self):
        self.log.append("fence_out")

    def record_sample(self, ptr, n, m):
        return sample_heads(ctypes.string_at(ptr, n) if n else b"", m)

    def partition_bytes_pieces_rounds(self, pieces, splitters, rounds, out_ptr, cap):
        """include/swarmgpu.h sg_dev_partition_bytes_pieces_rounds restated: part q = g * rounds
        + p, laid out round-major, every round at a 16-byte aligned offset."""
        self.log.append("partition")
        nparts = len(splitters) + 1
        parts = [b""] * nparts
        for ptr, n in pieces:
            for q, b in enumerate(route_parts(ctypes.string_at(ptr, n) if n else b"", splitters)):
                parts[q] += b
        G = nparts // rounds
        off = 0
        for p in range(rounds):
            off = (off + 15) & ~15
            for g in range(G):
                b = parts[g * rounds + p]
                assert off + len(b) <= cap
                ctypes.memmove(out_ptr + off, b, len(b))
                off += len(b)
        return [len(b) for b in parts], [len(S.parse_records(b)) for b in parts]

    def dedup_diff_into(self, cur_ptr, n, prior_ptr, pn, u_ptr, ucap, f_ptr, fcap):
        """sg_dev_dedup_diff_into restated with the oracle (outputs written at the caller's
        addresses)."""
        cur = ctypes.string_at(cur_ptr, n) if n else b""
        prior = ctypes.string_at(prior_ptr, pn) if pn else b""
        u, f = S.dedup_diff(cur, prior)
        assert len(u) <= ucap and (not f_ptr or len(f) <= fcap)
        ctypes.memmove(u_ptr, u, len(u))
        if f_ptr:
            ctypes.memmove(f_ptr, f, len(f))
        return _Res(len(u), len(f), len(S.parse_records(cur)), len(S.parse_records(u)), len(S.parse_records(f)))

    def partition_bytes(self, ptr, n, splitters, out_ptr, cap):
        self.log.append("partition")
        parts = route_parts(ctypes.string_at(ptr, n) if n else b"", splitters)
        blob = b"".join(parts)
        assert len(blob) <= cap
        ctypes.memmove(out_ptr, blob, len(blob))
        return [len(p) for p in parts], [len(S.parse_records(p)) for p in parts]
