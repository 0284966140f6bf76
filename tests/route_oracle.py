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


def key0(rec: bytes) -> int:
    """include/swarmgpu.h's first-chunk sort key restated: bytes [0, 7) big-endian in bits
    63..8 (zero past the end), tag = min(len, 8) in bits 7..0."""
    head = rec[:7] + b"\0" * (7 - min(len(rec), 7))
    return (int.from_bytes(head, "big") << 8) | min(len(rec), 8)


def _i64(v: int) -> int:
    return v - (1 << 64) if v >= 1 << 63 else v


M64 = (1 << 64) - 1


def span_mix(length: int, key: int) -> int:
    """include/swarmgpu.h sg_span_sum's per-record term restated: h = (key + length *
    0x9E3779B97F4A7C15) * 0xBF58476D1CE4E5B9 (mod 2^64), then h ^ h >> 31."""
    h = ((key + length * 0x9E3779B97F4A7C15) * 0xBF58476D1CE4E5B9) & M64
    return h ^ (h >> 31)


def span_sum(spans, keys) -> int:
    """sg_span_sum restated: sum mod 2^64 of span_mix(end - start, key) over the records."""
    return sum(span_mix(e - a, k & M64) for (a, e), k in zip(spans, keys)) & M64


CHK_SAMPLE = 256


def check_handover(buf: bytes, spans, keys, expect_sum: int) -> str:
    """sg_dev_dedup_diff_spans_into's check of a handed-over parse restated: '' when it holds,
    else why not (records tile the buffer, the checksum, every CHK_SAMPLE-th record's '\n'
    and key)."""
    n = len(buf)
    if not spans:
        return "" if n == 0 and (expect_sum & M64) == 0 else "no records for %d bytes" % n
    prev = -1
    for i, (a, e) in enumerate(spans):
        if not (a == prev + 1 and e > a and e < n):
            return "record %d (%d, %d) out of place" % (i, a, e)
        prev = e
        if i % CHK_SAMPLE == 0 and (buf[e] != 0x0A or key0(buf[a:e]) != keys[i] & M64):
            return "record %d does not match its bytes" % i
    if prev != n - 1:
        return "records end at %d of %d bytes" % (prev + 1, n)
    if span_sum(spans, keys) != expect_sum & M64:
        return "checksum mismatch"
    return ""


def _fake_pieces_count(self, pieces):
    return sum(len(S.parse_records(ctypes.string_at(p, n) if n else b"")) for p, n in pieces)


def _fake_rounds_spans(self, pieces, splitters, rounds, out_ptr, cap, sp_ptr, k_ptr, rec_cap):
    """sg_dev_partition_bytes_pieces_rounds_spans restated: the round-major byte layout of
    partition_bytes_pieces_rounds, plus every record's span (relative to its part's start) and
    key0, records in the same round-major part order."""
    pb, pr = self.partition_bytes_pieces_rounds(pieces, splitters, rounds, out_ptr, cap)
    nparts = len(pb)
    G = nparts // rounds
    ps = [0] * nparts
    # the parts' bytes as written (round-major), read back
    off, r = 0, 0
    sp = (ctypes.c_uint32 * (2 * max(rec_cap, 1))).from_address(sp_ptr)
    kk = (ctypes.c_int64 * max(rec_cap, 1)).from_address(k_ptr)
    for p in range(rounds):
        off = (off + 15) & ~15
        for g in range(G):
            q = g * rounds + p
            b = ctypes.string_at(out_ptr + off, pb[q]) if pb[q] else b""
            for a, e in S.record_spans(b):
                assert r < rec_cap
                sp[2 * r], sp[2 * r + 1] = a, e
                kk[r] = _i64(key0(b[a:e]))
                ps[q] = (ps[q] + span_mix(e - a, key0(b[a:e]))) & M64
                r += 1
            off += pb[q]
    return pb, pr, ps


REBASE_CHECK = 256


def _fake_rebase(self, buf_ptr, n, sp_ptr, n_rec, seg_first, seg_off):
    """sg_dev_rebase_spans restated: every span shifted by its source's offset, each source's
    first and last REBASE_CHECK records checked to end at a '\n' of the buffer."""
    sp = (ctypes.c_uint32 * (2 * max(n_rec, 1))).from_address(sp_ptr)
    buf = ctypes.string_at(buf_ptr, n) if n else b""
    first = list(seg_first) if seg_first else [0]
    bad = 0
    for s, f in enumerate(first):
        e_ = first[s + 1] if s + 1 < len(first) else n_rec
        o = seg_off[s] if seg_off else 0
        for i in range(f, e_):
            sp[2 * i] += o
            sp[2 * i + 1] += o
            if i - f < REBASE_CHECK or e_ - i <= REBASE_CHECK:
                a, e = sp[2 * i], sp[2 * i + 1]
                bad += 0 if (a <= e < n and buf[e] == 0x0A) else 1
    return bad


def _fake_spans_into(self, cur_ptr, n, sp_ptr, k_ptr, n_rec, ssum, prior_ptr, pn, u_ptr, ucap, f_ptr, fcap):
    """sg_dev_dedup_diff_spans_into restated: the library's check of the handed-over parse
    (check_handover: SG_E_CORRUPT when it fails), then dedup_diff_into."""
    from swarm_amd import _abi
    cur = ctypes.string_at(cur_ptr, n) if n else b""
    sp = (ctypes.c_uint32 * (2 * max(n_rec, 1))).from_address(sp_ptr)
    kk = (ctypes.c_int64 * max(n_rec, 1)).from_address(k_ptr)
    got = [(sp[2 * i], sp[2 * i + 1]) for i in range(n_rec)]
    why = check_handover(cur, got, [kk[i] & M64 for i in range(n_rec)], ssum)
    if why:
        raise _abi.SGError(_abi.SG_E_CORRUPT, "handed-over parse does not match the buffer: " + why)
    self.log.append("spans_into")
    return self.dedup_diff_into(cur_ptr, n, prior_ptr, pn, u_ptr, ucap, f_ptr, fcap)


FakeCtx.partition_pieces_count = _fake_pieces_count
FakeCtx.partition_bytes_pieces_rounds_spans = _fake_rounds_spans
FakeCtx.rebase_spans = _fake_rebase
FakeCtx.dedup_diff_spans_into = _fake_spans_into
