"""Host-side mirror of the scan-result hot path, over libswarmgpu.so (ctypes).

These are the functions the reference-side worker.py / server.py call:
  lines(buf)                 A3  module-output parsing             (worker/worker.py:83-98)
  dedup(buf) / dedup_chunks  A5+A7 merge + sort -u                  (server/server.py:399-412)
  diff(cur, prior)           A8  new records vs the prior scan      (README.md:11)
  dedup_diff(cur, prior)     A9  scan-completion step               (server/server.py:274-294)
  Matcher                    A4  literal (Aho-Corasick) / regex (DFA) signature matching
  nmap_ports(buf)            §8(f)2 nmap -oN -> host:port records  (worker/modules/nmap.json:2)
  json_fields(buf, keys)     §8(f)1 httpx -json -> field rows      (worker/modules/http2.json:2)
  Context                    device-resident path (HBM inputs, per-kernel timing)

Every call runs the HIP kernels; there is no CPU fallback. Inputs are bytes-like or numpy
uint8 arrays; outputs are bytes.
"""
from __future__ import annotations

import ctypes as C
import threading
from typing import List, Sequence, Tuple

import numpy as np

from . import _abi
from ._abi import check, lib


def part_offsets(part_bytes: Sequence[int], align16: bool = False) -> List[int]:
    """Start offset of every part in a partition_bytes_pieces output (align16: each part
    starts at the 16-byte aligned offset after the previous one)."""
    out, off = [], 0
    for n in part_bytes:
        out.append(off)
        off += n
        if align16:
            off = (off + 15) & ~15
    return out


def round_offsets(part_bytes: Sequence[int], rounds: int) -> List[int]:
    """Start offset of every round in a partition_bytes_pieces_rounds output (G x rounds parts,
    part q = g * rounds + p; round p = parts (0, p) .. (G - 1, p) back to back, each round at
    the 16-byte aligned offset after the previous one). rounds + 1 entries (the last = end)."""
    G = len(part_bytes) // rounds
    out, off = [], 0
    for p in range(rounds):
        off = (off + 15) & ~15
        out.append(off)
        off += sum(part_bytes[g * rounds + p] for g in range(G))
    out.append(off)
    return out


def _view(b) -> np.ndarray:
    if isinstance(b, np.ndarray):
        a = b.reshape(-1)
        if a.dtype != np.uint8:
            a = a.view(np.uint8)
        return np.ascontiguousarray(a)
    return np.frombuffer(memoryview(b), dtype=np.uint8)


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data if a.size else 0


def lines(buf) -> np.ndarray:
    """A3: (start, end) spans of the non-empty records, shape (R, 2), uint64."""
    a = _view(buf)
    n_rec = C.c_size_t(0)
    cap = a.size // 2 + 2
    spans = np.empty(2 * cap, dtype=np.uint64)
    check(lib.sg_lines(_ptr(a), a.size, spans.ctypes.data_as(C.POINTER(C.c_uint64)), cap,
                       C.byref(n_rec)))
    return spans[: 2 * n_rec.value].reshape(-1, 2)


def records(buf) -> List[bytes]:
    a = bytes(_view(buf))
    return [a[s:e] for s, e in lines(a).tolist()]


def dedup(buf) -> bytes:
    """A7: sort -u of a line-delimited buffer (empty records dropped)."""
    a = _view(buf)
    out = np.empty(a.size + 1, dtype=np.uint8)
    n = C.c_size_t(0)
    check(lib.sg_dedup(_ptr(a), a.size, out.ctypes.data, out.size, C.byref(n)))
    return out[: n.value].tobytes()


def dedup_chunks(chunks: Sequence[bytes]) -> bytes:
    """A5+A7: sort -u of the concatenation of chunk bodies, in the order given."""
    views = [_view(c) for c in chunks]
    k = len(views)
    ptrs = (C.c_void_p * max(k, 1))(*[_ptr(v) for v in views])
    lens = (C.c_size_t * max(k, 1))(*[v.size for v in views])
    total = sum(v.size for v in views)
    out = np.empty(total + 1, dtype=np.uint8)
    n = C.c_size_t(0)
    check(lib.sg_dedup_chunks(ptrs, lens, k, out.ctypes.data, out.size, C.byref(n)))
    return out[: n.value].tobytes()


def diff(cur, prior) -> bytes:
    """A8: sorted(set(cur) - set(prior)), '\\n'-terminated."""
    a, p = _view(cur), _view(prior)
    out = np.empty(a.size + 1, dtype=np.uint8)
    n = C.c_size_t(0)
    check(lib.sg_diff(_ptr(a), a.size, _ptr(p), p.size, out.ctypes.data, out.size, C.byref(n)))
    return out[: n.value].tobytes()


def dedup_diff(cur, prior) -> Tuple[bytes, bytes]:
    """A9: (sort -u of cur, new records of cur vs prior) in one pass."""
    a, p = _view(cur), _view(prior)
    u = np.empty(a.size + 1, dtype=np.uint8)
    f = np.empty(a.size + 1, dtype=np.uint8)
    un, fn = C.c_size_t(0), C.c_size_t(0)
    check(lib.sg_dedup_diff(_ptr(a), a.size, _ptr(p), p.size, u.ctypes.data, u.size, C.byref(un),
                            f.ctypes.data, f.size, C.byref(fn)))
    return u[: un.value].tobytes(), f[: fn.value].tobytes()


class Matcher:
    """A4 signature matcher compiled to a GPU automaton.

    kind="literal": Aho-Corasick, per record `sig in record` (LC_ALL=C grep -F [-i]).
    kind="regex":   DFA set, per record `re.search(sig, record)` on bytes (subset in
                    swarm_amd/csrc/sg_regex.hpp; unsupported constructs raise SGError).
    """

    def __init__(self, patterns: Sequence[bytes], kind: str = "literal", nocase: bool = False):
        pats = [bytes(p) for p in patterns]
        blob = b"".join(pats)
        offs = np.zeros(len(pats) + 1, dtype=np.uint32)
        np.cumsum([len(p) for p in pats], out=offs[1:])
        a = np.frombuffer(blob, dtype=np.uint8) if blob else np.zeros(1, dtype=np.uint8)
        self._h = C.c_void_p()
        fn = lib.sg_ac_compile if kind == "literal" else lib.sg_dfa_compile
        if kind not in ("literal", "regex"):
            raise ValueError("kind must be 'literal' or 'regex'")
        check(fn(a.ctypes.data, offs.ctypes.data_as(C.POINTER(C.c_uint32)), len(pats),
                 _abi.SG_NOCASE if nocase else 0, C.byref(self._h)))
        self.kind = kind
        self.n = len(pats)

    def close(self):
        if self._h:
            lib.sg_free(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def info(self) -> dict:
        st, gr, n = C.c_uint64(), C.c_uint32(), C.c_uint32()
        check(lib.sg_matcher_info(self._h, C.byref(st), C.byref(gr), C.byref(n)))
        return {"states": st.value, "automata": gr.value, "patterns": n.value}

    def match(self, buf) -> List[Tuple[int, int]]:
        """(record index, signature index) for every signature occurring in a record,
        sorted; record indices follow A3 (non-empty records in input order)."""
        a = _view(buf)
        cap = max(1024, a.size)
        while True:
            rec = np.empty(cap, dtype=np.uint64)
            sig = np.empty(cap, dtype=np.uint32)
            nh = C.c_size_t(0)
            rc = lib.sg_match(self._h, _ptr(a), a.size, rec.ctypes.data_as(C.POINTER(C.c_uint64)),
                              sig.ctypes.data_as(C.POINTER(C.c_uint32)), cap, C.byref(nh))
            if rc == _abi.SG_E_CAP:
                cap = nh.value
                continue
            check(rc)
            return list(zip(rec[: nh.value].tolist(), sig[: nh.value].tolist()))

    def match_lines(self, buf) -> bytes:
        """grep output: matched records in input order, '\\n'-terminated."""
        a = _view(buf)
        out = np.empty(a.size + 1, dtype=np.uint8)
        n = C.c_size_t(0)
        check(lib.sg_match_lines(self._h, _ptr(a), a.size, out.ctypes.data, out.size, C.byref(n)))
        return out[: n.value].tobytes()

    def match_lines_count(self, buf) -> Tuple[bytes, int]:
        """(grep output, number of non-empty input records) from one device pass."""
        import torch
        a = _view(buf)
        ctx = _shared_ctx()
        d = torch.from_numpy(np.array(a) if a.size else np.zeros(1, dtype=np.uint8)).cuda(ctx.device)
        ctx.fence_in()
        r = self.dev_match(ctx, d.data_ptr(), a.size)
        return ctx.to_bytes(r.lines, r.lines_bytes), int(r.in_records)

    def dev_match(self, ctx: "Context", d_buf: int, n: int) -> _abi.DevHits:
        r = _abi.DevHits()
        check(lib.sg_dev_match(ctx._h, self._h, C.c_void_p(d_buf), n, C.byref(r)))
        return r

    def dev_match_dedup_diff(self, ctx: "Context", d_buf: int, n: int, d_prior: int = 0, n_prior: int = 0,
                             count_hits: bool = True):
        """The metric's fused step on device buffers: parse -> match -> sort -u of the matched
        records -> new matched records vs the prior scan's matched set. Returns (DevResult,
        n_hits, matched_records) (include/swarmgpu.h sg_dev_match_dedup_diff). With
        count_hits=False n_hits is None: a literal matcher then only flags matched records
        (no (record, signature) hit list is built)."""
        r = _abi.DevResult()
        nh, nm = C.c_uint64(), C.c_uint64()
        check(lib.sg_dev_match_dedup_diff(ctx._h, self._h, C.c_void_p(d_buf), n,
                                          C.c_void_p(d_prior) if d_prior else None, n_prior, C.byref(r),
                                          C.byref(nh) if count_hits else None, C.byref(nm)))
        return r, (nh.value if count_hits else None), nm.value


def nmap_ports(buf) -> bytes:
    """nmap -oN text -> 'host:port' records (one per open port, input order), each
    '\n'-terminated (include/swarmgpu.h sg_nmap_ports)."""
    a = _view(buf)
    cap = 2 * a.size + 64
    while True:
        out = np.empty(cap, dtype=np.uint8)
        n = C.c_size_t(0)
        rc = lib.sg_nmap_ports(_ptr(a), a.size, out.ctypes.data, out.size, C.byref(n))
        if rc == _abi.SG_E_CAP:
            cap = n.value
            continue
        check(rc)
        return out[: n.value].tobytes()


def _keys_blob(keys: Sequence[bytes]):
    ks = [k.encode() if isinstance(k, str) else bytes(k) for k in keys]
    blob = np.frombuffer(b"".join(ks) or b"\0", dtype=np.uint8)
    offs = np.zeros(len(ks) + 1, dtype=np.uint32)
    np.cumsum([len(k) for k in ks], out=offs[1:])
    return blob, offs


def json_fields(buf, keys: Sequence[bytes]) -> Tuple[bytes, np.ndarray, np.ndarray]:
    """httpx -json lines -> (rows, row_rec, row_key): '\n'-terminated decoded values of the
    requested top-level keys (include/swarmgpu.h sg_json_fields), the input record and
    key index of each row."""
    a = _view(buf)
    blob, offs = _keys_blob(keys)
    cap, rcap = a.size + 64, a.size // 2 + 64
    out = np.empty(cap, dtype=np.uint8)
    rrec = np.empty(rcap, dtype=np.uint32)
    rkey = np.empty(rcap, dtype=np.uint32)
    n, nr = C.c_size_t(0), C.c_size_t(0)
    U32P = C.POINTER(C.c_uint32)
    check(lib.sg_json_fields(_ptr(a), a.size, blob.ctypes.data, offs.ctypes.data_as(U32P), len(offs) - 1,
                             out.ctypes.data, cap, C.byref(n), rrec.ctypes.data_as(U32P), rkey.ctypes.data_as(U32P),
                             rcap, C.byref(nr)))
    return out[: n.value].tobytes(), rrec[: nr.value].copy(), rkey[: nr.value].copy()


def hash64(rec: bytes) -> int:
    a = _view(rec)
    return int(lib.sg_hash64(_ptr(a), a.size))


def span_sum(spans: np.ndarray, keys: np.ndarray) -> int:
    """The handover checksum (include/swarmgpu.h sg_span_sum) of host spans (n x 2 uint32:
    start, end) and first-chunk keys (n uint64)."""
    sp = np.ascontiguousarray(spans, dtype=np.uint32).reshape(-1)
    k = np.ascontiguousarray(keys).view(np.uint64).reshape(-1)
    if sp.size != 2 * k.size:
        raise ValueError("%d span words for %d keys" % (sp.size, k.size))
    return int(lib.sg_span_sum(sp.ctypes.data, k.ctypes.data, k.size))


def device_count() -> int:
    n = C.c_int(0)
    check(lib.sg_device_count(C.byref(n)))
    return n.value


SPLIT_BYTES = 64  # include/swarmgpu.h SG_SPLIT_BYTES
_TLS = threading.local()


def _shared_ctx():
    """A per-thread context on torch's current device and stream (host helpers that stage
    through torch tensors). Held in thread-local storage: when a (short-lived request)
    thread ends, its contexts are released with it (Context.__del__ frees the HBM
    workspaces); a thread that switches streams gets a context on the new stream."""
    import torch
    dev = torch.cuda.current_device()
    key = (dev, torch.cuda.current_stream(dev).cuda_stream)
    pool = getattr(_TLS, "ctx", None)
    if pool is None:
        pool = _TLS.ctx = {}
    c = pool.get(key)
    if c is None:
        for k in [k for k in pool if k[0] == dev]:  # one context per device per thread
            pool.pop(k).close()
        c = pool[key] = Context(dev, key[1])
    return c


class Context:
    """A device context: one HIP device, one stream (torch's, if given), HBM workspaces,
    optional HIP-event timing of every kernel launch."""

    def __init__(self, device: int = 0, stream: int | None = None):
        self._h = C.c_void_p()
        # stream None: a context-owned stream; 0 (torch's default stream handle): the null
        # stream, so kernels order against torch work without explicit synchronisation
        s = None if stream is None else (C.c_void_p(stream) if stream else C.c_void_p(-1))
        check(lib.sg_ctx_create(device, s, C.byref(self._h)))
        self.device = device
        self.stream = stream

    @property
    def torch_device(self):
        """The context's device as a torch.device (where buffers for its calls are allocated)."""
        import torch
        return torch.device("cuda", self.device)

    def on_torch_stream(self) -> bool:
        """True when the context's kernels run on torch's current stream of its device, so
        torch allocations and library writes are ordered without extra synchronisation."""
        import torch
        return self.stream is not None and self.stream == torch.cuda.current_stream(self.device).cuda_stream

    def fence_in(self):
        """Before a library call that reads tensors torch produced (or writes into memory
        torch may still be reading): drain torch's stream unless the context shares it."""
        if not self.on_torch_stream():
            import torch
            torch.cuda.current_stream(self.device).synchronize()

    def fence_out(self):
        """After library writes into torch-owned memory that torch will read or free next:
        drain the context's stream unless it is torch's."""
        if not self.on_torch_stream():
            self.sync()

    def close(self):
        if self._h:
            lib.sg_ctx_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def sync(self):
        check(lib.sg_ctx_sync(self._h))

    def profile(self, on: bool = True, only: str = None):
        """HIP-event timing of every launch on the context stream (only: one kernel name)."""
        check(lib.sg_ctx_profile_only(self._h, (only or "").encode()))
        check(lib.sg_ctx_profile(self._h, 1 if on else 0))

    def reset_stats(self):
        check(lib.sg_ctx_reset_stats(self._h))

    def kernel_stats(self) -> dict:
        out = {}
        i = 0
        name = C.c_char_p()
        launches = C.c_uint64()
        ms = C.c_double()
        by = C.c_double()
        while lib.sg_ctx_kernel_stat(self._h, i, C.byref(name), C.byref(launches), C.byref(ms), C.byref(by)) == 0:
            out[name.value.decode()] = (launches.value, ms.value, by.value)
            i += 1
        return out

    def memcpy(self, dst: int, src: int, n: int):
        check(lib.sg_ctx_memcpy(self._h, C.c_void_p(dst), C.c_void_p(src), n))

    def to_bytes(self, dptr: int, n: int) -> bytes:
        out = np.empty(n, dtype=np.uint8)
        if n:
            self.memcpy(out.ctypes.data, dptr, n)
        return out.tobytes()

    def last_path(self):
        """(pipeline, flags) of the last dedup_diff on this context: ("radix", flags) — the only
        pipeline in the library; flags bit 0: hybrid sort (top digits global, groups finished
        in LDS), bit 1: the plain LSD sort ran again, bit 2: a group overflowed the local sort's
        LDS and its tiles were sorted again (k_rs_lsort_fix), bit 3: the all-segments mode
        (include/swarmgpu.h sg_ctx_last_path)."""
        p, f = C.c_int(), C.c_uint32()
        check(lib.sg_ctx_last_path(self._h, C.byref(p), C.byref(f)))
        return {0: "radix"}.get(p.value, str(p.value)), f.value

    def last_key_width(self) -> int:
        """Sort-key width in bytes (5..7) the last radix dedup chose on this context."""
        kw = C.c_uint32()
        check(lib.sg_ctx_last_key_width(self._h, C.byref(kw)))
        return kw.value

    def dedup_diff(self, d_cur: int, n_cur: int, d_prior: int = 0, n_prior: int = 0) -> _abi.DevResult:
        """Device pointers in, device result (context-owned) out."""
        r = _abi.DevResult()
        check(lib.sg_dev_dedup_diff(self._h, C.c_void_p(d_cur), n_cur,
                                    C.c_void_p(d_prior) if d_prior else None, n_prior, C.byref(r)))
        return r

    def nmap_ports(self, d_buf: int, n: int) -> _abi.DevText:
        r = _abi.DevText()
        check(lib.sg_dev_nmap_ports(self._h, C.c_void_p(d_buf), n, C.byref(r)))
        return r

    def json_fields(self, d_buf: int, n: int, keys: Sequence[bytes]) -> _abi.DevRows:
        blob, offs = _keys_blob(keys)
        r = _abi.DevRows()
        check(lib.sg_dev_json_fields(self._h, C.c_void_p(d_buf), n, blob.ctypes.data,
                                     offs.ctypes.data_as(C.POINTER(C.c_uint32)), len(offs) - 1, C.byref(r)))
        return r

    def partition_range(self, d_buf: int, n: int, splitters, d_out: int, out_cap: int):
        """Order-preserving routing by key0 splitters (len(splitters) + 1 parts); same output
        layout as partition(). Returns (bytes per part, records per part)."""
        sp = np.ascontiguousarray(np.asarray(splitters, dtype=np.uint64))
        parts = sp.size + 1
        pb = (C.c_uint64 * parts)()
        pr = (C.c_uint64 * parts)()
        arr = (C.c_uint64 * max(1, sp.size))(*sp.tolist())
        check(lib.sg_dev_partition_range(self._h, C.c_void_p(d_buf), n, arr, parts, C.c_void_p(d_out), out_cap,
                                         pb, pr))
        return list(pb), list(pr)

    def partition_bytes(self, d_buf: int, n: int, splitters: Sequence[bytes], d_out: int, out_cap: int):
        """Order-preserving routing by byte-string splitters (len(splitters) + 1 parts, each
        splitter cut to SPLIT_BYTES); same output layout as partition(). Returns (bytes per
        part, records per part)."""
        blob, offs = _keys_blob(list(splitters))
        parts = len(splitters) + 1
        pb = (C.c_uint64 * parts)()
        pr = (C.c_uint64 * parts)()
        check(lib.sg_dev_partition_bytes(self._h, C.c_void_p(d_buf), n, blob.ctypes.data,
                                         offs.ctypes.data_as(C.POINTER(C.c_uint32)), parts, C.c_void_p(d_out),
                                         out_cap, pb, pr))
        return list(pb), list(pr)

    def partition_bytes_pieces(self, pieces: Sequence[Tuple[int, int]], splitters: Sequence[bytes], d_out: int,
                               out_cap: int, align16: bool = False):
        """Route (device pointer, bytes) pieces into one part-contiguous buffer d_out. Returns
        (bytes per part, records per part), totals over the pieces. align16: part p starts at
        the 16-byte aligned offset after part p - 1 (part_offsets gives the starts)."""
        blob, offs = _keys_blob(list(splitters))
        parts = len(splitters) + 1
        k = len(pieces)
        ptrs = (C.c_void_p * max(1, k))(*[C.c_void_p(p) for p, _ in pieces])
        lens = (C.c_size_t * max(1, k))(*[n for _, n in pieces])
        pb = (C.c_uint64 * parts)()
        pr = (C.c_uint64 * parts)()
        fn = lib.sg_dev_partition_bytes_pieces_a16 if align16 else lib.sg_dev_partition_bytes_pieces
        check(fn(self._h, ptrs, lens, k, blob.ctypes.data, offs.ctypes.data_as(C.POINTER(C.c_uint32)), parts,
                 C.c_void_p(d_out) if d_out else None, out_cap, pb, pr))
        return list(pb), list(pr)

    def partition_bytes_pieces_rounds(self, pieces: Sequence[Tuple[int, int]], splitters: Sequence[bytes], rounds: int,
                                      d_out: int, out_cap: int):
        """Route pieces into G x rounds byte-range parts laid out round-major (include/swarmgpu.h
        sg_dev_partition_bytes_pieces_rounds; round_offsets gives each round's start). Returns
        (bytes per part, records per part) in part order."""
        blob, offs = _keys_blob(list(splitters))
        parts = len(splitters) + 1
        k = len(pieces)
        ptrs = (C.c_void_p * max(1, k))(*[C.c_void_p(p) for p, _ in pieces])
        lens = (C.c_size_t * max(1, k))(*[n for _, n in pieces])
        pb = (C.c_uint64 * parts)()
        pr = (C.c_uint64 * parts)()
        check(lib.sg_dev_partition_bytes_pieces_rounds(self._h, ptrs, lens, k, blob.ctypes.data,
                                                       offs.ctypes.data_as(C.POINTER(C.c_uint32)), parts, rounds,
                                                       C.c_void_p(d_out) if d_out else None, out_cap, pb, pr))
        return list(pb), list(pr)

    def partition_pieces_count(self, pieces: Sequence[Tuple[int, int]]) -> int:
        """The pieces' total record count (pass 0 of the piece partition, kept for the next
        partition call on the same pieces: include/swarmgpu.h sg_dev_partition_pieces_count)."""
        k = len(pieces)
        ptrs = (C.c_void_p * max(1, k))(*[C.c_void_p(p) for p, _ in pieces])
        lens = (C.c_size_t * max(1, k))(*[n for _, n in pieces])
        nr = C.c_uint64(0)
        check(lib.sg_dev_partition_pieces_count(self._h, ptrs, lens, k, C.byref(nr)))
        return int(nr.value)

    def partition_bytes_pieces_rounds_spans(self, pieces: Sequence[Tuple[int, int]], splitters: Sequence[bytes],
                                            rounds: int, d_out: int, out_cap: int, d_spans: int, d_keys: int,
                                            rec_cap: int):
        """partition_bytes_pieces_rounds that also writes every record's span (relative to its
        part's start) and first-chunk key into the caller's buffers (8 bytes each per record,
        round-major part order). Returns (bytes per part, records per part, handover checksum per
        part: include/swarmgpu.h sg_span_sum)."""
        blob, offs = _keys_blob(list(splitters))
        parts = len(splitters) + 1
        k = len(pieces)
        ptrs = (C.c_void_p * max(1, k))(*[C.c_void_p(p) for p, _ in pieces])
        lens = (C.c_size_t * max(1, k))(*[n for _, n in pieces])
        pb = (C.c_uint64 * parts)()
        pr = (C.c_uint64 * parts)()
        ps = (C.c_uint64 * parts)()
        check(lib.sg_dev_partition_bytes_pieces_rounds_spans(
            self._h, ptrs, lens, k, blob.ctypes.data, offs.ctypes.data_as(C.POINTER(C.c_uint32)), parts, rounds,
            C.c_void_p(d_out) if d_out else None, out_cap, pb, pr, C.c_void_p(d_spans) if d_spans else None,
            C.c_void_p(d_keys) if d_keys else None, rec_cap, ps))
        return list(pb), list(pr), list(ps)

    def rebase_spans(self, d_buf: int, n: int, d_spans: int, n_rec: int, seg_first: Sequence[int],
                     seg_off: Sequence[int]) -> int:
        """Received spans made relative to the receive buffer (segment s: records from
        seg_first[s] on get + seg_off[s]); returns how many records do not end before a '\n'
        of the buffer afterwards (0 for an intact transfer)."""
        ns = len(seg_first)
        sf = (C.c_uint64 * max(1, ns))(*[int(x) for x in seg_first])
        so = (C.c_uint64 * max(1, ns))(*[int(x) for x in seg_off])
        bad = C.c_uint64(0)
        check(lib.sg_dev_rebase_spans(self._h, C.c_void_p(d_buf) if d_buf else None, n,
                                      C.c_void_p(d_spans) if d_spans else None, n_rec, sf, so, ns, C.byref(bad)))
        return int(bad.value)

    def partition_bytes_pieces_spans(self, pieces: Sequence[Tuple[int, int]], splitters: Sequence[bytes], d_out: int,
                                     out_cap: int):
        """partition_bytes_pieces(align16=True) that also returns the parts' parse: (bytes per
        part, records per part, device spans pointer, device keys pointer, handover checksum per
        part for dedup_diff_spans_into); part p's records
        start at index sum(records[:p]) (8 bytes per record in each array; context-owned until
        the next call of this kind)."""
        blob, offs = _keys_blob(list(splitters))
        parts = len(splitters) + 1
        k = len(pieces)
        ptrs = (C.c_void_p * max(1, k))(*[C.c_void_p(p) for p, _ in pieces])
        lens = (C.c_size_t * max(1, k))(*[n for _, n in pieces])
        pb = (C.c_uint64 * parts)()
        pr = (C.c_uint64 * parts)()
        ps = (C.c_uint64 * parts)()
        sp, kp = C.c_void_p(), C.c_void_p()
        check(lib.sg_dev_partition_bytes_pieces_spans(self._h, ptrs, lens, k, blob.ctypes.data,
                                                      offs.ctypes.data_as(C.POINTER(C.c_uint32)), parts,
                                                      C.c_void_p(d_out) if d_out else None, out_cap, pb, pr,
                                                      C.byref(sp), C.byref(kp), ps))
        return list(pb), list(pr), sp.value or 0, kp.value or 0, list(ps)

    def dedup_diff_spans_into(self, d_cur: int, n_cur: int, d_spans: int, d_keys: int, n_rec: int, span_sum: int,
                              d_prior: int, n_prior: int, d_uniq: int, uniq_cap: int, d_fresh: int,
                              fresh_cap: int) -> _abi.DevResult:
        """dedup_diff_into for an aligned part whose records partition_bytes_pieces_spans
        already parsed (its n_rec spans and keys, and their handover checksum span_sum). The
        parse is checked against the bytes first (records tile the buffer, the checksum, sampled
        newlines and keys): SGError with rc SG_E_CORRUPT when it does not match. The spans and
        keys are consumed (the sort works in them)."""
        r = _abi.DevResult()
        check(lib.sg_dev_dedup_diff_spans_into(self._h, C.c_void_p(d_cur) if d_cur else None, n_cur,
                                               C.c_void_p(d_spans) if d_spans else None,
                                               C.c_void_p(d_keys) if d_keys else None, n_rec,
                                               int(span_sum) & 0xFFFFFFFFFFFFFFFF,
                                               C.c_void_p(d_prior) if d_prior else None, n_prior, C.c_void_p(d_uniq),
                                               uniq_cap, C.c_void_p(d_fresh) if d_fresh else None, fresh_cap,
                                               C.byref(r)))
        return r

    def dedup_diff_into(self, d_cur: int, n_cur: int, d_prior: int, n_prior: int, d_uniq: int, uniq_cap: int,
                        d_fresh: int, fresh_cap: int) -> _abi.DevResult:
        """dedup_diff with both outputs written at caller device addresses (capacities >= n_cur + 1)."""
        r = _abi.DevResult()
        check(lib.sg_dev_dedup_diff_into(self._h, C.c_void_p(d_cur) if d_cur else None, n_cur,
                                         C.c_void_p(d_prior) if d_prior else None, n_prior, C.c_void_p(d_uniq),
                                         uniq_cap, C.c_void_p(d_fresh) if d_fresh else None, fresh_cap, C.byref(r)))
        return r

    def record_sample(self, d_buf: int, n: int, m: int) -> Tuple[List[bytes], int]:
        """(the first SPLIT_BYTES bytes of m evenly spaced records — [] when the buffer has
        no records —, record count)."""
        heads = np.zeros((max(1, m), SPLIT_BYTES), dtype=np.uint8)
        lens = np.zeros(max(1, m), dtype=np.uint32)
        nr = C.c_uint64()
        check(lib.sg_dev_record_sample(self._h, C.c_void_p(d_buf), n, m, heads.ctypes.data,
                                       lens.ctypes.data_as(C.POINTER(C.c_uint32)), C.byref(nr)))
        if nr.value == 0:
            return [], 0
        return [heads[k, :lens[k]].tobytes() for k in range(m)], nr.value

    def key_sample(self, d_buf: int, n: int, m: int):
        """(m evenly spaced records' key0 values as uint64 (all ~0 if empty), record count)."""
        out = np.empty(max(1, m), dtype=np.uint64)
        nr = C.c_uint64()
        check(lib.sg_dev_key_sample(self._h, C.c_void_p(d_buf), n, m, out.ctypes.data_as(C.POINTER(C.c_uint64)),
                                    C.byref(nr)))
        return out[:m], nr.value

    def partition(self, d_buf: int, n: int, n_parts: int, d_out: int, out_cap: int):
        """Route records to part(hash64(record), n_parts), writing them grouped by partition
        into the caller's device buffer d_out (capacity >= n + 1). Returns (bytes per part,
        records per part)."""
        pb = (C.c_uint64 * n_parts)()
        pr = (C.c_uint64 * n_parts)()
        check(lib.sg_dev_partition(self._h, C.c_void_p(d_buf), n, n_parts, C.c_void_p(d_out),
                                   out_cap, pb, pr))
        return list(pb), list(pr)


class Templates:
    """nuclei matcher logic compiled for the GPU.

    templates: [{"condition": "and"|"or", "matchers": [{"type": "word"|"regex",
    "part": str, "condition": "and"|"or", "negative": bool, "case-insensitive": bool,
    "patterns": [bytes]}]}] — the matcher block of a nuclei template with `encoding: hex`
    words already decoded (tests/golden/gen_template_fixtures.py shows the conversion).
    A matcher whose part names one of `keys` reads that httpx -json field; any other part
    reads the whole record."""

    def __init__(self, templates, keys: Sequence[bytes] = ()):
        self.keys = [k.encode() if isinstance(k, str) else bytes(k) for k in keys]
        pats, ms, tflags = [], [], []
        for ti, t in enumerate(templates):
            tflags.append(_abi.SG_TM_AND if t.get("condition", "or") == "and" else 0)
            for m in t["matchers"]:
                part = m.get("part", "body")
                part = part.encode() if isinstance(part, str) else bytes(part)
                f = 0
                if m.get("condition", "or") == "and":
                    f |= _abi.SG_TM_AND
                if m.get("negative"):
                    f |= _abi.SG_TM_NEGATIVE
                if m.get("case-insensitive"):
                    f |= _abi.SG_TM_NOCASE
                kind = _abi.SG_TM_REGEX if m["type"] == "regex" else _abi.SG_TM_WORD
                ms.append(_abi.TmMatcher(kind, self.keys.index(part) + 1 if part in self.keys else 0, f, ti,
                                         len(pats), len(m["patterns"])))
                pats += [bytes(p) for p in m["patterns"]]
        blob = np.frombuffer(b"".join(pats) or b"\0", dtype=np.uint8)
        offs = np.zeros(len(pats) + 1, dtype=np.uint32)
        np.cumsum([len(p) for p in pats], out=offs[1:])
        marr = (_abi.TmMatcher * max(1, len(ms)))(*ms)
        tf = np.array(tflags or [0], dtype=np.uint32)
        kb, ko = _keys_blob(self.keys)
        U32P = C.POINTER(C.c_uint32)
        self._h = C.c_void_p()
        check(lib.sg_tmpl_compile(blob.ctypes.data, offs.ctypes.data_as(U32P), len(pats), marr, len(ms),
                                  tf.ctypes.data_as(U32P), len(tflags), kb.ctypes.data, ko.ctypes.data_as(U32P),
                                  len(self.keys), C.byref(self._h)))
        self.n = len(tflags)

    def close(self):
        if self._h:
            lib.sg_tmpl_free(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def info(self) -> dict:
        a, e, v = C.c_uint32(), C.c_uint32(), C.c_uint32()
        check(lib.sg_tmpl_info(self._h, C.byref(a), C.byref(e), C.byref(v)))
        return {"atoms": a.value, "engines": e.value, "vacuous": v.value, "templates": self.n}

    def match(self, buf) -> List[Tuple[int, int]]:
        """Sorted (record index, template index) pairs for which the template holds."""
        a = _view(buf)
        cap = max(1024, a.size // 8)
        while True:
            rec = np.empty(cap, dtype=np.uint32)
            tid = np.empty(cap, dtype=np.uint32)
            n = C.c_size_t(0)
            U32P = C.POINTER(C.c_uint32)
            rc = lib.sg_tmpl_eval(self._h, _ptr(a), a.size, rec.ctypes.data_as(U32P), tid.ctypes.data_as(U32P), cap,
                                  C.byref(n))
            if rc == _abi.SG_E_CAP:
                cap = n.value
                continue
            check(rc)
            return list(zip(rec[: n.value].tolist(), tid[: n.value].tolist()))

    def dev_match(self, ctx: "Context", d_buf: int, n: int, rows: _abi.DevRows = None,
                  rows_keys: Sequence[bytes] = None) -> _abi.DevTMatches:
        """rows (with rows_keys, the keys they were built with): the result of
        ctx.json_fields(d_buf, n, rows_keys) just before on the same context — the field
        rows are then not built a second time (include/swarmgpu.h sg_dev_tmpl_eval_rows)."""
        r = _abi.DevTMatches()
        if rows is not None:
            if [bytes(k) for k in (rows_keys or [])] != self.keys:
                raise ValueError("rows were built for keys %r, the templates use %r" % (rows_keys, self.keys))
            check(lib.sg_dev_tmpl_eval_rows(ctx._h, self._h, C.c_void_p(d_buf), n, C.byref(rows), C.byref(r)))
        else:
            check(lib.sg_dev_tmpl_eval(ctx._h, self._h, C.c_void_p(d_buf), n, C.byref(r)))
        return r


class Ingest:
    """Streamed /raw merge (§8(f) row 4): append chunk bodies (or pieces of them, as they
    stream from S3) in the A5 key order; finish() returns the merged body resident in HBM
    (device pointer, length), byte-identical to server/server.py:407-410's concatenation."""

    def __init__(self, ctx: "Context", size_hint: int = 0):
        self.ctx = ctx
        self._h = C.c_void_p()
        check(lib.sg_ingest_open(ctx._h, size_hint, C.byref(self._h)))

    def append(self, piece) -> None:
        a = _view(piece)
        if a.size:
            check(lib.sg_ingest_append(self._h, a.ctypes.data, a.size))

    def finish(self) -> Tuple[int, int]:
        d, n = C.c_void_p(), C.c_uint64()
        check(lib.sg_ingest_finish(self._h, C.byref(d), C.byref(n)))
        return d.value or 0, n.value

    def dedup_diff(self, prior=None) -> Tuple[bytes, bytes]:
        """(sort -u of the merged body, new records vs `prior`) as bytes."""
        d, n = self.finish()
        pd, pn, keep = 0, 0, None
        pv = _view(prior) if prior is not None else None
        if pv is not None and pv.size:
            import torch
            keep = torch.from_numpy(np.array(pv)).cuda(self.ctx.device)
            self.ctx.fence_in()
            pd, pn = keep.data_ptr(), keep.numel()
        r = self.ctx.dedup_diff(d, n, pd, pn)
        return self.ctx.to_bytes(r.uniq, r.uniq_bytes), self.ctx.to_bytes(r.fresh, r.fresh_bytes)

    def close(self):
        if self._h:
            lib.sg_ingest_close(self._h)
            self._h = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
