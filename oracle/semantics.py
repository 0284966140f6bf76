"""CPU ORACLE — test infrastructure only, never a product path.

Plain-Python restatement of the reference semantics for the scan-result hot path
(SURVEY.md §8(a) rows A1–A8). Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg import this module, and only as the checker / CPU baseline. The
product path (swarm_amd) never imports it and fails loudly without its HIP library.

Pinning:
  * A1/A5/A6/A2 are pinned against vectors produced by the reference's OWN code
    (tests/golden/reference_vectors.json, from gen_reference_fixtures.py).
  * A3/A7/A8 have no reference code (README.md:11 lists them as planned). Their
    semantics are fixed by BASELINE.json north_star ("sort -u / set semantics") and
    pinned against GNU coreutils `LC_ALL=C sort -u` / `comm -13`
    (tests/golden/coreutils_vectors.json, from gen_tool_fixtures.py).
  * A4 lives in absent third-party binaries (nuclei/httpx/nmap, unpinned versions;
    .MISSING_LARGE_BLOBS:1-4). It is pinned to grep-style semantics: literal ==
    `LC_ALL=C grep -F` (Python `sig in line`), regex == Python `re.search` on bytes,
    cross-checked against `grep -P`/`grep -E` on the common subset
    (tests/golden/grep_vectors.json).
"""
from __future__ import annotations

import re
from typing import Dict, Iterable, List, Sequence, Tuple

NL = b"\n"


# ----------------------------------------------------------------------------- A1
def client_readlines(data: bytes) -> List[str]:
    """client/swarm:20-21 — `open(file, 'r').readlines()`: UTF-8 decode with universal
    newlines ('\\r\\n' and lone '\\r' become '\\n'); every line keeps its '\\n'."""
    text = data.decode("utf-8")
    text = text.replace("\r\n", "\n").replace("\r", "\n")
    parts = text.split("\n")  # readlines splits on '\n' only (not on \x0b, \x85, ...)
    lines = [p + "\n" for p in parts[:-1]]
    if parts[-1]:
        lines.append(parts[-1])
    return lines


def server_chunks(file_content: Sequence[str], batch_size: int) -> List[bytes]:
    """server/server.py:433-447 — batch_size==0 means one chunk (:434-435);
    chunk_generator slices (:185-187); S3 body is '\\n'.join(chunk) (:447), UTF-8."""
    n = len(file_content)
    if batch_size == 0:
        batch_size = n
    if batch_size == 0:
        raise ValueError("range() arg 3 must not be zero")  # server raises: empty input, batch 0
    return ["\n".join(file_content[i:i + batch_size]).encode("utf-8")
            for i in range(0, n, batch_size)]


# ----------------------------------------------------------------------------- A5
S3_PAGE = 1000


def merge_keys(keys: Iterable[str], scan_id: str) -> List[str]:
    """server/server.py:403-404 — ListObjects under '{scan}/output/' (binary key order,
    one page of 1,000 keys, no pagination), keep keys ending in '.txt'."""
    prefix = "%s/output/" % scan_id
    listed = sorted(k for k in keys if k.startswith(prefix))[:S3_PAGE]
    return [k for k in listed if k.endswith(".txt")]


def merge_chunks(objects: Dict[str, bytes], scan_id: str) -> bytes:
    """server/server.py:407-412 — concatenate bodies in listed order, no separator."""
    return b"".join(objects[k] for k in merge_keys(objects.keys(), scan_id))


# ----------------------------------------------------------------------------- A3
def parse_records(buf: bytes) -> List[bytes]:
    """A3: split on '\\n', drop empty records (no trimming; '\\r' is kept)."""
    return [r for r in buf.split(NL) if r]


def record_spans(buf: bytes) -> List[Tuple[int, int]]:
    """A3 as (start, end) byte spans of the non-empty records, in input order."""
    out = []
    pos = 0
    n = len(buf)
    while pos <= n:
        q = buf.find(NL, pos)
        if q < 0:
            q = n
        if q > pos:
            out.append((pos, q))
        pos = q + 1
    return out


def serialize(records: Iterable[bytes]) -> bytes:
    recs = list(records)
    return b"".join(r + NL for r in recs)


# ----------------------------------------------------------------------------- A7 / A8
def dedup(buf: bytes) -> bytes:
    """A7: `sorted(set(buf.split(b'\\n')) - {b''})`, '\\n'-terminated == LC_ALL=C sort -u
    minus the empty line."""
    return serialize(sorted(set(buf.split(NL)) - {b""}))


def diff(cur: bytes, prior: bytes) -> bytes:
    """A8: `sorted(set(cur) - set(prior))` == LC_ALL=C comm -13 prior.sorted cur.sorted."""
    c = set(cur.split(NL)) - {b""}
    p = set(prior.split(NL))
    return serialize(sorted(c - p))


def dedup_diff(cur: bytes, prior: bytes) -> Tuple[bytes, bytes]:
    """The fused A7+A8 step the server runs at scan completion (A9)."""
    c = set(cur.split(NL)) - {b""}
    p = set(prior.split(NL))
    return serialize(sorted(c)), serialize(sorted(c - p))


# ----------------------------------------------------------------------------- A4
def _fold(b: bytes) -> bytes:
    return b.lower()  # bytes.lower() folds ASCII A-Z only == C-locale grep -i


def literal_hits(buf: bytes, sigs: Sequence[bytes], nocase: bool = False) -> List[Tuple[int, int]]:
    """A4 literal: for every non-empty record (A3 order) and every signature, does
    `sig in record` hold. Returns sorted (record_index, signature_index) pairs."""
    if any(len(s) == 0 for s in sigs):
        raise ValueError("empty signature")
    pats = [_fold(s) if nocase else s for s in sigs]
    hits = []
    for ri, rec in enumerate(parse_records(buf)):
        line = _fold(rec) if nocase else rec
        for si, p in enumerate(pats):
            if p in line:
                hits.append((ri, si))
    return hits


def regex_hits(buf: bytes, regexes: Sequence[bytes], nocase: bool = False) -> List[Tuple[int, int]]:
    """A4 regex: `re.search(pattern, record)` on bytes (unanchored search per record)."""
    flags = re.IGNORECASE if nocase else 0
    comp = [re.compile(r, flags) for r in regexes]
    hits = []
    for ri, rec in enumerate(parse_records(buf)):
        for si, c in enumerate(comp):
            if c.search(rec) is not None:
                hits.append((ri, si))
    return hits


def matched_lines(buf: bytes, hits: Sequence[Tuple[int, int]]) -> bytes:
    """Matched records in input order (one per record), '\\n'-terminated == grep output
    for lines that are non-empty."""
    recs = parse_records(buf)
    seen = sorted({r for r, _ in hits})
    return serialize(recs[r] for r in seen)


# ----------------------------------------------------------------------------- (e)
def hash_partition(records: Iterable[bytes], n_parts: int, hash_fn) -> List[List[bytes]]:
    """records go to partition hash(record) % G."""
    parts: List[List[bytes]] = [[] for _ in range(n_parts)]
    for r in records:
        parts[hash_fn(r) % n_parts].append(r)
    return parts
