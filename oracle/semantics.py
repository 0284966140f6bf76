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


# ----------------------------------------------------------------------------- §8(f)2 nmap -oN
# worker/modules/nmap.json:2 runs `nmap ... -oN {output}`; the reference uploads the text
# verbatim (worker/worker.py:96-98). The build turns it into C5-style host:port records.
_NMAP_REPORT = b"Nmap scan report for "
_NMAP_PORT = re.compile(rb"([0-9]{1,5})/(?:tcp|udp|sctp)[ \t]+open(?:[ \t]|$)")


def nmap_host_ports(buf: bytes) -> bytes:
    """One 'host:port' record per open-port line, in input order ('\\n'-terminated). host =
    the report line's text after 'Nmap scan report for ' up to the first space; port lines
    before any report line, or under a report with an empty host, are dropped."""
    host = None
    out = []
    for rec in parse_records(buf):
        if rec.startswith(_NMAP_REPORT):
            host = rec[len(_NMAP_REPORT):].split(b" ", 1)[0]
            continue
        m = _NMAP_PORT.match(rec)
        if m and host:
            out.append(host + b":" + m.group(1))
    return serialize(out)


# ----------------------------------------------------------------------------- §8(f)1 httpx -json
# worker/modules/http2.json:2 / web.json:2 run `httpx ... -json`: one JSON object per line.
# Byte-level restatement of json.loads for top-level member lookup (last duplicate wins)
# and string decoding; tests pin it against json.loads on valid lines.
_JWS = b" \t\r\n"


def _json_members(rec: bytes):
    """[(raw key, value start, value end)] of a line holding exactly one JSON object, or
    None (structural check: one top-level object, balanced strings/brackets, only
    whitespace around it)."""
    depth = 0
    in_str = esc = False
    done = False
    str_s = str_e = val_s = 0
    cur = None
    first = last = open_pos = close_pos = None
    members = []
    for i, ch in enumerate(rec):
        if ch not in _JWS:
            if first is None:
                first = i
            last = i
        if in_str:
            if esc:
                esc = False
            elif ch == 0x5C:
                esc = True
            elif ch == 0x22:
                in_str = False
                str_e = i
            continue
        if ch == 0x22:
            if depth == 0:
                return None
            in_str = True
            str_s = i + 1
        elif ch in b"{[:,}]" and done:
            return None
        elif ch in b"{[":
            if depth == 0:
                if ch != 0x7B:
                    return None
                open_pos = i
            depth += 1
        elif ch in b"}]":
            if depth == 0:
                return None
            if depth == 1:
                if ch != 0x7D:
                    return None
                if cur is not None:
                    members.append((cur, val_s, i))
                cur = None
                done = True
                close_pos = i
            depth -= 1
        elif ch == 0x3A and depth == 1:
            cur = _json_key(rec[str_s:str_e])
            val_s = i + 1
        elif ch == 0x2C and depth == 1:
            if cur is not None:
                members.append((cur, val_s, i))
            cur = None
    if in_str or depth or not done or first != open_pos or last != close_pos:
        return None
    return members


def _json_put_cp(out: bytearray, cp: int, nl: bytes) -> None:
    if cp == 0x0A:
        out += nl
    else:
        out += chr(cp).encode("utf-8", "surrogatepass")


def _json_key(raw: bytes) -> bytes:
    """A member key as json.loads sees it (escapes decoded, a newline stays one byte), in
    UTF-8; requested keys are compared with this."""
    return json_decode_string(raw, nl=b"\n") if b"\\" in raw else raw


def json_decode_string(s: bytes, nl: bytes = b"\\n") -> bytes:
    """JSON string body (between the quotes) -> bytes, as json.loads + UTF-8 encoding
    ('surrogatepass' for lone surrogates); a newline is written as `nl` (backslash-n in
    rows, so a row stays one line)."""
    out = bytearray()
    p, n = 0, len(s)
    hexd = b"0123456789abcdefABCDEF"

    def u4(q):
        if q + 4 > n or any(c not in hexd for c in s[q:q + 4]):
            return None
        return int(s[q:q + 4], 16)

    simple = {0x22: b'"', 0x5C: b"\\", 0x2F: b"/", 0x62: b"\x08", 0x66: b"\x0c", 0x6E: nl, 0x72: b"\r",
              0x74: b"\t"}
    while p < n:
        ch = s[p]
        if ch != 0x5C or p + 1 >= n:
            out.append(ch)
            p += 1
            continue
        e = s[p + 1]
        if e in simple:
            out += simple[e]
            p += 2
        elif e == 0x75:
            v = u4(p + 2)
            if v is None:
                out.append(ch)
                p += 1
                continue
            p += 6
            if 0xD800 <= v < 0xDC00 and p + 1 < n and s[p] == 0x5C and s[p + 1] == 0x75:
                lo = u4(p + 2)
                if lo is not None and 0xDC00 <= lo < 0xE000:
                    v = 0x10000 + ((v - 0xD800) << 10) + (lo - 0xDC00)
                    p += 6
            _json_put_cp(out, v, nl)
        else:
            out.append(ch)
            p += 1
    return bytes(out)


def _json_trim(v: bytes) -> bytes:
    return v.strip(_JWS)


def _json_item(v: bytes) -> List[bytes]:
    v = _json_trim(v)
    if not v:
        return []
    if len(v) >= 2 and v[0] == 0x22 and v[-1] == 0x22:
        return [json_decode_string(v[1:-1])] if len(v) > 2 else []
    return [v]


def json_value_rows(v: bytes) -> List[bytes]:
    """Rows of one member value: a string -> its decoded bytes; an array -> one row per
    element (strings decoded, others raw); anything else -> its raw text. Empty rows are
    dropped."""
    v = _json_trim(v)
    if not v:
        return []
    if v[0] != 0x5B:
        return _json_item(v)
    rows: List[bytes] = []
    depth = 0
    start = 1
    in_str = esc = False
    for p, ch in enumerate(v):
        if in_str:
            if esc:
                esc = False
            elif ch == 0x5C:
                esc = True
            elif ch == 0x22:
                in_str = False
            continue
        if ch == 0x22:
            in_str = True
        elif ch in b"[{":
            depth += 1
        elif ch in b"]}":
            if depth == 1:
                rows += _json_item(v[start:p])
                start = p + 1
            depth -= 1
        elif ch == 0x2C and depth == 1:
            rows += _json_item(v[start:p])
            start = p + 1
    return rows


def json_field_rows(buf: bytes, keys: Sequence[bytes]) -> Tuple[bytes, List[int], List[int]]:
    """(rows '\\n'-terminated, record index per row, key index per row): for each record
    (A3 order) holding one JSON object, each requested key in request order, the rows of
    its last occurrence."""
    rows, rrec, rkey = [], [], []
    for ri, rec in enumerate(parse_records(buf)):
        mem = _json_members(rec)
        if mem is None:
            continue
        last = {}
        for k, s, e in mem:
            last[k] = (s, e)
        for ki, k in enumerate(keys):
            if k in last:
                s, e = last[k]
                for row in json_value_rows(rec[s:e]):
                    rows.append(row)
                    rrec.append(ri)
                    rkey.append(ki)
    return serialize(rows), rrec, rkey


# ----------------------------------------------------------------------------- §8(f)3 nuclei matchers
# Matcher logic of nuclei templates (worker/modules/nuclei.json:2; the corpus is
# worker/artifacts/templates/**): matchers-condition and/or over matchers
# (technologies/tech-detect.yaml:16), each matcher words/regexes joined by its condition,
# `negative` (file/audit/cisco/disable-ip-source-route.yaml:19-22), `case-insensitive`
# (technologies/typo3-detect.yaml:23), `part` = the record, or an httpx -json field when the
# part names one of the requested keys (a pattern hits a field when it occurs in any of the
# field's rows). nuclei is an absent Go binary: this restates its documented semantics.
def _tm_part(part, keys: Sequence[bytes]) -> int:
    p = part.encode() if isinstance(part, str) else bytes(part)
    return keys.index(p) + 1 if p in keys else 0


def template_matches(buf: bytes, templates, keys: Sequence[bytes] = ()) -> List[Tuple[int, int]]:
    """Sorted (record index, template index) pairs for which the template holds."""
    keys = [k.encode() if isinstance(k, str) else bytes(k) for k in keys]
    norm = []
    for t in templates:
        ms = []
        for m in t["matchers"]:
            nc = bool(m.get("case-insensitive"))
            pats = [bytes(p) for p in m["patterns"]]
            if m["type"] == "regex":
                comp = [re.compile(p) for p in pats]  # case-insensitive is a word option; regexes use (?i)
                test = (lambda comp: lambda text: [c.search(text) is not None for c in comp])(comp)
            else:
                ws = [_fold(p) if nc else p for p in pats]
                test = (lambda ws, nc: lambda text: [w in (_fold(text) if nc else text) for w in ws])(ws, nc)
            ms.append((_tm_part(m.get("part", "body"), keys), test, m.get("condition", "or") == "and",
                       bool(m.get("negative"))))
        norm.append((t.get("condition", "or") == "and", ms))
    recs = parse_records(buf)
    rows_of = [dict() for _ in recs]
    if keys:
        rows, rrec, rkey = json_field_rows(buf, keys)
        for row, r, k in zip(rows.split(b"\n")[:-1], rrec, rkey):
            rows_of[r].setdefault(k + 1, []).append(row)
    out = []
    for ri, rec in enumerate(recs):
        for ti, (and_t, ms) in enumerate(norm):
            acc = and_t
            for part, test, and_m, neg in ms:
                texts = [rec] if part == 0 else rows_of[ri].get(part, [])
                hits = [False] * 0
                for text in texts:
                    h = test(text)
                    hits = h if not hits else [a or b for a, b in zip(hits, h)]
                if not hits:
                    ok = False
                else:
                    ok = all(hits) if and_m else any(hits)
                if neg:
                    ok = not ok
                acc = (acc and ok) if and_t else (acc or ok)
            if acc:
                out.append((ri, ti))
    return out
