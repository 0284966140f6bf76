"""Drop-in hooks for the reference's worker.py and server.py.

The REST API, the module contract and the client stay unchanged; these functions replace
the byte-level work at three points of the reference:

  server /raw/<scan_id>      server/server.py:399-412  -> raw_merge / raw_unique
  scan completion (100 %)    server/server.py:274-294  -> completion_dedup_diff
  worker after module run    worker/worker.py:83-98    -> postprocess_output
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional, Sequence, Tuple

from . import api

S3_PAGE = 1000  # one ListObjects page: server/server.py:403 does not paginate


def merge_keys(keys: Iterable[str], scan_id: str) -> List[str]:
    """server/server.py:403-404: keys under '{scan}/output/' in S3's binary key order,
    first page (1,000 keys) only, keeping those ending in '.txt'."""
    prefix = "%s/output/" % scan_id
    listed = sorted(k for k in keys if k.startswith(prefix))[:S3_PAGE]
    return [k for k in listed if k.endswith(".txt")]


def check_utf8(body: bytes, key: str = "") -> None:
    """server/server.py:410 decodes every chunk body on its own (`.decode('utf-8')`), so a body
    that is not valid UTF-8 — including a multibyte character split across two chunk files —
    makes /raw fail there. The GPU path works on bytes; the hooks keep the reference's
    behaviour by raising the same UnicodeDecodeError for such a body before any GPU work."""
    try:
        body.decode("utf-8")
    except UnicodeDecodeError as e:
        raise UnicodeDecodeError(e.encoding, e.object, e.start, e.end, "%s (chunk %s)" % (e.reason, key)) from None


def _bodies(objects: Dict[str, bytes], scan_id: str, strict_utf8: bool) -> List[bytes]:
    keys = merge_keys(objects.keys(), scan_id)
    if strict_utf8:
        for k in keys:
            check_utf8(objects[k], k)
    return [objects[k] for k in keys]


def raw_merge(objects: Dict[str, bytes], scan_id: str, strict_utf8: bool = True) -> bytes:
    """Byte-identical /raw body: concatenation in merge_keys order, no separator
    (server/server.py:407-410); invalid UTF-8 fails as the reference's decode does."""
    return b"".join(_bodies(objects, scan_id, strict_utf8))


def raw_unique(objects: Dict[str, bytes], scan_id: str, strict_utf8: bool = True) -> bytes:
    """sort -u of the /raw body, computed on the GPU straight from the chunk bodies."""
    return api.dedup_chunks(_bodies(objects, scan_id, strict_utf8))


def completion_dedup_diff(objects: Dict[str, bytes], scan_id: str,
                          prior_unique: Optional[bytes], strict_utf8: bool = True) -> Tuple[bytes, bytes]:
    """At scan completion: (sort -u of this scan, records new since the prior scan of the
    same module). `prior_unique` is the prior scan's stored sort -u output (or None)."""
    bodies = _bodies(objects, scan_id, strict_utf8)
    merged = b"".join(bodies) if len(bodies) != 1 else bodies[0]
    return api.dedup_diff(merged, prior_unique or b"")


def prior_scan_id(scans: Sequence[dict], module: str, scan_started: int) -> Optional[str]:
    """The prior scan of the same module: latest `scan_started` earlier than this one, from
    the asm.scans documents written at server/server.py:284-294."""
    best = None
    for s in scans:
        if s.get("module") != module or s.get("scan_status") != "complete":
            continue
        st = s.get("scan_started")
        if st is None or st >= scan_started:
            continue
        if best is None or st > best["scan_started"]:
            best = s
    return best["scan_id"] if best else None


def postprocess_output(output_file: str, matcher=None, matches_file: Optional[str] = None) -> int:
    """Worker hook between the module run and the upload (worker/worker.py:83-98): parse the
    module's line-delimited output on the GPU and, if a signature matcher is given, write
    the matched lines (grep output, input order) to `matches_file`. The output file itself
    is left untouched, so the upload contract (uploads/{scan}/output/chunk_{i}.txt) holds.
    Returns the number of non-empty records. One GPU pass: the match call parses the
    records itself (its in_records), so the file is not parsed twice."""
    with open(output_file, "rb") as f:
        data = f.read()
    if matcher is not None and matches_file:
        lines_out, n = matcher.match_lines_count(data)
        with open(matches_file, "wb") as f:
            f.write(lines_out)
        return n
    return len(api.lines(data))


def raw_stream_dedup_diff(ctx, keys: Iterable[str], scan_id: str, read_body, prior_unique: Optional[bytes] = None,
                          sizes: Optional[Dict[str, int]] = None) -> Tuple[bytes, bytes]:
    """/raw + completion without the `str +=` merge (server/server.py:399-412, §8(f) row 4):
    `read_body(key)` yields the pieces of one S3 object body (e.g. botocore's
    StreamingBody.iter_chunks()); they are appended straight into pinned staging buffers
    and copied to HBM in A5 key order while the next piece is read. `sizes` (key ->
    ContentLength from the listing) pre-sizes the device buffer."""
    order = merge_keys(keys, scan_id)
    hint = sum(sizes.get(k, 0) for k in order) if sizes else 0
    with api.Ingest(ctx, hint) as ing:
        for k in order:
            for piece in read_body(k):
                ing.append(piece)
        return ing.dedup_diff(prior_unique)
