#!/usr/bin/env python3
"""Extract nuclei templates (data) from the reference's template snapshot
(worker/artifacts/templates/**) into a committed fixture of
matcher logic: every template whose single matcher block uses only `word`, `regex` and
`binary` matchers (dsl/status/size/xpath/json are out of scope), with its
matchers-condition, and per matcher: type, part, condition, negative, case-insensitive
and the patterns as bytes (hex words / binary decoded). Regexes must compile as Python
bytes patterns and be accepted by swarm_amd's DFA compiler (tagged like signatures.json).

YAML is read with yaml.safe_load (no code execution). Run in the build container only:
    python3 tests/golden/gen_template_fixtures.py
"""
import base64
import ctypes
import json
import os
import re
import sys

import yaml

REF = "/root/reference/worker/artifacts/templates"
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
BLOCKS = ("requests", "http", "network", "tcp", "dns", "file", "ssl", "headless", "websocket")


def dfa_ok(lib, pat: bytes) -> bool:
    buf = (ctypes.c_uint8 * max(1, len(pat))).from_buffer_copy(pat or b"\0")
    offs = (ctypes.c_uint32 * 2)(0, len(pat))
    h = ctypes.c_void_p()
    rc = lib.sg_dfa_compile(buf, offs, 1, 0, ctypes.byref(h))
    if rc == 0:
        lib.sg_free(h)
    return rc == 0


def matcher_blocks(doc):
    out = []
    for k in BLOCKS:
        v = doc.get(k)
        if isinstance(v, list):
            for b in v:
                if isinstance(b, dict) and isinstance(b.get("matchers"), list):
                    out.append(b)
    return out


def convert(block, lib):
    ms = []
    for m in block["matchers"]:
        if not isinstance(m, dict) or m.get("internal"):
            return None
        t = m.get("type")
        if t == "word":
            ws = m.get("words") or []
            if not ws or not all(isinstance(w, str) for w in ws):
                return None
            if m.get("encoding") == "hex":
                try:
                    pats = [bytes.fromhex(w) for w in ws]
                except ValueError:
                    return None
            else:
                pats = [w.encode("utf-8") for w in ws]
            kind = "word"
        elif t == "binary":
            ws = m.get("binary") or []
            try:
                pats = [bytes.fromhex(w) for w in ws]
            except (ValueError, TypeError):
                return None
            kind = "word"
        elif t == "regex":
            rs = m.get("regex") or []
            if not rs or not all(isinstance(r, str) for r in rs):
                return None
            pats = [r.encode("utf-8") for r in rs]
            for p in pats:
                try:
                    re.compile(p)
                except re.error:
                    return None
                if not dfa_ok(lib, p):
                    return None
            kind = "regex"
        else:
            return None
        if not pats or any(len(p) == 0 for p in pats):
            return None
        ms.append({"type": kind, "part": str(m.get("part", "body")),
                   "condition": str(m.get("condition", "or")).lower(),
                   "negative": bool(m.get("negative", False)),
                   "case-insensitive": bool(m.get("case-insensitive", False)),
                   "patterns": [base64.b64encode(p).decode() for p in pats]})
    if not ms:
        return None
    return {"condition": str(block.get("matchers-condition", "or")).lower(), "matchers": ms}


def main():
    sys.path.insert(0, ROOT)
    from swarm_amd import _abi
    lib = _abi.lib
    out, n_files, skipped = [], 0, 0
    for dp, _, fns in sorted(os.walk(REF)):
        for fn in sorted(fns):
            if not fn.endswith(".yaml"):
                continue
            path = os.path.join(dp, fn)
            try:
                with open(path, "rb") as f:
                    doc = yaml.safe_load(f)
            except Exception:
                continue
            if not isinstance(doc, dict):
                continue
            n_files += 1
            blocks = matcher_blocks(doc)
            if len(blocks) != 1:
                skipped += 1
                continue
            t = convert(blocks[0], lib)
            if t is None:
                skipped += 1
                continue
            t["id"] = str(doc.get("id", fn))
            t["file"] = os.path.relpath(path, REF)
            t["severity"] = str((doc.get("info") or {}).get("severity", "")).lower()
            out.append(t)
    res = {"source": "worker/artifacts/templates/** (reference snapshot), yaml.safe_load",
           "files": n_files, "skipped": skipped, "templates": out}
    with open(os.path.join(HERE, "templates.json"), "w") as f:
        json.dump(res, f, separators=(",", ":"))
    print("files %d, kept %d, skipped %d" % (n_files, len(out), skipped))


if __name__ == "__main__":
    main()
