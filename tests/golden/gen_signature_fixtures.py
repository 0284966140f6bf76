#!/usr/bin/env python3
"""Extract the signature corpus (data) from the reference's nuclei template snapshot
(worker/artifacts/templates/**, SURVEY.md §2 "Signature corpus") into a committed fixture:

  words   : sorted unique `type: word` matcher words (encoding: hex excluded), as bytes
  regexes : sorted unique `type: regex` matcher patterns that compile under Python `re`
            as bytes patterns, each tagged with whether swarm_amd's DFA compiler accepts it
  info    : the subset from `severity: info` templates (worker/modules/nuclei.json:2 `-s info`)

YAML is read with yaml.safe_load (no code execution). Run in the build container only:
    python3 tests/golden/gen_signature_fixtures.py
"""
import base64
import json
import os
import re
import sys

import yaml

REF = "/root/reference/worker/artifacts/templates"
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))


def walk_matchers(doc):
    if isinstance(doc, dict):
        if "matchers" in doc and isinstance(doc["matchers"], list):
            for m in doc["matchers"]:
                if isinstance(m, dict):
                    yield m
        for v in doc.values():
            yield from walk_matchers(v)
    elif isinstance(doc, list):
        for v in doc:
            yield from walk_matchers(v)


def main():
    words, regexes = set(), set()
    info_words, info_regexes = set(), set()
    n_files = 0
    for dp, _, fns in os.walk(REF):
        for fn in fns:
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
            sev = str((doc.get("info") or {}).get("severity", "")).lower()
            for m in walk_matchers(doc):
                t = m.get("type")
                if t == "word" and m.get("encoding") != "hex":
                    for w in m.get("words") or []:
                        if isinstance(w, (str, int, float)):
                            b = str(w).encode("utf-8")
                            if b and b"\n" not in b:
                                words.add(b)
                                if sev == "info":
                                    info_words.add(b)
                elif t == "regex":
                    for r in m.get("regex") or []:
                        if isinstance(r, str):
                            b = r.encode("utf-8")
                            if b and b"\n" not in b:
                                regexes.add(b)
                                if sev == "info":
                                    info_regexes.add(b)
    sys.path.insert(0, ROOT)
    from swarm_amd import _abi  # compile-only check (host code, no GPU)
    import ctypes as C
    import numpy as np

    def dfa_ok(p):
        a = np.frombuffer(p, dtype=np.uint8)
        offs = np.array([0, len(p)], dtype=np.uint32)
        h = C.c_void_p()
        rc = _abi.lib.sg_dfa_compile(a.ctypes.data, offs.ctypes.data_as(C.POINTER(C.c_uint32)), 1, 0, C.byref(h))
        if rc == 0:
            _abi.lib.sg_free(h)
        return rc

    rx = []
    for r in sorted(regexes):
        try:
            re.compile(r)
        except re.error:
            continue
        rx.append({"p": base64.b64encode(r).decode(), "dfa_rc": dfa_ok(r), "info": r in info_regexes})
    out = {
        "note": "signature corpus extracted from the reference nuclei templates by "
                "tests/golden/gen_signature_fixtures.py (yaml.safe_load)",
        "templates": n_files,
        "words": [base64.b64encode(w).decode() for w in sorted(words)],
        "info_words": len(info_words),
        "regexes": rx,
    }
    with open(os.path.join(HERE, "signatures.json"), "w") as f:
        json.dump(out, f, indent=0)
    ok = sum(1 for r in rx if r["dfa_rc"] == 0)
    print("templates", n_files, "words", len(words), "regexes(py-ok)", len(rx), "dfa-ok", ok)


if __name__ == "__main__":
    main()
