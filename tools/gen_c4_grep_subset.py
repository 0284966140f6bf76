"""The 'agreeing subset' of the C4 signature set for the GNU `grep -E -f` CPU baseline
(BASELINE.md CPU-baseline plan): patterns whose POSIX-ERE reading gives the same matched
lines as Python's re.search on a sample of C4 banners. Syntactic filter first (no \\d-style
escapes, no (?...) groups, no lazy quantifiers, no backslash inside a bracket expression,
no range followed by '-'), then an empirical check per pattern with GNU grep on 3,000
banners. Writes tests/golden/c4_grep_subset.json (indices into corpus.c4_signatures' list)."""
import base64
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from swarm_amd import corpus  # noqa: E402

BAD = re.compile(rb"\\[dDsSwWbBAZzQEGh]|\(\?|[*+?}]\?|\\x|\{,|\\u|\\[0-9]|\[\^?\]|\\n|\\r|\\t|\\f|\\v|\\0|\\N|\\p|\\P"
                 rb"|\[[^\]]*\w-\w-|\[[^\]]*\\")


def main():
    sig = json.load(open(os.path.join(ROOT, "tests", "golden", "signatures.json")))
    pats, _ = corpus.c4_signatures([base64.b64decode(r["p"]) for r in sig["regexes"]])
    sample = corpus.lines_from_pool(corpus.banner_pool(), 3000, seed=3).tobytes()
    lines = sample.split(b"\n")[:-1]
    env = dict(os.environ, LC_ALL="C")
    keep = []
    for i, p in enumerate(pats):
        if BAD.search(p) or b"\n" in p:
            continue
        want = b"".join(ln + b"\n" for ln in lines if re.search(p, ln))
        r = subprocess.run(["grep", "-a", "-E", "-e", p.decode("latin1")], input=sample, env=env, stdout=subprocess.PIPE)
        if r.returncode in (0, 1) and r.stdout == want:
            keep.append(i)
    out = {"n_signatures": len(pats), "subset": keep,
           "note": "indices into corpus.c4_signatures(); grep -E agrees with re.search on 3,000 C4 banners"}
    with open(os.path.join(ROOT, "tests", "golden", "c4_grep_subset.json"), "w") as f:
        json.dump(out, f)
    print("%d of %d signatures" % (len(keep), len(pats)))


if __name__ == "__main__":
    main()
