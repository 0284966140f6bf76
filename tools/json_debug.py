"""Debug helper for the JSON field scan: runs one of the JSON test inputs through
swarm_amd.json_fields and the oracle and prints the first mismatching (record, key) rows
with the record's text.  python3 tools/json_debug.py <case>   (case: keys64 | random | httpx)"""
import json
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import swarm_amd as sg  # noqa: E402
from swarm_amd import corpus  # noqa: E402
from oracle import semantics as S  # noqa: E402  (checker only)


def case(name):
    if name == "keys64":
        keys = [b"k%d" % i for i in range(64)]
        rng = random.Random(3)
        lines = []
        for _ in range(300):
            obj = {("k%d" % rng.randrange(70)): rng.choice(["v", "", 5, [1, "x"], {"k1": "nested"}]) for _ in range(20)}
            lines.append(json.dumps(obj).encode())
        return b"\n".join(lines) + b"\n", keys
    if name == "httpx":
        return b"\n".join(corpus.httpx_json_pool(3000, seed=8)) + b"\n", [b"url", b"title", b"webserver", b"tech"]
    raise SystemExit("unknown case")


def main():
    data, keys = case(sys.argv[1])
    rows, rrec, rkey = sg.json_fields(data, keys)
    o_rows, o_rec, o_key = S.json_field_rows(data, keys)
    lines = data.split(b"\n")

    def group(rows, rec, key):
        out = {}
        for row, r, k in zip(rows.split(b"\n"), rec, key):
            out.setdefault((r, k), []).append(row)
        return out

    g = group(rows, list(rrec.tolist()), list(rkey.tolist()))
    o = group(o_rows, o_rec, o_key)
    bad = sorted(set(g) | set(o))
    n = 0
    for rk in bad:
        if g.get(rk) != o.get(rk):
            r, k = rk
            print("record %d key %s: gpu %r oracle %r" % (r, keys[k], g.get(rk), o.get(rk)))
            print("   line:", lines[r][:400])
            n += 1
            if n >= 6:
                break
    print("mismatches shown:", n)


if __name__ == "__main__":
    main()
