#!/usr/bin/env python3
"""Golden vectors for the rows with no reference code (A3/A7/A8) and for A4, produced by
GNU tools in the C locale:

  A7 dedup  == `LC_ALL=C sort -u`           (minus the empty line)
  A8 diff   == `LC_ALL=C comm -13 prior cur` (both sort -u'd)
  A4 literal== `LC_ALL=C grep -F [-i] -n`    (one run per signature)
  A4 regex  == `LC_ALL=C grep -P -n`         (PCRE; Python `re` on bytes agrees on the subset)

Run in the build container:  python3 tests/golden/gen_tool_fixtures.py
Writes tests/golden/coreutils_vectors.json and tests/golden/grep_vectors.json.
"""
import base64
import json
import os
import random
import subprocess
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ENV = dict(os.environ, LC_ALL="C")


def b64(b):
    return base64.b64encode(b).decode()


def run(cmd, inp=None):
    return subprocess.run(cmd, input=inp, stdout=subprocess.PIPE, env=ENV, check=False).stdout


def sort_u(data: bytes) -> bytes:
    out = run(["sort", "-u"], data)
    if out.startswith(b"\n"):  # the empty record sorts first in C locale; A7 drops it
        out = out[1:]
    return out


def comm13(prior_sorted: bytes, cur_sorted: bytes) -> bytes:
    with tempfile.TemporaryDirectory() as d:
        a, b = os.path.join(d, "p"), os.path.join(d, "c")
        open(a, "wb").write(prior_sorted)
        open(b, "wb").write(cur_sorted)
        return run(["comm", "-13", a, b])


def subdomains(rng, n, pool):
    labels = []
    for _ in range(pool):
        L = rng.randint(1, 14)
        lab = "".join(rng.choice("abcdefghijklmnopqrstuvwxyz0123456789") for _ in range(L))
        opt = rng.choice(["", "", "api.", "dev.", "www.", "mail."])
        labels.append(("%s.%starget%d.com" % (lab, opt, rng.randrange(64))).encode())
    return b"".join(rng.choice(labels) + b"\n" for _ in range(n))


def dedup_cases():
    rng = random.Random(7)
    cases = {
        "empty": b"",
        "only_newlines": b"\n\n\n",
        "basic": b"b.com\na.com\nb.com\n\nc.com\na.com\n",
        "unterminated": b"z\ny\nz",
        "prefixes": b"ab\nab\x00\nabc\na\nab\nabcdefg\nabcdefgh\nabcdefg\x00\nabcdefghijklmn\n"
                    b"abcdefghijklmno\nabcdefghijklm\n\x00\n\x00\x00\n",
        "cr_kept": b"a.com\r\na.com\nb.com\r\n\r\n",
        "high_bytes": bytes([0xff, 0x0a, 0x80, 0x0a, 0x7f, 0x0a, 0xc3, 0xbc, 0x0a, 0x41, 0x0a]),
        "long_common_prefix": b"".join(b"https://www.example.com/path/segment/%d\n" % i
                                       for i in (5, 3, 30, 3, 100, 1, 10, 5)),
        "exact_7_8_14": b"1234567\n12345678\n12345678901234\n1234567\n1234567890123\n123456789012345\n",
        "subdomains_2k": subdomains(rng, 2000, 900),
        "identical_long": b"x" * 40 + b"\n" + (b"x" * 40 + b"\n") * 70 + b"x" * 39 + b"\n",
    }
    out = []
    for name, data in cases.items():
        out.append({"name": name, "input": b64(data), "sort_u": b64(sort_u(data))})
    return out


def diff_cases():
    rng = random.Random(11)
    cur = subdomains(rng, 3000, 1500)
    recs = sorted(set(cur.split(b"\n")) - {b""})
    prior_recs = [r for r in recs if rng.random() < 0.9] + [b"gone.target1.com", b"zzz.old.net"]
    prior = b"".join(r + b"\n" for r in sorted(set(prior_recs)))
    cases = [
        ("subdomains", cur, prior),
        ("empty_prior", b"a\nb\na\n", b""),
        ("empty_cur", b"", b"a\nb\n"),
        ("all_known", b"b\na\n", b"a\nb\nc\n"),
        ("prefix_edges", b"ab\nab\x00\nabc\nabcdefgh\nabcdefghi\n", b"ab\x00\nabcdefgh\n"),
        ("cr_distinct", b"a.com\r\na.com\n", b"a.com\n"),
    ]
    out = []
    for name, c, p in cases:
        out.append({"name": name, "cur": b64(c), "prior": b64(p),
                    "comm13": b64(comm13(sort_u(p), sort_u(c)))})
    return out


def grep_lines_to_records(data: bytes):
    """grep -n numbers every line (empty ones too); map to A3 record indices."""
    m = {}
    ri = 0
    parts = data.split(b"\n")
    if data.endswith(b"\n") or not data:
        parts = parts[:-1]
    for ln, line in enumerate(parts, 1):
        if line:
            m[ln] = ri
            ri += 1
    return m


def grep_hits(data: bytes, pats, mode):
    m = grep_lines_to_records(data)
    hits = []
    with tempfile.TemporaryDirectory() as d:
        fn = os.path.join(d, "in")
        open(fn, "wb").write(data)
        for si, p in enumerate(pats):
            r = subprocess.run(["grep", "-n", "-a"] + mode + ["--", p, fn], stdout=subprocess.PIPE,
                               env=ENV)
            for line in r.stdout.split(b"\n"):
                if line:
                    ln = int(line.split(b":", 1)[0])
                    hits.append([m[ln], si])
    return sorted(hits)


def banner_corpus(rng, n):
    servers = [b"Apache/2.4.41 (Ubuntu)", b"nginx/1.18.0", b"Microsoft-IIS/10.0", b"cloudflare",
               b"LiteSpeed", b"openresty/1.19.3.1", b"Jetty(9.4.z)", b"gunicorn/20.0.4"]
    titles = [b"Welcome to nginx!", b"Index of /", b"Grafana", b"Jenkins", b"phpMyAdmin",
              b"WordPress &rsaquo; Setup", b"Apache Tomcat/9.0.31", b"Login", b"IIS Windows Server"]
    lines = []
    for i in range(n):
        k = rng.random()
        if k < 0.3:
            lines.append(b"SSH-2.0-OpenSSH_%d.%dp1 Ubuntu-4ubuntu0.%d" % (rng.randrange(5, 9), rng.randrange(10), rng.randrange(5)))
        elif k < 0.45:
            lines.append(b"220 mail%d.example.org ESMTP Postfix (Ubuntu)" % rng.randrange(100))
        elif k < 0.5:
            lines.append(b"")
        else:
            lines.append(b"https://h%d.target%d.com [%d] [%s] [%s]" % (
                rng.randrange(10000), rng.randrange(64), rng.choice([200, 301, 403, 404, 500]),
                rng.choice(titles), rng.choice(servers)))
    return b"\n".join(lines) + b"\n"


def literal_cases():
    rng = random.Random(3)
    data = banner_corpus(rng, 1500)
    sigs = [b"nginx", b"Apache", b"OpenSSH_7", b"Postfix", b"Tomcat", b"Index of", b"&rsaquo;",
            b"Jenkins", b"IIS", b"ngin", b"x/1.18", b"[200]", b"Ubuntu", b"h99.", b"openresty",
            b"gunicorn/20.0.4", b"ESMTP", b"phpMyAdmin", b"Jetty(", b"notpresent-xyz"]
    out = [{"name": "banners", "input": b64(data), "sigs": [b64(s) for s in sigs], "nocase": False,
            "hits": grep_hits(data, sigs, ["-F"])}]
    sigs_i = [b"NGINX", b"apache", b"welcome TO", b"ssh-2.0", b"grafana", b"LOGIN"]
    out.append({"name": "banners_nocase", "input": b64(data), "sigs": [b64(s) for s in sigs_i],
                "nocase": True, "hits": grep_hits(data, sigs_i, ["-F", "-i"])})
    tricky = b"aaaa\nabab\nbaba\n\nxyzxyz\nhello world\nHELLO\n\x00\x01\x02\n\xff\xfe\n"
    sigs_t = [b"aa", b"aaa", b"aba", b"bab", b"zx", b"lo w", b"hello", b"\x01\x02", b"\xfe", b"a"]
    out.append({"name": "overlaps", "input": b64(tricky), "sigs": [b64(s) for s in sigs_t],
                "nocase": False, "hits": grep_hits(tricky, sigs_t, ["-F"])})
    return out


def regex_cases():
    rng = random.Random(5)
    data = banner_corpus(rng, 1500)
    pats = [rb"^SSH-2\.0-OpenSSH_([\w.]+)", rb"OpenSSH_[78]\.\dp1", rb"^220 [\w.-]+ ESMTP",
            rb"\[(200|301)\]", rb"nginx/1\.1[0-9]\.\d+", rb"Apache/2\.4\.\d+ \(Ubuntu\)$",
            rb"(?i)welcome to nginx", rb"Jetty\(9\.[0-9.z]+\)", rb"h[0-9]{4}\.target6[0-3]",
            rb"Ubuntu-4ubuntu0\.[0-2]$", rb"^https?://", rb"(Grafana|Jenkins|Login)\]",
            rb"[^a-z ]{3,}Admin", rb"IIS.*Server", rb"x{2,3}", rb"\d\d\d\] \[Index", rb"(ab|cd)+ef?",
            rb"\sPostfix\s", rb"gunicorn/20\.0\.[4-9]\]$", rb"Microsoft-IIS/1[0-9]\.0"]
    return [{"name": "banners", "input": b64(data), "regexes": [b64(p) for p in pats],
             "hits": grep_hits(data, pats, ["-P"])}]


def main():
    with open(os.path.join(HERE, "coreutils_vectors.json"), "w") as f:
        json.dump({"note": "LC_ALL=C GNU coreutils 8.32 sort -u / comm -13",
                   "dedup": dedup_cases(), "diff": diff_cases()}, f, indent=1)
    with open(os.path.join(HERE, "grep_vectors.json"), "w") as f:
        json.dump({"note": "LC_ALL=C GNU grep 3.7: -F (literal), -F -i, -P (regex)",
                   "literal": literal_cases(), "regex": regex_cases()}, f, indent=1)
    print("ok")


if __name__ == "__main__":
    main()
