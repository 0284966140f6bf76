"""GPU parity for A4 signature matching: Aho-Corasick literals (== grep -F / `in`) and the
regex DFA set (== Python re.search on bytes), against the grep golden vectors, the nuclei
signature corpus and random fuzz cases."""
import base64
import random
import re

import pytest

from conftest import b64d, load_golden
from oracle import semantics as S

pytestmark = pytest.mark.gpu

GR = load_golden("grep_vectors.json")
SIG = load_golden("signatures.json")
WORDS = [base64.b64decode(w) for w in SIG["words"]]
REGEXES = [base64.b64decode(r["p"]) for r in SIG["regexes"]]


@pytest.fixture(scope="module", params=["auto", "litfilter", "joint"])
def sg(request):
    """Run every literal test with the engine the compiler picks, with the hashed q-gram
    filter forced (SG_FORCE_LITFILTER is read at compile time) in its two-class scheme, and
    forced in its joint scheme (SG_LIT_SCHEME=1; large inputs pick one by timing both)."""
    import os
    import swarm_amd
    assert swarm_amd.device_count() > 0
    if request.param in ("litfilter", "joint"):
        os.environ["SG_FORCE_LITFILTER"] = "1"
        os.environ["SG_LIT_SCHEME"] = "0" if request.param == "litfilter" else "1"
    yield swarm_amd
    os.environ.pop("SG_FORCE_LITFILTER", None)
    os.environ.pop("SG_LIT_SCHEME", None)


@pytest.mark.parametrize("case", GR["literal"], ids=lambda c: c["name"])
def test_literal_golden(sg, case):
    data = b64d(case["input"])
    sigs = [b64d(s) for s in case["sigs"]]
    m = sg.Matcher(sigs, "literal", nocase=case["nocase"])
    assert [list(h) for h in m.match(data)] == case["hits"]
    hits = S.literal_hits(data, sigs, case["nocase"])
    assert m.match_lines(data) == S.matched_lines(data, hits)


@pytest.mark.parametrize("case", GR["regex"], ids=lambda c: c["name"])
def test_regex_golden(sg, case):
    data = b64d(case["input"])
    pats = [b64d(s) for s in case["regexes"]]
    m = sg.Matcher(pats, "regex")
    assert [list(h) for h in m.match(data)] == case["hits"]


def planted_corpus(rng, n, sigs, frac=0.05):
    base = [b"https://h%d.target%d.com [%d] [%s] [%s]" % (
        rng.randrange(99999), rng.randrange(64), rng.choice([200, 301, 403, 404]),
        rng.choice([b"Login", b"Index of /", b"Dashboard", b"Welcome"]),
        rng.choice([b"nginx/1.18.0", b"Apache/2.4.41 (Ubuntu)", b"cloudflare"])) for _ in range(n)]
    for i in range(n):
        if rng.random() < frac:
            s = rng.choice(sigs)
            k = rng.randrange(len(base[i]) + 1)
            base[i] = base[i][:k] + s + base[i][k:]
    return b"\n".join(x.replace(b"\n", b" ") for x in base) + b"\n"


def test_literal_corpus_2k(sg):
    """C3-style: 2,000 corpus words (len >= 4, seed 0) over planted httpx lines."""
    rng = random.Random(0)
    pool = [w for w in WORDS if len(w) >= 4]
    sigs = rng.sample(pool, 2000)
    data = planted_corpus(rng, 1500, sigs)
    m = sg.Matcher(sigs, "literal")
    assert m.match(data) == S.literal_hits(data, sigs)


def test_literal_corpus_all_words_nocase(sg):
    rng = random.Random(1)
    data = planted_corpus(rng, 400, WORDS, 0.2)
    m = sg.Matcher(WORDS, "literal", nocase=True)
    assert m.match(data) == S.literal_hits(data, WORDS, nocase=True)


def test_regex_corpus_subset(sg):
    rng = random.Random(2)
    pats = rng.sample(REGEXES, 60)
    frags = [b"<title>Grafana</title>", b"Server: nginx", b"X-Powered-By: PHP/7.4.3", b"wp-content/plugins/",
             b"ORA-01756", b"jenkins", b"SSH-2.0-OpenSSH_8.2p1", b"Apache Tomcat/9.0", b"phpMyAdmin",
             b"Dell", b" asp.net ", b"APP_KEY=base64", b"DB_HOST=db", b"Location: https://interact.sh"]
    data = planted_corpus(rng, 600, frags, 0.5)
    m = sg.Matcher(pats, "regex")
    assert m.match(data) == S.regex_hits(data, pats)


def rand_regex(rng, depth=0):
    atoms = [b"a", b"b", b"c", b".", b"[ab]", b"[^a]", b"\\d", b"\\w", b"\\s", b"x", b"(?:ab|c)", b"\\b", b"\\B"]
    parts = []
    for _ in range(rng.randint(1, 4)):
        if depth < 2 and rng.random() < 0.2:
            a = b"(" + rand_regex(rng, depth + 1) + b")"
        else:
            a = rng.choice(atoms)
        q = rng.choice([b"", b"", b"", b"*", b"+", b"?", b"{1,2}", b"{2}", b"*?"])
        if a in (b"\\b", b"\\B"):
            q = b""
        parts.append(a + q)
    r = b"".join(parts)
    if depth == 0:
        if rng.random() < 0.2:
            r = b"^" + r
        if rng.random() < 0.2:
            r = r + b"$"
        if rng.random() < 0.15:
            r = r + b"|" + rand_regex(rng, 1)
    return r


@pytest.mark.parametrize("seed", range(8))
def test_regex_fuzz(sg, seed):
    rng = random.Random(1000 + seed)
    pats = []
    while len(pats) < 25:
        p = rand_regex(rng)
        try:
            re.compile(p)
        except re.error:
            continue
        pats.append(p)
    nocase = seed % 2 == 1
    lines = [bytes(rng.choice(b"abcx 1_-A") for _ in range(rng.randint(1, 12))) for _ in range(300)]
    data = b"\n".join(lines) + b"\n"
    m = sg.Matcher(pats, "regex", nocase=nocase)
    assert m.match(data) == S.regex_hits(data, pats, nocase=nocase)


@pytest.mark.parametrize("seed", range(4))
def test_literal_fuzz_overlaps(sg, seed):
    rng = random.Random(2000 + seed)
    sigs = list({bytes(rng.choice(b"abc") for _ in range(rng.randint(1, 5))) for _ in range(40)})
    data = b"\n".join(bytes(rng.choice(b"abcd") for _ in range(rng.randint(1, 30))) for _ in range(500)) + b"\n"
    m = sg.Matcher(sigs, "literal")
    assert m.match(data) == S.literal_hits(data, sigs)


def test_device_match_lines(sg):
    import torch
    rng = random.Random(9)
    sigs = rng.sample([w for w in WORDS if len(w) >= 4], 300)
    data = planted_corpus(rng, 3000, sigs)
    m = sg.Matcher(sigs, "literal")
    d = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    ctx = sg.Context(0, torch.cuda.current_stream().cuda_stream)
    r = m.dev_match(ctx, d.data_ptr(), d.numel())
    hits = S.literal_hits(data, sigs)
    assert r.n_hits == len(hits)
    assert ctx.to_bytes(r.lines, r.lines_bytes) == S.matched_lines(data, hits)
    ctx.close()


@pytest.mark.parametrize("nocase", [False, True])
def test_literal_tile_edges(sg, nocase):
    """Every pattern-length class (1..3 whole, 4..7 and >= 8 anchored), records longer than a
    parse tile (16 KiB) and patterns planted across tile boundaries and at buffer ends."""
    rng = random.Random(77 + nocase)
    alpha = b"abcdefgh/:.-ABCD"
    sigs = list({bytes(rng.choice(alpha) for _ in range(L)) for L in list(range(1, 12)) * 6 + [16, 23, 31, 40] * 4})
    sigs = [s for s in sigs if s]
    parts = []
    for i in range(60):
        L = rng.choice([0, 1, 5, 40, 300, 5000, 20000])
        line = bytearray(rng.choice(b"xyzXYZ0123 ") for _ in range(L))
        for _ in range(rng.randint(0, 6)):
            s = rng.choice(sigs)
            if nocase:
                s = bytes(c ^ 0x20 if 97 <= c <= 122 and rng.random() < 0.5 else c for c in s)
            k = rng.randrange(len(line) + 1)
            line[k:k] = s
        parts.append(bytes(line))
    data = b"\n".join(parts)
    # plant patterns straddling the 16 KiB tile edges
    data = bytearray(data)
    for edge in range(16384, len(data) - 64, 16384):
        s = rng.choice(sigs)
        off = edge - rng.randrange(len(s) + 1)
        data[off:off + len(s)] = s
    data = bytes(data)
    m = sg.Matcher(sigs, "literal", nocase=nocase)
    assert m.match(data) == S.literal_hits(data, sigs, nocase=nocase)
    assert m.match(data + b"\n") == S.literal_hits(data + b"\n", sigs, nocase=nocase)


@pytest.mark.parametrize("nocase", [False, True])
def test_literal_strided_class_alignments(sg, nocase):
    """The 8-gram class is probed at every 4th position only (its patterns file 4 consecutive
    grams): patterns of lengths 10..20, periodic ones among them, planted at every start
    residue, overlapping each other and at record/buffer ends."""
    rng = random.Random(4242 + nocase)
    sigs = [b"abababababab", b"aaaaaaaaaaaaaaa", b"xyzxyzxyzxyz", b"0123456789", b"01234567890",
            b"abcdefghijklmnopqrst", b"Hello-World!", b"aaaaaaaaaab"]
    sigs += [bytes(rng.choice(b"abcdef") for _ in range(L)) for L in range(10, 21)]
    sigs = list(dict.fromkeys(sigs))
    lines = []
    for i in range(400):
        line = bytearray(rng.choice(b"abcdefxyz ") for _ in range(rng.randint(0, 60)))
        for _ in range(rng.randint(0, 3)):
            s = rng.choice(sigs)
            if nocase:
                s = bytes(c ^ 0x20 if 97 <= c <= 122 and rng.random() < 0.5 else c for c in s)
            k = rng.randrange(len(line) + 1)
            line[k:k] = s
        lines.append(bytes(line))
    for pad in range(8):  # every start residue mod 4, twice
        lines.append(b"." * pad + b"abababababababab" + b"aaaaaaaaaaaaaaaaaaab")
    data = b"\n".join(lines)
    m = sg.Matcher(sigs, "literal", nocase=nocase)
    assert m.match(data) == S.literal_hits(data, sigs, nocase=nocase)
    assert m.match(data + b"\n") == S.literal_hits(data + b"\n", sigs, nocase=nocase)


def test_regex_c4_banners_full_signature_set(sg):
    """C4 shape: nmap-style banners against the full ~10k regex set (corpus regexes +
    synthetic nmap `match` families), bit-exact vs re.search on a sample."""
    from swarm_amd import corpus
    pats = REGEXES + corpus.nmap_signatures()
    pool = corpus.banner_pool(pool=400, seed=21)
    data = b"\n".join(pool) + b"\n"
    m = sg.Matcher(pats, "regex")
    got = m.match(data)
    exp = S.regex_hits(data, pats)
    assert got == exp
    assert len(exp) > 50


def test_regex_verify_blocks_over_two_automata(sg):
    """Enough prefilter candidates (> 4096) that the verify sorts them by pattern and its
    256-candidate blocks straddle the boundary between two patterns' runs: such a block
    stages both automata (or the first) in LDS; every hit equals re.search."""
    import random
    from swarm_amd import corpus
    pats = corpus.nmap_signatures(n_products=60)
    rows = corpus.banner_pool(n_products=60, pool=1500, match_frac=0.6, seed=33)
    rng = random.Random(33)
    data = b"".join(rng.choice(rows) + b"\n" for _ in range(9000))
    m = sg.Matcher(pats, "regex")
    got = m.match(data)
    exp = S.regex_hits(data, pats)
    assert got == exp
    assert len(exp) > 4096


@pytest.mark.parametrize("multi", ["1", "0"])
def test_regex_factorless_groups_packed_and_single(sg, multi, monkeypatch):
    """Factor-less patterns whose DFAs split into several groups: walked together by the
    packed multi-group kernel (SG_DFA_MULTI=1, default) or one launch per group (0); both
    bit-exact vs re.search, including start-state accepts (x?) and end-of-record anchors."""
    import random
    monkeypatch.setenv("SG_DFA_MULTI", multi)
    pats = [rb"[a-z]{%d,9}[0-9]{2,%d}[a-z]" % (i % 3 + 1, i % 4 + 2) for i in range(12)]
    pats += [rb"^\w+\s\d+$", rb"x?", rb"(a|b)*c$", rb"[0-9]+\.[0-9]+\.[0-9]+"]
    pats += [rb"[ab][^\n]{%d}[cd]" % k for k in range(6, 12)]
    m = sg.Matcher(pats, "regex")
    assert m.info()["automata"] >= 4
    rng = random.Random(5)
    alpha = b"abcdxyz0123456789. "
    lines = [bytes(rng.choice(alpha) for _ in range(rng.randrange(0, 90))) for _ in range(3000)]
    lines += [b"", b"abc", b"word 123", b"aaaaaaaaaaaac", b"1.2.3", b"b0123456789d"]
    data = b"\n".join(lines) + b"\n"
    got = m.match(data)
    assert got == S.regex_hits(data, pats)
    assert len(got) > 3000


def test_repeated_calls_keep_workspace_bounded():
    """Hundreds of matches on one context reuse the hit workspace instead of growing it
    (a capacity fed back from the slot size used to compound by the slot headroom)."""
    import torch
    import numpy as np
    import swarm_amd
    data = b"".join(b"host%d nginx login\n" % i for i in range(2000))
    d = torch.from_numpy(np.frombuffer(data, dtype=np.uint8).copy()).cuda()
    ctx = swarm_amd.Context(0, torch.cuda.current_stream().cuda_stream)
    lit = swarm_amd.Matcher([b"nginx", b"login"], "literal")
    rx = swarm_amd.Matcher([rb"host[0-9]+ ", rb"login$"], "regex")
    for _ in range(400):
        r1 = lit.dev_match(ctx, d.data_ptr(), d.numel())
        r2 = rx.dev_match(ctx, d.data_ptr(), d.numel())
    assert r1.n_hits == 4000 and r2.n_hits == 4000
    ctx.close()


OVERSIZE = rb"<[^>]{1,512}\bwire:"  # the corpus regex whose search DFA exceeds 65,535 states


def test_regex_oversize_corpus_pattern(sg):
    """Verified by its anchored DFA from every start offset: '<' at distances around the
    {1,512} bounds, '>' in between, several '<', word/non-word bytes before 'wire:'."""
    rng = random.Random(4)
    lines = []
    for d in list(range(0, 8)) + list(range(505, 520)) + [rng.randrange(1, 700) for _ in range(200)]:
        for pre in (b" ", b"x", b"<", b"_", b"-", b">"):
            body = bytes(rng.choice(b"abc <_/=\"") for _ in range(max(d - 1, 0)))
            lines.append(b"<" + body[: max(d - 1, 0)] + (pre if d > 0 else b"") + b"wire:x")
            lines.append(b"<" * rng.randint(1, 3) + body + b">" + pre + b"wire:")
    lines += [b"wire:", b"<wire:", b"< wire:", b"<a wire:", b"<awire:", b"<a>b wire:", b"<" + b"a" * 511 + b" wire:",
              b"<" + b"a" * 512 + b" wire:", b"<" + b"a" * 600 + b"<" + b"b wire:"]
    data = b"\n".join(lines) + b"\n"
    pats = [OVERSIZE, rb"wire:", rb"<[a-z]+>"]
    m = sg.Matcher(pats, "regex")
    assert m.match(data) == S.regex_hits(data, pats)


@pytest.mark.parametrize("seed", range(4))
def test_regex_fuzz_anchored_verify(sg, seed):
    """Every prefiltered pattern verified by its anchored DFA (SG_REGEX_ANCHORED, read at
    compile time): random patterns around a literal factor, with ^ $ \\b \\B and classes."""
    import os
    rng = random.Random(2000 + seed)
    pats = []
    while len(pats) < 25:
        p = rand_regex(rng, 1) + rng.choice([b"abc", b"cab", b"xax"]) + rand_regex(rng, 1)
        if rng.random() < 0.2:
            p = b"^" + p
        if rng.random() < 0.2:
            p = p + b"$"
        try:
            re.compile(p)
        except re.error:
            continue
        pats.append(p)
    lines = [bytes(rng.choice(b"abcx 1_-A") for _ in range(rng.randint(1, 16))) for _ in range(400)]
    lines += [b"abc", b"cab", b"xax", b" abc ", b"aabcc", b"xaxabcab"]
    data = b"\n".join(lines) + b"\n"
    os.environ["SG_REGEX_ANCHORED"] = "1"
    try:
        m = sg.Matcher(pats, "regex", nocase=seed % 2 == 1)
    finally:
        os.environ.pop("SG_REGEX_ANCHORED", None)
    assert m.match(data) == S.regex_hits(data, pats, nocase=seed % 2 == 1)


@pytest.mark.parametrize("dense", [False, True])
def test_hit_sort_buckets_vs_radix(dense, monkeypatch):
    """Hits sorted by record buckets in LDS equal the radix sort's (SG_HIT_RADIX=1) and the
    oracle's; the dense case (thousands of hits per record: every occurrence is a hit
    before de-duplication) overflows the buckets and falls back to the radix sort."""
    import swarm_amd
    rng = random.Random(77 + dense)
    if dense:
        sigs = [b"a", b"b", b"ab", b"ba", b"aba", b"bab", b"abab"]
        data = b"\n".join(bytes(rng.choice(b"ab") for _ in range(rng.randint(1, 3000))) for _ in range(300)) + b"\n"
    else:
        sigs = rng.sample([w for w in WORDS if len(w) >= 4], 300)
        data = planted_corpus(rng, 40000, sigs, frac=0.3)
    m = swarm_amd.Matcher(sigs, "literal")
    a = m.match(data)
    la = m.match_lines(data)
    monkeypatch.setenv("SG_HIT_RADIX", "1")
    b = m.match(data)
    hits = S.literal_hits(data, sigs)
    assert a == b == hits
    assert la == m.match_lines(data) == S.matched_lines(data, hits)
    m.close()
