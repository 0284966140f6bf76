"""GPU parity: A3 parse, A5+A7 merge/dedup, A8 diff and the partition through the C-ABI,
bit-exact against the CPU oracle and the GNU-tool golden vectors."""
import random

import numpy as np
import pytest

from conftest import b64d, load_golden
from hash_oracle import hash64 as py_hash64, part_of
from oracle import semantics as S

pytestmark = pytest.mark.gpu

CU = load_golden("coreutils_vectors.json")
REF = load_golden("reference_vectors.json")


@pytest.fixture(scope="module")
def sg():
    import swarm_amd
    assert swarm_amd.device_count() > 0, "GPU tests need a HIP device"
    return swarm_amd


def rand_buf(rng, n_lines, alphabet=b"ab\x00\r\xff.", maxlen=20, p_empty=0.1, tail=True):
    out = []
    for _ in range(n_lines):
        if rng.random() < p_empty:
            out.append(b"")
            continue
        L = rng.randint(1, maxlen)
        out.append(bytes(rng.choice(alphabet) for _ in range(L)))
    b = b"\n".join(out)
    return b + b"\n" if tail else b


# ------------------------------------------------------------------ A3
@pytest.mark.parametrize("size", [0, 1, 7, 8, 8191, 8192, 8193, 16384, 16385, 40000])
@pytest.mark.parametrize("pattern", ["mixed", "nl_only", "no_nl", "tile_edges"])
def test_lines_spans(sg, size, pattern):
    rng = random.Random(size * 7 + len(pattern))
    if pattern == "mixed":
        b = bytes(rng.choice(b"xy\n\r") for _ in range(size))
    elif pattern == "nl_only":
        b = b"\n" * size
    elif pattern == "no_nl":
        b = bytes(rng.choice(b"pq") for _ in range(size))
    else:
        a = bytearray(b"z" * size)
        for p in range(8191, size, 8192):
            a[p] = 0x0A
        b = bytes(a)
    got = [tuple(x) for x in sg.lines(b).tolist()]
    assert got == S.record_spans(b)


# ------------------------------------------------------------------ A7
@pytest.mark.parametrize("case", CU["dedup"], ids=lambda c: c["name"])
def test_dedup_golden(sg, case):
    assert sg.dedup(b64d(case["input"])) == b64d(case["sort_u"])


@pytest.mark.parametrize("seed", range(6))
def test_dedup_random_bytes(sg, seed):
    rng = random.Random(seed)
    b = rand_buf(rng, 3000, maxlen=rng.choice([3, 9, 30]), tail=seed % 2 == 0)
    assert sg.dedup(b) == S.dedup(b)


def test_dedup_long_shared_prefixes(sg):
    """Big groups of equal 7-byte prefixes force the radix refinement rounds."""
    rng = random.Random(5)
    pre = b"https://www.example.com/very/long/shared/prefix/"
    recs = [pre + b"%d/%s" % (rng.randrange(300), rng.choice([b"a", b"b", b"ab", b""]))
            for _ in range(20000)]
    recs += [pre[:k] for k in range(0, len(pre), 3)]
    rng.shuffle(recs)
    b = b"\n".join(recs) + b"\n"
    assert sg.dedup(b) == S.dedup(b)


def test_dedup_identical_long_records(sg):
    b = (b"q" * 100 + b"\n") * 5000 + (b"q" * 99 + b"\n") * 7 + (b"q" * 101 + b"\n") * 3
    assert sg.dedup(b) == S.dedup(b)


def test_dedup_subdomains_200k(sg):
    from swarm_amd import corpus
    buf, _ = corpus.subdomains(200_000, seed=99)
    b = buf.tobytes()
    assert sg.dedup(b) == S.dedup(b)


@pytest.mark.parametrize("case", REF["a5_merge"], ids=lambda c: c["name"])
def test_merge_dedup_reference_chunks(sg, case):
    """A5 -> A7: the reference /raw merge order, then sort -u, from the chunk bodies."""
    from swarm_amd import hooks
    objs = {"%s/output/%s" % (case["scan_id"], k): b64d(v) for k, v in case["objects"].items()}
    merged = S.merge_chunks(objs, case["scan_id"])
    assert merged == b64d(case["raw"])
    bodies = [objs[k] for k in hooks.merge_keys(objs.keys(), case["scan_id"])]
    assert sg.dedup_chunks(bodies) == S.dedup(merged)


# ------------------------------------------------------------------ A8
@pytest.mark.parametrize("case", CU["diff"], ids=lambda c: c["name"])
def test_diff_golden(sg, case):
    assert sg.diff(b64d(case["cur"]), b64d(case["prior"])) == b64d(case["comm13"])


@pytest.mark.parametrize("seed", range(4))
def test_dedup_diff_random(sg, seed):
    rng = random.Random(100 + seed)
    cur = rand_buf(rng, 4000, alphabet=b"abc\x00", maxlen=12)
    prior_recs = sorted(set(S.parse_records(rand_buf(rng, 3000, alphabet=b"abc\x00", maxlen=12))))
    prior = b"".join(r + b"\n" for r in prior_recs)
    u, f = sg.dedup_diff(cur, prior)
    eu, ef = S.dedup_diff(cur, prior)
    assert u == eu and f == ef


def test_diff_unsorted_prior(sg):
    rng = random.Random(3)
    cur = rand_buf(rng, 3000, alphabet=b"xyz", maxlen=9)
    prior = rand_buf(rng, 3000, alphabet=b"xyz", maxlen=9)  # unsorted, duplicated
    assert sg.diff(cur, prior) == S.diff(cur, prior)


def test_dedup_diff_c1(sg):
    """C1: 1M subdomains in 16 worker chunks merged in S3 key order, deduped, diffed."""
    from swarm_amd import corpus, hooks
    buf, ids = corpus.subdomains(1_000_000, seed=1234)
    chunks = corpus.chunk_layout(buf, 16)
    objs = {"c1_1/output/chunk_%d.txt" % i: ch.tobytes() for i, ch in enumerate(chunks)}
    merged = S.merge_chunks(objs, "c1_1")
    prior = corpus.prior_of(ids).tobytes()
    u, f = hooks.completion_dedup_diff(objs, "c1_1", prior)
    eu, ef = S.dedup_diff(merged, prior)
    assert u == eu and f == ef


# ------------------------------------------------------------------ device path + C2
def test_device_path_torch_tensors(sg):
    import torch
    from swarm_amd import corpus
    buf, ids = corpus.subdomains(300_000, seed=7)
    prior = corpus.prior_of(ids)
    d_cur = torch.from_numpy(buf).cuda()
    d_pri = torch.from_numpy(prior).cuda()
    ctx = sg.Context(0, torch.cuda.current_stream().cuda_stream)
    r = ctx.dedup_diff(d_cur.data_ptr(), d_cur.numel(), d_pri.data_ptr(), d_pri.numel())
    u = ctx.to_bytes(r.uniq, r.uniq_bytes)
    f = ctx.to_bytes(r.fresh, r.fresh_bytes)
    eu, ef = S.dedup_diff(buf.tobytes(), prior.tobytes())
    assert u == eu and f == ef
    assert r.uniq_records == eu.count(b"\n") and r.fresh_records == ef.count(b"\n")
    # misaligned device pointer (offset 3) still works
    d_pad = torch.zeros(buf.size + 3, dtype=torch.uint8, device="cuda")
    d_pad[3:] = d_cur
    r2 = ctx.dedup_diff(d_pad.data_ptr() + 3, buf.size, d_pri.data_ptr(), d_pri.numel())
    assert ctx.to_bytes(r2.fresh, r2.fresh_bytes) == ef
    ctx.close()


def test_c2_full_size_bit_exact(sg):
    """C2 (10M lines) at the BASELINE size, bit-exact: sort -u and the diff equal an
    independent numpy reference (fixed-width row sort of the rendered names; np.isin for
    the set difference)."""
    import torch
    from swarm_amd import corpus
    buf, ids = corpus.subdomains(10_000_000, seed=1234)
    prior = corpus.prior_of(ids)
    d_cur = torch.from_numpy(buf).cuda()
    d_pri = torch.from_numpy(prior).cuda()
    ctx = sg.Context(0, torch.cuda.current_stream().cuda_stream)
    r = ctx.dedup_diff(d_cur.data_ptr(), d_cur.numel(), d_pri.data_ptr(), d_pri.numel())
    u = ctx.to_bytes(r.uniq, r.uniq_bytes)
    f = ctx.to_bytes(r.fresh, r.fresh_bytes)
    urows = corpus.sorted_unique_rows(ids)
    prow = corpus.prior_rows(ids)
    frows = urows[~np.isin(urows, prow)]
    assert r.in_records == 10_000_000
    assert r.uniq_records == urows.size and r.fresh_records == frows.size
    assert u == corpus.serialize_rows(urows).tobytes()
    assert f == corpus.serialize_rows(frows).tobytes()
    ctx.close()


# ------------------------------------------------------------------ partition (§8(e))
@pytest.mark.parametrize("parts,maxlen", [(1, 25), (2, 25), (3, 25), (8, 25), (256, 90), (255, 17)])
def test_partition_matches_hash_oracle(sg, parts, maxlen):
    """Records of every length and start alignment (the device hash joins aligned words)."""
    import torch
    rng = random.Random(parts)
    b = rand_buf(rng, 5000, alphabet=b"abcdef.", maxlen=maxlen, tail=False)
    recs = S.parse_records(b)
    d = torch.frombuffer(bytearray(b), dtype=torch.uint8).cuda()
    ctx = sg.Context(0, torch.cuda.current_stream().cuda_stream)
    dout = torch.empty(d.numel() + 1, dtype=torch.uint8, device="cuda")
    pbytes, precs = ctx.partition(d.data_ptr(), d.numel(), parts, dout.data_ptr(), dout.numel())
    out = ctx.to_bytes(dout.data_ptr(), sum(pbytes))
    exp = [[] for _ in range(parts)]
    for r in recs:
        exp[part_of(py_hash64(r), parts)].append(r)
    assert precs == [len(e) for e in exp]
    assert pbytes == [sum(len(r) + 1 for r in e) for e in exp]
    assert out == b"".join(r + b"\n" for e in exp for r in e)
    ctx.close()


@pytest.mark.parametrize("k", [2, 3, 63, 64, 65, 66, 129, 200])
def test_dedup_segment_sizes(sg, k):
    """Segments of k distinct records sharing their first 7+ bytes: <= 64 are sorted by one
    wave in LDS (run sort), > 64 go through the radix refinement rounds first."""
    rng = random.Random(k)
    recs = [b"shared_" + bytes(rng.choice(b"xyz\x00\xff") for _ in range(rng.randint(0, 6))) for _ in range(k)]
    recs += rng.sample(recs, min(len(recs), 10))  # duplicates inside the segment
    recs += [b"other%d" % i for i in range(50)]
    rng.shuffle(recs)
    b = b"\n".join(recs) + b"\n"
    assert sg.dedup(b) == S.dedup(b)


def test_dedup_long_records_segment_mirror(sg):
    """A segment whose bytes exceed the per-wave LDS window (global mirror path)."""
    rng = random.Random(77)
    recs = [b"samepre" + bytes(rng.choice(b"ab") for _ in range(rng.randint(200, 700))) for _ in range(40)]
    recs += recs[:5]
    rng.shuffle(recs)
    b = b"\n".join(recs) + b"\n"
    assert sg.dedup(b) == S.dedup(b)


def test_dedup_unsorted_prior_long(sg):
    """An unsorted prior goes through the full sort/unique pipeline before the diff."""
    rng = random.Random(8)
    pool = [b"host%05d.example.com" % i for i in range(3000)]
    cur = b"\n".join(rng.choice(pool) for _ in range(5000)) + b"\n"
    prior = b"\n".join(rng.choice(pool) for _ in range(4000)) + b"\n"
    u, f = sg.dedup_diff(cur, prior)
    eu, ef = S.dedup_diff(cur, prior)
    assert u == eu and f == ef


@pytest.mark.parametrize("maxlen", [1, 15, 16, 31, 32, 33, 63, 64, 65, 200])
def test_dedup_slot_width_boundaries(sg, maxlen):
    """Longest record just below / at / above the fixed-slot widths (32, 64 bytes) and the
    packed fallback; records start at every source alignment."""
    rng = random.Random(maxlen)
    recs = [bytes(rng.choice(b"ab\x00\xff") for _ in range(rng.randint(1, maxlen))) for _ in range(3000)]
    recs.append(b"z" * maxlen)
    recs += rng.sample(recs, 500)
    rng.shuffle(recs)
    b = b"\n".join(recs) + b"\n"
    assert sg.dedup(b) == S.dedup(b)
    prior = b"".join(r + b"\n" for r in sorted(set(recs[:1500])))
    u, f = sg.dedup_diff(b, prior)
    eu, ef = S.dedup_diff(b, prior)
    assert u == eu and f == ef


# ------------------------------------------------------------------ prior sortedness check
def _swapped_prior(recs, i):
    r = list(recs)
    r[i], r[i + 1] = r[i + 1], r[i]
    return b"".join(x + b"\n" for x in r)


@pytest.mark.parametrize("off", list(range(8, 61)) + [70, 100])
def test_prior_one_swapped_pair_past_key0(sg, off):
    """A prior sorted except for one adjacent pair that shares key0 (the first 7 bytes) and
    differs at byte `off` must be detected as unsorted (rec_cmp_w fast path)."""
    base = b"abcdefg" + bytes(range(0x41, 0x41 + max(0, off - 7)))[: max(0, off - 7)]
    a, b = base[:off] + b"A" + b"tail", base[:off] + b"B" + b"tail"
    others = [b"aaa", b"abcdefa", b"zzz-%d" % off, b"zzzz"]
    recs = sorted(set(others + [a, b]))
    i = recs.index(a)
    prior = _swapped_prior(recs, i)
    cur = b"".join(x + b"\n" for x in [a, b, b"new-1", b"zzz-%d" % off])
    assert sg.dedup_diff(cur, prior) == S.dedup_diff(cur, prior)
    assert sg.diff(cur, prior) == S.dedup_diff(cur, prior)[1]


@pytest.mark.parametrize("pair", [(b"abcdefghX", b"abcdefgh"), (b"abcdefgh" * 7 + b"Z", b"abcdefgh" * 7),
                                  (b"0123456789abcdef", b"0123456789abcde"), (b"k" * 49, b"k" * 48)])
@pytest.mark.parametrize("align", range(16))
def test_prior_length_only_pair_every_alignment(sg, pair, align):
    """Descending pair differing only in length (a record and its prefix), at every 16-B
    alignment of the prior's records."""
    pad = b"p" * align
    head = [b"!" + pad] if align else []
    recs = head + [pair[1], pair[0]]  # ascending
    prior_sorted = b"".join(x + b"\n" for x in recs)
    prior_bad = b"".join(x + b"\n" for x in head + [pair[0], pair[1]])
    cur = pair[0] + b"\n" + pair[1] + b"\nother\n"
    for prior in (prior_sorted, prior_bad):
        assert sg.dedup_diff(cur, prior) == S.dedup_diff(cur, prior)


# ------------------------------------------------------------------ common-prefix keying
def _url_recs(rng, n, hosts=300, scheme=b"https://"):
    hs = [b"www.h%d.example.com" % rng.randrange(hosts) for _ in range(hosts)]
    return [scheme + rng.choice(hs) + b"/" + b"p" * rng.randrange(0, 30) for _ in range(n)]


@pytest.mark.parametrize("seed", range(3))
def test_dedup_diff_url_common_prefix(sg, seed):
    """Every record starts with 'https://www.h' (13 shared bytes): the radix pipeline keys
    from the common prefix; results stay those of sorted(set())."""
    rng = random.Random(seed)
    cur = b"\n".join(_url_recs(rng, 20_000)) + b"\n"
    prior = b"".join(r + b"\n" for r in sorted(set(_url_recs(rng, 8_000))))
    assert sg.dedup_diff(cur, prior) == S.dedup_diff(cur, prior)


@pytest.mark.parametrize("case", ["prefix_is_record", "all_identical", "prior_breaks_prefix", "long_prefix"])
def test_common_prefix_edges(sg, case):
    rng = random.Random(11)
    if case == "prefix_is_record":
        recs = [b"https://"] + [b"https://" + bytes([rng.randrange(97, 123)]) * rng.randrange(1, 9) for _ in range(3000)]
        prior = b"https://\nhttps://a\n"
    elif case == "all_identical":
        recs = [b"x" * 300] * 500
        prior = b"x" * 299 + b"\n"
    elif case == "prior_breaks_prefix":
        recs = _url_recs(rng, 3000)
        prior = b"".join(r + b"\n" for r in sorted(set(_url_recs(rng, 500) + [b"http://a", b"zzz"])))
    else:
        pre = b"P" * 250
        recs = [pre + bytes(rng.choice(b"ab\x00\xff") for _ in range(rng.randrange(0, 20))) for _ in range(4000)]
        prior = b"".join(r + b"\n" for r in sorted(set(recs[::3])))
    cur = b"\n".join(recs) + b"\n"
    assert sg.dedup_diff(cur, prior) == S.dedup_diff(cur, prior)
    assert sg.dedup(cur) == S.dedup(cur)


@pytest.mark.parametrize("prior_ok", [True, False], ids=["sorted_prior", "swapped_prior"])
@pytest.mark.parametrize("second", ["same_prefix", "longer_prefix", "shorter_prefix", "no_prefix"])
def test_prior_check_on_speculative_keys(prior_ok, second):
    """The prior's sortedness is checked on its keys at the last call's common prefix (URL
    lists: keys from byte 0 all tie); when the prefix comes out elsewhere the check runs again
    on keys from byte 0. One swapped pair past the prefix is caught either way, and a sorted
    prior is trusted either way (both give the oracle's output)."""
    import numpy as np
    import torch
    rng = random.Random(7)
    c = _kw_ctx()

    def run(recs, prior_recs, swap):
        pr = sorted(set(prior_recs))
        if swap:
            i = len(pr) // 2
            pr[i], pr[i + 1] = pr[i + 1], pr[i]
        cur, prior = b"\n".join(recs) + b"\n", b"".join(r + b"\n" for r in pr)
        dc = torch.from_numpy(np.frombuffer(cur, dtype=np.uint8).copy()).cuda()
        dp = torch.from_numpy(np.frombuffer(prior, dtype=np.uint8).copy()).cuda()
        r = c.dedup_diff(dc.data_ptr(), len(cur), dp.data_ptr(), len(prior))
        eu, ef = S.dedup_diff(cur, prior)
        assert c.to_bytes(r.uniq, r.uniq_bytes) == eu and c.to_bytes(r.fresh, r.fresh_bytes) == ef

    try:
        first = _url_recs(rng, 6000)  # common prefix 'https://www.h' (13 bytes): kept by the context
        run(first, first[::3], False)
        if second == "same_prefix":
            recs = _url_recs(rng, 6000)
        elif second == "longer_prefix":
            recs = [b"https://www.h7" + r[14:] for r in _url_recs(rng, 6000)]
        elif second == "shorter_prefix":
            recs = [r if i % 2 else b"https://a" + r[13:] for i, r in enumerate(_url_recs(rng, 6000))]
        else:
            recs = [bytes(rng.choice(b"abcdefgh/.:") for _ in range(rng.randint(1, 30))) for _ in range(6000)]
        run(recs, recs[::2] + [recs[0] + b"-old"], not prior_ok)
    finally:
        c.close()


def _kw_ctx():
    import torch
    import swarm_amd
    return swarm_amd.Context(0, torch.cuda.current_stream().cuda_stream)


@pytest.mark.parametrize("seed", [1, 2])
def test_narrowed_key_widths_with_tie_segments(seed):
    """High-entropy records (narrowed 6/5-byte sort keys) where many distinct records share
    exactly 5, 6 or 7 bytes, records shorter than the key, duplicates, NUL/0xff bytes; the
    width chosen is reported and the result equals the oracle and the 7-byte-key run."""
    import os
    import random
    import numpy as np
    import torch
    rng = random.Random(seed)
    alpha = bytes(range(33, 127)) + b"\x00\xff"
    heads = [bytes(rng.choice(alpha) for _ in range(rng.choice([5, 6, 7]))) for _ in range(60_000)]
    recs = []
    for _ in range(200_000):
        h = rng.choice(heads)
        k = rng.random()
        recs.append(h[: rng.randint(1, len(h))] if k < 0.05 else h + bytes(rng.choice(alpha) for _ in range(rng.randint(0, 9))))
    recs += recs[: 30_000]  # duplicates
    rng.shuffle(recs)
    cur = b"\n".join(recs) + b"\n"
    prior = S.dedup(b"\n".join(recs[::3]) + b"\n")
    c = _kw_ctx()
    try:
        dc = torch.from_numpy(np.frombuffer(cur, dtype=np.uint8).copy()).cuda()
        dp = torch.from_numpy(np.frombuffer(prior, dtype=np.uint8).copy()).cuda()
        r = c.dedup_diff(dc.data_ptr(), len(cur), dp.data_ptr(), len(prior))
        kw = c.last_key_width()
        eu, ef = S.dedup_diff(cur, prior)
        assert c.to_bytes(r.uniq, r.uniq_bytes) == eu and c.to_bytes(r.fresh, r.fresh_bytes) == ef
        assert kw in (5, 6)
    finally:
        c.close()


def test_low_entropy_keeps_seven_byte_key():
    import numpy as np
    import torch
    recs = [b"10.%d.%d.%d:%d" % (a, b, d, p) for a in range(4) for b in range(40) for d in range(40) for p in (22, 80, 443)]
    cur = b"\n".join(recs) + b"\n"
    c = _kw_ctx()
    try:
        dc = torch.from_numpy(np.frombuffer(cur, dtype=np.uint8).copy()).cuda()
        r = c.dedup_diff(dc.data_ptr(), len(cur), 0, 0)
        assert c.to_bytes(r.uniq, r.uniq_bytes) == S.dedup(cur)
        assert c.last_key_width() == 7
    finally:
        c.close()


@pytest.mark.parametrize("alpha", ["ip", "wide", "nul_bytes"])
def test_refinement_packed_chunk_keys(sg, alpha):
    """Big groups whose next chunks use a small alphabet (IP digits: 4-bit packed keys), a
    wide one (no packing) or NUL bytes inside records (rank 0 shared with the filler past a
    record's end, told apart by the tag): dedup and diff equal the oracle's."""
    rng = random.Random(71)
    if alpha == "ip":
        recs = [b"10.%d.%d.%d:%d" % (rng.randrange(3), rng.randrange(256), rng.randrange(256),
                                     rng.choice([22, 80, 443, 8080, 3389])) for _ in range(60000)]
    elif alpha == "wide":
        recs = [b"shared-prefix/" + bytes(rng.choice(range(1, 256)) for _ in range(rng.randint(0, 12))).replace(b"\n", b"")
                for _ in range(30000)]
    else:
        recs = [b"grp" + bytes(rng.choice(b"\x00a1") for _ in range(rng.randint(0, 14))) for _ in range(30000)]
    prior_recs = sorted(set(rng.sample(recs, len(recs) // 3)))
    cur = b"\n".join(recs) + b"\n"
    prior = b"".join(r + b"\n" for r in prior_recs)
    assert sg.dedup(cur) == S.dedup(cur)
    assert sg.dedup_diff(cur, prior) == S.dedup_diff(cur, prior)


# ------------------------------------------------------------------ hybrid radix sort
def test_hybrid_sort_subdomains(sg):
    """1.5M C2-shaped records: the sort runs its top key digits globally and finishes every
    group in LDS (flags bit 0); output equals the independent numpy reference."""
    import torch
    from swarm_amd import corpus
    buf, ids = corpus.subdomains(1_500_000, seed=77)
    prior = corpus.prior_of(ids)
    d_cur = torch.from_numpy(buf).cuda()
    d_pri = torch.from_numpy(prior).cuda()
    ctx = sg.Context(0, torch.cuda.current_stream().cuda_stream)
    try:
        r = ctx.dedup_diff(d_cur.data_ptr(), d_cur.numel(), d_pri.data_ptr(), d_pri.numel())
        assert ctx.last_path()[1] & 3 == 1
        urows = corpus.sorted_unique_rows(ids)
        frows = urows[~np.isin(urows, corpus.prior_rows(ids))]
        assert ctx.to_bytes(r.uniq, r.uniq_bytes) == corpus.serialize_rows(urows).tobytes()
        assert ctx.to_bytes(r.fresh, r.fresh_bytes) == corpus.serialize_rows(frows).tobytes()
    finally:
        ctx.close()


@pytest.mark.parametrize("shape", ["overflow", "ties"])
def test_hybrid_sort_overflow_and_ties(sg, shape):
    """overflow: half the records share their first 3 bytes, so the groups the global digits
    leave are far larger than one block's LDS: the local sort flags them and the fix-up sorts
    those groups' members by one radix sort (flags bits 0 and 2, no full re-sort: bit 1). ties: distinct records sharing all sorted key bytes,
    short records (live length tag), duplicates: the local sort keeps them in input order
    like the full sort. Both equal the oracle."""
    import torch
    rng = np.random.default_rng(5 if shape == "overflow" else 6)
    alpha = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789", dtype=np.uint8)
    n = 1_200_000
    if shape == "overflow":
        body = alpha[rng.integers(0, 36, size=(n, 11))]
        body[: n // 2, :3] = ord("a")
        recs = [bytes(r) for r in body]
    else:
        heads = alpha[rng.integers(0, 36, size=(n // 3, 8))]
        recs = []
        for i in range(n):
            h = bytes(heads[rng.integers(0, n // 3)])
            k = int(rng.integers(0, 10))
            recs.append(h[: 3 + k % 5] if k < 2 else h + bytes(alpha[rng.integers(0, 36, size=k % 4)]))
    rng.shuffle(recs)
    cur = b"\n".join(recs) + b"\n"
    prior = S.dedup(b"\n".join(recs[::4]) + b"\n")
    dc = torch.from_numpy(np.frombuffer(cur, dtype=np.uint8).copy()).cuda()
    dp = torch.from_numpy(np.frombuffer(prior, dtype=np.uint8).copy()).cuda()
    ctx = sg.Context(0, torch.cuda.current_stream().cuda_stream)
    try:
        r = ctx.dedup_diff(dc.data_ptr(), len(cur), dp.data_ptr(), len(prior))
        flags = ctx.last_path()[1]
        eu, ef = S.dedup_diff(cur, prior)
        assert ctx.to_bytes(r.uniq, r.uniq_bytes) == eu
        assert ctx.to_bytes(r.fresh, r.fresh_bytes) == ef
        if shape == "overflow":
            assert flags & 5 == 5 and not flags & 2  # fixed up, no full re-sort
        else:
            assert flags & 1
    finally:
        ctx.close()


def test_hybrid_sort_repeated_record(sg):
    """one record repeated ~10k times among ~1.2M distinct ones (40 of them sharing
    its first 3 bytes) forms a group of equal top digits larger than one block's LDS: the
    fix-up sorts only that group's members (flags bit 2), never the whole input again (bit 1
    clear); output exact."""
    import torch
    rng = np.random.default_rng(8)
    alpha = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789", dtype=np.uint8)
    n = 1_200_000
    body = alpha[rng.integers(0, 36, size=(n, 12))]
    recs = [bytes(r) for r in body] + [b"rep" + bytes(r[3:]) for r in body[:40]]
    recs += [b"repeated.target7.com"] * 10_000
    rng.shuffle(recs)
    cur = b"\n".join(recs) + b"\n"
    prior = S.dedup(b"\n".join(recs[::4]) + b"\n")
    dc = torch.from_numpy(np.frombuffer(cur, dtype=np.uint8).copy()).cuda()
    dp = torch.from_numpy(np.frombuffer(prior, dtype=np.uint8).copy()).cuda()
    ctx = sg.Context(0, torch.cuda.current_stream().cuda_stream)
    try:
        r = ctx.dedup_diff(dc.data_ptr(), len(cur), dp.data_ptr(), len(prior))
        flags = ctx.last_path()[1]
        eu, ef = S.dedup_diff(cur, prior)
        assert ctx.to_bytes(r.uniq, r.uniq_bytes) == eu
        assert ctx.to_bytes(r.fresh, r.fresh_bytes) == ef
        assert flags & 5 == 5 and not flags & 2
    finally:
        ctx.close()


@pytest.mark.parametrize("shape", ["rare", "tags", "prefix_rare"])
def test_key_stats_rare_digits(sg, shape):
    """The sort skips a digit pass only on the keys' exact varying bits (OR ^ AND gathered
    with the common-prefix scan, or with the re-key at the prefix), never on the sampled
    histograms: a digit that one record in 300K carries must still be sorted. rare: key
    bytes 1-3 constant but for single records; tags: lengths 1-12 (the length tag varies,
    also after narrowing); prefix_rare: every record starts "https://" (re-keyed at the
    prefix) with the rare bytes after it. Equal to the oracle."""
    import torch
    rng = np.random.default_rng({"rare": 11, "tags": 12, "prefix_rare": 13}[shape])
    alpha = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789", dtype=np.uint8)
    n = 300_000
    if shape == "tags":
        lens = rng.integers(1, 13, size=n)
        body = alpha[rng.integers(0, 36, size=(n, 12))]
        recs = [bytes(body[i, : lens[i]]) for i in range(n)]
    else:
        body = alpha[rng.integers(0, 36, size=(n, 14))]
        body[:, 1:4] = ord("q")
        for j, i in enumerate(rng.choice(n, size=6, replace=False)):
            body[i, 1 + j % 3] = ord("a") + j  # a rare digit at bytes 1..3
        body[rng.integers(0, n), 0] = ord("~")  # byte 0 varies: no common prefix there
        recs = [bytes(r) for r in body]
        if shape == "prefix_rare":
            recs = [b"https://" + r for r in recs]
    recs += recs[: n // 5]  # duplicates
    rng.shuffle(recs)
    cur = b"\n".join(recs) + b"\n"
    prior = S.dedup(b"\n".join(recs[::3]) + b"\n")
    dc = torch.from_numpy(np.frombuffer(cur, dtype=np.uint8).copy()).cuda()
    dp = torch.from_numpy(np.frombuffer(prior, dtype=np.uint8).copy()).cuda()
    ctx = sg.Context(0, torch.cuda.current_stream().cuda_stream)
    try:
        r = ctx.dedup_diff(dc.data_ptr(), len(cur), dp.data_ptr(), len(prior))
        eu, ef = S.dedup_diff(cur, prior)
        assert ctx.to_bytes(r.uniq, r.uniq_bytes) == eu
        assert ctx.to_bytes(r.fresh, r.fresh_bytes) == ef
    finally:
        ctx.close()


# ------------------------------------------------------------------ record shapes x segment modes
@pytest.mark.parametrize("shape", ["mixed_long", "slot_edges", "url_prefix", "nul_cr"])
@pytest.mark.parametrize("segall", ["0", "1", "2"])
def test_dedup_shapes_seg_modes(sg, monkeypatch, shape, segall):
    """Record shapes against the oracle in every segment mode: mixed_long: short records
    beside long ones, many sharing their first 7+ bytes (segment sorts, byte compares past the
    chunk keys); slot_edges: lengths 29..34 past a shared 28-byte head; url_prefix: a common
    'https://' prefix (keys taken past it); nul_cr: NUL, CR and 0xff bytes (a NUL byte must not
    tie with the record end). segall=2: the all-segments mode (no byte compares in the
    adjacent pass, every segment of 2+ records ranked by the segment sorts); 0: compare mode;
    1: chosen by the context's last unique fraction."""
    import torch
    monkeypatch.setenv("SG_SEG_ALL", segall)
    rng = np.random.default_rng({"mixed_long": 21, "slot_edges": 22, "url_prefix": 23, "nul_cr": 24}[shape])
    n = 200_000
    if shape == "mixed_long":
        heads = [bytes(rng.choice(list(b"abc"), size=int(rng.integers(1, 12)))) for _ in range(3000)]
        recs = []
        for _ in range(n):
            h = heads[int(rng.integers(0, len(heads)))]
            tail = b"x" * int(rng.integers(25, 45)) + bytes(rng.choice(list(b"pq"), size=3)) if rng.random() < 0.25 else b""
            recs.append(h + tail)
    elif shape == "slot_edges":
        base = bytes(rng.choice(list(b"mn"), size=28))
        recs = [base + bytes(rng.choice(list(b"01"), size=int(rng.integers(1, 7)))) for _ in range(n // 4)]
        recs += [bytes(rng.choice(list(b"abc"), size=int(rng.integers(3, 10)))) for _ in range(3 * n // 4)]
    elif shape == "url_prefix":
        recs = [b"https://h%d.t%d.example.com" % (int(rng.integers(0, 60_000)), int(rng.integers(0, 9))) for _ in range(n)]
        recs += [b"https://" + b"y" * int(k) for k in rng.integers(20, 50, size=3000)]
    else:
        recs = [bytes(rng.choice([0, 13, 255, 97, 98], size=int(rng.integers(1, 9)))) for _ in range(n)]
        recs += [r + b"\x00" for r in recs[:5000]]
    rng.shuffle(recs)
    cur = b"\n".join(recs) + b"\n"
    prior = S.dedup(b"\n".join(recs[::3]) + b"\n")
    dc = torch.from_numpy(np.frombuffer(cur, dtype=np.uint8).copy()).cuda()
    dp = torch.from_numpy(np.frombuffer(prior, dtype=np.uint8).copy()).cuda()
    ctx = sg.Context(0, torch.cuda.current_stream().cuda_stream)
    try:
        r = ctx.dedup_diff(dc.data_ptr(), len(cur), dp.data_ptr(), len(prior))
        eu, ef = S.dedup_diff(cur, prior)
        assert ctx.to_bytes(r.uniq, r.uniq_bytes) == eu
        assert ctx.to_bytes(r.fresh, r.fresh_bytes) == ef
    finally:
        ctx.close()


def test_diff_prior_shapes(sg):
    """The diff against priors that stress its per-tile prior ranges: a prior far denser than
    cur (tiles whose staged prior range overflows the LDS), runs of prior records sharing key0
    with distinct tails (binary search by full compare), a prior sharing only some keys, and a
    cur whose last records sort above every prior record."""
    import torch
    rng = np.random.default_rng(31)
    alpha = np.frombuffer(b"abcdefgh", dtype=np.uint8)
    body = alpha[rng.integers(0, 8, size=(120_000, 9))]
    recs = [bytes(r) for r in body]
    prior_recs = set(recs[::2])
    prior_recs |= {b"abcdefgh" + bytes(alpha[rng.integers(0, 8, size=6)]) for _ in range(60_000)}
    prior_recs |= {bytes(alpha[rng.integers(0, 8, size=5)]) for _ in range(20_000)}
    cur = b"\n".join(recs + [b"zzzz-last", b"abcdefghabc"]) + b"\n"
    prior = S.serialize(sorted(prior_recs))
    dc = torch.from_numpy(np.frombuffer(cur, dtype=np.uint8).copy()).cuda()
    dp = torch.from_numpy(np.frombuffer(prior, dtype=np.uint8).copy()).cuda()
    ctx = sg.Context(0, torch.cuda.current_stream().cuda_stream)
    try:
        r = ctx.dedup_diff(dc.data_ptr(), len(cur), dp.data_ptr(), len(prior))
        eu, ef = S.dedup_diff(cur, prior)
        assert ctx.to_bytes(r.uniq, r.uniq_bytes) == eu
        assert ctx.to_bytes(r.fresh, r.fresh_bytes) == ef
        assert r.fresh_records == ef.count(b"\n")
    finally:
        ctx.close()


@pytest.mark.parametrize("segall", ["2", "0"])
@pytest.mark.parametrize("names", ["digits", "letters"])
def test_seg_all_mode_hostports(sg, monkeypatch, segall, names):
    """host:port records (a host's ports share key0: segments of near-duplicates, C5's shape)
    with repeats, short records held whole by key0 repeated > 64 times, and a big group
    sharing 7+ bytes (refinement rounds, then the mode's pass over the sub-segments): the
    all-segments mode (2) and the compare mode (0) both equal the oracle. digits: low-entropy
    names keep the 7-byte key (marking pass first, as C5's range parts); letters: a narrowed
    key (the adjacent pass runs before the big-group count comes back)."""
    import torch
    monkeypatch.setenv("SG_SEG_ALL", segall)
    rng = np.random.default_rng(41)
    if names == "digits":
        hosts = [b"h%05d.t%d.example.com" % (int(rng.integers(0, 30_000)), int(rng.integers(0, 5))) for _ in range(8000)]
    else:
        alpha = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz", dtype=np.uint8)
        hosts = [bytes(alpha[rng.integers(0, 26, size=int(rng.integers(6, 14)))]) + b".example.net" for _ in range(8000)]
    ports = [b"22", b"80", b"443", b"8080", b"3389", b"21"]
    recs = [hosts[int(rng.integers(0, len(hosts)))] + b":" + ports[int(rng.integers(0, 6))] for _ in range(150_000)]
    recs += [b"a:1"] * 200 + [b"b"] * 90
    recs += [b"sharedprefix-" + b"%d" % int(k) for k in rng.integers(0, 500, size=3000)]
    rng.shuffle(recs)
    cur = b"\n".join(recs) + b"\n"
    prior = S.dedup(b"\n".join(recs[::5]) + b"\n")
    dc = torch.from_numpy(np.frombuffer(cur, dtype=np.uint8).copy()).cuda()
    dp = torch.from_numpy(np.frombuffer(prior, dtype=np.uint8).copy()).cuda()
    ctx = sg.Context(0, torch.cuda.current_stream().cuda_stream)
    try:
        for _ in range(2):  # the second call sees the first one's unique fraction (auto mode)
            r = ctx.dedup_diff(dc.data_ptr(), len(cur), dp.data_ptr(), len(prior))
            eu, ef = S.dedup_diff(cur, prior)
            assert ctx.to_bytes(r.uniq, r.uniq_bytes) == eu
            assert ctx.to_bytes(r.fresh, r.fresh_bytes) == ef
            assert bool(ctx.last_path()[1] & 8) == (segall == "2")
            assert (ctx.last_key_width() == 7) == (names == "digits")
    finally:
        ctx.close()


@pytest.mark.gpu
def test_prefix_key_speculation_sequence(sg):
    """Keys taken speculatively at the last call's common prefix (>= 8 bytes): a sequence of
    calls on one context whose prefix stays, grows, shrinks and vanishes, each output against
    the oracle (a wrong speculation falls back to re-keying)."""
    import torch
    rng = np.random.default_rng(57)

    def urls(prefix, n, extra=b""):
        return [prefix + bytes(rng.choice(list(b"abcdefgh./"), size=int(rng.integers(1, 20)))) + extra
                for _ in range(n)]

    seq = [
        urls(b"https://", 60_000),                      # base 8 (speculation armed)
        urls(b"https://", 60_000),                      # base 8 again: speculative keys used
        urls(b"https://www.", 60_000),                  # base 12 != 8: re-keyed
        urls(b"https://www.", 50_000) + [b"https://x"],  # prefix drops back to 8
        urls(b"http://", 60_000),                       # base 7: no speculation next
        urls(b"", 60_000),                              # no common prefix
        urls(b"https://", 60_000),
    ]
    ctx = sg.Context(0, torch.cuda.current_stream().cuda_stream)
    try:
        for recs in seq:
            cur = b"\n".join(recs) + b"\n"
            prior = S.dedup(b"\n".join(recs[::4]) + b"\n")
            dc = torch.from_numpy(np.frombuffer(cur, dtype=np.uint8).copy()).cuda()
            dp = torch.from_numpy(np.frombuffer(prior, dtype=np.uint8).copy()).cuda()
            r = ctx.dedup_diff(dc.data_ptr(), len(cur), dp.data_ptr(), len(prior))
            eu, ef = S.dedup_diff(cur, prior)
            assert ctx.to_bytes(r.uniq, r.uniq_bytes) == eu
            assert ctx.to_bytes(r.fresh, r.fresh_bytes) == ef
    finally:
        ctx.close()


@pytest.mark.parametrize("segall", ["2", "0"])
def test_segment_ranks_every_group_size(sg, monkeypatch, segall):
    """Segments of every size 1..64 (the 16-lane, the paired 32-lane and the whole-wave
    rankers), their members differing in chunk 0, 1, 2, 3 or past the fourth chunk (byte
    compares), some records ending inside a chunk, with duplicates, against the oracle."""
    import torch
    monkeypatch.setenv("SG_SEG_ALL", segall)
    rng = np.random.default_rng(53)
    alpha = np.frombuffer(b"0123456789abcdefghij:.-", dtype=np.uint8)
    recs = []
    for g in range(1, 65):
        for rep in range(3):
            head = b"g%02dr%d-" % (g, rep)  # 7 bytes: the segment's key0
            mid = bytes(alpha[rng.integers(0, len(alpha), size=int(rng.choice([0, 5, 12, 19, 26, 33])))])
            distinct = max(1, g // int(rng.choice([1, 2, 4])))
            tails = [bytes(alpha[rng.integers(0, len(alpha), size=int(rng.integers(0, 9)))]) for _ in range(distinct)]
            members = [head + mid + tails[int(rng.integers(0, distinct))] for _ in range(g)]
            recs += members
    rng.shuffle(recs)
    cur = b"\n".join(recs) + b"\n"
    prior = S.dedup(b"\n".join(recs[::7]) + b"\n")
    dc = torch.from_numpy(np.frombuffer(cur, dtype=np.uint8).copy()).cuda()
    dp = torch.from_numpy(np.frombuffer(prior, dtype=np.uint8).copy()).cuda()
    ctx = sg.Context(0, torch.cuda.current_stream().cuda_stream)
    try:
        for _ in range(2):
            r = ctx.dedup_diff(dc.data_ptr(), len(cur), dp.data_ptr(), len(prior))
            eu, ef = S.dedup_diff(cur, prior)
            assert ctx.to_bytes(r.uniq, r.uniq_bytes) == eu
            assert ctx.to_bytes(r.fresh, r.fresh_bytes) == ef
    finally:
        ctx.close()
