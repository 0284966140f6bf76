"""GPU parity of the metric's fused step (sg_dev_match_dedup_diff): raw module output ->
parse -> signature match -> sort -u of the matched records -> diff against the prior scan's
matched set, bit-exact against the oracle (`sig in line` / re.search, sorted(set()), set
difference)."""
import base64
import json
import os
import random

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import semantics as S
from swarm_amd import corpus

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import torch
    import swarm_amd
    assert swarm_amd.device_count() > 0
    c = swarm_amd.Context(0, torch.cuda.current_stream().cuda_stream)
    yield c
    c.close()


@pytest.fixture(scope="module")
def sigs():
    sig = json.load(open(os.path.join(GOLDEN, "signatures.json")))
    words = [base64.b64decode(w) for w in sig["words"]]
    return random.Random(0).sample([w for w in words if len(w) >= 4], 300)


def dev(b):
    import torch
    return torch.from_numpy(np.frombuffer(b + b"\0", dtype=np.uint8).copy()).cuda()


def fused(ctx, m, data, prior, count_hits=True):
    d, p = dev(data), dev(prior)
    r, nh, nm = m.dev_match_dedup_diff(ctx, d.data_ptr(), len(data), p.data_ptr() if prior else 0, len(prior),
                                       count_hits=count_hits)
    return ctx.to_bytes(r.uniq, r.uniq_bytes), ctx.to_bytes(r.fresh, r.fresh_bytes), r, nh, nm


def oracle(data, sigs, prior, kind="literal"):
    hits = S.literal_hits(data, sigs) if kind == "literal" else S.regex_hits(data, sigs)
    matched = S.matched_lines(data, hits)
    u, f = S.dedup_diff(matched, prior)
    return u, f, hits, matched


@pytest.mark.parametrize("count_hits", [True, False])
@pytest.mark.parametrize("n,seed", [(1500, 1), (4000, 2)])
def test_fused_literal_httpx(ctx, sigs, n, seed, count_hits):
    import swarm_amd
    tails = corpus.httpx_tails(sigs, n_tails=512, seed=seed)
    buf, ids = corpus.httpx_hosts(n, tails, seed=seed, universe=n // 2)
    data = buf.tobytes()
    m = swarm_amd.Matcher(sigs, "literal")
    prior_all = corpus.httpx_rows(corpus.prior_ids(ids), tails).tobytes()
    prior = S.dedup(S.matched_lines(prior_all, S.literal_hits(prior_all, sigs)))
    u, f, r, nh, nm = fused(ctx, m, data, prior, count_hits)
    eu, ef, hits, matched = oracle(data, sigs, prior)
    assert u == eu and f == ef
    assert nm == len(S.parse_records(matched))
    assert nh == (len(hits) if count_hits else None)
    assert r.in_records == len(S.parse_records(data))
    assert r.uniq_records == len(S.parse_records(eu)) and r.fresh_records == len(S.parse_records(ef))


def test_fused_no_prior_and_no_match(ctx, sigs):
    import swarm_amd
    m = swarm_amd.Matcher([b"zzzz-never"], "literal")
    data = b"alpha\nbeta\nalpha\n"
    u, f, r, nh, nm = fused(ctx, m, data, b"")
    assert (u, f, nh, nm) == (b"", b"", 0, 0)
    m2 = swarm_amd.Matcher([b"alp", b"et"], "literal")
    u, f, r, nh, nm = fused(ctx, m2, data + b"\r\nalphabet", b"")
    eu, ef, _, _ = oracle(data + b"\r\nalphabet", [b"alp", b"et"], b"")
    assert u == eu and f == ef == eu


def test_fused_regex_banners(ctx):
    import swarm_amd
    pats = corpus.nmap_signatures(n_products=40)
    rows = corpus.banner_pool(n_products=40, pool=600, match_frac=0.3, seed=3)
    rng = random.Random(5)
    data = b"".join(rng.choice(rows) + b"\n" for _ in range(2500))
    prior_rows = b"".join(r + b"\n" for r in rows[:300])
    prior = S.dedup(S.matched_lines(prior_rows, S.regex_hits(prior_rows, pats)))
    m = swarm_amd.Matcher(pats, "regex")
    u, f, r, nh, nm = fused(ctx, m, data, prior)
    eu, ef, hits, _ = oracle(data, pats, prior, kind="regex")
    assert u == eu and f == ef and nh == len(hits)


@pytest.mark.parametrize("seed", [3, 4])
def test_fused_flag_path_edge_records(ctx, seed, monkeypatch):
    """The flag path (no hit count): matched records taken in place from the input — empty
    lines, CR, an unterminated last record, URL-like shared prefixes, every record matching
    or none, a record matching several signatures several times."""
    import swarm_amd
    monkeypatch.setenv("SG_FORCE_LITFILTER", "1")  # the flag path is the q-gram filter's
    rng = random.Random(seed)
    sigs = [b"alpha", b"beta-", b"\r", b"zz", b"https://h1"]
    recs = []
    for i in range(3000):
        k = rng.random()
        if k < 0.05:
            recs.append(b"")
        elif k < 0.5:
            recs.append(b"https://h%d.example/%s" % (rng.randrange(50), rng.choice([b"alpha", b"betazz", b"x"])))
        else:
            recs.append(b"%s beta-beta-%d alpha\r" % (rng.choice([b"a", b"zz", b"q"]), rng.randrange(100)))
    data = b"\n".join(recs) + b"\nunterminated alpha"
    prior = S.dedup(S.matched_lines(data[: len(data) // 3], S.literal_hits(data[: len(data) // 3], sigs)))
    m = swarm_amd.Matcher(sigs, "literal")
    for pr in (prior, b""):
        u, f, r, nh, nm = fused(ctx, m, data, pr, count_hits=False)
        eu, ef, hits, matched = oracle(data, sigs, pr)
        assert u == eu and f == ef and nm == len(S.parse_records(matched)) and nh is None
    none = swarm_amd.Matcher([b"never-there"], "literal")
    u, f, r, nh, nm = fused(ctx, none, data, prior, count_hits=False)
    assert (u, f, nm) == (b"", b"", 0)


def test_fused_prefix_key_speculation(sigs):
    """Repeated fused steps on one context: the matched records' keys are also taken at the
    last call's common prefix (>= 8 bytes: httpx lines start with https://), used when the
    prefix comes out the same, re-keyed otherwise; every output against the oracle."""
    import torch
    import swarm_amd
    c = swarm_amd.Context(0, torch.cuda.current_stream().cuda_stream)
    try:
        m = swarm_amd.Matcher(sigs, "literal")
        tails = corpus.httpx_tails(sigs, n_tails=512, seed=7)
        for step, (n, seed, swap) in enumerate([(30000, 7, None), (30000, 8, None), (30000, 9, (b"https://", b"http://x")),
                                                 (30000, 10, None)]):
            buf, ids = corpus.httpx_hosts(n, tails, seed=seed, universe=n // 2)
            data = buf.tobytes()
            if swap:
                data = data.replace(swap[0], swap[1])
            prior_all = corpus.httpx_rows(corpus.prior_ids(ids), tails).tobytes()
            prior = S.dedup(S.matched_lines(prior_all, S.literal_hits(prior_all, sigs)))
            for count_hits in (False, True):
                u, f, r, nh, nm = fused(c, m, data, prior, count_hits)
                eu, ef, hits, matched = oracle(data, sigs, prior)
                assert u == eu and f == ef, (step, count_hits)
    finally:
        c.close()
