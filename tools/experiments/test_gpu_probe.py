"""GPU parity of the probe path (opt-in, SG_PROBE=1; a strictly increasing prior: the current
records are looked up in a hash table of the prior, only the new ones are sorted, and the
unique output is the prior's found records merged with them) against the oracle's sort -u /
comm -13.

Every case also runs with the hash weakened (SG_PROBE_FPMASK=0: one fingerprint for all
records, SG_PROBE_SLOTS=1.01: a nearly full table), so each probe walks long runs of slots
and every candidate goes through the byte compare and the terminator check."""
import random

import numpy as np
import pytest

from oracle import semantics as S

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import torch
    import swarm_amd
    c = swarm_amd.Context(0, torch.cuda.current_stream().cuda_stream)
    yield c
    c.close()


@pytest.fixture(autouse=True)
def probe_on(monkeypatch):
    monkeypatch.setenv("SG_PROBE", "1")  # opt-in path


@pytest.fixture(params=["default", "weak_hash"])
def mode(request, monkeypatch):
    if request.param == "weak_hash":
        monkeypatch.setenv("SG_PROBE_FPMASK", "0")
        monkeypatch.setenv("SG_PROBE_SLOTS", "1.01")
    return request.param


def dev(b: bytes):
    import torch
    return torch.from_numpy(np.frombuffer(b + b"\0", dtype=np.uint8).copy()).cuda()


def sorted_prior(recs) -> bytes:
    return b"".join(r + b"\n" for r in sorted(set(recs)))


def run(ctx, cur: bytes, prior: bytes, path="probe"):
    dc, dp = dev(cur), dev(prior)
    r = ctx.dedup_diff(dc.data_ptr(), len(cur), dp.data_ptr(), len(prior))
    u = ctx.to_bytes(r.uniq, r.uniq_bytes)
    f = ctx.to_bytes(r.fresh, r.fresh_bytes)
    eu, ef = S.dedup_diff(cur, prior)
    assert u == eu
    assert f == ef
    assert r.in_records == len(S.parse_records(cur))
    assert r.uniq_records == eu.count(b"\n") and r.fresh_records == ef.count(b"\n")
    if path:
        assert ctx.last_path()[0] == path
    return r


def rand_rec(rng, alphabet, lo, hi):
    return bytes(rng.choice(alphabet) for _ in range(rng.randint(lo, hi)))


@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("overlap", [0.0, 0.5, 0.9, 1.0])
def test_random_bytes_overlaps(ctx, mode, seed, overlap):
    rng = random.Random(1000 * seed + int(overlap * 10))
    universe = list({rand_rec(rng, b"ab\x00\r\xff.", 1, 14) for _ in range(3000)})
    rng.shuffle(universe)
    k = int(len(universe) * overlap)
    prior = sorted_prior(universe[:k] + [rand_rec(rng, b"xyz", 1, 6) for _ in range(300)])
    cur_recs = [rng.choice(universe) for _ in range(5000)]
    cur = b"\n".join(cur_recs) + b"\n"
    run(ctx, cur, prior)


def test_cur_subset_of_prior_no_new(ctx, mode):
    recs = [b"h%05d.example.org" % i for i in range(4000)]
    prior = sorted_prior(recs)
    cur = b"\n".join(recs[::3] * 2) + b"\n"
    r = run(ctx, cur, prior)
    assert r.fresh_records == 0


def test_disjoint_prior_all_new(ctx, mode):
    prior = sorted_prior([b"a%05d" % i for i in range(3000)])
    cur = b"\n".join(b"b%05d" % (i % 1700) for i in range(5000)) + b"\n"
    run(ctx, cur, prior)


def test_prefix_records_and_terminators(ctx, mode):
    """Records that are prefixes of each other (the terminator check), NUL/CR bytes, and a
    prior whose last record has no trailing newline."""
    base = [b"abc", b"abcd", b"abc\x00", b"ab", b"abc\r", b"abcde" * 20, b"abcde" * 20 + b"f", b"a"]
    prior_recs = sorted(set(base[::2] + [b"zz%03d" % i for i in range(200)]))
    prior = b"\n".join(prior_recs)  # no trailing newline
    cur = b"\n".join(base * 3 + [b"zz%03d" % i for i in range(0, 200, 3)] + [b"zz199"])  # no trailing newline
    run(ctx, cur, prior)
    run(ctx, cur + b"\n", prior + b"\n")


@pytest.mark.parametrize("maxlen", [7, 16, 47, 48, 49, 100, 300])
def test_long_records_hash_windows(ctx, mode, maxlen):
    rng = random.Random(maxlen)
    stem = b"x" * max(0, maxlen - 6)
    universe = list({stem[: rng.randint(0, len(stem))] + rand_rec(rng, b"pqrs", 1, 6) for _ in range(2500)})
    prior = sorted_prior(universe[: len(universe) * 2 // 3])
    cur = b"\n".join(rng.choice(universe) for _ in range(4000)) + b"\n"
    run(ctx, cur, prior)


def test_new_records_tie_prior_keys(ctx, mode):
    """New records share their first 7+ bytes with runs of prior records: the insertion
    point comes from the bytewise search inside the equal-key run."""
    prior_recs = [b"samekey-%04d" % (2 * i) for i in range(3000)]
    prior = sorted_prior(prior_recs)
    new = [b"samekey-%04d" % (2 * i + 1) for i in range(0, 3000, 7)]
    new += [b"samekey-", b"samekey-0000x", b"samekey-9999", b"samekey-59999", b"samekez", b"samekex"]
    cur_recs = prior_recs[::2] + new + new[:50]
    random.Random(5).shuffle(cur_recs)
    run(ctx, b"\n".join(cur_recs) + b"\n", prior)


def test_url_common_prefix(ctx, mode):
    rng = random.Random(9)
    urls = list({b"https://%s.example.com/%s" % (rand_rec(rng, b"abcdefgh", 3, 9), rand_rec(rng, b"0123", 0, 5))
                 for _ in range(4000)})
    prior = sorted_prior(urls[:3000])
    cur = b"\n".join(rng.choice(urls) for _ in range(6000)) + b"\n"
    run(ctx, cur, prior)


@pytest.mark.parametrize("case", ["one_cur", "one_prior", "one_each_equal", "one_each_new"])
def test_single_records(ctx, mode, case):
    if case == "one_cur":
        cur, prior = b"m\n", sorted_prior([b"a", b"m", b"z"])
    elif case == "one_prior":
        cur, prior = b"b\na\nc\na\n", b"b\n"
    elif case == "one_each_equal":
        cur, prior = b"same\n", b"same\n"
    else:
        cur, prior = b"new\n", b"old\n"
    run(ctx, cur, prior)


def test_unsorted_prior_keeps_radix(ctx):
    run(ctx, b"a\nb\nc\n", b"b\na\n", path="radix")


def test_full_segment_falls_back_to_radix(ctx, monkeypatch):
    """Segments of 4 slots: some segment gets no free slot, the call runs the radix pipeline."""
    monkeypatch.setenv("SG_PROBE_SEGBITS", "2")
    recs = [b"r%05d" % i for i in range(3000)]
    run(ctx, b"\n".join(recs[::2] + [b"new%d" % i for i in range(50)]) + b"\n", sorted_prior(recs), path="radix")


def test_probe_disabled_by_env(ctx, monkeypatch):
    monkeypatch.setenv("SG_PROBE", "0")
    run(ctx, b"a\nb\nc\n", b"a\nb\n", path="radix")


def test_caller_output_buffers_misaligned(ctx, mode):
    """dedup_diff_into (the C5 part path) with outputs at odd device addresses."""
    import torch
    from swarm_amd import corpus
    buf, ids = corpus.subdomains(50_000, seed=21)
    prior = corpus.prior_of(ids)
    dc, dp = dev(buf.tobytes()), dev(prior.tobytes())
    out = torch.zeros(2 * (buf.size + 64), dtype=torch.uint8, device="cuda")
    ou, of = out.data_ptr() + 5, out.data_ptr() + buf.size + 64 + 11
    r = ctx.dedup_diff_into(dc.data_ptr(), buf.size, dp.data_ptr(), prior.size, ou, buf.size + 1, of, buf.size + 1)
    assert ctx.last_path()[0] == "probe"
    eu, ef = S.dedup_diff(buf.tobytes(), prior.tobytes())
    assert ctx.to_bytes(r.uniq, r.uniq_bytes) == eu and r.uniq == ou
    assert ctx.to_bytes(r.fresh, r.fresh_bytes) == ef and r.fresh == of


def test_subdomains_300k_matches_radix(ctx, monkeypatch):
    from swarm_amd import corpus
    buf, ids = corpus.subdomains(300_000, seed=3)
    prior = corpus.prior_of(ids).tobytes()
    cur = buf.tobytes()
    r = run(ctx, cur, prior)
    monkeypatch.setenv("SG_PROBE", "0")
    r2 = run(ctx, cur, prior, path="radix")
    assert (r.uniq_records, r.fresh_records) == (r2.uniq_records, r2.fresh_records)


def test_fused_x1_matches_radix(ctx, monkeypatch):
    """The fused match -> sort -u -> diff step on 300k httpx lines: probe path output equals
    the radix pipeline's byte for byte (long records, many merge tiles)."""
    import base64
    import json
    import os
    import torch
    import swarm_amd
    from swarm_amd import corpus
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sig = json.load(open(os.path.join(root, "tests", "golden", "signatures.json")))
    words = [base64.b64decode(w) for w in sig["words"]]
    sigs = random.Random(0).sample([w for w in words if len(w) >= 4], 2000)
    tails = corpus.httpx_tails(sigs)
    buf, ids = corpus.httpx_hosts(300_000, tails, seed=77)
    d = torch.from_numpy(buf).cuda()
    m = swarm_amd.Matcher(sigs, "literal")
    dp_in = torch.from_numpy(corpus.httpx_rows(corpus.prior_ids(ids), tails)).cuda()
    r0, _, _ = m.dev_match_dedup_diff(ctx, dp_in.data_ptr(), dp_in.numel())
    n_prior = int(r0.uniq_bytes)
    d_prior = torch.empty(max(n_prior, 1), dtype=torch.uint8, device="cuda")
    ctx.memcpy(d_prior.data_ptr(), r0.uniq, n_prior)
    outs = []
    for mode in ("1", "0"):
        monkeypatch.setenv("SG_PROBE", mode)
        r, _, _ = m.dev_match_dedup_diff(ctx, d.data_ptr(), d.numel(), d_prior.data_ptr(), n_prior, count_hits=False)
        outs.append((ctx.to_bytes(r.uniq, r.uniq_bytes), ctx.to_bytes(r.fresh, r.fresh_bytes), ctx.last_path()[0]))
    assert outs[0][2] == "probe" and outs[1][2] == "radix"
    assert outs[0][:2] == outs[1][:2]
    m.close()
