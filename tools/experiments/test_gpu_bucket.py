"""GPU parity of the bucket sample-sort dedup+diff path (sg_bucket.hip): splitters taken from
the prior scan, two bucket passes, per-bucket LDS sort/dedup/diff, compaction. Forced onto
small inputs with SG_BUCKET_MIN=0 and a small SG_BUCKET_TARGET so thousands of buckets form;
every output is compared bit for bit with the oracle (sorted(set()) and set difference), and
the path that served the call is asserted (inputs outside the LDS bounds must hand over to
the radix pipeline and still be exact)."""
import os
import random

import numpy as np
import pytest

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


@pytest.fixture(autouse=True)
def small_buckets(monkeypatch):
    monkeypatch.setenv("SG_BUCKET", "1")
    monkeypatch.setenv("SG_BUCKET_MIN", "0")
    monkeypatch.setenv("SG_BUCKET_TARGET", "2500")


def dev(b):
    import torch
    return torch.from_numpy(np.frombuffer(b, dtype=np.uint8).copy()).cuda()


def run(ctx, cur: bytes, prior: bytes):
    dc, dp = dev(cur + b"\0"), dev(prior + b"\0")
    r = ctx.dedup_diff(dc.data_ptr(), len(cur), dp.data_ptr(), len(prior))
    u = ctx.to_bytes(r.uniq, r.uniq_bytes)
    f = ctx.to_bytes(r.fresh, r.fresh_bytes)
    return u, f, r, ctx.last_path()


def check(ctx, cur, prior, path="bucket"):
    u, f, r, (p, flags) = run(ctx, cur, prior)
    eu, ef = S.dedup_diff(cur, prior)
    assert u == eu
    assert f == ef
    assert r.in_records == len(S.parse_records(cur))
    assert r.uniq_records == len(S.parse_records(eu)) and r.fresh_records == len(S.parse_records(ef))
    if path:
        assert p == path, (p, flags)
    return flags


def subdomain_pair(n, seed):
    buf, ids = corpus.subdomains(n, seed=seed)
    return buf.tobytes(), corpus.prior_of(ids).tobytes()


@pytest.mark.parametrize("n,seed", [(20_000, 1), (60_000, 2), (200_000, 3)])
def test_subdomains(ctx, n, seed):
    cur, prior = subdomain_pair(n, seed)
    check(ctx, cur, prior)
    assert S.parse_records(prior)  # the prior is what the splitters come from


def test_prior_records_counted(ctx):
    cur, prior = subdomain_pair(50_000, 4)
    _, _, r, (p, _) = run(ctx, cur, prior)
    assert p == "bucket" and r.prior_records == len(S.parse_records(prior))


@pytest.mark.parametrize("seed", range(4))
def test_random_bytes_with_nul_cr_ff(ctx, seed):
    """Records over a small alphabet with NUL, CR, 0xff and '.', many sharing 7+ bytes
    (key0 ties with splitters and inside buckets), empty lines, no final newline."""
    rng = random.Random(seed)
    alpha = b"ab\x00\r\xff."
    recs = [bytes(rng.choice(alpha) for _ in range(rng.randint(1, 24))) for _ in range(30_000)]
    prior_set = sorted(set(r for r in recs if rng.random() < 0.7))
    prior = b"".join(r + b"\n" for r in prior_set)
    cur = b"\n".join(recs[i] if i % 50 else b"" for i in range(len(recs)))  # empty lines, unterminated
    check(ctx, cur, prior)


def test_long_shared_prefixes_url_like(ctx):
    """URL-like records: every record shares 'https://' and many share far more than the
    7-byte key0 (ties resolved by byte compares in classification, sort and diff)."""
    rng = random.Random(7)
    hosts = ["www.example%d.com" % rng.randrange(400) for _ in range(2000)]
    recs = [("https://%s/%s" % (rng.choice(hosts), "a" * rng.randrange(0, 40))).encode() for _ in range(40_000)]
    prior = b"".join(r + b"\n" for r in sorted(set(recs[::3])))
    check(ctx, b"\n".join(recs) + b"\n", prior)


def test_lengths_around_key_and_word_sizes(ctx):
    base = b"abcdefghijklmnopqrstuvwxyz0123456789"
    recs = [base[:k] + bytes([c]) for k in range(0, 30) for c in range(0x61, 0x61 + 40)]
    recs += [base[:k] for k in range(1, 36)]
    rng = random.Random(8)
    cur_l = recs * 3
    rng.shuffle(cur_l)
    prior = b"".join(r + b"\n" for r in sorted(set(recs[::2])))
    check(ctx, b"\n".join(cur_l) + b"\n", prior)


def test_heavy_duplicates(ctx):
    cur, prior = subdomain_pair(5_000, 9)
    cur = cur * 8
    check(ctx, cur, prior)


def test_extreme_duplication_hands_over(ctx):
    """Thousands of copies of a few records land in one bucket past its LDS budget: the radix
    pipeline takes over, exactly."""
    cur, prior = subdomain_pair(20_000, 22)
    recs = S.parse_records(cur)
    cur = cur + b"".join(recs[i % 7] + b"\n" for i in range(30_000))
    check(ctx, cur, prior, path=None)


def test_records_equal_to_splitters_and_prior_extremes(ctx):
    """Every prior record also in cur (some splitters reappear), plus records below the first
    and above the last prior record."""
    cur, prior = subdomain_pair(40_000, 10)
    cur = prior + cur + b"\x00\x00\n\xff\xff\xff\n!\n"
    check(ctx, cur, prior)


def test_cur_without_prior_overlap(ctx):
    cur, _ = subdomain_pair(30_000, 11)
    _, prior = subdomain_pair(30_000, 12)
    check(ctx, cur, prior)


def test_unsorted_prior_hands_over(ctx):
    cur, prior = subdomain_pair(40_000, 13)
    recs = S.parse_records(prior)
    i = len(recs) // 2
    recs[i], recs[i + 1] = recs[i + 1], recs[i]
    bad = b"".join(r + b"\n" for r in recs)
    flags = check(ctx, cur, bad, path="radix")
    assert flags & 8


def test_duplicated_prior_hands_over(ctx):
    cur, prior = subdomain_pair(40_000, 14)
    recs = S.parse_records(prior)
    recs.insert(100, recs[100])
    check(ctx, cur, b"".join(r + b"\n" for r in recs), path="radix")


def test_long_record_hands_over(ctx):
    cur, prior = subdomain_pair(60_000, 15)
    cur = cur[: len(cur) // 2] + b"L" * 5000 + b"\n" + cur[len(cur) // 2:]
    flags = check(ctx, cur, prior, path=None)
    p, _ = ctx.last_path()
    assert p in ("radix", "probe") and flags & 1 or p == "bucket"


def test_skewed_bucket_hands_over(ctx):
    """All cur records fall between two adjacent splitters: one bucket over its LDS budget."""
    cur_recs = [b"mmm-%06d.example" % i for i in range(20_000)]
    prior = b"".join(b"%s%05d\n" % (c, i) for c in (b"a", b"z") for i in range(2000))
    flags = check(ctx, b"\n".join(cur_recs) + b"\n", prior, path="radix")
    assert flags & 2


def test_default_threshold_keeps_small_inputs_on_radix(ctx, monkeypatch):
    monkeypatch.delenv("SG_BUCKET_MIN")
    cur, prior = subdomain_pair(20_000, 16)
    check(ctx, cur, prior, path="radix")


def test_disabled_by_env(ctx, monkeypatch):
    monkeypatch.setenv("SG_BUCKET", "0")
    cur, prior = subdomain_pair(20_000, 17)
    check(ctx, cur, prior, path="radix")


def test_host_api_uses_bucket_path(ctx):
    import swarm_amd
    cur, prior = subdomain_pair(30_000, 18)
    assert swarm_amd.dedup_diff(cur, prior) == S.dedup_diff(cur, prior)
    assert swarm_amd.diff(cur, prior) == S.dedup_diff(cur, prior)[1]


def test_repeated_calls_reuse_workspaces(ctx):
    for seed in (19, 20, 21):
        cur, prior = subdomain_pair(30_000 + 5_000 * seed, seed)
        check(ctx, cur, prior)
