"""GPU parity for shards larger than one call (C5 sizes): order-preserving range routing by
key0 splitters, then per-part dedup/diff whose concatenation is the global sort -u /
comm -13 output, bit-exact against the oracle."""
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


def dev(b):
    import torch
    return torch.from_numpy(np.frombuffer(b, dtype=np.uint8).copy()).cuda()


def test_range_parts_are_ordered_and_complete(ctx):
    import torch
    from swarm_amd import sharded
    buf, _ = corpus.subdomains(200_000, seed=31)
    data = buf.tobytes() + b"a\nzz\n\xff\xff\n\x00\nsame-prefix-1\nsame-prefix-2\n"
    d = dev(data)
    sp = sharded.choose_splitters(ctx.key_sample(d.data_ptr(), d.numel(), 4096)[0], 9)
    out = torch.empty(d.numel() + 16, dtype=torch.uint8, device=d.device)
    pb, pr = ctx.partition_range(d.data_ptr(), d.numel(), sp, out.data_ptr(), out.numel())
    assert sum(pb) == len(data) and sum(pr) == len(S.parse_records(data))
    got = out[: sum(pb)].cpu().numpy().tobytes()
    off, prev_max = 0, None
    for b in range(len(pb)):
        recs = S.parse_records(got[off:off + pb[b]])
        assert len(recs) == pr[b]
        if recs:
            if prev_max is not None:
                assert prev_max < min(recs)
            prev_max = max(recs)
        off += pb[b]
    assert sorted(S.parse_records(got)) == sorted(S.parse_records(data))


@pytest.mark.parametrize("part_bytes,piece", [(4 << 20, 5 << 20), (1 << 20, 3 << 20), (64 << 20, 64 << 20)])
def test_dedup_diff_large_matches_global_oracle(ctx, part_bytes, piece):
    from swarm_amd import sharded
    buf, ids = corpus.subdomains(1_200_000, seed=32)
    prior = corpus.prior_of(ids)
    cur_p = sharded.split_at_newlines(dev(buf.tobytes()), piece)
    pri_p = sharded.split_at_newlines(dev(prior.tobytes()), piece)
    u, f, st = sharded.dedup_diff_large(ctx, cur_p, pri_p, part_bytes=part_bytes)
    eu, ef = S.dedup_diff(buf.tobytes(), prior.tobytes())
    assert u.cpu().numpy().tobytes() == eu
    assert f.cpu().numpy().tobytes() == ef
    assert st["in_records"] == 1_200_000


def test_dedup_large_unsorted_prior_and_no_prior(ctx):
    from swarm_amd import sharded
    a, _ = corpus.subdomains(300_000, seed=33, universe=200_000)
    b, _ = corpus.subdomains(300_000, seed=34, universe=200_000)
    cur = a.tobytes() + b"tail-without-newline"
    u, f, st = sharded.dedup_diff_large(ctx, sharded.split_at_newlines(dev(cur), 1 << 20),
                                        sharded.split_at_newlines(dev(b.tobytes()), 1 << 20), part_bytes=2 << 20)
    eu, ef = S.dedup_diff(cur, b.tobytes())
    assert u.cpu().numpy().tobytes() == eu and f.cpu().numpy().tobytes() == ef
    u2, f2, _ = sharded.dedup_diff_large(ctx, [dev(cur)], (), part_bytes=1 << 20)
    assert u2.cpu().numpy().tobytes() == eu and f2.cpu().numpy().tobytes() == eu


def test_many_tiny_parts_and_skewed_keys(ctx):
    """Up to 256 parts (the routing maximum), many empty ones, and a key0 value shared by a
    large run of records (it cannot be split: it stays in one part)."""
    from swarm_amd import sharded
    buf, ids = corpus.subdomains(100_000, seed=35)
    same = b"".join(b"samekey-%d.example\n" % (i % 5000) for i in range(60_000))
    cur = buf.tobytes() + same
    prior = S.dedup(same[: len(same) // 3])
    u, f, st = sharded.dedup_diff_large(ctx, sharded.split_at_newlines(dev(cur), 512 << 10), [dev(prior)],
                                        part_bytes=16 << 10)
    assert st["parts"] == 256
    eu, ef = S.dedup_diff(cur, prior)
    assert u.cpu().numpy().tobytes() == eu and f.cpu().numpy().tobytes() == ef


def test_private_stream_context_is_fenced():
    """A Context without a stream argument runs on its own non-blocking stream; the sharded
    path must still order torch allocations against library writes."""
    import swarm_amd
    from swarm_amd import sharded
    c = swarm_amd.Context(0)
    try:
        assert not c.on_torch_stream()
        buf, ids = corpus.subdomains(400_000, seed=36)
        prior = corpus.prior_of(ids)
        for _ in range(3):  # reuse of freed torch blocks between rounds is the hazard
            u, f, _ = sharded.dedup_diff_large(c, sharded.split_at_newlines(dev(buf.tobytes()), 1 << 20),
                                               sharded.split_at_newlines(dev(prior.tobytes()), 1 << 20),
                                               part_bytes=1 << 20)
            eu, ef = S.dedup_diff(buf.tobytes(), prior.tobytes())
            assert u.cpu().numpy().tobytes() == eu and f.cpu().numpy().tobytes() == ef
    finally:
        c.close()
