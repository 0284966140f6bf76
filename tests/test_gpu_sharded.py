"""GPU parity for shards larger than one call (C5 sizes): order-preserving range routing by
byte-string (and key0) splitters, then per-part dedup/diff whose concatenation is the global
sort -u / comm -13 output, bit-exact against the oracle. The byte routing itself is checked
against bisect over the cut splitters (Python bytes order is sort's byte order)."""
import random

import numpy as np
import pytest

from oracle import semantics as S
from route_oracle import route_parts, sample_heads
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
    """Up to 256 parts (the routing maximum), many empty ones, and a large run of records
    sharing their first 8 bytes (byte splitters divide it; equal records stay together)."""
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


def shared_prefix_records(n, seed):
    """Records sharing long prefixes: lengths around the 8-byte word and 64-byte cut
    boundaries, NUL / 0xff bytes, equal 64-byte heads with different tails."""
    rng = random.Random(seed)
    heads = [b"https://www.example.com/" + bytes(rng.choice(b"ab\x00\xff/") for _ in range(rng.randint(0, 48)))
             for _ in range(300)]
    recs = []
    for _ in range(n):
        h = rng.choice(heads)
        k = rng.random()
        if k < 0.3:
            recs.append(h)
        elif k < 0.6:
            recs.append((h + b"X" * 80)[:rng.choice([56, 63, 64, 65, 71, 72, 100])])
        else:
            recs.append(h + bytes(rng.choice(b"az\x00") for _ in range(rng.randint(1, 30))))
    return recs


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_byte_partition_matches_bisect(ctx, seed):
    import torch
    recs = shared_prefix_records(20_000, seed)
    data = b"\n".join(recs) + b"\n\n" + b"no-newline-tail"
    rng = random.Random(seed + 10)
    sp = sorted(rng.sample(recs, 40) + [b"", b"https://www.example.com/" + b"a" * 70, b"\xff" * 3])
    d = dev(data)
    out = torch.empty(d.numel() + 16, dtype=torch.uint8, device=d.device)
    pb, pr = ctx.partition_bytes(d.data_ptr(), d.numel(), sp, out.data_ptr(), out.numel())
    want = route_parts(data, sp)
    assert pb == [len(w) for w in want]
    assert pr == [len(S.parse_records(w)) for w in want]
    assert out[: sum(pb)].cpu().numpy().tobytes() == b"".join(want)


def test_byte_partition_edge_cases(ctx):
    import torch
    from swarm_amd._abi import SGError
    d = dev(b"b\na\n")
    out = torch.empty(32, dtype=torch.uint8, device=d.device)
    assert ctx.partition_bytes(d.data_ptr(), d.numel(), [], out.data_ptr(), out.numel()) == ([4], [2])
    with pytest.raises(SGError):
        ctx.partition_bytes(d.data_ptr(), d.numel(), [b"b", b"a"], out.data_ptr(), out.numel())
    with pytest.raises(SGError):  # equal after the 64-byte cut, then shorter
        ctx.partition_bytes(d.data_ptr(), d.numel(), [b"x" * 64 + b"1", b"x" * 63], out.data_ptr(), out.numel())
    e = dev(b"\n\n")
    assert ctx.partition_bytes(e.data_ptr(), 2, [b"m"], out.data_ptr(), out.numel()) == ([0, 0], [0, 0])


def test_record_sample_heads(ctx):
    recs = shared_prefix_records(5_000, 4)
    data = b"\n".join(recs) + b"\n"
    d = dev(data)
    heads, n = ctx.record_sample(d.data_ptr(), d.numel(), 777)
    R = S.parse_records(data)
    assert n == len(R)
    assert heads == [R[(k * len(R)) // 777][:64] for k in range(777)] == sample_heads(data, 777)[0]
    e = dev(b"\n\n\n")
    assert ctx.record_sample(e.data_ptr(), 3, 16) == ([], 0)


@pytest.mark.parametrize("kind", ["urls", "ips"])
def test_shared_prefix_data_splits_evenly(ctx, kind):
    """URL and 10.x.y.z:port records (key0 = 'https:/' / '10.x.y.' for whole runs) still
    route into balanced parts, and the part outputs are the global result."""
    import torch
    from swarm_amd import sharded
    if kind == "urls":
        recs = shared_prefix_records(150_000, 7)
        cur = b"\n".join(recs) + b"\n"
        prior = S.dedup(b"\n".join(recs[::3]) + b"\n")
    else:
        pool = corpus.ip_pool_torch(56_000, seed=5, device="cuda")
        cur = b"".join(p.cpu().numpy().tobytes() for p in corpus.hostport_pieces(pool, 200_000, 0, 800_000, seed=1,
                                                                               ports_per_host=16))
        prior = S.dedup(b"".join(p.cpu().numpy().tobytes() for p in corpus.hostport_pieces(
            pool, 150_000, 80_000, 880_000, seed=2, ports_per_host=16)))
    u, f, st = sharded.dedup_diff_large(ctx, sharded.split_at_newlines(dev(cur), 1 << 20), [dev(prior)],
                                        part_bytes=len(cur) // 8)
    eu, ef = S.dedup_diff(cur, prior)
    assert u.cpu().numpy().tobytes() == eu and f.cpu().numpy().tobytes() == ef
    pbytes = st["part_bytes"]
    assert len(pbytes) >= 8
    assert max(pbytes) <= 1.5 * (sum(pbytes) / len(pbytes))


def test_oversize_part_is_routed_again(ctx, monkeypatch):
    from swarm_amd import sharded
    monkeypatch.setattr(sharded, "PART_LIMIT", 300_000)
    buf, ids = corpus.subdomains(100_000, seed=37)
    prior = corpus.prior_of(ids)
    u, f, st = sharded.dedup_diff_large(ctx, [dev(buf.tobytes())], [dev(prior.tobytes())], splitters=[b"m"])
    eu, ef = S.dedup_diff(buf.tobytes(), prior.tobytes())
    assert u.cpu().numpy().tobytes() == eu and f.cpu().numpy().tobytes() == ef
    assert st["rerouted_parts"] >= 2 and max(st["part_bytes"]) <= 300_000


def test_identical_records_past_the_limit_raise(ctx, monkeypatch):
    from swarm_amd import sharded
    monkeypatch.setattr(sharded, "PART_LIMIT", 100_000)
    same = b"".join(b"x" * 70 + b"%d\n" % (i % 3) for i in range(5_000))
    with pytest.raises(ValueError, match="share their first 64 bytes"):
        sharded.dedup_diff_large(ctx, [dev(same)], (), part_bytes=50_000)


def test_partition_pieces_part_contiguous(ctx):
    """k pieces (unaligned starts, an empty piece, no final newline) routed into one buffer:
    part p = the pieces' part-p records in piece order (route_parts per piece, joined)."""
    import torch
    recs = shared_prefix_records(30_000, 11)
    data = b"\n".join(recs) + b"\n"
    cuts = [0, 7, len(data) // 3, len(data) // 3, len(data)]
    cuts = [c if c in (0, len(data)) else data.index(b"\n", c) + 1 for c in cuts]
    d = dev(b"#" + data)  # pieces start at odd addresses
    pieces = [d[1 + a:1 + b] for a, b in zip(cuts, cuts[1:])]
    sp = sorted(random.Random(12).sample(recs, 20))
    out = torch.full((len(data) + 64,), 0x55, dtype=torch.uint8, device=d.device)
    pb, pr = ctx.partition_bytes_pieces([(p.data_ptr(), p.numel()) for p in pieces], sp, out.data_ptr(), out.numel())
    per_piece = [route_parts(data[a:b], sp) for a, b in zip(cuts, cuts[1:])]
    want = [b"".join(pp[q] for pp in per_piece) for q in range(len(sp) + 1)]
    assert pb == [len(w) for w in want]
    assert pr == [len(S.parse_records(w)) for w in want]
    got = out.cpu().numpy().tobytes()
    assert got[: sum(pb)] == b"".join(want)
    assert set(got[sum(pb):]) == {0x55}


@pytest.mark.parametrize("shift", [0, 1, 7, 15])
def test_dedup_diff_into_any_address(ctx, shift):
    import torch
    buf, ids = corpus.subdomains(30_000, seed=40 + shift)
    prior = corpus.prior_of(ids).tobytes()
    cur = buf.tobytes()
    dc, dp = dev(cur), dev(prior)
    cap = len(cur) + 1
    ub = torch.full((cap + 64,), 0xEE, dtype=torch.uint8, device=dc.device)
    fb = torch.full((cap + 64,), 0xEE, dtype=torch.uint8, device=dc.device)
    r = ctx.dedup_diff_into(dc.data_ptr(), len(cur), dp.data_ptr(), len(prior), ub.data_ptr() + shift, cap,
                            fb.data_ptr() + shift, cap)
    eu, ef = S.dedup_diff(cur, prior)
    u, f = ub.cpu().numpy().tobytes(), fb.cpu().numpy().tobytes()
    assert u[shift:shift + r.uniq_bytes] == eu and f[shift:shift + r.fresh_bytes] == ef
    assert set(u[:shift] + u[shift + r.uniq_bytes:]) <= {0xEE} and set(f[:shift] + f[shift + r.fresh_bytes:]) <= {0xEE}
    assert r.uniq == ub.data_ptr() + shift and r.fresh == fb.data_ptr() + shift
    # no prior: the new records are all unique records, copied into the fresh output
    r = ctx.dedup_diff_into(dc.data_ptr(), len(cur), 0, 0, ub.data_ptr() + shift, cap, fb.data_ptr() + shift, cap)
    assert ctx.to_bytes(r.fresh, r.fresh_bytes) == eu == ctx.to_bytes(r.uniq, r.uniq_bytes)
    from swarm_amd._abi import SGError
    with pytest.raises(SGError):
        ctx.dedup_diff_into(dc.data_ptr(), len(cur), 0, 0, ub.data_ptr(), len(cur), fb.data_ptr(), cap)


def test_stored_prior_parts_skip_routing(ctx):
    """The C5 step with the stored prior split at its own part boundaries (no prior routing)
    equals the routed path and the oracle."""
    from swarm_amd import sharded
    buf, ids = corpus.subdomains(400_000, seed=44)
    prior_raw = corpus.prior_of(ids).tobytes()
    pieces = sharded.split_at_newlines(dev(prior_raw), 1 << 20)
    sp = sharded.choose_splitters(sharded.sample_records(ctx, pieces, 256), 6)
    pu, _, pst = sharded.dedup_diff_large(ctx, pieces, (), splitters=sp)
    assert len(pst["uniq_part_bytes"]) == len(sp) + 1 and sum(pst["uniq_part_bytes"]) == pu.numel()
    parts = sharded.split_parts(pu, pst["uniq_part_bytes"])
    cur = sharded.split_at_newlines(dev(buf.tobytes()), 1 << 20)
    u, f, _ = sharded.dedup_diff_large(ctx, cur, (), splitters=sp, prior_parts=parts)
    eu, ef = S.dedup_diff(buf.tobytes(), prior_raw)
    assert u.cpu().numpy().tobytes() == eu and f.cpu().numpy().tobytes() == ef
    u2, f2, _ = sharded.dedup_diff_large(ctx, cur, [pu], splitters=sp)
    assert u2.cpu().numpy().tobytes() == eu and f2.cpu().numpy().tobytes() == ef


def test_partition_pieces_aligned_parts(ctx):
    """align16: every part starts at a 16-byte aligned offset of the output, bytes and
    records as the back-to-back variant, padding untouched."""
    import torch
    from swarm_amd.api import part_offsets
    recs = shared_prefix_records(20_000, 13)
    data = b"\n".join(recs) + b"\n"
    cuts = [0, len(data) // 4, len(data) // 2, len(data)]
    cuts = [c if c in (0, len(data)) else data.index(b"\n", c) + 1 for c in cuts]
    d = dev(b"#" + data)
    pieces = [d[1 + a:1 + b] for a, b in zip(cuts, cuts[1:])]
    sp = sorted(random.Random(14).sample(recs, 12))
    out = torch.full((len(data) + 16 * 14 + 64,), 0x55, dtype=torch.uint8, device=d.device)
    pb, pr = ctx.partition_bytes_pieces([(p.data_ptr(), p.numel()) for p in pieces], sp, out.data_ptr(), out.numel(),
                                        align16=True)
    per_piece = [route_parts(data[a:b], sp) for a, b in zip(cuts, cuts[1:])]
    want = [b"".join(pp[q] for pp in per_piece) for q in range(len(sp) + 1)]
    assert pb == [len(w) for w in want]
    assert pr == [len(S.parse_records(w)) for w in want]
    got = out.cpu().numpy().tobytes()
    offs = part_offsets(pb, align16=True)
    for o, w in zip(offs, want):
        assert o % 16 == 0
        assert got[o:o + len(w)] == w
    # the padding between parts is never written
    used = set()
    for o, w in zip(offs, want):
        used.update(range(o, o + len(w)))
    assert {got[i] for i in range(len(got)) if i not in used} == {0x55}


def test_partition_spans_handover(ctx):
    """partition_bytes_pieces_spans: aligned parts plus every part's parse (spans relative
    to the part, equal to the parser's on that part; keys as the dedup's own), and the dedup
    fed that parse (dedup_diff_spans_into) equals the oracle's sort -u / comm -13 per part."""
    import swarm_amd
    import torch
    from swarm_amd.api import part_offsets, span_sum
    from route_oracle import key0, span_sum as py_span_sum
    recs = shared_prefix_records(25_000, 17) + [b"", b"x", b"x" * 300]
    random.Random(18).shuffle(recs)
    data = b"\n".join(recs) + b"\n"
    cuts = [0, len(data) // 3, 2 * len(data) // 3, len(data)]
    cuts = [c if c in (0, len(data)) else data.index(b"\n", c) + 1 for c in cuts]
    d = dev(b"#" + data)
    pieces = [d[1 + a:1 + b] for a, b in zip(cuts, cuts[1:])]
    sp = sorted(random.Random(19).sample([r for r in recs if r], 9))
    out = torch.full((len(data) + 16 * 11 + 64,), 0x55, dtype=torch.uint8, device=d.device)
    pb, pr, dsp, dkp, ps = ctx.partition_bytes_pieces_spans([(p.data_ptr(), p.numel()) for p in pieces], sp,
                                                            out.data_ptr(), out.numel())
    nrec = sum(pr)
    spans = np.frombuffer(ctx.to_bytes(dsp, 8 * nrec), dtype=np.uint32).reshape(-1, 2)
    keys = np.frombuffer(ctx.to_bytes(dkp, 8 * nrec), dtype=np.uint64)
    got = out.cpu().numpy().tobytes()
    prior_recs = sorted(set(random.Random(20).sample([r for r in recs if r], 5000)))
    r0 = 0
    for o, n, nr, ssum in zip(part_offsets(pb, align16=True), pb, pr, ps):
        part = got[o:o + n]
        assert np.array_equal(spans[r0:r0 + nr].astype(np.uint64), swarm_amd.lines(part))
        # the part's handover checksum, as the restatement computes it from the part's bytes
        assert ssum == py_span_sum(S.record_spans(part), [key0(part[a:e]) for a, e in S.record_spans(part)])
        assert ssum == span_sum(spans[r0:r0 + nr], keys[r0:r0 + nr])
        if n:
            lo, hi = S.parse_records(part)[0], S.parse_records(part)[-1]
            prior = b"".join(r + b"\n" for r in prior_recs if lo <= r <= hi)
            dp = dev(prior)
            ub = torch.empty(n + 64, dtype=torch.uint8, device=d.device)
            fb = torch.empty(n + 64, dtype=torch.uint8, device=d.device)
            r = ctx.dedup_diff_spans_into(out.data_ptr() + o, n, dsp + 8 * r0, dkp + 8 * r0, nr, ssum, dp.data_ptr(),
                                          len(prior), ub.data_ptr() + 3, n + 1, fb.data_ptr() + 5, n + 1)
            eu, ef = S.dedup_diff(part, prior)
            assert ctx.to_bytes(r.uniq, r.uniq_bytes) == eu
            assert ctx.to_bytes(r.fresh, r.fresh_bytes) == ef
        r0 += nr
    assert r0 == len(S.parse_records(data))


@pytest.mark.parametrize("world,rounds", [(2, 3), (3, 1), (1, 4)])
def test_partition_pieces_rounds_layout(ctx, world, rounds):
    """sg_dev_partition_bytes_pieces_rounds: world x rounds byte ranges, part q = g * rounds
    + p, laid out round-major (round p = parts (0, p) .. (world - 1, p) back to back, every
    round 16-byte aligned): each round is one contiguous all-to-all send buffer. Checked
    against route_parts per piece; padding between rounds never written."""
    import torch
    from swarm_amd.api import round_offsets
    from route_oracle import FakeCtx
    recs = shared_prefix_records(20_000, 21 + world)
    data = b"\n".join(recs) + b"\n"
    cuts = [0, len(data) // 3, len(data) // 3, len(data)]  # an empty piece in the middle
    cuts = [c if c in (0, len(data)) else data.index(b"\n", c) + 1 for c in cuts]
    d = dev(b"#" + data)
    pieces = [d[1 + a:1 + b] for a, b in zip(cuts, cuts[1:])]
    sp = sorted(random.Random(22).sample(recs, world * rounds - 1))
    cap = len(data) + len(pieces) + 16 * (rounds + 1)
    out = torch.full((cap + 64,), 0x55, dtype=torch.uint8, device=d.device)
    pb, pr = ctx.partition_bytes_pieces_rounds([(p.data_ptr(), p.numel()) for p in pieces], sp, rounds,
                                               out.data_ptr(), cap)
    got = out.cpu().numpy().tobytes()
    host = np.frombuffer(bytearray(data), dtype=np.uint8)
    want_buf = bytearray(b"\x55" * (cap + 64))
    wb = (np.frombuffer(want_buf, dtype=np.uint8))
    hp = [np.frombuffer(bytearray(data[a:b] or b"\0"), dtype=np.uint8) for a, b in zip(cuts, cuts[1:])]
    wpb, wpr = FakeCtx().partition_bytes_pieces_rounds([(h.ctypes.data, b - a) for h, (a, b) in
                                                        zip(hp, zip(cuts, cuts[1:]))], sp, rounds, wb.ctypes.data, cap)
    assert (pb, pr) == (wpb, wpr)
    assert got == bytes(want_buf)
    offs = round_offsets(pb, rounds)
    assert all(o % 16 == 0 for o in offs[:-1]) and offs[-1] <= cap
    del host


@pytest.mark.parametrize("world,rounds", [(2, 3), (3, 1), (1, 4)])
def test_partition_pieces_rounds_spans(ctx, world, rounds):
    """sg_dev_partition_bytes_pieces_rounds_spans (after sg_dev_partition_pieces_count): the
    round-major bytes of the plain call, plus every record's span (relative to its part) and
    key0 in the same round-major order, equal to the host restatement; then a round received
    from the parts of several sources (concatenated) is rebased to its own buffer with every
    record checked to end at a '\n', and a damaged copy of it is reported."""
    import torch
    from swarm_amd.api import round_offsets
    from route_oracle import FakeCtx
    recs = shared_prefix_records(20_000, 41 + world)
    data = b"\n".join(recs) + b"\n"
    cuts = [0, len(data) // 3, len(data) // 3, len(data)]  # an empty piece in the middle
    cuts = [c if c in (0, len(data)) else data.index(b"\n", c) + 1 for c in cuts]
    d = dev(b"#" + data)
    pieces = [d[1 + a:1 + b] for a, b in zip(cuts, cuts[1:])]
    plist = [(p.data_ptr(), p.numel()) for p in pieces]
    sp = sorted(random.Random(42).sample(recs, world * rounds - 1))
    cap = len(data) + len(pieces) + 16 * (rounds + 1)
    nrec = ctx.partition_pieces_count(plist)
    assert nrec == len(recs)
    out = torch.full((cap + 64,), 0x55, dtype=torch.uint8, device=d.device)
    dsp = torch.zeros(2 * nrec, dtype=torch.int32, device=d.device)
    dk = torch.zeros(nrec, dtype=torch.int64, device=d.device)
    pb, pr, ps = ctx.partition_bytes_pieces_rounds_spans(plist, sp, rounds, out.data_ptr(), cap, dsp.data_ptr(),
                                                         dk.data_ptr(), nrec)
    hp = [np.frombuffer(bytearray(data[a:b] or b"\0"), dtype=np.uint8) for a, b in zip(cuts, cuts[1:])]
    wb = np.full(cap + 64, 0x55, dtype=np.uint8)
    wsp = np.zeros(2 * nrec, dtype=np.uint32)
    wk = np.zeros(nrec, dtype=np.int64)
    wpb, wpr, wps = FakeCtx().partition_bytes_pieces_rounds_spans([(h.ctypes.data, b - a) for h, (a, b) in
                                                                   zip(hp, zip(cuts, cuts[1:]))], sp, rounds,
                                                                  wb.ctypes.data, cap, wsp.ctypes.data, wk.ctypes.data,
                                                                  nrec)
    assert (pb, pr, ps) == (wpb, wpr, wps)
    assert out.cpu().numpy().tobytes() == wb.tobytes()
    assert np.array_equal(dsp.cpu().numpy().view(np.uint32), wsp)
    assert np.array_equal(dk.cpu().numpy(), wk)
    # a receiver's round p: the sources' parts (g, p) concatenated, spans relative to each
    offs = round_offsets(pb, rounds)
    G = world
    for p in range(rounds):
        o, r0 = offs[p], sum(pr[g * rounds + q] for q in range(p) for g in range(G))
        n, nr = sum(pb[g * rounds + p] for g in range(G)), sum(pr[g * rounds + p] for g in range(G))
        if not nr:
            continue
        recv = out[o:o + n].clone()
        rsp = dsp[2 * r0:2 * (r0 + nr)].clone()
        seg_first, seg_off, fr, fo = [], [], 0, 0
        for g in range(G):
            seg_first.append(fr)
            seg_off.append(fo)
            fr += pr[g * rounds + p]
            fo += pb[g * rounds + p]
        assert ctx.rebase_spans(recv.data_ptr(), n, rsp.data_ptr(), nr, seg_first, seg_off) == 0
        part = recv.cpu().numpy().tobytes()
        assert [tuple(x) for x in rsp.cpu().numpy().view(np.uint32).reshape(-1, 2).tolist()] == S.record_spans(part)
        bad = out[o:o + n].clone()
        bad[n // 2:] = 0xAB  # the upper half never delivered
        rsp2 = dsp[2 * r0:2 * (r0 + nr)].clone()
        assert ctx.rebase_spans(bad.data_ptr(), n, rsp2.data_ptr(), nr, seg_first, seg_off) > 0


def test_stored_prior_aligned_parts(ctx):
    """dedup_diff_large(align_parts=True): every part's unique output starts 16-byte aligned
    ('\\n' padding: the buffer's records are still the sort -u records) and those parts,
    handed back as prior_parts, are read in place with results equal to the oracle."""
    from swarm_amd import sharded
    buf, ids = corpus.subdomains(300_000, seed=45)
    prior_raw = corpus.prior_of(ids).tobytes()
    pieces = sharded.split_at_newlines(dev(prior_raw), 1 << 20)
    sp = sharded.choose_splitters(sharded.sample_records(ctx, pieces, 256), 7)
    pu, _, pst = sharded.dedup_diff_large(ctx, pieces, (), splitters=sp, align_parts=True)
    parts = sharded.stored_parts(pu, pst)
    assert len(parts) == len(sp) + 1
    assert all(p is None or p.data_ptr() % 16 == 0 for p in parts)
    assert S.serialize(S.parse_records(pu.cpu().numpy().tobytes())) == S.dedup(prior_raw)
    cur = sharded.split_at_newlines(dev(buf.tobytes()), 1 << 20)
    u, f, _ = sharded.dedup_diff_large(ctx, cur, (), splitters=sp, prior_parts=parts)
    eu, ef = S.dedup_diff(buf.tobytes(), prior_raw)
    assert u.cpu().numpy().tobytes() == eu and f.cpu().numpy().tobytes() == ef


def test_private_stream_last_part_without_prior():
    """on a context with its own stream, a part with no prior records copies its
    unique output into the caller's new-record buffer; the call must not return before that
    copy has landed (torch reads or frees the buffer next)."""
    import swarm_amd
    import torch
    from swarm_amd import sharded
    c = swarm_amd.Context(0)
    try:
        assert not c.on_torch_stream()
        buf, ids = corpus.subdomains(300_000, seed=46)
        cur = buf.tobytes()
        # the prior only holds records below "m": every part above has no prior records
        prior = b"".join(r + b"\n" for r in S.parse_records(corpus.prior_of(ids).tobytes()) if r < b"m")
        for _ in range(3):
            u, f, st = sharded.dedup_diff_large(c, sharded.split_at_newlines(dev(cur), 1 << 20), [dev(prior)],
                                                splitters=[b"f", b"m", b"t"])
            fh = f.cpu().numpy().tobytes()  # read on torch's stream right away
            del f
            torch.empty(len(fh) + 4096, dtype=torch.uint8, device="cuda").fill_(0)  # reuse freed blocks
            eu, ef = S.dedup_diff(cur, prior)
            assert u.cpu().numpy().tobytes() == eu and fh == ef
    finally:
        c.close()
