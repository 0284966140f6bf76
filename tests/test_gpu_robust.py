"""GPU robustness of the dedup/diff on parts of pathological content.

Round 4's 1-rank RCCL rounds step handed the dedup a 1.65 GB received part whose upper
bytes RCCL had not delivered (the all-to-all of > 1 GiB messages is wrong on this image's
RCCL; tools/rccl_probe.py detail). Whatever bytes a part holds, the library must return the
exact `sort -u` / `comm -13` result of those bytes, never touch memory outside its buffers.
These cases feed `sg_dev_dedup_diff_into` (the entry the rounds step calls) parts that no
scanner emits: one giant record, NUL runs with and without newlines, random bytes of every
value, a zero-filled tail after valid records, only newlines, 1-byte records, and groups of
identical long records (the refinement rounds). Expected results come from the oracle
(`oracle/semantics.py`, few records) or from numpy (many tiny records)."""
import random

import numpy as np
import pytest

from oracle import semantics as S

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    import torch
    import swarm_amd
    assert swarm_amd.device_count() > 0, "GPU tests need a HIP device"
    ctx = swarm_amd.Context(0, torch.cuda.current_stream().cuda_stream)
    yield torch, ctx
    ctx.close()


def run_into(torch, ctx, cur: bytes, prior: bytes = b""):
    """dedup_diff_into with caller outputs (the rounds step's call), outputs copied back."""
    d_cur = torch.frombuffer(bytearray(cur), dtype=torch.uint8).cuda() if cur else torch.zeros(16, dtype=torch.uint8,
                                                                                               device="cuda")
    d_pri = torch.frombuffer(bytearray(prior), dtype=torch.uint8).cuda() if prior else None
    n = len(cur)
    ou = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    of = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    r = ctx.dedup_diff_into(d_cur.data_ptr(), n, d_pri.data_ptr() if prior else 0, len(prior),
                            ou.data_ptr(), ou.numel(), of.data_ptr(), of.numel())
    torch.cuda.synchronize()
    u = bytes(ou[:r.uniq_bytes].cpu().numpy())
    f = bytes(of[:r.fresh_bytes].cpu().numpy())
    return r, u, f


def check(torch, ctx, cur: bytes, prior: bytes = b""):
    r, u, f = run_into(torch, ctx, cur, prior)
    eu, ef = S.dedup_diff(cur, prior)
    assert u == eu
    assert f == ef
    assert r.uniq_records == eu.count(b"\n") and r.fresh_records == ef.count(b"\n")


MB = 1 << 20


def _rand_bytes(seed, n, exclude_nl=False):
    rng = np.random.default_rng(seed)
    a = rng.integers(0, 256, n, dtype=np.uint8)
    if exclude_nl:
        a[a == 0x0A] = 0x0B
    return a.tobytes()


@pytest.mark.parametrize("seg_all", ["0", "2"])
@pytest.mark.parametrize("case", ["nul_no_newline", "random_no_newline", "nul_no_newline_unaligned"])
def test_one_giant_record(env, monkeypatch, case, seg_all):
    torch, ctx = env
    monkeypatch.setenv("SG_SEG_ALL", seg_all)
    if case == "nul_no_newline":
        cur = bytes(48 * MB)
    elif case == "random_no_newline":
        cur = _rand_bytes(1, 48 * MB, exclude_nl=True)
    else:
        cur = bytes(48 * MB - 13)
    check(torch, ctx, cur)
    check(torch, ctx, cur, prior=cur + b"\n")   # the same record in the prior: nothing new
    check(torch, ctx, cur, prior=b"a\nb\n")


@pytest.mark.parametrize("tail", ["zeros", "garbage"])
def test_valid_records_then_stale_tail(env, tail):
    """A part whose lower bytes are records and whose upper bytes were never delivered."""
    torch, ctx = env
    rng = random.Random(5)
    recs = [b"h%d.example%d.com:%d" % (rng.randrange(50_000), rng.randrange(9), rng.choice((80, 443, 8080)))
            for _ in range(600_000)]
    head = b"\n".join(recs)  # (cut inside the last record: the tail continues it)
    if tail == "zeros":
        cur = head + bytes(24 * MB)
    else:
        g = bytearray(_rand_bytes(2, 24 * MB))
        cur = head + bytes(g)
    check(torch, ctx, cur)
    check(torch, ctx, cur, prior=S.dedup(head[: len(head) // 2]))


@pytest.mark.parametrize("seg_all", ["0", "2"])
def test_giant_duplicates_and_small(env, monkeypatch, seg_all):
    """Three copies of a 6 MB record among small ones: the byte compares of equal giants."""
    torch, ctx = env
    monkeypatch.setenv("SG_SEG_ALL", seg_all)
    big = _rand_bytes(3, 6 * MB, exclude_nl=True)
    big2 = big[:-1] + bytes([big[-1] ^ 1])  # differs in its last byte
    rng = random.Random(3)
    small = [bytes(rng.choice(b"abc\x00\xff") for _ in range(rng.randint(1, 30))) for _ in range(20_000)]
    recs = small[:5000] + [big] + small[5000:10000] + [big, big2] + small[10000:] + [big]
    cur = b"\n".join(recs) + b"\n"
    check(torch, ctx, cur)
    check(torch, ctx, cur, prior=S.dedup(big + b"\n" + b"\n".join(small[:7000])))


@pytest.mark.parametrize("reclen", [300, 3000])
def test_identical_long_records_refinement(env, reclen):
    """> 64 copies of the same long record (refinement rounds until the records end) next to
    near-copies that differ at the end."""
    torch, ctx = env
    rng = random.Random(reclen)
    base = bytes(rng.choice(b"xyz") for _ in range(reclen))
    near = [base[:-1] + bytes([c]) for c in b"ABCDEFGHIJ"]
    recs = [base] * 200 + near * 30 + [base[: reclen // 2]] * 70
    rng.shuffle(recs)
    cur = b"\n".join(recs) + b"\n"
    check(torch, ctx, cur)
    check(torch, ctx, cur, prior=S.dedup(b"\n".join(near[:5]) + b"\n"))


def test_only_newlines(env):
    torch, ctx = env
    r, u, f = run_into(torch, ctx, b"\n" * (32 * MB))
    assert r.in_records == 0 and u == b"" and f == b""


@pytest.mark.parametrize("seg_all", ["0", "2"])
def test_many_one_byte_records(env, monkeypatch, seg_all):
    """16M records of one byte (every value but '\\n'): 255 unique, huge duplicate runs."""
    torch, ctx = env
    monkeypatch.setenv("SG_SEG_ALL", seg_all)
    rng = np.random.default_rng(7)
    v = rng.integers(0, 255, 16 * MB, dtype=np.uint8)
    v[v >= 0x0A] += 1  # 0..255 without 0x0a
    a = np.empty(2 * v.size, dtype=np.uint8)
    a[0::2] = v
    a[1::2] = 0x0A
    cur = a.tobytes()
    prior = b"".join(bytes([x]) + b"\n" for x in range(0, 256, 3) if x != 0x0A)
    r, u, f = run_into(torch, ctx, cur, prior)
    want = sorted(set(v.tolist()))
    assert u == b"".join(bytes([x]) + b"\n" for x in want)
    assert f == b"".join(bytes([x]) + b"\n" for x in want if x % 3)
    assert r.in_records == v.size


def test_nul_records_of_many_lengths(env):
    """Records of NUL bytes only (1..40 long): every record is a repeat of one of 40."""
    torch, ctx = env
    rng = np.random.default_rng(9)
    lens = rng.integers(1, 41, 1_000_000)
    cur = b"\n".join(bytes(int(k)) for k in lens) + b"\n"
    prior = b"".join(bytes(k) + b"\n" for k in range(1, 41, 2))
    r, u, f = run_into(torch, ctx, cur, prior)
    present = sorted(set(lens.tolist()))
    assert u == b"".join(bytes(k) + b"\n" for k in present)
    assert f == b"".join(bytes(k) + b"\n" for k in present if k % 2 == 0)


@pytest.mark.parametrize("seed", [11, 12])
def test_uniform_random_bytes(env, seed):
    """64 MB of uniformly random bytes (a '\\n' every ~256 bytes on average, NUL, CR, 0xff)."""
    torch, ctx = env
    cur = _rand_bytes(seed, 64 * MB)
    check(torch, ctx, cur, prior=S.dedup(cur[: 8 * MB]))


@pytest.mark.parametrize("seg_all", ["1", "2"])
def test_large_part_with_stale_record_tail(env, monkeypatch, seg_all):
    """Round 4's faulting shape with NON-zero stale bytes: 1.65 GB = 1.05 GB of
    host:port records + 0.6 GB of another host:port buffer's bytes, starting mid-record and
    cut mid-record (what a caching allocator's reused block holds), plus a prior. The dedup
    must not fault, and its result must equal the sort -u / comm -13 of the union of the two
    halves' records, computed by deduping each half on its own and then their outputs
    together (and the diff against the prior the same way)."""
    torch, ctx = env
    monkeypatch.setenv("SG_SEG_ALL", seg_all)
    from swarm_amd import corpus
    pool = corpus.host_pool_torch(8_000_000, seed=71)
    (head,) = corpus.hostport_pieces(pool, 33_500_000, 0, 32_000_000, seed=72, per_piece=33_500_000, ports_per_host=4)
    (old,) = corpus.hostport_pieces(pool, 20_000_000, 0, 32_000_000, seed=73, per_piece=20_000_000, ports_per_host=4)
    (pri,) = corpus.hostport_pieces(pool, 4_000_000, 0, 32_000_000, seed=74, per_piece=4_000_000, ports_per_host=4)
    del pool
    a = 17
    tail = old[a:a + min(600 * MB, old.numel() - a - 5)]  # starts and ends inside records
    assert int(tail[0]) != 0x0A and int(tail[-1]) != 0x0A
    d = torch.cat([head, tail])
    n = d.numel()

    def run(buf, prior):
        ou = torch.empty(buf.numel() + 64, dtype=torch.uint8, device="cuda")
        of = torch.empty(buf.numel() + 64, dtype=torch.uint8, device="cuda")
        r = ctx.dedup_diff_into(buf.data_ptr(), buf.numel(), prior.data_ptr(), prior.numel(), ou.data_ptr(), ou.numel(),
                                of.data_ptr(), of.numel())
        torch.cuda.synchronize()
        return r, ou[:r.uniq_bytes], of[:r.fresh_bytes]

    r, u, f = run(d, pri)
    rh, uh, fh = run(head, pri)
    rt, ut, ft = run(tail.clone(), pri)
    assert r.in_records == rh.in_records + rt.in_records
    _, u2, _ = run(torch.cat([uh, ut]), pri[:0])
    _, f2, _ = run(torch.cat([fh, ft]), pri[:0])
    assert torch.equal(u, u2)
    assert torch.equal(f, f2)
    assert int(u[-1]) == 10 and r.uniq_records < r.in_records
    del d, u, f, u2, f2, head, tail, old
    torch.cuda.empty_cache()


def test_large_part_with_zero_tail(env):
    """The shape of round 4's faulting part: 1.65 GB = 1.05 GB of records (a 105 MB subdomain
    buffer repeated 10 times) + 0.6 GB that stayed zero. Expected: the NUL-only record first
    (byte 0 sorts below every subdomain), then sort -u of the base buffer (numpy reference)."""
    torch, ctx = env
    from swarm_amd import corpus
    base, ids = corpus.subdomains(4_000_000, seed=21)
    urows = corpus.sorted_unique_rows(ids)
    want_u = corpus.serialize_rows(urows).tobytes()
    nb = base.size
    reps = 10
    ztail = 600 * MB
    n = nb * reps + ztail
    d = torch.zeros(n, dtype=torch.uint8, device="cuda")
    db = torch.from_numpy(base).cuda()
    for k in range(reps):
        d[k * nb:(k + 1) * nb] = db
    del db
    ou = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    r = ctx.dedup_diff_into(d.data_ptr(), n, 0, 0, ou.data_ptr(), ou.numel(), 0, 0)
    torch.cuda.synchronize()
    assert r.in_records == 4_000_000 * reps + 1
    assert r.uniq_records == urows.size + 1
    head = ou[:ztail + 1].cpu().numpy()
    assert not head[:ztail].any() and head[ztail] == 0x0A
    got = bytes(ou[ztail + 1:r.uniq_bytes].cpu().numpy())
    assert got == want_u
    del d, ou
    torch.cuda.empty_cache()
