"""The handed-over parse is checked before any kernel reads through it.

sg_dev_dedup_diff_spans_into dedups a part (or an exchange round) with the spans and keys the
routing pass wrote, instead of parsing it again. Those arrive through the same all-to-alls as
the bytes, so a record's span may come back out of range, reversed or shifted, and its key
changed. The library checks them in its common-prefix scan, before the first byte is read
through a span: the records must tile the buffer, their span_mix checksum must equal the
producer's (sg_span_sum), and every 256th record must end at a '\n' and carry its own key. A
mismatch is SG_E_CORRUPT — never a fault, never a wrong success. Also: sg_dev_rebase_spans
with more sources than one launch's table, offsets and empty sources, pinned to
the host parse."""
import random

import numpy as np
import pytest

from oracle import semantics as S
from route_oracle import key0, span_sum as py_span_sum

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    import torch
    import swarm_amd
    assert swarm_amd.device_count() > 0, "GPU tests need a HIP device"
    ctx = swarm_amd.Context(0, torch.cuda.current_stream().cuda_stream)
    yield torch, ctx
    ctx.close()


@pytest.fixture(scope="module")
def big_part(env):
    """One 50M-record host:port part (~1.6 GB, C5's record shape) with the parse the routing
    pass hands over (one part: no splitters), copied into tensors the tests may damage, and a
    prior of 5M of its records."""
    torch, ctx = env
    from swarm_amd import corpus
    n_rec = 50_000_000
    pool = corpus.host_pool_torch(4_000_000, seed=61)
    (cur,) = corpus.hostport_pieces(pool, n_rec, 0, 16_000_000, seed=62, per_piece=n_rec, ports_per_host=4)
    (pri,) = corpus.hostport_pieces(pool, 5_000_000, 0, 16_000_000, seed=63, per_piece=5_000_000, ports_per_host=4)
    n = cur.numel()
    out = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    ctx.fence_in()
    pb, pr, dsp, dkp, ps = ctx.partition_bytes_pieces_spans([(cur.data_ptr(), n)], [], out.data_ptr(), out.numel())
    assert pb == [n] and pr == [n_rec]
    sp = torch.empty(2 * n_rec, dtype=torch.int32, device="cuda")
    kk = torch.empty(n_rec, dtype=torch.int64, device="cuda")
    ctx.memcpy(sp.data_ptr(), dsp, 8 * n_rec)
    ctx.memcpy(kk.data_ptr(), dkp, 8 * n_rec)
    ctx.sync()
    del pool
    yield out[:n], sp, kk, ps[0], pri
    del out, sp, kk, pri, cur


def _into(torch, ctx, buf, sp, kk, nr, ssum, pri):
    """spans_into on copies of the parse (the call sorts the handed-over arrays in place)."""
    sp, kk = sp.clone(), kk.clone()
    n = buf.numel()
    ou = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    of = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    r = ctx.dedup_diff_spans_into(buf.data_ptr(), n, sp.data_ptr(), kk.data_ptr(), nr, ssum, pri.data_ptr(),
                                  pri.numel(), ou.data_ptr(), ou.numel(), of.data_ptr(), of.numel())
    torch.cuda.synchronize()
    return r, ou[:r.uniq_bytes], of[:r.fresh_bytes]


def test_big_part_intact_equals_own_parse(env, big_part):
    """The intact handover: the checksum the partition returned matches, and the result is
    byte-identical to the dedup that parses the part itself."""
    torch, ctx = env
    buf, sp, kk, ssum, pri = big_part
    nr = kk.numel()
    r, u, f = _into(torch, ctx, buf, sp, kk, nr, ssum, pri)
    n = buf.numel()
    ou = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    of = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    r2 = ctx.dedup_diff_into(buf.data_ptr(), n, pri.data_ptr(), pri.numel(), ou.data_ptr(), ou.numel(),
                             of.data_ptr(), of.numel())
    torch.cuda.synchronize()
    assert r.in_records == nr == r2.in_records
    assert (r.uniq_records, r.fresh_records) == (r2.uniq_records, r2.fresh_records)
    assert torch.equal(u, ou[:r2.uniq_bytes]) and torch.equal(f, of[:r2.fresh_bytes])
    # sort -u properties at full size: strictly increasing records, each a record of the input
    assert int(u[-1]) == 10 and r.uniq_records < nr


DAMAGE = ["end_out_of_range", "reversed", "wrong_key", "shifted_boundary", "start_past_end_of_buffer",
          "first_record_out_of_range", "dropped_tail", "wrong_checksum"]


@pytest.mark.parametrize("damage", DAMAGE)
def test_big_part_damaged_parse_is_rejected(env, big_part, damage):
    """One damaged record in the middle of the 50M-record part (outside the rebase's sampled
    ends, and not a multiple of the sampled stride), or a wrong checksum: SG_E_CORRUPT, no
    fault; the context works afterwards."""
    torch, ctx = env
    from swarm_amd._abi import SGError, SG_E_CORRUPT
    buf, sp0, kk0, ssum, pri = big_part
    nr = kk0.numel()
    n = buf.numel()
    sp, kk = sp0.clone(), kk0.clone()
    m = nr // 2 + 12_345
    v = sp.view(-1, 2)
    if damage == "end_out_of_range":
        v[m, 1] = n + 4096
    elif damage == "reversed":
        v[m] = v[m].flip(0).clone()
    elif damage == "wrong_key":
        kk[m] ^= 1 << 40
    elif damage == "shifted_boundary":  # still tiles the buffer: only the checksum sees it
        v[m, 1] += 1
        v[m + 1, 0] += 1
    elif damage == "start_past_end_of_buffer":
        v[m, 0] = -16  # 0xfffffff0 as uint32
    elif damage == "first_record_out_of_range":  # the common-prefix scan's reference record
        v[0, 1] = n + 100_000
    elif damage == "dropped_tail":
        v[nr - 1, 1] -= 1
    bad_sum = (ssum ^ 1) if damage == "wrong_checksum" else ssum
    with pytest.raises(SGError) as ei:
        _into(torch, ctx, buf, sp, kk, nr, bad_sum, pri)
    assert ei.value.rc == SG_E_CORRUPT, str(ei.value)
    # the context is intact: the undamaged handover still gives the right answer
    r, _, _ = _into(torch, ctx, buf, sp0, kk0, nr, ssum, pri)
    assert r.in_records == nr


def test_records_handed_over_must_tile_the_buffer(env):
    """Small cases: a parse of a buffer with a blank line (spans that skip bytes), no records
    for non-empty bytes, and a handover whose last record stops before the buffer's end are
    all rejected; an intact one equals the oracle."""
    torch, ctx = env
    from swarm_amd._abi import SGError, SG_E_CORRUPT
    recs = [b"b.example.com", b"a", b"x" * 70, b"a", b"\xffz"]
    data = b"\n".join(recs) + b"\n"
    spans, keys, off = [], [], 0
    for r in recs:
        spans.append((off, off + len(r)))
        keys.append(key0(r))
        off += len(r) + 1
    d = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()

    def call(buf, sp, kk, ssum, n=None):
        t_sp = torch.tensor(np.array(sp, dtype=np.uint32).view(np.int32).reshape(-1) if sp else [0, 0],
                            dtype=torch.int32, device="cuda")
        t_k = torch.tensor(np.array(kk, dtype=np.uint64).view(np.int64) if kk else [0], dtype=torch.int64,
                           device="cuda")
        nb = buf.numel() if n is None else n
        ou = torch.empty(nb + 64, dtype=torch.uint8, device="cuda")
        r = ctx.dedup_diff_spans_into(buf.data_ptr(), nb, t_sp.data_ptr(), t_k.data_ptr(), len(sp), ssum, 0, 0,
                                      ou.data_ptr(), ou.numel(), 0, 0)
        torch.cuda.synchronize()
        return bytes(ou[:r.uniq_bytes].cpu().numpy())

    assert call(d, spans, keys, py_span_sum(spans, keys)) == S.dedup(data)
    # a blank line inside: the records no longer tile the buffer
    data2 = data.replace(b"\na\n", b"\n\na\n", 1)
    d2 = torch.frombuffer(bytearray(data2), dtype=torch.uint8).cuda()
    sp2 = [(a + (1 if i >= 1 else 0), e + (1 if i >= 1 else 0)) for i, (a, e) in enumerate(spans)]
    for args in [(d2, sp2, keys, py_span_sum(sp2, keys)), (d, [], [], 0), (d, spans, keys, py_span_sum(spans, keys),
                                                                            len(data) + 1)]:
        with pytest.raises(SGError) as ei:
            call(*args)
        assert ei.value.rc == SG_E_CORRUPT


@pytest.mark.parametrize("nsrc", [3, 70, 130])
def test_rebase_many_sources_pinned_to_host_parse(env, nsrc):
    """An exchange round from nsrc sources (more than one launch's SG_REBASE_SEGS table, some
    sources empty, non-zero offsets): rebased spans equal the host parse of the round, and the
    round deduped with them (checksum = the sources' sums) equals the oracle."""
    torch, ctx = env
    rng = random.Random(nsrc)
    msgs, sps, kks = [], [], []
    for s in range(nsrc):
        k = 0 if s % 7 == 3 else rng.randrange(1, 300)
        recs = [b"h%d.t%d.com:%d" % (rng.randrange(5000), s % 5, rng.choice([22, 80, 443])) for _ in range(k)]
        msg = b"".join(r + b"\n" for r in recs)
        msgs.append(msg)
        sps.append(S.record_spans(msg))
        kks.append([key0(msg[a:e]) for a, e in sps[-1]])
    data = b"".join(msgs)
    seg_first, seg_off, fr, fo = [], [], 0, 0
    for m, sp in zip(msgs, sps):
        seg_first.append(fr)
        seg_off.append(fo)
        fr += len(sp)
        fo += len(m)
    flat_sp = np.array([x for sp in sps for x in sp], dtype=np.uint32).reshape(-1)
    flat_k = np.array([x for kk in kks for x in kk], dtype=np.uint64)
    d = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    t_sp = torch.from_numpy(flat_sp.view(np.int32).copy()).cuda()
    t_k = torch.from_numpy(flat_k.view(np.int64).copy()).cuda()
    nr = len(flat_k)
    assert ctx.rebase_spans(d.data_ptr(), len(data), t_sp.data_ptr(), nr, seg_first, seg_off) == 0
    got = [tuple(x) for x in t_sp.cpu().numpy().view(np.uint32).reshape(-1, 2).tolist()]
    assert got == S.record_spans(data)
    ssum = sum(py_span_sum(sp, kk) for sp, kk in zip(sps, kks)) & ((1 << 64) - 1)
    ou = torch.empty(len(data) + 64, dtype=torch.uint8, device="cuda")
    r = ctx.dedup_diff_spans_into(d.data_ptr(), len(data), t_sp.data_ptr(), t_k.data_ptr(), nr, ssum, 0, 0,
                                  ou.data_ptr(), ou.numel(), 0, 0)
    torch.cuda.synchronize()
    assert bytes(ou[:r.uniq_bytes].cpu().numpy()) == S.dedup(data)
    # a source whose message arrived short: its last records no longer end at a '\n'
    if nsrc > 3:
        bad = d.clone()
        s = max(range(nsrc), key=lambda j: len(msgs[j]))
        a = seg_off[s]
        bad[a + len(msgs[s]) // 2:a + len(msgs[s])] = 0
        t_sp2 = torch.from_numpy(flat_sp.view(np.int32).copy()).cuda()
        assert ctx.rebase_spans(bad.data_ptr(), len(data), t_sp2.data_ptr(), nr, seg_first, seg_off) > 0
