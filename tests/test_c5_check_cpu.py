"""The C5 full-size checker (oracle/c5_check.py) pinned against the oracle on CPU tensors:
its id-level expectation must accept the oracle's own sort -u / comm -13 output of the
rendered records, and reject a dropped record, a duplicated one and a swapped pair. The pool
carries duplicated host names, so the exact host canonicalisation is exercised."""
import numpy as np
import torch

from oracle import c5_check as C
from oracle import semantics as S


def _setup():
    from swarm_amd import corpus
    mat, lens = corpus.host_pool_torch(3000, seed=5, device="cpu")
    # hosts 3000..3099 render the same names as hosts 0..99 (and 3100 as 7)
    mat = torch.cat([mat, mat[:100], mat[7:8]])
    lens = torch.cat([lens, lens[:100], lens[7:8]])
    pool = (mat, lens)
    K = 4
    U = mat.shape[0] * K
    args_c = (20_000, 0, U, 1, 7_000)
    args_p = (15_000, U // 10, U, 2, 7_000)
    cur = corpus.hostport_pieces(pool, *args_c, ports_per_host=K)
    prior = corpus.hostport_pieces(pool, *args_p, ports_per_host=K)
    cb = b"".join(p.numpy().tobytes() for p in cur)
    pb = S.dedup(b"".join(p.numpy().tobytes() for p in prior))
    ids = lambda a: corpus.hostport_ids(*a, device="cpu")  # noqa: E731
    return pool, K, ids(args_c), ids(args_p), cb, pb, (lambda: ids(args_c)), (lambda: ids(args_p))


def _t(b):
    return torch.from_numpy(np.frombuffer(b, dtype=np.uint8).copy())


def test_c5_checker_accepts_oracle_output():
    pool, K, ci, pi, cb, pb, _, _ = _setup()
    eu, ef = S.dedup_diff(cb, pb)
    r = C.check_step(pool, K, K, ci, pi, _t(eu), _t(ef))
    assert r["full_size_bit_exact"], r
    assert r["expected_unique"] == len(S.parse_records(eu))
    assert r["expected_new"] == len(S.parse_records(ef))


def test_c5_checker_rejects_wrong_outputs():
    pool, K, _, _, cb, pb, ci, pi = _setup()
    eu, ef = S.dedup_diff(cb, pb)
    recs = S.parse_records(eu)
    dropped = S.serialize(recs[:5] + recs[6:])
    duped = S.serialize(recs[:5] + [recs[5]] + recs[5:-1])
    swapped = S.serialize(recs[:5] + [recs[6], recs[5]] + recs[7:])
    for bad in (dropped, duped, swapped):
        assert not C.check_step(pool, K, K, ci(), pi(), _t(bad), _t(ef))["full_size_bit_exact"]
    fr = S.parse_records(ef)
    assert not C.check_step(pool, K, K, ci(), pi(), _t(eu), _t(S.serialize(fr[1:])))["full_size_bit_exact"]
