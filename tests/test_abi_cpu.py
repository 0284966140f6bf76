"""C-ABI checks that need no GPU: the library loads, exports every symbol the header
declares, reports no device cleanly, and its host-side hash matches the restatement."""
import os
import re

import pytest

from conftest import ROOT
from hash_oracle import hash64 as py_hash64


def header_functions():
    txt = open(os.path.join(ROOT, "include", "swarmgpu.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(sg_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    from swarm_amd import _abi
    names = header_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(_abi.lib, n), n
    assert set(names) == set(_abi.EXPORTS)


def test_version_and_device_count():
    from swarm_amd import _abi
    assert _abi.lib.sg_version() >= 10000
    import ctypes
    n = ctypes.c_int(-1)
    assert _abi.lib.sg_device_count(ctypes.byref(n)) == 0
    assert n.value >= 0


@pytest.mark.parametrize("rec", [b"", b"a", b"abcdefg", b"abcdefgh", b"abcdefghi",
                                 b"x.target12.com", bytes(range(256)), b"\x00" * 17])
def test_hash64_host_matches_restatement(rec):
    from swarm_amd import hash64
    assert hash64(rec) == py_hash64(rec)


def test_span_sum_host_matches_restatement():
    """sg_span_sum (the handover checksum the partition returns and the dedup checks) equals
    its restatement in route_oracle, keys with the top bit set included; order-free."""
    import random
    import numpy as np
    from route_oracle import key0, span_sum as py_span_sum
    from swarm_amd.api import span_sum
    rng = random.Random(3)
    recs = [bytes(rng.randrange(256) for _ in range(rng.randrange(1, 40))) for _ in range(500)]
    recs = [r.replace(b"\n", b"x") for r in recs] + [b"\xff" * 9, b"a"]
    spans, keys, off = [], [], 0
    for r in recs:
        spans.append((off, off + len(r)))
        keys.append(key0(r))
        off += len(r) + 1
    sp = np.array(spans, dtype=np.uint32)
    k = np.array(keys, dtype=np.uint64)
    want = py_span_sum(spans, keys)
    assert span_sum(sp, k) == want
    perm = np.random.default_rng(4).permutation(len(recs))
    assert span_sum(sp[perm], k[perm]) == want
    assert span_sum(np.zeros((0, 2), np.uint32), np.zeros(0, np.uint64)) == 0
    k2 = k.copy()
    k2[7] ^= np.uint64(1)
    assert span_sum(sp, k2) != want


def test_no_gpu_fails_loudly_not_silently():
    """Without a device the product path raises instead of computing on the CPU."""
    from swarm_amd import device_count, dedup
    from swarm_amd._abi import SGError
    if device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(SGError):
        dedup(b"b\na\n")


def test_choose_splitters_quantiles():
    import numpy as np
    from swarm_amd import sharded
    s = np.array([5, 1, 9, 3, 7, 0xFFFFFFFFFFFFFFFF], dtype=np.uint64)
    sp = sharded.choose_splitters(s, 3)
    assert sp.tolist() == [3, 7]
    assert sharded.choose_splitters(s, 1).size == 0
    assert np.all(np.diff(sharded.choose_splitters(np.arange(1000, dtype=np.uint64), 17).astype(np.int64)) >= 0)


def test_choose_byte_splitters():
    from swarm_amd import sharded
    samples = [b"m", b"a", b"zz", b"b", b"ab", b"ab", b"\x00", b"\xff"]
    sp = sharded.choose_splitters(samples, 4)
    assert sp == sorted(sp) and len(sp) == 3
    assert sharded.choose_splitters([], 4) == [] and sharded.choose_splitters(samples, 1) == []
    assert sharded.n_splitters(sp) == 3


def test_part_overflow_message_names_the_limit():
    from swarm_amd import sharded
    msg = sharded.part_overflow_message([b"a"], 1, 10, 20)
    assert "share their first 64 bytes" in msg and str(sharded.PART_LIMIT) in msg


def test_shard_bounds_newline_aligned():
    import numpy as np
    from swarm_amd.distributed import shard_bounds
    data = b"a\nbb\n\nccc\nd"
    for world in (1, 2, 3, 5, 20):
        cuts = shard_bounds(np.frombuffer(data, dtype=np.uint8), world)
        assert cuts[0] == 0 and cuts[-1] == len(data) and len(cuts) == world + 1
        assert all(b >= a for a, b in zip(cuts, cuts[1:]))
        assert all(data[c - 1:c] == b"\n" for c in cuts[1:-1] if 0 < c < len(data))
        assert b"".join(data[a:b] for a, b in zip(cuts, cuts[1:])) == data


def test_ip_pool_is_distinct_10_slash_8():
    import torch
    from swarm_amd import corpus
    mat, lens = corpus.ip_pool_torch(5000, seed=5, device="cpu")
    ips = {bytes(mat[i, :lens[i]].tolist()) for i in range(5000)}
    assert len(ips) == 5000
    assert all(ip.startswith(b"10.") and ip.count(b".") == 3 for ip in ips)
    assert all(0 <= int(o) <= 255 for ip in list(ips)[:500] for o in ip.split(b"."))
