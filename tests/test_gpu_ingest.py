"""GPU parity for streamed merge ingestion (§8(f) row 4): pieces appended in A5 key order
land in HBM byte-identical to the reference's /raw concatenation, and dedup/diff on the
ingested body equals the oracle."""
import random

import numpy as np
import pytest

from conftest import b64d, load_golden
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


def pieces(rng, body, max_piece):
    out, i = [], 0
    while i < len(body):
        k = rng.randint(0, max_piece)
        out.append(body[i:i + k])
        i += k
    return out


@pytest.mark.parametrize("hint", [0, 1])
def test_reference_raw_vectors_streamed(ctx, hint):
    import swarm_amd
    from swarm_amd import hooks
    rng = random.Random(3)
    for case in load_golden("reference_vectors.json")["a5_merge"]:
        objs = {"%s/output/%s" % (case["scan_id"], k): b64d(v) for k, v in case["objects"].items()}
        want = b64d(case["raw"])
        order = hooks.merge_keys(objs.keys(), case["scan_id"])
        with swarm_amd.Ingest(ctx, len(want) if hint else 0) as ing:
            for k in order:
                for p in pieces(rng, objs[k], 7):
                    ing.append(p)
            d, n = ing.finish()
            assert ctx.to_bytes(d, n) == want


def test_large_streamed_merge_dedup_diff(ctx):
    import swarm_amd
    from swarm_amd import hooks
    rng = random.Random(4)
    body = corpus.subdomains(1_500_000, seed=21)[0].tobytes()  # ~38 MB: several staging buffers
    chunks = corpus.chunk_layout(np.frombuffer(body, dtype=np.uint8), 23)
    objs = {"s/output/chunk_%d.txt" % i: c.tobytes() for i, c in enumerate(chunks)}
    order = hooks.merge_keys(objs.keys(), "s")
    want = b"".join(objs[k] for k in order)
    prior = S.dedup(corpus.subdomains(300_000, seed=22)[0].tobytes())
    uniq, fresh = hooks.raw_stream_dedup_diff(ctx, objs.keys(), "s", lambda k: pieces(rng, objs[k], 3 << 20), prior)
    assert uniq == S.dedup(want)
    assert fresh == S.diff(want, prior)
    # growth path without a size hint, tiny and huge pieces
    with swarm_amd.Ingest(ctx) as ing:
        for k in order:
            for p in pieces(rng, objs[k], 20 << 20) + [b""]:
                ing.append(p)
        d, n = ing.finish()
        assert n == len(want) and ctx.to_bytes(d, n) == want


def test_empty_ingest(ctx):
    import swarm_amd
    with swarm_amd.Ingest(ctx) as ing:
        assert ing.finish()[1] == 0
        assert ing.dedup_diff(None) == (b"", b"")


def test_byte_by_byte_pieces(ctx):
    import swarm_amd
    body = b"".join(b"r%d.example.com\n" % (i % 977) for i in range(5000))
    with swarm_amd.Ingest(ctx) as ing:
        for i in range(len(body)):
            ing.append(body[i:i + 1])
        u, f = ing.dedup_diff(b"r1.example.com\n")
    eu, ef = S.dedup_diff(body, b"r1.example.com\n")
    assert u == eu and f == ef
