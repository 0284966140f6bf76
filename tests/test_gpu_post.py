"""GPU runs of the drop-in pieces around the hot path: the worker post-step module entry
(`python -m swarm_amd.post`, one subprocess per op as a module command would run it), the
hooks (worker postprocess, /raw unique, completion dedup+diff with the reference's UTF-8
behaviour), and re-entrancy of the host API from concurrent threads (Flask serves requests
on threads, flask/app.py threaded=True)."""
import os
import random
import subprocess
import sys
import threading

import numpy as np
import pytest

from conftest import ROOT
from oracle import semantics as S
from swarm_amd import corpus

pytestmark = pytest.mark.gpu


def run_post(*args):
    p = subprocess.run([sys.executable, "-m", "swarm_amd.post"] + [str(a) for a in args], cwd=ROOT,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=120)
    return p.returncode, p.stderr.decode()


def test_post_match_literal(tmp_path):
    sigs = [b"admin", b"Login", b"nginx/1.18"]
    rows = corpus.httpx_pool(sigs, 500, 0.2, seed=3)
    data = b"\n".join(random.Random(1).choice(rows) for _ in range(3000)) + b"\n\n"
    (tmp_path / "s.txt").write_bytes(b"\n".join(sigs) + b"\n")
    (tmp_path / "in").write_bytes(data)
    rc, err = run_post("match", "--literal", tmp_path / "s.txt", tmp_path / "in", tmp_path / "out")
    assert rc == 0, err
    assert (tmp_path / "out").read_bytes() == S.matched_lines(data, S.literal_hits(data, sigs))


def test_post_nmap_dedup_diff_lines(tmp_path):
    rep = corpus.nmap_report(200, seed=4)
    (tmp_path / "r.nmap").write_bytes(rep)
    rc, err = run_post("nmap", tmp_path / "r.nmap", tmp_path / "hp")
    assert rc == 0, err
    hp = (tmp_path / "hp").read_bytes()
    assert hp == S.nmap_host_ports(rep)
    rc, err = run_post("dedup", tmp_path / "hp", tmp_path / "u")
    assert rc == 0, err
    assert (tmp_path / "u").read_bytes() == S.dedup(hp)
    prior = S.dedup(b"".join(r + b"\n" for r in S.parse_records(hp)[::2]))
    (tmp_path / "prior").write_bytes(prior)
    rc, err = run_post("diff", tmp_path / "prior", tmp_path / "hp", tmp_path / "new")
    assert rc == 0, err
    assert (tmp_path / "new").read_bytes() == S.dedup_diff(hp, prior)[1]
    (tmp_path / "raw").write_bytes(b"\n\na\r\n\nb\nc")
    rc, err = run_post("lines", tmp_path / "raw", tmp_path / "l")
    assert rc == 0, err
    assert (tmp_path / "l").read_bytes() == b"a\r\nb\nc\n"


def test_post_json_fields(tmp_path):
    lines = b"".join(corpus.httpx_json_pool(64, seed=2)[i] + b"\n" for i in range(64))
    (tmp_path / "in").write_bytes(lines)
    rc, err = run_post("json", "url,title,tech", tmp_path / "in", tmp_path / "out")
    assert rc == 0, err
    assert (tmp_path / "out").read_bytes() == S.json_field_rows(lines, [b"url", b"title", b"tech"])[0]


def test_hook_postprocess_output_single_pass(tmp_path):
    import swarm_amd
    from swarm_amd import hooks
    sigs = [b"Grafana", b"Index of"]
    data = b"\n".join(corpus.httpx_pool(sigs, 400, 0.3, seed=5)) + b"\n\n"
    (tmp_path / "chunk_0.txt").write_bytes(data)
    m = swarm_amd.Matcher(sigs, "literal")
    n = hooks.postprocess_output(str(tmp_path / "chunk_0.txt"), m, str(tmp_path / "m.txt"))
    assert n == len(S.parse_records(data))
    assert (tmp_path / "m.txt").read_bytes() == S.matched_lines(data, S.literal_hits(data, sigs))
    assert (tmp_path / "chunk_0.txt").read_bytes() == data  # the upload contract is untouched
    assert hooks.postprocess_output(str(tmp_path / "chunk_0.txt")) == n


def _objects(n_chunks=12):
    buf, ids = corpus.subdomains(30_000, seed=6)
    parts = corpus.chunk_layout(buf, n_chunks)
    return {"scanA/output/chunk_%d.txt" % i: p.tobytes() for i, p in enumerate(parts)}, ids


def test_hook_raw_unique_and_completion():
    from swarm_amd import hooks
    objs, ids = _objects()
    objs["scanA/output/notes.log"] = b"ignored\n"
    merged = S.merge_chunks(objs, "scanA")
    assert hooks.raw_merge(objs, "scanA") == merged
    assert hooks.raw_unique(objs, "scanA") == S.dedup(merged)
    prior = corpus.prior_of(ids).tobytes()
    assert hooks.completion_dedup_diff(objs, "scanA", prior) == S.dedup_diff(merged, prior)
    assert hooks.completion_dedup_diff(objs, "scanA", None) == S.dedup_diff(merged, b"")


@pytest.mark.parametrize("bad", [b"ok\n\xff\xfe\n", "café\n".encode()[:-2]])
def test_hook_invalid_utf8_fails_like_the_reference(bad):
    """server/server.py:410 decodes each body; a bad body (or a multibyte character cut at the
    chunk edge) raises UnicodeDecodeError there, so the hooks raise it too."""
    from swarm_amd import hooks
    objs = {"s/output/chunk_0.txt": b"a\n", "s/output/chunk_1.txt": bad}
    for fn in (hooks.raw_merge, hooks.raw_unique):
        with pytest.raises(UnicodeDecodeError):
            fn(objs, "s")
    with pytest.raises(UnicodeDecodeError):
        hooks.completion_dedup_diff(objs, "s", None)
    assert hooks.raw_unique(objs, "s", strict_utf8=False) == S.dedup(b"a\n" + bad)


def test_host_api_reentrant_threads():
    """8 threads, each calling dedup_diff and Matcher.match on its own data 6 times, at once."""
    import swarm_amd
    m = swarm_amd.Matcher([b"api.", b"mail", b"target3"], "literal")
    jobs = []
    for t in range(8):
        buf, ids = corpus.subdomains(40_000 + 3_000 * t, seed=100 + t)
        jobs.append((buf.tobytes(), corpus.prior_of(ids).tobytes()))
    want = [S.dedup_diff(c, p) for c, p in jobs]
    want_hits = [S.literal_hits(c[:60_000], [b"api.", b"mail", b"target3"]) for c, _ in jobs]
    errors = []

    def worker(t):
        try:
            c, p = jobs[t]
            for _ in range(6):
                if swarm_amd.dedup_diff(c, p) != want[t]:
                    errors.append("dedup_diff mismatch in thread %d" % t)
                if m.match(c[:60_000]) != want_hits[t]:
                    errors.append("match mismatch in thread %d" % t)
        except Exception as e:  # noqa: BLE001
            errors.append("thread %d: %r" % (t, e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=300)
    assert not errors, errors[:3]
