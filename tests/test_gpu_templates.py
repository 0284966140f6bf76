"""GPU parity for nuclei matcher logic (§8(f) row 3): (record, template) results of the
C-ABI template engine vs the oracle, on hand cases, random templates and the template
corpus extracted from the reference (tests/golden/templates.json)."""
import random

import numpy as np
import pytest

from oracle import semantics as S
from swarm_amd import corpus
from test_templates_oracle import BUF, CASES, R, W, corpus_templates

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sg():
    import swarm_amd
    assert swarm_amd.device_count() > 0
    return swarm_amd


def test_hand_cases_together(sg):
    T = [t for t, _ in CASES]
    assert sg.Templates(T).match(BUF) == S.template_matches(BUF, T)


@pytest.mark.parametrize("i", range(len(CASES)))
def test_hand_case(sg, i):
    t = CASES[i][0]
    assert sg.Templates([t]).match(BUF) == S.template_matches(BUF, [t])


VOCAB = [b"nginx", b"Apache", b"PHP", b"Login", b"admin", b"WordPress", b"jQuery", b"200", b"OK", b"x-api",
         b"Server", b"ssh", b"LOGIN", b"Admin Panel"]


def random_templates(rng, n, parts):
    out = []
    for _ in range(n):
        ms = []
        for _ in range(rng.randint(1, 3)):
            part = rng.choice(parts)
            if rng.random() < 0.2:
                m = R(*[rng.choice([rb"PHP/[0-9]", rb"(?i)login", rb"^\{", rb"Admin\b", rb"nginx/1\.[0-9]+"])
                        for _ in range(rng.randint(1, 2))], part=part)
            else:
                m = W(*[rng.choice(VOCAB) for _ in range(rng.randint(1, 3))], part=part)
                m["case-insensitive"] = rng.random() < 0.3
            m["condition"] = rng.choice(["and", "or"])
            m["negative"] = rng.random() < 0.15
            ms.append(m)
        out.append({"condition": rng.choice(["and", "or"]), "matchers": ms})
    return out


def random_lines(rng, n):
    lines = []
    for _ in range(n):
        ws = [rng.choice(VOCAB + [b"foo", b"bar", b"nginx/1.18", b"PHP/7.4"]) for _ in range(rng.randint(0, 6))]
        lines.append(b" ".join(ws) or b"-")
    return lines


def test_random_templates_on_records(sg):
    rng = random.Random(5)
    T = random_templates(rng, 300, ["body"])
    data = b"\n".join(random_lines(rng, 3000)) + b"\n"
    assert sg.Templates(T).match(data) == S.template_matches(data, T)


def test_random_templates_on_json_fields(sg):
    rng = random.Random(6)
    keys = [b"title", b"webserver", b"tech"]
    T = random_templates(rng, 200, ["body", "title", "webserver", "tech"])
    data = b"\n".join(corpus.httpx_json_pool(2500, seed=13)) + b"\n"
    got = sg.Templates(T, keys).match(data)
    assert got == S.template_matches(data, T, keys)
    assert len(got) > 100


def planted_lines(rng, T, n):
    base = corpus.httpx_pool([], pool=1024, seed=3)
    out = []
    for _ in range(n):
        line = rng.choice(base)
        if rng.random() < 0.6:
            t = rng.choice(T)
            for m in t["matchers"]:
                if m["type"] != "word" or m.get("negative"):
                    continue
                ps = m["patterns"] if m.get("condition") == "and" else [rng.choice(m["patterns"])]
                for p in ps:
                    if b"\n" not in p:
                        line += b" " + p
        out.append(line)
    return out


def test_corpus_templates_planted(sg):
    rng = random.Random(7)
    T = corpus_templates()
    data = b"\n".join(planted_lines(rng, T, 6000)) + b"\n"
    got = sg.Templates(T).match(data)
    want = S.template_matches(data, T)
    assert got == want
    assert len(want) > 6000  # vacuous (negative-only) templates fire everywhere


def test_corpus_templates_device_path(sg):
    import torch
    rng = random.Random(8)
    T = corpus_templates()
    data = b"\n".join(planted_lines(rng, T, 2000)) + b"\n"
    d = torch.from_numpy(np.frombuffer(data, dtype=np.uint8).copy()).cuda()
    ctx = sg.Context(0, torch.cuda.current_stream().cuda_stream)
    tm = sg.Templates(T)
    r = tm.dev_match(ctx, d.data_ptr(), d.numel())
    n = int(r.n)
    rec = np.frombuffer(ctx.to_bytes(r.rec_idx, 4 * n), dtype=np.uint32)
    tid = np.frombuffer(ctx.to_bytes(r.tmpl_id, 4 * n), dtype=np.uint32)
    assert list(zip(rec.tolist(), tid.tolist())) == S.template_matches(data, T)
    assert r.in_records == 2000
    ctx.close()


@pytest.mark.parametrize("data", [b"", b"\n", b"only one line\n"])
def test_edges(sg, data):
    T = [{"condition": "or", "matchers": [W(b"nginx", negative=True)]},
         {"condition": "and", "matchers": [W(b"line"), W(b"one")]}]
    assert sg.Templates(T).match(data) == S.template_matches(data, T)


@pytest.mark.parametrize("case", ["records", "fields", "corpus"])
def test_record_wave_matches_sort_path(sg, monkeypatch, case):
    """The record-wave evaluation (default: per-record LDS matcher counts, no expansion sort)
    and the sort-based evaluation (SG_TM_SORT=1) give the same pairs, both equal to the
    oracle's."""
    rng = random.Random(11)
    keys = None
    if case == "records":
        T = random_templates(rng, 400, ["body"])
        data = b"\n".join(random_lines(rng, 4000)) + b"\n"
    elif case == "fields":
        keys = [b"title", b"webserver", b"tech"]
        T = random_templates(rng, 300, ["body", "title", "webserver", "tech"])
        data = b"\n".join(corpus.httpx_json_pool(3000, seed=17)) + b"\n"
    else:
        T = corpus_templates()
        data = b"\n".join(planted_lines(rng, T, 3000)) + b"\n"
    want = S.template_matches(data, T, keys) if keys else S.template_matches(data, T)
    outs = []
    for mode in ("0", "1"):
        monkeypatch.setenv("SG_TM_SORT", mode)
        tm = sg.Templates(T, keys) if keys else sg.Templates(T)
        outs.append(tm.match(data))
    assert outs[0] == want
    assert outs[1] == want


def test_record_wave_many_hits_per_record(sg):
    """Records holding every word of every matcher (long per-record hit lists, every template
    touched, `and` matchers at their full count) next to empty and hit-free records."""
    words = [b"w%03d" % i for i in range(120)]
    T = []
    for i in range(0, 120, 4):
        T.append({"condition": "and", "matchers": [W(*words[i:i + 4], condition="and"), W(words[(i + 7) % 120])]})
        T.append({"condition": "or", "matchers": [W(*words[i:i + 2], condition="and", negative=True)]})
    full = b" ".join(words)
    lines = [full, b"", b"nothing here", full[: len(full) // 2], b" ".join(reversed(words))] * 40
    data = b"\n".join(lines) + b"\n"
    assert sg.Templates(T).match(data) == S.template_matches(data, T)


def test_wide_matcher_uses_sort_path(sg):
    """A matcher with more than 255 distinct words does not fit the record-wave 8-bit counts:
    the handle evaluates with the sort-based path, same results."""
    words = [b"k%04d" % i for i in range(300)]
    T = [{"condition": "or", "matchers": [W(*words, condition="and")]},
         {"condition": "or", "matchers": [W(*words[:10])]},
         {"condition": "and", "matchers": [W(*words[:20], condition="and"), W(b"zz", negative=True)]}]
    lines = [b" ".join(words), b" ".join(words[:299]), b" ".join(words[:20]), b"zz " + b" ".join(words[:20]), b""] * 20
    data = b"\n".join(lines) + b"\n"
    assert sg.Templates(T).match(data) == S.template_matches(data, T)


def test_field_rows_repeat_atoms(sg):
    """One record's field rows hit the same word several times (array rows, repeated keys'
    rows) across engines: each (record, atom) counts once for `and` matchers."""
    keys = [b"title", b"tech"]
    lines = [b'{"title":"nginx nginx","tech":["nginx","nginx:1.2","PHP","nginx"]}',
             b'{"title":"x","tech":["PHP","PHP"]}',
             b'{"tech":["a","b"],"title":"PHP nginx"}',
             b'{"title":"none"}', b"not json nginx PHP"]
    T = [{"condition": "or", "matchers": [W(b"nginx", b"PHP", part="tech", condition="and")]},
         {"condition": "or", "matchers": [W(b"nginx", part="title"), W(b"PHP", part="tech")]},
         {"condition": "and", "matchers": [W(b"nginx", part="title"), W(b"nginx"), W(b"PHP", part="tech")]},
         {"condition": "or", "matchers": [R(rb"ngin.", part="tech"), W(b"zzz", part="title", negative=True)]},
         {"condition": "or", "matchers": [W(b"nginx", b"PHP", b"Apache", condition="and")]}]
    data = b"\n".join(lines * 30) + b"\n"
    assert sg.Templates(T, keys).match(data) == S.template_matches(data, T, keys)


def test_device_eval_with_given_field_rows(sg):
    """The fields step parses the JSON once: the rows of ctx.json_fields handed to the
    template evaluation (sg_dev_tmpl_eval_rows) give the same (record, template) pairs as
    building them inside, and as the oracle; rows built for other keys are refused."""
    import torch
    rng = random.Random(31)
    keys = [b"title", b"webserver", b"tech"]
    T = random_templates(rng, 80, ["body", "title", "webserver", "tech"])
    data = b"\n".join(corpus.httpx_json_pool(4000, seed=23)) + b"\n"
    d = torch.from_numpy(np.frombuffer(data, dtype=np.uint8).copy()).cuda()
    ctx = sg.Context(0, torch.cuda.current_stream().cuda_stream)
    try:
        tm = sg.Templates(T, keys)
        r1 = tm.dev_match(ctx, d.data_ptr(), d.numel())
        pairs1 = list(zip(np.frombuffer(ctx.to_bytes(r1.rec_idx, 4 * r1.n), dtype=np.uint32).tolist(),
                          np.frombuffer(ctx.to_bytes(r1.tmpl_id, 4 * r1.n), dtype=np.uint32).tolist()))
        rows = ctx.json_fields(d.data_ptr(), d.numel(), keys)
        r2 = tm.dev_match(ctx, d.data_ptr(), d.numel(), rows=rows, rows_keys=keys)
        pairs2 = list(zip(np.frombuffer(ctx.to_bytes(r2.rec_idx, 4 * r2.n), dtype=np.uint32).tolist(),
                          np.frombuffer(ctx.to_bytes(r2.tmpl_id, 4 * r2.n), dtype=np.uint32).tolist()))
        assert pairs1 == pairs2 == S.template_matches(data, T, keys)
        with pytest.raises(ValueError):
            tm.dev_match(ctx, d.data_ptr(), d.numel(), rows=rows, rows_keys=[b"url"])
    finally:
        ctx.close()
