"""GPU parity for the §8(f) module-output formats: nmap -oN -> host:port records and
httpx -json -> field rows, through the C-ABI, bit-exact against the oracle."""
import json
import random

import numpy as np
import pytest

from oracle import semantics as S
from swarm_amd import corpus
from test_formats_oracle import NMAP_EXPECT, NMAP_FIXTURE

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sg():
    import swarm_amd
    assert swarm_amd.device_count() > 0
    return swarm_amd


# ------------------------------------------------------------------ nmap
def test_nmap_fixture(sg):
    assert sg.nmap_ports(NMAP_FIXTURE) == NMAP_EXPECT


@pytest.mark.parametrize("data", [b"", b"\n\n", b"Nmap scan report for x\n", b"22/tcp open ssh\n",
                                  b"Nmap scan report for h\n22/tcp open", b"Nmap scan report for h\n1/udp\topen\t\n",
                                  b"Nmap scan report for h\n99999/tcp open\n100000/tcp open\n"])
def test_nmap_edges(sg, data):
    assert sg.nmap_ports(data) == S.nmap_host_ports(data)


@pytest.mark.parametrize("hosts,seed", [(50, 1), (5000, 2), (60000, 3)])
def test_nmap_generated(sg, hosts, seed):
    txt = corpus.nmap_report(hosts, seed=seed)
    assert sg.nmap_ports(txt) == S.nmap_host_ports(txt)


def test_nmap_device_path_feeds_dedup(sg):
    import torch
    txt = corpus.nmap_report(20000, seed=4) * 3  # every host:port three times
    d = torch.from_numpy(np.frombuffer(txt, dtype=np.uint8).copy()).cuda()
    ctx = sg.Context(0, torch.cuda.current_stream().cuda_stream)
    r = ctx.nmap_ports(d.data_ptr(), d.numel())
    want = S.nmap_host_ports(txt)
    assert r.records == want.count(b"\n")
    assert ctx.to_bytes(r.data, r.bytes) == want
    # host:port records -> sort -u (C5 shape) straight from HBM
    u = ctx.dedup_diff(r.data, r.bytes)
    assert ctx.to_bytes(u.uniq, u.uniq_bytes) == S.dedup(want)
    ctx.close()


# ------------------------------------------------------------------ httpx -json
KEYS = [b"url", b"title", b"webserver", b"tech", b"status_code", b"a", b"hash", b"input"]


def check(sg, data, keys):
    rows, rrec, rkey = sg.json_fields(data, keys)
    o_rows, o_rec, o_key = S.json_field_rows(data, keys)
    assert rows == o_rows
    assert rrec.tolist() == o_rec
    assert rkey.tolist() == o_key


def test_json_httpx_pool(sg):
    data = b"\n".join(corpus.httpx_json_pool(3000, seed=8)) + b"\n"
    check(sg, data, KEYS)


def test_json_single_key_and_missing_keys(sg):
    data = b"\n".join(corpus.httpx_json_pool(500, seed=9)) + b"\n"
    check(sg, data, [b"tech"])
    check(sg, data, [b"nope", b"ur", b"urls", b"title"])


def test_json_64_keys(sg):
    keys = [b"k%d" % i for i in range(64)]
    rng = random.Random(3)
    lines = []
    for _ in range(300):
        obj = {("k%d" % rng.randrange(70)): rng.choice(["v", "", 5, [1, "x"], {"k1": "nested"}]) for _ in range(20)}
        lines.append(json.dumps(obj).encode())
    check(sg, b"\n".join(lines) + b"\n", keys)


def backslash_lines():
    """Strings whose backslash runs and escaped quotes straddle the 64-byte chunk edges."""
    out = []
    for pad in range(0, 70):
        for run in (1, 2, 3, 4, 63, 64, 65, 127, 128):
            val = "x" * pad + "\\" * run + '"' + "y"
            line = json.dumps({"title": val, "url": "u%d" % pad}, separators=(",", ":"))
            out.append(line.encode())
    return out


def test_json_backslash_runs_across_chunks(sg):
    data = b"\n".join(backslash_lines()) + b"\n"
    check(sg, data, [b"title", b"url"])


def test_json_random_objects(sg):
    from test_formats_oracle import _rand_val
    rng = random.Random(21)
    keys = [b"k0", b"k1", b"title", b"tech"]
    lines = []
    for _ in range(4000):
        obj = {rng.choice(["k0", "k1", "title", "tech", "z"]): _rand_val(rng) for _ in range(rng.randint(0, 6))}
        s = json.dumps(obj, ensure_ascii=rng.random() < 0.5, separators=rng.choice([(",", ":"), (" , ", " : ")]))
        lines.append(s.encode("utf-8", "surrogatepass"))
    check(sg, b"\n".join(lines) + b"\n", keys)


def test_json_duplicates_malformed_and_whitespace(sg):
    lines = [b'{"title":"first","x":1,"title":"second","tech":["a"],"tech":[]}',
             b"not json", b'{"title":1', b'{"title":"x}', b"[1,2]", b'"str"', b'{"title":1} x',
             b'{"title":1}{"b":2}', b"{", b"}", b'{"title":[1,2}', b'x {"title":1}',
             b'  {"title" : "v" }\t', b'{"title":"a\\u0000b","tech":["\\ud83d\\ude00","\\ud800x","",null,[1]]}',
             b'{"title":"' + b"w" * 5000 + b'","url":"' + b"\\n" * 2000 + b'"}',
             b'{"deep":{"title":"nested, not top-level"},"title":"top"}', b"{}", b'{"title":{}}']
    check(sg, b"\n".join(lines) + b"\n", [b"title", b"tech", b"url"])


def test_json_plain_arrays(sg):
    """Array values without backslashes take the scan's 16-byte SWAR counter (rows and bytes
    must equal the byte walk's): nesting, blanks around and inside items, empty strings,
    separators and brackets inside strings, empty items, text after the closing bracket, a
    second array in the same value, at every alignment of the value inside 16-byte blocks."""
    vals = [b'[]', b'[ ]', b'[,]', b'[1,,2]', b'["a" , "" ,"b"]', b'[ "x,y]" , "[z" ]', b'[[1,2],{"k":[3]},4]',
            b'[ "" ]', b'[""]', b'["\t"]', b'[  1  2 , 3 ]', b'[1] x', b'[1] [2]',
            b'["' + b"q" * 40 + b'", "' + b"r" * 17 + b'"]', b'[{"a":"]"},"}",["[",","]]', b'[ true , null , -1.5e3 ]',
            b'[1,[2,[3,[4]]],5]', b'["a"\t,\r"b" ]', b'[ "a" "b" ]', b'["]"]']
    lines = []
    for pad in range(0, 17):
        for v in vals:
            lines.append(b'{"' + b"p" * pad + b'":1,"tech":' + v + b',"title":"t"}')
            lines.append(b'{"tech" :  ' + v + b'  }')
    check(sg, b"\n".join(lines) + b"\n", [b"tech", b"title"])


def test_json_device_rows_match_and_feed_matcher(sg):
    """Rows are a line buffer: the A4 matcher runs on them directly (part-scoped match)."""
    import torch
    data = b"\n".join(corpus.httpx_json_pool(4000, seed=12)) + b"\n"
    d = torch.from_numpy(np.frombuffer(data, dtype=np.uint8).copy()).cuda()
    ctx = sg.Context(0, torch.cuda.current_stream().cuda_stream)
    r = ctx.json_fields(d.data_ptr(), d.numel(), [b"title", b"webserver"])
    rows = ctx.to_bytes(r.data, r.bytes)
    o_rows, o_rec, o_key = S.json_field_rows(data, [b"title", b"webserver"])
    assert rows == o_rows and r.rows == len(o_rec) and r.in_records == 4000
    m = sg.Matcher([b"nginx", b"Login", b"\xe6\x97\xa5"], "literal")
    assert m.match(rows) == S.literal_hits(o_rows, [b"nginx", b"Login", b"\xe6\x97\xa5"])
    ctx.close()


def test_json_long_lines_and_many_rows(sg):
    """Lines of 100 KB+ (a long title, a 5,000-element tech array) and rows past 2^16."""
    big = json.dumps({"title": "t" * 120_000 + "é", "tech": ["x%d" % i for i in range(5000)],
                      "url": "u"}).encode()
    lines = [big] + corpus.httpx_json_pool(20_000, seed=17)
    check(sg, b"\n".join(lines) + b"\n", [b"title", b"tech", b"url"])


def test_nmap_many_hosts_crlf(sg):
    txt = corpus.nmap_report(100_000, seed=9).replace(b"\n", b"\r\n")
    assert sg.nmap_ports(txt) == S.nmap_host_ports(txt)


def test_json_escaped_keys(sg):
    """Keys written with JSON escapes (and requested keys that need them) match by their
    decoded form, as json.loads would."""
    from test_formats_oracle import ESC_KEYS, escaped_key_lines
    keys = [k.encode("utf-8") for k in ESC_KEYS] + [b"k\\n", b"tit"]
    check(sg, b"\n".join(escaped_key_lines(3000, seed=6)) + b"\n", keys)
