"""CPU checks of the §8(f) format oracles (nmap -oN -> host:port, httpx -json -> field
rows): hand-written fixtures, and the JSON restatement pinned against Python's json
module on valid lines (the reference semantics: json.loads, last duplicate key wins)."""
import json
import random

import pytest

from oracle import semantics as S
from swarm_amd import corpus

NMAP_FIXTURE = (
    b"# Nmap 7.80 scan initiated as: nmap -sV -oN out\n"
    b"22/tcp open ssh (before any report: dropped)\n"
    b"Nmap scan report for a.example.com (10.0.0.1)\n"
    b"Host is up (0.010s latency).\n"
    b"PORT     STATE    SERVICE VERSION\n"
    b"22/tcp   open     ssh     OpenSSH 8.2p1\n"
    b"25/tcp   closed   smtp\n"
    b"53/udp   open|filtered domain\n"
    b"80/tcp   open     http    nginx\n"
    b"443/tcp\topen\n"
    b"123456/tcp open x\n"
    b"8080/tcp opened x\n"
    b"\n"
    b"Nmap scan report for 10.0.0.2\r\n"
    b"3306/tcp open  mysql\r\n"
    b"Nmap scan report for \n"
    b"21/tcp open ftp\n"
    b"Nmap scan report for b.example.com\n"
    b"5432/sctp open pg\n"
    b"# Nmap done\n")
NMAP_EXPECT = (b"a.example.com:22\na.example.com:80\na.example.com:443\n10.0.0.2\r:3306\n"
               b"b.example.com:5432\n")


def test_nmap_fixture():
    assert S.nmap_host_ports(NMAP_FIXTURE) == NMAP_EXPECT


def test_nmap_generated_report_counts():
    txt = corpus.nmap_report(300, seed=3)
    out = S.nmap_host_ports(txt)
    opened = sum(1 for ln in txt.split(b"\n") if b" open " in ln and b"/tcp" in ln or b"/udp open " in ln)
    assert out.count(b"\n") == opened
    assert all(b":" in r for r in out.split(b"\n")[:-1])


def _enc(s: str) -> bytes:
    return s.encode("utf-8", "surrogatepass").replace(b"\n", b"\\n")


def json_reference_rows(line: bytes, keys):
    """What json.loads says: per key, (kind, value) items."""
    obj = json.loads(line)
    out = []
    for ki, k in enumerate(keys):
        kk = k.decode()
        if not isinstance(obj, dict) or kk not in obj:
            continue
        v = obj[kk]
        items = v if isinstance(v, list) else [v]
        for el in items:
            if isinstance(el, str):
                if el:
                    out.append((ki, "s", _enc(el)))
            else:
                out.append((ki, "v", el))
    return out


def check_line_against_json(line: bytes, keys):
    rows, rrec, rkey = S.json_field_rows(line + b"\n", keys)
    got = rows.split(b"\n")[:-1]
    ref = json_reference_rows(line, keys)
    assert len(got) == len(ref), (line, got, ref)
    for g, k, (ki, kind, v) in zip(got, rkey, ref):
        assert k == ki
        if kind == "s":
            assert g == v
        else:
            assert json.loads(g) == v


def test_json_oracle_matches_json_module_on_httpx_lines():
    keys = [b"url", b"title", b"webserver", b"tech", b"status_code", b"a", b"hash", b"failed", b"missing"]
    for line in corpus.httpx_json_pool(1500, seed=2):
        check_line_against_json(line, keys)


def _rand_str(rng):
    pool = ["a", "Z", " ", '"', "\\", "/", "\n", "\t", "\r", "\x00", "\x1f", "\x7f", "é", "€",
            "\U0001F600", "\ud800", "\udc00", "<", "&", ",", ":", "{", "}", "[", "]"]
    return "".join(rng.choice(pool) for _ in range(rng.randint(0, 12)))


def _rand_val(rng, depth=0):
    r = rng.random()
    if r < 0.35 or depth > 2:
        return _rand_str(rng)
    if r < 0.5:
        return rng.choice([0, -1, 3.5, 1e-7, 10 ** 20, True, False, None])
    if r < 0.8:
        return [_rand_val(rng, depth + 1) for _ in range(rng.randint(0, 4))]
    return {_rand_str(rng): _rand_val(rng, depth + 1) for _ in range(rng.randint(0, 3))}


@pytest.mark.parametrize("ascii_only", [True, False])
def test_json_oracle_matches_json_module_on_random_objects(ascii_only):
    rng = random.Random(17 + ascii_only)
    keys = [b"k0", b"k1", b"k2", b"title", b"tech"]
    for _ in range(1500):
        obj = {}
        for _ in range(rng.randint(0, 6)):
            k = rng.choice(["k0", "k1", "k2", "title", "tech", "other", "k"])
            obj[k] = _rand_val(rng)
        sep = rng.choice([(",", ":"), (", ", ": "), (" ,  ", " :\t")])
        s = json.dumps(obj, ensure_ascii=ascii_only, separators=sep)
        if rng.random() < 0.2:
            s = "  " + s + " \t"
        try:
            line = s.encode("utf-8", "surrogatepass")
            line.decode("utf-8")
        except UnicodeDecodeError:
            continue  # lone surrogates written raw are not valid UTF-8 input for json.loads
        check_line_against_json(line, keys)


def test_json_duplicate_keys_last_wins():
    line = b'{"title":"first","x":1,"title":"second","tech":["a"],"tech":[]}'
    rows, rrec, rkey = S.json_field_rows(line + b"\n", [b"title", b"tech"])
    assert rows == b"second\n"
    assert json.loads(line)["title"] == "second"


@pytest.mark.parametrize("line", [b"not json", b'{"a":1', b'{"a":"x}', b"[1,2]", b'"str"', b'{"a":1} x',
                                  b'{"a":1}{"b":2}', b"{", b"}", b'{"a":[1,2}', b"x {\"a\":1}", b"7"])
def test_json_malformed_lines_yield_nothing(line):
    try:
        assert not isinstance(json.loads(line), dict)
    except ValueError:
        pass
    assert S.json_field_rows(line + b"\n", [b"a", b"b"]) == (b"", [], [])


def test_json_whitespace_around_object_is_valid():
    rows, rrec, rkey = S.json_field_rows(b'  {"a" : "v" }\t\n', [b"a"])
    assert rows == b"v\n" and rrec == [0] and rkey == [0]


ESC_KEYS = ["title", 'ti"tle', "a\\b", "k\n", "tab\t", "é", "\U0001F600", "/x", "\x01"]


def escaped_key_lines(n, seed):
    """Objects whose top-level keys need (or are written with) JSON escapes."""
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        obj = {rng.choice(ESC_KEYS): _rand_val(rng) for _ in range(rng.randint(1, 5))}
        s = json.dumps(obj, ensure_ascii=rng.random() < 0.5, separators=rng.choice([(",", ":"), (" , ", " : ")]))
        if rng.random() < 0.3:  # spell a plain key with escapes, as another writer might
            s = s.replace('"title"', rng.choice(['"\\u0074itle"', '"t\\u0069tl\\u0065"', '"titl\\u0065"']))
        if rng.random() < 0.2:
            s = s.replace('"/x"', '"\\/x"')
        out.append(s.encode("utf-8", "surrogatepass"))
    out += [b'{"\\u0074itle":"a","title":"b"}', b'{"title":"a","\\u0074itle":"b"}', b'{"ti\\"tle":"q"}',
            b'{"\\ud83d\\ude00":"smile"}', b'{"k\\n":"nl","k\\\\n":"bs"}']
    return out


def test_json_escaped_keys_match_json_module():
    keys = [k.encode("utf-8") for k in ESC_KEYS] + [b"k\\n", b"tit"]
    for line in escaped_key_lines(1500, seed=5):
        try:
            line.decode("utf-8")
        except UnicodeDecodeError:
            continue
        check_line_against_json(line, keys)
