"""CPU checks of the nuclei matcher-logic oracle (§8(f) row 3) on hand cases, and of the
template fixture extracted from the reference corpus (compiles without a GPU)."""
import base64

import pytest

from conftest import load_golden
from oracle import semantics as S


def W(*ws, **kw):
    m = {"type": "word", "part": "body", "patterns": list(ws)}
    m.update(kw)
    return m


def R(*rs, **kw):
    m = {"type": "regex", "part": "body", "patterns": list(rs)}
    m.update(kw)
    return m


BUF = (b"Server: nginx/1.18 X-Powered-By: PHP/7.4\n"
       b"<meta name=\"generator\" content=\"WordPress 5.8\">\n"
       b"plain text line\n"
       b"X-TYPO3-Parsetime: 12ms\n")

CASES = [
    ({"condition": "or", "matchers": [W(b"nginx")]}, [0]),
    ({"condition": "or", "matchers": [W(b"nginx", b"WordPress")]}, [0, 1]),
    ({"condition": "or", "matchers": [W(b"nginx", b"PHP", condition="and")]}, [0]),
    ({"condition": "or", "matchers": [W(b"nginx", b"WordPress", condition="and")]}, []),
    ({"condition": "and", "matchers": [W(b"nginx"), W(b"Apache", negative=True)]}, [0]),
    ({"condition": "or", "matchers": [W(b"nginx", negative=True)]}, [1, 2, 3]),
    ({"condition": "or", "matchers": [W(b"x-typo3-parsetime:", **{"case-insensitive": True})]}, [3]),
    ({"condition": "or", "matchers": [W(b"x-typo3-parsetime:")]}, []),
    ({"condition": "or", "matchers": [R(rb"PHP/[0-9]+\.[0-9]+")]}, [0]),
    ({"condition": "and", "matchers": [R(rb"^<meta"), W(b"5.8")]}, [1]),
    ({"condition": "or", "matchers": [R(rb"(?i)WORDPRESS")]}, [1]),
    ({"condition": "or", "matchers": [W(b"a\nb")]}, []),
]


@pytest.mark.parametrize("tmpl,recs", CASES)
def test_oracle_hand_cases(tmpl, recs):
    assert S.template_matches(BUF, [tmpl]) == [(r, 0) for r in recs]


def test_oracle_json_parts():
    buf = (b'{"title":"Admin Login","webserver":"nginx","tech":["PHP:7.4","jQuery"]}\n'
           b'{"title":"Welcome","tech":["WordPress"]}\n'
           b"not json but nginx Login\n")
    keys = [b"title", b"webserver", b"tech"]
    t = [{"condition": "or", "matchers": [W(b"Login", part="title")]},
         {"condition": "or", "matchers": [W(b"PHP", b"jQuery", part="tech", condition="and")]},
         {"condition": "or", "matchers": [W(b"PHP:7.4jQuery", part="tech")]},  # rows are matched one by one
         {"condition": "or", "matchers": [W(b"nginx", part="body")]},
         {"condition": "or", "matchers": [W(b"nginx", part="webserver", negative=True)]}]
    assert S.template_matches(buf, t, keys) == [(0, 0), (0, 1), (0, 3), (1, 4), (2, 3), (2, 4)]


def corpus_templates():
    d = load_golden("templates.json")
    return [dict(t, matchers=[dict(m, patterns=[base64.b64decode(p) for p in m["patterns"]]) for m in t["matchers"]])
            for t in d["templates"]]


def test_template_fixture_compiles_without_gpu():
    import swarm_amd
    T = corpus_templates()
    assert len(T) > 900
    t = swarm_amd.Templates(T, keys=[b"title", b"webserver"])
    info = t.info()
    assert info["templates"] == len(T) and info["atoms"] > 1000 and info["engines"] >= 2
    assert info["vacuous"] == sum(1 for x in T if S.template_matches(b"\x01\n", [x]) == [(0, 0)])
