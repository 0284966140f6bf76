"""The CPU oracle against every golden vector (reference-generated and GNU-tool-generated)."""
import pytest

from conftest import b64d, load_golden
from oracle import semantics as S

REF = load_golden("reference_vectors.json")
CU = load_golden("coreutils_vectors.json")
GR = load_golden("grep_vectors.json")


@pytest.mark.parametrize("case", REF["a1_chunking"], ids=lambda c: c["name"])
def test_a1_chunk_layout(case):
    fc = S.client_readlines(b64d(case["file"]))
    assert fc == case["file_content"]
    assert S.server_chunks(fc, case["batch_size"]) == [b64d(x) for x in case["chunks"]]


@pytest.mark.parametrize("case", REF["a5_merge"], ids=lambda c: c["name"])
def test_a5_merge(case):
    objs = {"%s/output/%s" % (case["scan_id"], k): b64d(v) for k, v in case["objects"].items()}
    assert S.merge_chunks(objs, case["scan_id"]) == b64d(case["raw"])


def test_a6_get_chunk():
    c = REF["a6_get_chunk"][0]
    assert c["json"]["contents"].encode() == b64d(c["object"])


def test_a2_module_commands_keep_contract():
    cmds = REF["a2_module_cmds"]
    assert set(cmds) == {"dnsx", "http2", "httprobe", "httpx", "nmap", "nuclei", "web"}
    for c in cmds.values():
        assert "uploads/s_1/output/chunk_7.txt" in c and "downloads/chunk_7.txt" in c


@pytest.mark.parametrize("case", CU["dedup"], ids=lambda c: c["name"])
def test_a7_dedup_vs_sort_u(case):
    assert S.dedup(b64d(case["input"])) == b64d(case["sort_u"])


@pytest.mark.parametrize("case", CU["diff"], ids=lambda c: c["name"])
def test_a8_diff_vs_comm(case):
    assert S.diff(b64d(case["cur"]), b64d(case["prior"])) == b64d(case["comm13"])


@pytest.mark.parametrize("case", GR["literal"], ids=lambda c: c["name"])
def test_a4_literal_vs_grep_F(case):
    hits = S.literal_hits(b64d(case["input"]), [b64d(s) for s in case["sigs"]], case["nocase"])
    assert [list(h) for h in hits] == case["hits"]


@pytest.mark.parametrize("case", GR["regex"], ids=lambda c: c["name"])
def test_a4_regex_vs_grep_P(case):
    hits = S.regex_hits(b64d(case["input"]), [b64d(s) for s in case["regexes"]])
    assert [list(h) for h in hits] == case["hits"]


def test_record_spans_agree_with_parse():
    buf = b"\n\na\r\nbb\n\n\nccc"
    assert [buf[s:e] for s, e in S.record_spans(buf)] == S.parse_records(buf)


def test_prior_scan_id_picks_latest_complete_earlier_scan_of_module():
    """server/server.py:277-294 writes asm.scans documents; the prior of a scan is the latest
    completed scan of the same module that started earlier."""
    from swarm_amd.hooks import prior_scan_id
    scans = [
        {"scan_id": "a", "module": "dnsx", "scan_status": "complete", "scan_started": 100},
        {"scan_id": "b", "module": "dnsx", "scan_status": "complete", "scan_started": 300},
        {"scan_id": "c", "module": "dnsx", "scan_status": "running", "scan_started": 350},
        {"scan_id": "d", "module": "httpx", "scan_status": "complete", "scan_started": 390},
        {"scan_id": "e", "module": "dnsx", "scan_status": "complete", "scan_started": 500},
        {"scan_id": "f", "module": "dnsx", "scan_status": "complete"},
    ]
    assert prior_scan_id(scans, "dnsx", 400) == "b"
    assert prior_scan_id(scans, "dnsx", 300) == "a"
    assert prior_scan_id(scans, "dnsx", 100) is None
    assert prior_scan_id(scans, "httpx", 1000) == "d"
    assert prior_scan_id(scans, "nmap", 1000) is None


def test_check_utf8_matches_reference_decode():
    from swarm_amd.hooks import check_utf8
    check_utf8("déjà vu\n".encode())
    with pytest.raises(UnicodeDecodeError):
        check_utf8(b"\xe2\x82")  # a character cut at a chunk edge
