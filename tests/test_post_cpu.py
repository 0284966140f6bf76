"""The worker post-step entry (swarm_amd.post): argument parsing, signature files and the
example module JSONs' command strings — no GPU work. The GPU runs are in test_gpu_post.py."""
import glob
import json
import os

import pytest

from conftest import ROOT
from swarm_amd import post


def test_parser_ops():
    ap = post.build_parser()
    a = ap.parse_args(["match", "--literal", "s.txt", "in", "out"])
    assert (a.op, a.literal, a.regex, a.inp, a.out) == ("match", "s.txt", None, "in", "out")
    assert ap.parse_args(["diff", "p", "i", "o"]).prior == "p"
    assert ap.parse_args(["json", "url,title", "i", "o"]).keys == "url,title"
    with pytest.raises(SystemExit):
        ap.parse_args(["match", "in", "out"])  # --literal or --regex is required


def test_read_signatures_skips_blank_lines(tmp_path):
    f = tmp_path / "s.txt"
    f.write_bytes(b"admin\n\nLogin\r\nx\n")
    assert post.read_signatures(str(f)) == [b"admin", b"Login\r", b"x"]


def test_missing_input_exits_1(tmp_path, capsys):
    assert post.main(["dedup", str(tmp_path / "nope"), str(tmp_path / "out")]) == 1
    assert "swarm_amd.post dedup" in capsys.readouterr().err


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(ROOT, "examples", "modules", "*.json"))))
def test_example_modules_keep_the_contract(path):
    """Each example substitutes like worker/worker.py:27-33 and ends by writing {output}."""
    cmd = json.load(open(path))["command"]
    assert "{input}" in cmd and "{output}" in cmd
    sub = cmd.replace("{input}", "downloads/chunk_3.txt").replace("{output}", "uploads/s/output/chunk_3.txt")
    assert sub.rstrip().endswith(" uploads/s/output/chunk_3.txt")
    assert "python3 -m swarm_amd.post " in sub
    op = sub.split("python3 -m swarm_amd.post ", 1)[1].split()
    post.build_parser().parse_args(op)
