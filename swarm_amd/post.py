"""Worker post-step as a module command: `python -m swarm_amd.post <op> ...`.

The reference runs every module as one shell command with `{input}` / `{output}`
substituted (worker/worker.py:27-33, :83) and uploads `{output}` when the command exits 0
(:96-98); a non-zero exit marks the job `cmd failed` (:89). A module JSON can therefore chain
the GPU step after the scanner without any change to worker.py, e.g.

  {"command": "httpx -l {input} -silent -title -o {output}.raw && python3 -m swarm_amd.post match --literal sigs.txt {output}.raw {output}"}

(examples/modules/ holds such files). Operations (all run the HIP kernels; no CPU path):

  lines  IN OUT                    A3: the non-empty records of IN, '\\n'-terminated
  match  (--literal|--regex) SIGS IN OUT [--nocase]
                                   A4: grep output — the records with a signature hit
  nmap   IN OUT                    §8(f)2: nmap -oN report -> host:port records
  json   KEYS IN OUT               §8(f)1: httpx -json lines -> rows of the comma-separated keys
  dedup  IN OUT                    A7: sort -u
  diff   PRIOR IN OUT              A8: records of IN not in PRIOR (sorted, unique)

SIGS is a file of one signature per line (blank lines ignored). Exit status 0 on success,
1 on any error (message on stderr), as the worker expects of a module command.
"""
from __future__ import annotations

import argparse
import sys
from typing import List


def _read(path: str) -> bytes:
    with open(path, "rb") as f:
        return f.read()


def _write(path: str, data: bytes) -> None:
    with open(path, "wb") as f:
        f.write(data)


def read_signatures(path: str) -> List[bytes]:
    """One signature per line; a trailing '\\r' is kept (it is part of the bytes a record
    would have to contain); empty lines are skipped."""
    return [s for s in _read(path).split(b"\n") if s]


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="python -m swarm_amd.post", description=__doc__.split("\n\n")[0])
    sub = ap.add_subparsers(dest="op", required=True)
    p = sub.add_parser("lines")
    p.add_argument("inp")
    p.add_argument("out")
    p = sub.add_parser("match")
    g = p.add_mutually_exclusive_group(required=True)
    g.add_argument("--literal", metavar="SIGS")
    g.add_argument("--regex", metavar="SIGS")
    p.add_argument("--nocase", action="store_true")
    p.add_argument("inp")
    p.add_argument("out")
    p = sub.add_parser("nmap")
    p.add_argument("inp")
    p.add_argument("out")
    p = sub.add_parser("json")
    p.add_argument("keys", help="comma-separated top-level keys, e.g. url,title,webserver,tech")
    p.add_argument("inp")
    p.add_argument("out")
    p = sub.add_parser("dedup")
    p.add_argument("inp")
    p.add_argument("out")
    p = sub.add_parser("diff")
    p.add_argument("prior")
    p.add_argument("inp")
    p.add_argument("out")
    return ap


def run(args) -> int:
    from . import api
    data = _read(args.inp)
    if args.op == "lines":
        spans = api.lines(data)
        out = b"".join(data[s:e] + b"\n" for s, e in spans.tolist())
    elif args.op == "match":
        kind = "literal" if args.literal else "regex"
        sigs = read_signatures(args.literal or args.regex)
        out = api.Matcher(sigs, kind, nocase=args.nocase).match_lines(data)
    elif args.op == "nmap":
        out = api.nmap_ports(data)
    elif args.op == "json":
        keys = [k.encode() for k in args.keys.split(",") if k]
        out, _, _ = api.json_fields(data, keys)
    elif args.op == "dedup":
        out = api.dedup(data)
    else:
        out = api.diff(data, _read(args.prior))
    _write(args.out, out)
    return 0


def main(argv=None) -> int:
    args = build_parser().parse_args(argv)
    try:
        return run(args)
    except Exception as e:  # the worker reads only the exit status (worker/worker.py:86-90)
        print("swarm_amd.post %s: %s" % (args.op, e), file=sys.stderr)
        return 1


if __name__ == "__main__":
    sys.exit(main())
