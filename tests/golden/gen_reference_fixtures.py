#!/usr/bin/env python3
"""Generate golden vectors by running the REFERENCE's own Python code (stub-imported).

Run in the build container only (it reads /root/reference, which never travels to the
GPU box):

    cd /tmp && PYTHONDONTWRITEBYTECODE=1 python3 -B /root/repo/tests/golden/gen_reference_fixtures.py

What is pinned:
  A1  chunk bytes the server writes to S3 for a client file + batch_size
      (client/swarm:18-32 readlines, server/server.py:414-461 '\\n'.join)
  A5  the /raw merge output for a set of output-chunk objects (server/server.py:399-412)
  A6  the /get-chunk JSON (server/server.py:338-345)
  A2  worker module command strings (worker/worker.py:27-33, worker/modules/*.json)

Stand-ins are placed in sys.modules BEFORE import: an in-memory redis, a fake boto3 S3
client (lexicographic list order, 1,000-key page like S3's ListObjects v1), a
botocore.exceptions stub and a requests stub that never touches the network
(server.py:52/59 calls the DigitalOcean API at import time). The fake S3 is the only
part of the chain that is not reference code; its two behaviours (key order and page
size) are S3's documented ListObjects semantics and are noted in the fixture.
"""
import base64
import importlib.machinery
import importlib.util
import io
import json
import os
import sys
import tempfile
import types

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_vectors.json")


# ----------------------------------------------------------------------------- stand-ins
class FakeRedis:
    def __init__(self, *a, **k):
        self.h, self.l = {}, {}

    def hset(self, name, key, value):
        if isinstance(key, str):
            key = key.encode()
        if isinstance(value, str):
            value = value.encode()
        self.h.setdefault(name, {})[key] = value

    def hget(self, name, key):
        if isinstance(key, str):
            key = key.encode()
        return self.h.get(name, {}).get(key)

    def hkeys(self, name):
        return list(self.h.get(name, {}).keys())

    def rpush(self, name, v):
        if isinstance(v, str):
            v = v.encode()
        self.l.setdefault(name, []).append(v)

    def lpop(self, name):
        q = self.l.get(name, [])
        return q.pop(0) if q else None

    def flushall(self):
        self.h.clear()
        self.l.clear()


class FakeS3:
    PAGE = 1000  # S3 ListObjects (v1) default/maximum page size

    def __init__(self):
        self.objs = {}

    def put_object(self, Body, Bucket, Key):
        if isinstance(Body, str):
            Body = Body.encode("utf-8")  # boto3 encodes str bodies as UTF-8
        self.objs[Key] = bytes(Body)

    def get_object(self, Bucket, Key):
        return {"Body": io.BytesIO(self.objs[Key])}

    def list_objects(self, Bucket, Prefix):
        keys = sorted(k for k in self.objs if k.startswith(Prefix))  # UTF-8 binary order
        return {"Contents": [{"Key": k} for k in keys[: self.PAGE]]}

    def upload_file(self, fn, Bucket, Key):
        with open(fn, "rb") as f:
            self.objs[Key] = f.read()

    def download_file(self, Bucket, Key, fn):
        with open(fn, "wb") as f:
            f.write(self.objs[Key])


S3 = FakeS3()


class _Resp:
    status_code = 599
    text = "offline"

    def json(self):
        return {}


class FakeRequests(types.ModuleType):
    last_post = None

    def get(self, *a, **k):
        return _Resp()

    def post(self, url, headers=None, json=None, **k):
        FakeRequests.last_post = json
        return _Resp()

    def delete(self, *a, **k):
        return _Resp()


def install_stubs():
    redis = types.ModuleType("redis")
    redis.Redis = FakeRedis
    boto3 = types.ModuleType("boto3")
    boto3.client = lambda *a, **k: S3
    botocore = types.ModuleType("botocore")
    bexc = types.ModuleType("botocore.exceptions")

    class NoCredentialsError(Exception):
        pass

    bexc.NoCredentialsError = NoCredentialsError
    botocore.exceptions = bexc
    sys.modules.update({"redis": redis, "boto3": boto3, "botocore": botocore,
                        "botocore.exceptions": bexc, "requests": FakeRequests("requests")})
    pt = types.ModuleType("prettytable")
    pt.PrettyTable = object
    sys.modules.setdefault("prettytable", pt)


def load(name, path):
    loader = importlib.machinery.SourceFileLoader(name, path)
    spec = importlib.util.spec_from_loader(name, loader)
    mod = importlib.util.module_from_spec(spec)
    loader.exec_module(mod)
    return mod


def b64(b):
    return base64.b64encode(b).decode()


# ----------------------------------------------------------------------------- cases
def main():
    sys.dont_write_bytecode = True
    install_stubs()
    scratch = tempfile.mkdtemp(prefix="sg_ref_")
    os.chdir(scratch)  # server.py makes uploads/ in cwd at import (server.py:20-21)
    server = load("ref_server", os.path.join(REF, "server/server.py"))
    client = load("ref_client", os.path.join(REF, "client/swarm"))
    worker = load("ref_worker", os.path.join(REF, "worker/worker.py"))
    app = server.app
    tc = app.test_client()
    auth = {"Authorization": "Bearer yoloswag"}
    vectors = {"note": "generated by tests/golden/gen_reference_fixtures.py from the reference "
                       "(stub-imported); fake S3 lists keys in binary order, 1,000 per page",
               "a1_chunking": [], "a5_merge": [], "a6_get_chunk": [], "a2_module_cmds": {}}

    # ---- A1: client readlines -> POST /queue -> S3 input chunk bodies
    a1_cases = [
        ("ten_b4", b"".join(b"h%d.example.com\n" % i for i in range(10)), 4),
        ("ten_b0", b"".join(b"h%d.example.com\n" % i for i in range(10)), 0),
        ("unterminated_b3", b"a.com\nb.com\nc.com\nd.com", 3),
        ("batch_gt_len", b"x.org\ny.org\n", 50),
        ("b1", b"p\nq\nr\n", 1),
        ("crlf_and_cr", b"a.com\r\nb.com\rc.com\n\nd.com\r\n", 2),
        ("blank_lines", b"\n\nu.io\n\n\nv.io\n", 3),
        ("many_chunks", b"".join(b"s%02d.t.net\n" % i for i in range(23)), 2),
        ("utf8", "münchen.de\nété.fr\nplain.com\n".encode(), 2),
        ("single_line_no_nl", b"only.example", 0),
    ]
    for name, data, batch in a1_cases:
        S3.objs.clear()
        fn = os.path.join(scratch, name + ".txt")
        with open(fn, "wb") as f:
            f.write(data)
        jc = client.JobClient("http://offline", "yoloswag")
        jc.start_scan(fn, "dnsx", 0, batch, scan_id="scan_%s" % name.replace("_", ""))
        body = FakeRequests.last_post
        r = tc.post("/queue", json=body, headers=auth)
        sid = body["scan_id"]
        chunks = []
        i = 0
        while True:
            k = "%s/input/chunk_%d.txt" % (sid, i)
            if k not in S3.objs:
                break
            chunks.append(b64(S3.objs[k]))
            i += 1
        vectors["a1_chunking"].append({"name": name, "file": b64(data), "batch_size": batch,
                                       "file_content": body["file_content"],
                                       "status": r.status_code, "chunks": chunks})

    # ---- A5: output chunks -> GET /raw
    def raw_case(name, objs, scan="merge_1700000000"):
        S3.objs.clear()
        for k, v in objs.items():
            S3.objs["%s/output/%s" % (scan, k)] = v
        r = tc.get("/raw/" + scan, headers=auth)
        vectors["a5_merge"].append({"name": name, "scan_id": scan,
                                    "objects": {k: b64(v) for k, v in objs.items()},
                                    "status": r.status_code, "raw": b64(r.data)})

    raw_case("twelve_chunks", {"chunk_%d.txt" % i: b"out%da\nout%db\n" % (i, i) for i in range(12)})
    raw_case("no_trailing_newline", {"chunk_0.txt": b"a\nb", "chunk_1.txt": b"c\nd",
                                     "chunk_2.txt": b"e\n"})
    raw_case("non_txt_filtered", {"chunk_0.txt": b"k1\n", "chunk_1.txt.part": b"zz\n",
                                  "notes.json": b"{}\n", "chunk_1.txt": b"k2\n"})
    raw_case("empty_chunks", {"chunk_0.txt": b"", "chunk_1.txt": b"x\n", "chunk_2.txt": b""})
    raw_case("utf8_and_cr", {"chunk_0.txt": "ü.de\r\n".encode(), "chunk_1.txt": b"\r\n\n"})
    raw_case("page_limit_1005", {"chunk_%d.txt" % i: b"r%d\n" % i for i in range(1005)})

    # ---- A6: /get-chunk JSON
    S3.objs.clear()
    S3.objs["g_1/output/chunk_3.txt"] = b"alpha\nbeta\n"
    r = tc.get("/get-chunk/g_1/3", headers=auth)
    vectors["a6_get_chunk"].append({"scan_id": "g_1", "chunk_id": "3", "object": b64(b"alpha\nbeta\n"),
                                    "json": r.get_json(), "status": r.status_code})

    # ---- A2: worker module command templates
    os.chdir(os.path.join(REF, "worker"))
    jp = worker.JobProcessor("http://offline", "k", "w1", 1, "", "")
    for fn in sorted(os.listdir("modules")):
        mod = fn[:-5]
        vectors["a2_module_cmds"][mod] = jp.get_module_cmd(mod, "downloads/chunk_7.txt",
                                                           "uploads/s_1/output/chunk_7.txt")
    os.chdir(scratch)

    with open(OUT, "w") as f:
        json.dump(vectors, f, indent=1, sort_keys=True)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
