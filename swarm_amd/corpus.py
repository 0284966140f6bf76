"""Deterministic synthetic corpora for the BASELINE.json configs.

C1/C2 subdomains: label [a-z0-9]{3,14} + '.' + optional one of api./dev./www./mail. +
target{0..63}.com, one per line. Records are draws from a universe of `n` names (seeded),
so about 63 % of lines are unique (n draws from n items). The prior scan is the sorted
unique set minus every name whose universe id is divisible by 10 (90 % of it).

All generation is vectorized numpy: 10M lines take a few seconds.
"""
from __future__ import annotations

import numpy as np

ALPHA = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789", dtype=np.uint8)
OPTS = [b"", b"api.", b"dev.", b"www.", b"mail."]


def _mix(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64, copy=True)
    with np.errstate(over="ignore"):
        x ^= x >> np.uint64(30)
        x *= np.uint64(0xBF58476D1CE4E5B9)
        x ^= x >> np.uint64(27)
        x *= np.uint64(0x94D049BB133111EB)
        x ^= x >> np.uint64(31)
    return x


def render_names(ids: np.ndarray, salt: int = 0) -> tuple:
    """Render universe ids to subdomain bytes. Returns (matrix (m, W) uint8, lengths)."""
    ids = ids.astype(np.uint64)
    with np.errstate(over="ignore"):
        h = _mix(ids * np.uint64(0x9E3779B97F4A7C15) + np.uint64(salt))
    m = ids.size
    L = (3 + (h % np.uint64(12))).astype(np.int64)                 # label length 3..14
    lab = np.empty((m, 14), dtype=np.uint8)
    g = h
    for j in range(14):
        with np.errstate(over="ignore"):
            g = _mix(g + np.uint64(j + 1))
        lab[:, j] = ALPHA[(g % np.uint64(36)).astype(np.int64)]
    opt = ((h >> np.uint64(40)) % np.uint64(5)).astype(np.int64)
    tgt = ((h >> np.uint64(48)) % np.uint64(64)).astype(np.int64)
    # middle: '.' + opt (padded to 6)
    mid = np.zeros((m, 6), dtype=np.uint8)
    mid[:, 0] = ord(".")
    mid_len = np.ones(m, dtype=np.int64)
    for k, o in enumerate(OPTS):
        sel = opt == k
        if o:
            mid[sel, 1:1 + len(o)] = np.frombuffer(o, dtype=np.uint8)
            mid_len[sel] = 1 + len(o)
    # tail: target{i}.com
    tail = np.zeros((m, 13), dtype=np.uint8)
    tail[:, :6] = np.frombuffer(b"target", dtype=np.uint8)
    two = tgt >= 10
    d0 = np.where(two, tgt // 10, tgt)
    tail[:, 6] = ord("0") + d0
    tail[two, 7] = ord("0") + tgt[two] % 10
    nd = np.where(two, 2, 1)
    com = np.frombuffer(b".com", dtype=np.uint8)
    for j in range(4):
        col = 6 + nd + j
        tail[np.arange(m), col] = com[j]
    tail_len = 6 + nd + 4
    W = 14 + 6 + 13
    mat = np.zeros((m, W), dtype=np.uint8)
    msk = np.zeros((m, W), dtype=bool)
    mat[:, :14] = lab
    msk[:, :14] = np.arange(14)[None, :] < L[:, None]
    mat[:, 14:20] = mid
    msk[:, 14:20] = np.arange(6)[None, :] < mid_len[:, None]
    mat[:, 20:33] = tail
    msk[:, 20:33] = np.arange(13)[None, :] < tail_len[:, None]
    return mat, msk


def _flatten(mat: np.ndarray, msk: np.ndarray, sep: int = 0x0A) -> np.ndarray:
    m, W = mat.shape
    full = np.empty((m, W + 1), dtype=np.uint8)
    full[:, :W] = mat
    full[:, W] = sep
    fm = np.empty((m, W + 1), dtype=bool)
    fm[:, :W] = msk
    fm[:, W] = True
    return full[fm]


def subdomains(n: int, seed: int = 1234, universe: int | None = None, chunk: int = 1 << 20) -> tuple:
    """(n subdomain lines as a '\\n'-terminated uint8 array, their universe ids)."""
    U = universe or max(n, 1)
    rng = np.random.default_rng(seed)
    ids = rng.integers(0, U, size=n, dtype=np.uint64)
    parts = []
    for i in range(0, n, chunk):
        mat, msk = render_names(ids[i:i + chunk])
        parts.append(_flatten(mat, msk))
    return np.concatenate(parts) if parts else np.zeros(0, dtype=np.uint8), ids


def name_rows(ids: np.ndarray) -> np.ndarray:
    """Names of `ids` as left-compacted fixed-width rows (dtype S33). Rows compare like
    their byte strings: no name contains NUL, and a shorter name is a 0-padded prefix."""
    mat, msk = render_names(ids)
    W = mat.shape[1]
    comp = np.zeros_like(mat)
    lens = msk.sum(axis=1)
    flat = mat[msk]
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    valid = np.arange(W)[None, :] < lens[:, None]
    idx = starts[:, None] + np.arange(W)[None, :]
    comp[valid] = flat[idx[valid]]
    return comp.view("S%d" % W).reshape(-1)


def serialize_rows(rows: np.ndarray) -> np.ndarray:
    """Fixed-width S rows -> '\n'-terminated byte buffer."""
    W = rows.dtype.itemsize
    mat = rows.view(np.uint8).reshape(-1, W)
    return _flatten(mat, mat != 0)


def sorted_unique_rows(ids: np.ndarray) -> np.ndarray:
    return np.unique(name_rows(np.unique(ids)))


def prior_rows(ids: np.ndarray) -> np.ndarray:
    u = np.unique(ids)
    return np.unique(name_rows(u[(u % np.uint64(10)) != 0]))


def prior_of(ids: np.ndarray) -> np.ndarray:
    """The prior scan: sort -u of the names of the drawn ids except ids % 10 == 0 (about
    90 % of this scan's unique set), serialized."""
    return serialize_rows(prior_rows(ids))


TITLES = [b"Welcome to nginx!", b"Index of /", b"Grafana", b"Jenkins", b"phpMyAdmin", b"Login",
          b"IIS Windows Server", b"Apache2 Ubuntu Default Page: It works", b"Dashboard", b"404 Not Found",
          b"Sign in", b"Kibana", b"GitLab", b"RabbitMQ Management", b"Swagger UI", b"Home"]
SERVERS = [b"nginx/1.18.0", b"Apache/2.4.41 (Ubuntu)", b"Microsoft-IIS/10.0", b"cloudflare", b"LiteSpeed",
           b"openresty/1.19.3.1", b"Jetty(9.4.z-SNAPSHOT)", b"gunicorn/20.0.4", b"envoy", b"AmazonS3"]


def httpx_pool(sigs, pool: int = 1 << 16, plant: float = 0.01, seed: int = 0):
    """A pool of httpx-style result lines `url [status] [title] [server]` (~100 B); a
    `plant` fraction carries a signature inside the title."""
    import random
    rng = random.Random(seed)
    rows = []
    for _ in range(pool):
        title = rng.choice(TITLES)
        if sigs and rng.random() < plant:
            s = rng.choice(sigs)
            k = rng.randrange(len(title) + 1)
            title = title[:k] + s + title[k:]
        rows.append(b"https://%s.target%d.com/%s [%d] [%s] [%s] [%d]" % (
            b"".join(bytes([rng.choice(b"abcdefghijklmnopqrstuvwxyz0123456789")]) for _ in range(rng.randint(3, 12))),
            rng.randrange(64), rng.choice([b"", b"login", b"admin/", b"index.php", b"api/v1/status"]),
            rng.choice([200, 301, 302, 403, 404, 500]), title.replace(b"\n", b" "), rng.choice(SERVERS),
            rng.randrange(100, 99999)))
    return rows


def lines_from_pool(rows, n: int, seed: int = 0, chunk: int = 1 << 20) -> np.ndarray:
    """n lines drawn uniformly from `rows`, '\\n'-terminated (vectorized, chunked)."""
    W = max(len(r) for r in rows)
    mat = np.zeros((len(rows), W), dtype=np.uint8)
    lens = np.array([len(r) for r in rows], dtype=np.int64)
    for i, r in enumerate(rows):
        mat[i, :len(r)] = np.frombuffer(r, dtype=np.uint8)
    msk = np.arange(W)[None, :] < lens[:, None]
    rng = np.random.default_rng(seed)
    parts = []
    for i in range(0, n, chunk):
        idx = rng.integers(0, len(rows), size=min(chunk, n - i))
        parts.append(_flatten(mat[idx], msk[idx]))
    return np.concatenate(parts) if parts else np.zeros(0, dtype=np.uint8)


def chunk_layout(lines_arr: np.ndarray, n_chunks: int) -> list:
    """Split a '\\n'-terminated buffer into n_chunks worker-output chunks at line boundaries
    (the per-chunk outputs the server merges, server/server.py:399-412)."""
    nl = np.flatnonzero(lines_arr == 0x0A)
    R = nl.size
    bounds = [0]
    for k in range(1, n_chunks):
        r = (R * k) // n_chunks
        bounds.append(int(nl[r - 1]) + 1 if r > 0 else 0)
    bounds.append(lines_arr.size)
    return [lines_arr[bounds[i]:bounds[i + 1]] for i in range(n_chunks)]


# ------------------------------------------------------------------ C4: nmap-style banners
_SYL = [b"Open", b"Pure", b"Pro", b"Free", b"Net", b"Cyber", b"Micro", b"Mega", b"Secure", b"Fast", b"Quick",
        b"Blue", b"Red", b"Iron", b"Cloud", b"Data", b"Web", b"Mail", b"File", b"Core", b"Edge", b"Star",
        b"Nova", b"Zen", b"Arc", b"Hyper", b"Ultra", b"Smart", b"Tiny", b"Big"]
_SUF = [b"SSH", b"FTPd", b"Mail", b"Web", b"Srv", b"Box", b"Gate", b"Hub", b"Link", b"Wall", b"Stack", b"Store",
        b"Proxy", b"DB", b"Cache", b"Queue", b"Vault", b"Shell", b"Port", b"Node"]

# nmap-service-probes-style `match` templates ({p} = product). Each yields one signature
# per product; the banner generator renders matching lines with concrete versions.
_FAMILIES = [
    (rb"^SSH-2\.0-{p}[_-]([\d.]+)(?:p\d+)?", b"SSH-2.0-{p}_{v}p1 Debian-{b}"),
    (rb"^220 [\w.-]+ ESMTP {p}(?: \(([\w ]+)\))?", b"220 mx{b}.mail.example.net ESMTP {p} (Ubuntu) ready at {v}"),
    (rb"^220[- ]{p} FTP [Ss]erver \(Version ([\w.]+)\)", b"220 {p} FTP server (Version {v}) ready."),
    (rb"^HTTP/1\.[01] \d{3} .*Server: {p}/([\d.]+)",
     b"HTTP/1.1 200 OK Date: Mon, 12 Oct 2026 10:{b} GMT Content-Type: text/html Server: {p}/{v}"),
    (rb"^\+OK {p} POP3 (?:server )?ready", b"+OK {p} POP3 server ready <{b}@host>"),
    (rb"^\* OK \[CAPABILITY IMAP4rev1[^\]]*\] {p} ready", b"* OK [CAPABILITY IMAP4rev1 IDLE] {p} ready"),
    (rb"^{p} ([\d.]+) \(build (\d+)\)", b"{p} {v} (build {b})"),
    (rb"^-ERR unknown command '{p}[^']*'", b"-ERR unknown command '{p}-{b}'"),
]


def nmap_products(n: int, seed: int = 7) -> list:
    rng = np.random.default_rng(seed)
    out, seen = [], set()
    while len(out) < n:
        a, b = _SYL[rng.integers(len(_SYL))], _SUF[rng.integers(len(_SUF))]
        p = a + b + (b"%d" % rng.integers(100) if rng.random() < 0.7 else b"")
        if p not in seen:
            seen.add(p)
            out.append(p)
    return out


def nmap_signatures(n_products: int = 1100, seed: int = 7) -> list:
    """len(_FAMILIES) * n_products regexes (C4's synthetic nmap-style families)."""
    prods = nmap_products(n_products, seed)
    return [t.replace(b"{p}", p) for t, _ in _FAMILIES for p in prods]


def banner_pool(n_products: int = 1100, pool: int = 1 << 16, match_frac: float = 0.3, seed: int = 9) -> list:
    """Port-banner lines (~60 B): match_frac render a signature family with a known product,
    the rest the same shapes with unknown products."""
    rng = np.random.default_rng(seed)
    prods = nmap_products(n_products, 7)
    rows = []
    for _ in range(pool):
        fam = _FAMILIES[rng.integers(len(_FAMILIES))][1]
        if rng.random() < match_frac:
            p = prods[rng.integers(len(prods))]
        else:
            p = b"Unk" + _SUF[rng.integers(len(_SUF))] + b"%d" % rng.integers(1000)
        v = b"%d.%d.%d" % (rng.integers(10), rng.integers(20), rng.integers(30))
        rows.append(fam.replace(b"{p}", p).replace(b"{v}", v).replace(b"{b}", b"%d" % rng.integers(100000)))
    return rows


# ------------------------------------------------------------------ §8(f): module-output formats
_TECH = [b"Nginx:1.18.0", b"PHP:7.4.3", b"jQuery", b"Bootstrap:4.5.2", b"WordPress:5.8", b"Cloudflare", b"React",
         b"Amazon S3", b"Apache HTTP Server:2.4.41", b"Ubuntu", b"Google Font API", b"Font Awesome", b"HSTS",
         b"Varnish", b"Express", b"Node.js", b"Jenkins:2.303", b"Grafana:8.1.2", b"Kibana", b"GitLab"]
_UNI = ["\u00e9t\u00e9", "\u65e5\u672c\u8a9e", "\U0001F600 smile", "caf\u00e9 \u2014 menu", "\u0414\u043e\u043c"]


def httpx_json_pool(pool: int = 1 << 12, seed: int = 5) -> list:
    """httpx -json result lines (the keys and value shapes httpx v1 prints), serialized the
    way Go's encoding/json does (HTML characters escaped as \\u003c etc., non-ASCII kept)."""
    import json
    import random
    rng = random.Random(seed)
    rows = []
    for _ in range(pool):
        host = "%s.target%d.com" % ("".join(rng.choice("abcdefghijklmnopqrstuvwxyz0123456789")
                                           for _ in range(rng.randint(3, 12))), rng.randrange(64))
        scheme = rng.choice(["http", "https"])
        port = {"http": "80", "https": "443"}[scheme]
        title = rng.choice(TITLES).decode()
        r = rng.random()
        if r < 0.1:
            title = rng.choice(_UNI)
        elif r < 0.15:
            title = title + ' <b>"quoted"</b> & \\ back'
        elif r < 0.17:
            title = "line1\nline2\ttab"
        elif r < 0.19:
            title = ""
        obj = {
            "timestamp": "2026-10-12T10:%02d:%02d.%06d+00:00" % (rng.randrange(60), rng.randrange(60),
                                                                 rng.randrange(10 ** 6)),
            "hash": {"body_md5": "%032x" % rng.getrandbits(128), "header_md5": "%032x" % rng.getrandbits(128)},
            "port": port,
            "url": "%s://%s" % (scheme, host),
            "input": host,
            "title": title,
            "scheme": scheme,
            "webserver": rng.choice(SERVERS).decode(),
            "content_type": rng.choice(["text/html", "application/json", "text/plain"]),
            "method": "GET",
            "host": "%d.%d.%d.%d" % tuple(rng.randrange(256) for _ in range(4)),
            "path": "/",
            "time": "%.6fms" % (rng.random() * 900),
            "a": ["%d.%d.%d.%d" % tuple(rng.randrange(256) for _ in range(4)) for _ in range(rng.randint(1, 3))],
            "tech": [t.decode() for t in rng.sample(_TECH, rng.randint(0, 4))],
            "words": rng.randrange(5000),
            "lines": rng.randrange(500),
            "status_code": rng.choice([200, 301, 302, 403, 404, 500]),
            "content_length": rng.randrange(100000),
            "failed": False,
            "knowledgebase": {"PageType": "nonerror", "pHash": 0},
        }
        if rng.random() < 0.3:
            del obj["tech"]
        s = json.dumps(obj, ensure_ascii=False, separators=(",", ":"))
        s = s.replace("<", "\\u003c").replace(">", "\\u003e").replace("&", "\\u0026")
        rows.append(s.encode("utf-8"))
    return rows


def nmap_report(n_hosts: int, seed: int = 11, max_ports: int = 6) -> bytes:
    """nmap -sV -oN text for n_hosts hosts (header, per-host report, port table, footer)."""
    import random
    rng = random.Random(seed)
    svc = [(22, b"ssh", b"OpenSSH 8.2p1 Ubuntu 4ubuntu0.5 (Ubuntu Linux; protocol 2.0)"),
           (25, b"smtp", b"Postfix smtpd"), (53, b"domain", b"ISC BIND 9.16.1"), (80, b"http", b"nginx 1.18.0"),
           (443, b"ssl/http", b"nginx 1.18.0"), (3306, b"mysql", b"MySQL 5.7.33"),
           (8080, b"http-proxy", b""), (8443, b"ssl/https-alt", b"")]
    out = [b"# Nmap 7.80 scan initiated Mon Oct 12 10:00:00 2026 as: nmap -sV -iL input -oN output"]
    for h in range(n_hosts):
        name = b"h%d.target%d.com" % (rng.randrange(10 ** 6), rng.randrange(64))
        ip = b"%d.%d.%d.%d" % tuple(rng.randrange(256) for _ in range(4))
        out.append(b"Nmap scan report for %s (%s)" % (name, ip) if rng.random() < 0.8
                   else b"Nmap scan report for %s" % ip)
        out.append(b"Host is up (0.0%dms latency)." % rng.randrange(100))
        out.append(b"Not shown: 996 filtered ports")
        out.append(b"PORT     STATE  SERVICE  VERSION")
        for port, name_, ver in rng.sample(svc, rng.randint(0, max_ports)):
            state = rng.choice([b"open", b"open", b"open", b"closed", b"filtered"])
            proto = b"tcp" if port != 53 or rng.random() < 0.5 else b"udp"
            out.append(b"%s/%s %s %s %s" % (b"%d" % port, proto, state, name_, ver))
        if rng.random() < 0.3:
            out.append(b"Service Info: OS: Linux; CPE: cpe:/o:linux:linux_kernel")
        out.append(b"")
    out.append(b"Service detection performed. Please report any incorrect results at https://nmap.org/submit/ .")
    out.append(b"# Nmap done at Mon Oct 12 10:05:00 2026 -- %d IP addresses (%d hosts up) scanned in 300.00 seconds"
               % (n_hosts, n_hosts))
    return b"\n".join(out) + b"\n"


# ------------------------------------------------------------------ C5: host:port records
PORTS = [b"21", b"22", b"23", b"25", b"53", b"80", b"81", b"110", b"111", b"135", b"139", b"143", b"443", b"445",
         b"465", b"587", b"993", b"995", b"1433", b"1723", b"2049", b"3000", b"3306", b"3389", b"5432", b"5900",
         b"6379", b"8000", b"8080", b"8443", b"9200", b"27017"]


def host_pool_gpu(n_hosts: int, seed: int = 5, device="cuda", chunk: int = 1 << 21):
    """n_hosts subdomain names rendered on the host (render_names), left-aligned on the GPU:
    (matrix (n_hosts, 33) uint8, lengths int32)."""
    import torch
    mats, lens = [], []
    for i in range(0, n_hosts, chunk):
        ids = np.arange(i, min(n_hosts, i + chunk), dtype=np.uint64)
        mat, msk = render_names(ids, salt=seed)
        m = torch.from_numpy(mat).to(device)
        k = torch.from_numpy(msk).to(device)
        order = torch.sort((~k).to(torch.uint8), dim=1, stable=True).indices
        mats.append(torch.gather(m, 1, order))
        lens.append(k.sum(1).to(torch.int32))
    return torch.cat(mats), torch.cat(lens)


_ALPHA_T = b"abcdefghijklmnopqrstuvwxyz0123456789"


def _tmix(x):
    """splitmix64 finalizer on int64 tensors (wrapping multiplies, logical shifts)."""
    def shr(v, k):
        return (v >> k) & ((1 << (64 - k)) - 1)
    c1 = 0xBF58476D1CE4E5B9 - (1 << 64)
    c2 = 0x94D049BB133111EB - (1 << 64)
    x = x ^ shr(x, 30)
    x = x * c1
    x = x ^ shr(x, 27)
    x = x * c2
    return x ^ shr(x, 31)


def host_pool_torch(n_hosts: int, seed: int = 5, device="cuda", chunk: int = 1 << 23):
    """n_hosts host names rendered on the GPU (label of 6..14 [a-z0-9], optional
    api./dev./www./mail., target{0..63}.com), left-aligned: (matrix (n, 33) uint8, lengths)."""
    import torch
    alpha = torch.frombuffer(bytearray(_ALPHA_T), dtype=torch.uint8).to(device)
    opts = [b"", b"api", b"dev", b"www", b"mail"]
    optm = torch.zeros((5, 6), dtype=torch.uint8)
    optl = torch.zeros(5, dtype=torch.int64)
    for k, o in enumerate(opts):
        b = (b"." + o) if o else b""
        optm[k, :len(b)] = torch.frombuffer(bytearray(b or b"\0"), dtype=torch.uint8)[:len(b)]
        optl[k] = len(b)
    optm, optl = optm.to(device), optl.to(device)
    tails = torch.zeros((64, 13), dtype=torch.uint8)
    taill = torch.zeros(64, dtype=torch.int64)
    for t in range(64):
        b = b".target%d.com" % t
        tails[t, :len(b)] = torch.frombuffer(bytearray(b), dtype=torch.uint8)
        taill[t] = len(b)
    tails, taill = tails.to(device), taill.to(device)
    mats, lens = [], []
    for i in range(0, n_hosts, chunk):
        ids = torch.arange(i, min(n_hosts, i + chunk), dtype=torch.int64, device=device)
        h = _tmix(ids * 0x1E3779B97F4A7C15 + seed)
        m = ids.numel()
        L = 6 + (h & 0x7FFFFFFF) % 9
        row = torch.zeros((m, 33), dtype=torch.uint8, device=device)
        msk = torch.zeros((m, 33), dtype=torch.bool, device=device)
        g = h
        for j in range(14):
            g = _tmix(g + (j + 1))
            row[:, j] = alpha[(g & 0x7FFFFFFF) % 36]
        col = torch.arange(33, device=device)
        msk[:, :14] = col[None, :14] < L[:, None]
        o = ((h >> 40) & 0xFFFFFF) % 5
        row[:, 14:20] = optm[o]
        msk[:, 14:20] = col[None, :6] < optl[o][:, None]
        t = ((h >> 48) & 0xFFFF) % 64
        row[:, 20:33] = tails[t]
        msk[:, 20:33] = col[None, :13] < taill[t][:, None]
        order = torch.sort((~msk).to(torch.uint8), dim=1, stable=True).indices
        mats.append(torch.gather(row, 1, order))
        lens.append(msk.sum(1).to(torch.int32))
    return torch.cat(mats), torch.cat(lens)


def ip_pool_torch(n_hosts: int, seed: int = 5, device="cuda", chunk: int = 1 << 23):
    """n_hosts (<= 2**26) distinct IPv4 addresses rendered on the GPU — all in 10.0.0.0/8
    when n_hosts <= 2**24 (an internal-range port scan: every record shares its first 3
    bytes and many their first 7), else 10.x.y.z .. 13.x.y.z — left-aligned: (matrix (n, 15)
    uint8, lengths). Host h -> address (h * odd + seed) mod 2**bits above 10.0.0.0, a
    bijection, so hosts never collide."""
    import torch
    if n_hosts > 1 << 26:
        raise ValueError("ip_pool_torch: at most 2**26 hosts")
    bits = 24 if n_hosts <= 1 << 24 else 26
    mats, lens = [], []
    for i in range(0, n_hosts, chunk):
        ids = torch.arange(i, min(n_hosts, i + chunk), dtype=torch.int64, device=device)
        x = (ids * 0x2F0B3A5 + seed) & ((1 << bits) - 1)
        octs = [10 + (x >> 24), (x >> 16) & 255, (x >> 8) & 255, x & 255]
        m = ids.numel()
        row = torch.zeros((m, 15), dtype=torch.uint8, device=device)
        msk = torch.zeros((m, 15), dtype=torch.bool, device=device)
        col = 0
        for k, o in enumerate(octs):
            row[:, col], msk[:, col] = (48 + o // 100).to(torch.uint8), o >= 100
            row[:, col + 1], msk[:, col + 1] = (48 + (o // 10) % 10).to(torch.uint8), o >= 10
            row[:, col + 2], msk[:, col + 2] = (48 + o % 10).to(torch.uint8), True
            col += 3
            if k < 3:
                row[:, col], msk[:, col] = 46, True
                col += 1
        order = torch.sort((~msk).to(torch.uint8), dim=1, stable=True).indices
        mats.append(torch.gather(row, 1, order))
        lens.append(msk.sum(1).to(torch.int32))
    return torch.cat(mats), torch.cat(lens)


def hostport_ids(n: int, lo: int, hi: int, seed: int, per_piece: int = 50_000_000, device="cuda"):
    """The combo ids hostport_pieces draws (uniform in [lo, hi), one torch.Generator seeded
    with `seed`), yielded piece by piece: the same stream for the same arguments."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    for s in range(0, n, per_piece):
        m = min(per_piece, n - s)
        yield torch.randint(lo, hi, (m,), generator=g, device=device, dtype=torch.int64)


def hostport_port(c, ports_per_host: int | None = None):
    """Port index (into PORTS) of combo ids c: with k = ports_per_host slots per host, a hash
    of the combo (a host keeps a few open ports); without it, c % len(PORTS)."""
    P = len(PORTS)
    return (c % P) if ports_per_host is None else ((_tmix(c * 0x2545F4914F6CDD1D) & 0x7FFFFFFF) % P)


def hostport_pieces(pool, n: int, lo: int, hi: int, seed: int, per_piece: int = 50_000_000,
                    ports_per_host: int | None = None):
    """n 'host:port' records ('\\n'-terminated) for combo ids drawn uniformly from [lo, hi),
    rendered on the GPU, as a list of device byte tensors of <= per_piece records each (each
    ends at a record boundary). Combo c: host c // k and, with ports_per_host = k, the k-slot
    port PORTS[hash(c) % 32] (a host keeps a few open ports, as in a port scan); without it,
    k = len(PORTS) and port c % k."""
    import torch
    mat, lens = pool
    dev = mat.device
    P = len(PORTS)
    K = ports_per_host or P
    pm = torch.zeros((P, 8), dtype=torch.uint8)
    pl = torch.zeros(P, dtype=torch.int64)
    for i, p in enumerate(PORTS):
        b = b":" + p + b"\n"
        pm[i, :len(b)] = torch.frombuffer(bytearray(b), dtype=torch.uint8)
        pl[i] = len(b)
    pm, pl = pm.to(dev), pl.to(dev)
    W = mat.shape[1]
    if (hi - 1) // K >= mat.shape[0]:  # host ids index the pool on the GPU: check here
        raise ValueError("combo ids up to %d need %d hosts; the pool has %d" % (hi - 1, (hi - 1) // K + 1, mat.shape[0]))
    out = []
    cols = torch.arange(W + 8, device=dev)
    for c in hostport_ids(n, lo, hi, seed, per_piece, dev):
        m = c.numel()
        h = c // K
        p = hostport_port(c, ports_per_host)
        rows = torch.zeros((m, W + 8), dtype=torch.uint8, device=dev)
        rows[:, :W] = mat[h]
        hl = lens[h].to(torch.int64)
        rows.scatter_(1, hl[:, None] + torch.arange(8, device=dev)[None, :], pm[p])
        out.append(rows[cols[None, :] < (hl + pl[p])[:, None]])
        del rows, c, h, p, hl
    return out


# ------------------------------------------------------------------ X1: httpx host lines
def httpx_tails(sigs, n_tails: int = 4096, plant: float = 0.05, seed: int = 0) -> tuple:
    """A pool of httpx result tails `/path [status] [title] [server] [size]` as a masked byte
    matrix; a `plant` fraction of titles carries one of `sigs`."""
    rows = [r.split(b".com", 1)[1] for r in httpx_pool(sigs, n_tails, plant, seed=seed)]
    W = max(len(r) for r in rows)
    mat = np.zeros((len(rows), W), dtype=np.uint8)
    lens = np.array([len(r) for r in rows], dtype=np.int64)
    for i, r in enumerate(rows):
        mat[i, :len(r)] = np.frombuffer(r, dtype=np.uint8)
    return mat, np.arange(W)[None, :] < lens[:, None]


def httpx_rows(ids: np.ndarray, tails: tuple, chunk: int = 1 << 20) -> np.ndarray:
    """One httpx line per universe id: `https://` + the id's subdomain name + the tail the id
    always gets (a URL answers with the same title and server on every scan), so two lines
    are equal exactly when their ids are. '\\n'-terminated."""
    tmat, tmsk = tails
    pre = np.frombuffer(b"https://", dtype=np.uint8)
    parts = []
    for i in range(0, ids.size, chunk):
        sub = ids[i:i + chunk]
        nmat, nmsk = render_names(sub)
        t = (_mix(sub.astype(np.uint64) ^ np.uint64(0x5bd1e995)) % np.uint64(tmat.shape[0])).astype(np.int64)
        m = sub.size
        mat = np.concatenate([np.broadcast_to(pre, (m, pre.size)), nmat, tmat[t]], axis=1)
        msk = np.concatenate([np.ones((m, pre.size), dtype=bool), nmsk, tmsk[t]], axis=1)
        parts.append(_flatten(mat, msk))
    return np.concatenate(parts) if parts else np.zeros(0, dtype=np.uint8)


def httpx_hosts(n: int, tails: tuple, seed: int = 1234, universe: int | None = None) -> tuple:
    """(n httpx lines drawn from a universe of n URLs like the C2 subdomains, their ids)."""
    U = universe or max(n, 1)
    ids = np.random.default_rng(seed).integers(0, U, size=n, dtype=np.uint64)
    return httpx_rows(ids, tails), ids


def prior_ids(ids: np.ndarray) -> np.ndarray:
    """The prior scan's ids: this scan's distinct ids except those divisible by 10."""
    u = np.unique(ids)
    return u[(u % np.uint64(10)) != 0]


def generic_regexes(pats, probe_banners: int = 400, max_frac: float = 0.1, seed: int = 17) -> list:
    """Indices of the regexes that fire on more than `max_frac` of banners from UNKNOWN products
    (a deterministic probe): extractor-style patterns such as
    `([a-zA-Z0-9.-]+).([a-z0-9]+).([a-z0-9]+).\\w+` that say nothing about a service. A service
    fingerprint set (nmap-service-probes `match` lines) has none of them; C4 leaves them out
    so that the fraction of banners matched reflects the known-product share."""
    import re
    probe = banner_pool(pool=probe_banners, match_frac=0.0, seed=seed)
    out = []
    for i, p in enumerate(pats):
        try:
            c = re.compile(p)
        except re.error:
            continue
        if sum(1 for b in probe if c.search(b)) > max_frac * len(probe):
            out.append(i)
    return out


def c4_signatures(corpus_regexes) -> tuple:
    """(C4 signature list, number of corpus regexes left out as generic): the nuclei corpus
    regexes minus generic_regexes(), plus the nmap-style families."""
    gen = set(generic_regexes(corpus_regexes))
    return [p for i, p in enumerate(corpus_regexes) if i not in gen] + nmap_signatures(), len(gen)
