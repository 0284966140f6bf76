"""Python model of the round-5 wave-per-line JSON scan (k_json_scan_w in
json_scan_wave_per_line_r5.patch, a measured loss kept out of the tree), lane by lane, used
to debug the kernel's logic on the CPU: python3 tools/experiments/json_wave_model.py.
Compares the member spans it keeps (last occurrence per key, line ok flag) with the
oracle's _json_members on random and test-suite-like lines at every alignment."""
import json
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from oracle import semantics as S  # noqa: E402

NONE = 0xffffffff
T = {(0, 0): 0, (0, 1): 1, (0, 2): 0, (1, 0): 1, (1, 1): 0, (1, 2): 2, (2, 0): 1, (2, 1): 1, (2, 2): 1}


def bits(m):
    j = 0
    while m:
        if m & 1:
            yield j
        m >>= 1
        j += 1


def hib(m):
    return m.bit_length() - 1


def lob(m):
    return (m & -m).bit_length() - 1


def scan_line(buf, sx, sy, keys):
    st, depth, bad, done = 0, 0, False, False
    open_pos = close_pos = NONE
    lo1 = lb1 = 0
    ls = (False, 0, 0, False)
    pm_on, pm_vbs, pm_c, pm_key = False, False, 0, 0
    own = {}
    cb = sx & ~15
    while cb < sy and not bad:
        L = []
        for lane in range(64):
            lb = cb + 16 * lane
            vm = 0
            if lb < sy and lb + 16 > sx:
                lo = sx - lb if sx > lb else 0
                hi = min(sy - lb, 16)
                vm = ((1 << hi) - 1) & ~((1 << lo) - 1)
            m = dict(lb=lb, vm=vm, qm=0, bsm=0, om=0, cm=0, clm=0, cmm=0, by={})
            for j in range(16):
                if vm >> j & 1:
                    b = buf[lb + j]
                    m["by"][j] = b
                    if b == 0x22: m["qm"] |= 1 << j
                    if b == 0x5c: m["bsm"] |= 1 << j
                    if b in b"{[": m["om"] |= 1 << j
                    if b in b"}]": m["cm"] |= 1 << j
                    if b == 0x3a: m["clm"] |= 1 << j
                    if b == 0x2c: m["cmm"] |= 1 << j
            L.append(m)
        # string state per lane start
        s = st
        for m in L:
            m["s_in"] = s
            inb = oq = cq = 0
            for j in range(16):
                cls = (m["qm"] >> j & 1) | ((m["bsm"] >> j & 1) << 1)
                if s != 0: inb |= 1 << j
                if cls == 1:
                    if s == 0: oq |= 1 << j
                    elif s == 1: cq |= 1 << j
                s = T[(s, cls)]
            m.update(inb=inb, oq=oq, cq=cq)
        st_next = s
        d = depth
        for m in L:
            out = ~m["inb"] & m["vm"]
            m["o_om"], m["o_cm"], m["o_cl"], m["o_cma"] = m["om"] & out, m["cm"] & out, m["clm"] & out, m["cmm"] & out
            m["d0"] = d
            d += bin(m["o_om"]).count("1") - bin(m["o_cm"]).count("1")
        depth_next = d
        for m in L:
            E = m["oq"] | m["o_om"] | m["o_cm"] | m["o_cl"] | m["o_cma"]
            m["E"] = E
            d1cl = d1cm = d1cb = 0
            d0op = 16
            lbad = False
            d = m["d0"]
            for j in bits(E):
                bit = 1 << j
                if m["oq"] & bit:
                    if d == 0: lbad = True
                elif m["o_om"] & bit:
                    if d == 0:
                        if m["by"][j] == ord("["): lbad = True
                        if d0op == 16: d0op = j
                    d += 1
                elif m["o_cm"] & bit:
                    if d == 0: lbad = True
                    elif d == 1:
                        if m["by"][j] == ord("]"): lbad = True
                        d1cb |= bit
                    d -= 1
                elif d == 1:
                    if m["o_cl"] & bit: d1cl |= bit
                    else: d1cm |= bit
            m.update(d1cl=d1cl, d1cm=d1cm, d1cb=d1cb, d0op=d0op, lbad=lbad)
        bad = bad or any(m["lbad"] for m in L)
        if open_pos == NONE:
            for m in L:
                if m["d0op"] < 16:
                    open_pos = m["lb"] + m["d0op"]; break
        if not done:
            for m in L:
                if m["d1cb"]:
                    done = True
                    close_pos = m["lb"] + lob(m["d1cb"])
                    bad = bad or any(mm["E"] and mm["lb"] + hib(mm["E"]) > close_pos for mm in L)
                    break
        else:
            bad = bad or any(mm["E"] for mm in L)
        depth, st = depth_next, st_next
        if bad:
            break
        # before-lane values
        for i, m in enumerate(L):
            src = [k for k in range(i) if L[k]["oq"]]
            m["lo_prev"] = (L[src[-1]]["lb"] + hib(L[src[-1]]["oq"]) + 1) if src else lo1
            src = [k for k in range(i) if L[k]["bsm"]]
            m["lb_prev"] = (L[src[-1]]["lb"] + hib(L[src[-1]]["bsm"]) + 1) if src else lb1

        def str_info(m, jq):
            ob = m["oq"] & ((1 << jq) - 1)
            s = m["lb"] + hib(ob) + 1 if ob else m["lo_prev"]
            frm = s - m["lb"] if s > m["lb"] else 0
            k = (m["bsm"] & ((1 << jq) - 1) & ~((1 << frm) - 1)) != 0 or (s < m["lb"] and m["lb_prev"] > s)
            return s, k

        for m in L:
            if m["cq"]:
                jq = hib(m["cq"])
                m["lq"] = (str_info(m, jq), m["lb"] + jq)
        for i, m in enumerate(L):
            src = [k for k in range(i) if L[k]["cq"]]
            if src:
                (s_, k_), e_ = L[src[-1]]["lq"]
                m["ps"] = (True, s_, e_, k_)
            else:
                m["ps"] = ls
            m["d1"] = m["d1cl"] | m["d1cm"] | m["d1cb"]
        for i, m in enumerate(L):
            nxt = [k for k in range(i + 1, 64) if L[k]["d1"]]
            if nxt:
                mm = L[nxt[0]]
                j = lob(mm["d1"])
                m["nd"] = (mm["lb"] + j, 0 if mm["d1cl"] >> j & 1 else 1)
            else:
                m["nd"] = None
            nb = [k for k in range(i + 1, 64) if L[k]["bsm"]]
            m["nb"] = L[nb[0]]["lb"] + lob(L[nb[0]]["bsm"]) if nb else NONE
        if pm_on:
            f1 = [m for m in L if m["d1"]]
            fbl = [m for m in L if m["bsm"]]
            fb = fbl[0]["lb"] + lob(fbl[0]["bsm"]) if fbl else NONE
            if not f1:
                pm_vbs = pm_vbs or bool(fbl)
            else:
                m = f1[0]
                j = lob(m["d1"])
                t = m["lb"] + j
                if not (m["d1cl"] >> j & 1):
                    own[pm_key] = (pm_c + 1, t, pm_vbs or fb < t)
                pm_on = False
        best = {}
        pend = None
        for m in L:
            for j in bits(m["d1cl"]):
                c = m["lb"] + j
                nx = m["d1"] & ~((2 << j) - 1)
                has_t, term = True, True
                if nx:
                    jt = lob(nx)
                    t = m["lb"] + jt
                    term = not (m["d1cl"] >> jt & 1)
                elif m["nd"]:
                    t, kind = m["nd"]
                    term = kind != 0
                else:
                    has_t = False
                if not term:
                    continue
                cqb = m["cq"] & ((1 << j) - 1)
                if cqb:
                    jq = hib(cqb)
                    (ks, kesc) = str_info(m, jq)
                    ke = m["lb"] + jq
                elif m["ps"][0]:
                    _, ks, ke, kesc = m["ps"]
                else:
                    ks = ke = 0; kesc = False
                kb = bytes(buf[ks:ke])
                if kesc:
                    try:
                        kb = json.loads(b'"' + kb + b'"').encode("utf-8", "surrogatepass")
                    except ValueError:
                        kb = None
                key = keys.index(kb) if kb in keys else -1
                if key < 0:
                    continue
                if not has_t:
                    pend = (c, key)
                    continue
                ab = m["bsm"] & ~((2 << j) - 1)
                fb = m["lb"] + lob(ab) if ab else m["nb"]
                best[key] = max(best.get(key, (0,)), (c + 1, t, fb < t))
        for k, (vs, t, vbs) in best.items():
            own[k] = (vs, t, vbs)
        if pend:
            pm_on = True
            pm_c, pm_key = pend
            pm_vbs = any(m["bsm"] and m["lb"] + hib(m["bsm"]) > pm_c for m in L)
        src = [m for m in L if m["oq"]]
        if src: lo1 = src[-1]["lb"] + hib(src[-1]["oq"]) + 1
        src = [m for m in L if m["bsm"]]
        if src: lb1 = src[-1]["lb"] + hib(src[-1]["bsm"]) + 1
        src = [m for m in L if m["cq"]]
        if src:
            (s_, k_), e_ = src[-1]["lq"]
            ls = (True, s_, e_, k_)
        cb += 1024
    ws = b" \t\r\n"
    ok = not bad and st == 0 and depth == 0 and done and open_pos != NONE
    if ok:
        ok = all(buf[q] in ws for q in range(sx, open_pos)) and all(buf[q] in ws for q in range(close_pos + 1, sy))
    return ok, own


def check(rec, keys, pad):
    buf = bytearray(b"x" * pad + rec + b"\n" + b"\0" * 1100)
    ok, own = scan_line(buf, pad, pad + len(rec), keys)
    mem = S._json_members(rec)
    want = None
    if mem is not None:
        want = {}
        for k, s, e in mem:
            if k in keys:
                want[keys.index(k)] = (s, e)
    got = {k: (vs - pad, ve - pad) for k, (vs, ve, _) in own.items()} if ok else None
    return got == want, got, want


def main():
    rng = random.Random(3)
    keys = [b"k%d" % i for i in range(64)]
    fails = 0
    for it in range(300):
        obj = {("k%d" % rng.randrange(70)): rng.choice(["v", "", 5, [1, "x"], {"k1": "nested"}]) for _ in range(20)}
        rec = json.dumps(obj).encode()
        for pad in (0, 5, 12, 15):
            good, got, want = check(rec, keys, pad)
            if not good:
                fails += 1
                if fails < 4:
                    print("FAIL pad", pad, rec[:200])
                    print("  got ", got)
                    print("  want", want)
    # long lines (several chunks), backslashes, escaped keys, malformed variants
    keys2 = [b"url", b"title", b"a\\b", b"q\"k", b"tech", b"k1"]
    def rnd_str(n):
        al = 'ab"\\/\n{}[]:, \u00e9'
        return "".join(rng.choice(al) for _ in range(n))
    for it in range(400):
        obj = {}
        for _ in range(rng.randrange(1, 12)):
            k = rng.choice(["url", "title", "a\\b", 'q"k', "tech", "k1", "zz", rnd_str(3)])
            v = rng.choice([rnd_str(rng.randrange(0, 40)), rnd_str(rng.randrange(500, 1500)), 7,
                            [rnd_str(5), 3, {"k1": rnd_str(4)}], {"url": rnd_str(8)}, None, True])
            obj[k] = v
        rec = json.dumps(obj, ensure_ascii=rng.random() < 0.5).encode()
        if rng.random() < 0.3:  # duplicate keys: append a raw member
            rec = rec[:-1] + b', "url": "dup\\\\", "title": [1, "\\"x"]}'
        variants = [rec, b"  " + rec + b" \t", rec[:-1], rec + b"x", b"[" + rec[1:], rec.replace(b":", b"", 1)]
        for vr in variants:
            for pad in (0, 7, 15):
                good, got, want = check(vr, keys2, pad)
                if not good:
                    fails += 1
                    if fails < 6:
                        print("FAIL2 pad", pad, len(vr), vr[:160])
                        print("  got ", got)
                        print("  want", want)
    print("fails", fails)


if __name__ == "__main__":
    main()
