#!/usr/bin/env python3
"""Benchmark of the scan-result hot path (BASELINE.json metric: records/s and GB/s vs the HBM
roofline for match+dedup+diff, 1 and 8 GPUs).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload ...]

N = 1 (default workload c2): ONE JSON line whose headline is BASELINE configs[1] ("C2": 10M
synthetic subdomain lines, sort -u + diff against the prior scan, inputs resident in HBM),
carrying the other configs measured in the same run as sub-objects, each with its own
roofline and CPU baseline: `c1` (configs[0], the reference's CPU-runnable case through the
drop-in completion hook), `c3` (configs[2], 50M httpx lines x 2,000 literals), `c5`
(configs[4], 1B host:port records on one GPU), `fused_x1` (the metric's match+dedup+diff as
one call) and `urls`.
N > 1 (default workload c5): C5 STRONG scaling — 1B host:port records in total, byte-range
sharded over the N ranks with the round-pipelined RCCL all-to-all (swarm_amd.distributed
.dedup_diff_rounds_step) — with the C2 weak-scaling step (10M lines per rank) as a `c2_weak`
sub-object. The launcher starts N ranks itself when no torch.distributed launcher wraps it.

`roofline` is the dominant kernel's algorithmic bytes ÷ its average launch time (HIP events
on the launch stream, live in the timed region); `cpu_baseline` is the oracle's Python
restatement of the reference semantics timed on this host (1 thread), plus GNU coreutils /
grep across the host's core share.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: 8.0 TB/s spec
HBM_COPY_GBS = 6290.0      # measured float4 copy (same guide)
METRIC = "scan records/sec + GB/s (vs HBM roofline) for match+dedup+diff, 1 and 8 GPUs"


# library stat name -> HIP kernel symbol (rocprofv3 -T names) for the PMC traffic lookup
KERNEL_SYMBOL = {"rs_pass": "k_rs_down", "emit_sorted": "k_emit_sorted", "emit_uniq": ("k_emit_uniq_s", "k_emit_uniq"),
                 "emit_fresh": "k_emit_fresh", "diff_tile": "k_diff_tile", "adjacent": ("k_adjacent2", "k_adjacent"),
                 "rs_lsort": "k_rs_lsort", "rs_lbounds": "k_rs_lbounds", "seg_heads": "k_sel_count",
                 "lines": "k_lines", "lit_match": "k_lit_scan", "dfa_match": "k_dfa_match", "ac_match": "k_ac_match",
                 "re_prefilter": "k_lit_scan", "re_verify": "k_verify", "json_scan": ("k_json_scan_t", "k_json_scan"),
                 "json_emit": "k_json_emit", "tm_eval": "k_tm_eval", "tm_collect": "k_tm_collect",
                 "bk_sort": "k_bk_sort", "bk_l1_apply": "k_bp_apply", "bk_l2_apply": "k_bp_apply",
                 "bk_l1_count": "k_bp_count", "bk_l2_count": "k_bp_count", "bk_compact": "k_bk_compact",
                 "part_emit": "k_part_apply", "range_bytes": "k_range_bytes", "gather_spans": "k_gather_spans",
                 "gather_matched": "k_gather_matched", "seg_wave": "k_seg_wave", "seg_small": "k_seg_small",
                 "rs_up": "k_rs_up", "lcp": "k_lcp", "rekey": "k_rekey", "key_sample": "k_key_sample",
                 "key_stats": "k_key_stats", "rs_dsum": "k_rs_dsum"}


def pmc_traffic(workload, kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 FETCH_SIZE/WRITE_SIZE
    passes (profiles/pmc_traffic.json, written by tools/pmc_summary.py; FETCH_SIZE doubled per
    MI355X_MICROARCH.md). None when no pass covers this kernel."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    syms = KERNEL_SYMBOL.get(kernel, kernel)
    try:
        table = json.load(open(path))[workload]
    except (OSError, KeyError, ValueError):
        return None
    for sym in ((syms,) if isinstance(syms, str) else syms):  # launch form first (template variants)
        if sym in table:
            return table[sym]
    return None


def roofline_of(stats, kernel=None, workload=None, full=None):
    """The dominant kernel and its achieved GB/s: the algorithmic bytes the library credited
    to its launches (SURVEY.md §8(d) model) over the HIP-event time of the
    same launches, recorded on the launch stream inside the timed region. A kernel whose
    byte model needs a profiling-only count (the segment sorts) takes its bytes per launch
    from the fully profiled step `full`."""
    if not stats:
        return None
    if kernel is None:
        kernel = max(stats.items(), key=lambda kv: kv[1][1])[0]
    if kernel not in stats:
        return None
    launches, ms, by = stats[kernel]
    if not launches or ms <= 0:
        return None
    if not by and full and kernel in full and full[kernel][0]:
        by = full[kernel][2] / full[kernel][0] * launches
    ach = by / (ms * 1e-3) / 1e9
    out = {"kernel": kernel, "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
           "bytes_per_launch": int(by / launches), "avg_launch_us": round(ms / launches * 1e3, 2),
           "frac_of_measured_copy_bw": round(ach / HBM_COPY_GBS, 4)}
    t = pmc_traffic(workload, kernel) if workload else None
    if t:
        out["traffic"] = t["bytes"]
        out["traffic_source"] = "profiles/" + t["source"] + " (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, per launch)"
    return out


def _exact_flags(d, out, depth=0):
    """Every bit-exactness flag of a cpu_baseline object (and its nested GNU legs)."""
    for k, v in (d or {}).items():
        if isinstance(v, bool) and "exact" in k:
            out.append(v)
        elif isinstance(v, dict) and depth < 2:
            _exact_flags(v, out, depth + 1)
    return out


def legs_summary(line):
    """A compact per-leg digest for the end of the JSON line (the driver keeps only the line's
    tail): ms per step, records/s, the dominant kernel's roofline fraction, its measured HBM
    traffic over its algorithmic bytes, and whether every bit-exactness check of the leg held."""
    out = {}
    for name, leg in [("c2", line)] + [(k, line[k]) for k in ("fused_x1", "urls", "c1", "c3", "c4", "c5", "fields")
                                       if isinstance(line.get(k), dict)]:
        if "error" in leg:
            out[name] = {"error": str(leg["error"])[:120]}
            continue
        rf = leg.get("roofline") or {}
        flags = _exact_flags(leg.get("cpu_baseline"), [])
        d = {"ms": leg.get("ms_per_step"), "value": leg.get("value"), "kernel": rf.get("kernel"),
             "frac": rf.get("frac"), "traffic_x": None, "bit_exact": (all(flags) if flags else None)}
        if rf.get("traffic") and rf.get("bytes_per_launch"):
            d["traffic_x"] = round(rf["traffic"] / rf["bytes_per_launch"], 2)
        out[name] = d
    return out


def kernel_table(stats):
    out = {}
    for k, (l, ms, by) in sorted(stats.items(), key=lambda kv: -kv[1][1]):
        out[k] = {"launches": l, "ms_total": round(ms, 3)}
        if by and ms:
            out[k]["gbps"] = round(by / (ms * 1e-3) / 1e9, 1)
    return out


def timed_steps(ctx, run, args, world: int = 1):
    """W warmup steps; one fully profiled untimed step (per-kernel table, dominant kernel:
    rank 0's, agreed across ranks); then K timed steps with HIP events only around the
    dominant kernel's launches, bracketed by a barrier + device sync on both sides; the
    elapsed time is the max over ranks. Returns (elapsed_s, full_stats, timed_stats,
    dominant, last_result)."""
    import torch
    import torch.distributed as dist
    r = None
    for _ in range(args.warmup):
        r = None
        r = run()
    torch.cuda.synchronize()
    ctx.reset_stats()
    ctx.profile(True)
    r = None
    r = run()
    torch.cuda.synchronize()
    ctx.profile(False)
    full = ctx.kernel_stats()
    dominant = max(full.items(), key=lambda kv: kv[1][1])[0] if full else None
    if world > 1:
        names = [None] * world
        dist.all_gather_object(names, dominant)
        dominant = names[0]
    ctx.reset_stats()
    ctx.profile(True, only=dominant)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        r = None
        r = run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    ctx.profile(False)
    if world > 1:
        from swarm_amd import distributed as D
        el = D.all_max_float(el)
    return el, full, ctx.kernel_stats(), dominant, r


def sub_leg(name, fn, keys=None):
    """Run one sub-leg of the default line; a failure is recorded in the line (never hidden,
    never fatal to the headline). keys: the fields of the leg's own line to keep."""
    import torch
    try:
        torch.cuda.empty_cache()
        out = fn()
        if keys:
            out = {k: out[k] for k in keys if k in out}
        return out
    except Exception as e:  # noqa: BLE001 - reported in the JSON line
        import traceback
        traceback.print_exc()
        return {"error": "%s: %s" % (type(e).__name__, e)}
    finally:
        torch.cuda.empty_cache()


SUB_KEYS = ("value", "unit", "ms_per_step", "steps", "warmup", "config", "gbps", "hbm_frac_step", "records",
            "roofline", "cpu_baseline", "dedup_path", "kernels_top", "scaling", "n_gpus")


def bench_c3(args, ctx=None, emit=True):
    """BASELINE.json configs[2] (C3): 50M httpx-style response lines x 2,000 literal
    signatures (sampled, seed 0, from the nuclei template words of length >= 4), 1 GPU. One
    step = parse + match + hits sorted by record + the matched lines serialised (grep
    output). Algorithmic bytes (SURVEY.md §8(d) match model): input + matched output."""
    import numpy as np
    import torch

    import swarm_amd
    from swarm_amd import corpus

    own = ctx is None
    if own:
        torch.cuda.set_device(0)
        ctx = swarm_amd.Context(0, torch.cuda.current_stream().cuda_stream)
    sigs = c3_signatures()
    n_lines = args.c3_lines
    pool = corpus.httpx_pool(sigs, 1 << 16, 0.01, seed=0)
    buf = corpus.lines_from_pool(pool, n_lines, seed=1)
    d = torch.from_numpy(buf).cuda()
    m = swarm_amd.Matcher(sigs, "literal")
    run = lambda: m.dev_match(ctx, d.data_ptr(), d.numel())  # noqa: E731
    el, full, stats, dominant, r = timed_steps(ctx, run, args)
    R = int(r.in_records)
    step_bytes = int(d.numel()) + int(r.lines_bytes)
    cpu = None
    if not args.no_cpu_baseline:
        from oracle import semantics as S
        m_s = 20_000
        cut = int(np.flatnonzero(buf == 10)[m_s - 1]) + 1
        sample = buf[:cut].tobytes()
        tc = time.perf_counter()
        hits = S.literal_hits(sample, sigs)
        tc = time.perf_counter() - tc
        cpu = {"value": round(m_s / tc, 1), "unit": "records/s", "cores": 1, "kind": "port",
               "sample": "%d C3 lines x 2000 literals, oracle `sig in line`, 1 thread, %.2f s" % (m_s, tc),
               "host_cpus": os.cpu_count()}
        cpu["gpu_hits_bit_exact_on_sample"] = (m.match(sample) == hits)
        if not args.no_gnu:
            # GNU grep -F over the whole C3 input on the host cores, checked against the GPU's
            # full matched-line output (full-size parity)
            cores = host_cores()
            g = gnu_grep(buf.tobytes(), sigs, cores, "-F")
            if g:
                gm, secs = g
                r_full = m.dev_match(ctx, d.data_ptr(), d.numel())
                cpu["gnu_grep"] = {"value": round(R / secs, 1), "unit": "records/s", "cores": cores, "seconds": secs,
                                   "sample": "the full input (%d lines, %d B)" % (R, d.numel()),
                                   "command": "LC_ALL=C grep -a -F -f sigs (x%d line-aligned splits)" % cores,
                                   "bit_exact_full": ctx.to_bytes(r_full.lines, r_full.lines_bytes) == gm}
                del gm
    out = {
        "metric": METRIC, "value": round(R * args.steps / el, 1), "unit": "records/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el * 1e3 / args.steps, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (httpx-style lines, 1 % planted signatures, SURVEY.md §8(d) C3)",
        "config": {"workload": "C3: %dM httpx lines x 2000 literal signatures, 1 GPU" % (n_lines // 1_000_000),
                   "engine": "lit_match" if "lit_match" in full else "ac_match",
                   "bytes": int(d.numel()), "automaton_states": m.info()["states"]},
        "gbps": round(step_bytes * args.steps / el / 1e9, 2),
        "hbm_frac_step": round(step_bytes * args.steps / el / 1e9 / HBM_PEAK_GBS, 4),
        "records": {"in": R, "hits": int(r.n_hits), "matched": int(r.matched_records),
                    "matched_bytes": int(r.lines_bytes)},
        "roofline": roofline_of(stats, dominant, "c3", full),
        "cpu_baseline": cpu,
        "kernels": kernel_table(full),
        "kernels_note": "per-kernel table from one fully profiled untimed step; the timed steps record "
                        "HIP events only around the dominant kernel",
    }
    out["kernels_top"] = dict(list(out["kernels"].items())[:8])
    if emit:
        print(json.dumps(out), flush=True)
    del d, buf, r
    m.close()
    if own:
        ctx.close()
    return out


def bench_c4(args, ctx=None, emit=True):
    """BASELINE.json configs[3] (C4): nmap-service-probes-style port banners x ~10k regex
    signatures (the 1,176 DFA-compilable nuclei template regexes + 8,800 synthetic
    nmap-style `match` families), regex-DFA with literal-factor prefilter. Per GPU: the
    8-GPU config's share, 12.5M banners; weak scaling with --gpus. ctx given: a sub-leg of
    the default line (1 GPU, the caller's context; returns the leg's dict)."""
    import base64

    import numpy as np
    import torch

    import swarm_amd
    from swarm_amd import corpus

    import torch.distributed as dist
    from swarm_amd import distributed as D

    own = ctx is None
    if own:
        world, rank, local = dist_setup(args)
        if world > 1:
            local = local % max(torch.cuda.device_count(), 1)
            torch.cuda.set_device(local)
            dist.init_process_group(args.dist_backend)
        else:
            torch.cuda.set_device(0)
    else:
        world, rank, local = 1, 0, 0
    sig = json.load(open(os.path.join(ROOT, "tests", "golden", "signatures.json")))
    pats, n_generic = corpus.c4_signatures([base64.b64decode(r["p"]) for r in sig["regexes"]])
    n_lines = args.c4_lines
    pool = corpus.banner_pool()
    buf = corpus.lines_from_pool(pool, n_lines, seed=3 + rank)  # rank r's contiguous input shard
    d = torch.from_numpy(buf).cuda()
    if own:
        ctx = swarm_amd.Context(local, torch.cuda.current_stream().cuda_stream)
    tc0 = time.perf_counter()
    m = swarm_amd.Matcher(pats, "regex")  # replicated automata
    compile_s = time.perf_counter() - tc0
    tot = {}

    def run():
        r, tot["g"] = D.match_step(ctx, m, d)
        return r
    el, full, stats, dominant, r = timed_steps(ctx, run, args, world)
    g_rec, g_hits, g_matched = tot["g"]
    R = int(r.in_records)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import semantics as S
        m_s = 1000
        cut = int(np.flatnonzero(buf == 10)[m_s - 1]) + 1
        sample = buf[:cut].tobytes()
        tc = time.perf_counter()
        hits = S.regex_hits(sample, pats)
        tc = time.perf_counter() - tc
        cpu = {"value": round(m_s / tc, 1), "unit": "records/s", "cores": 1, "kind": "port",
               "sample": "%d C4 banners x %d regexes, oracle re.search, 1 thread, %.2f s" % (m_s, len(pats), tc),
               "host_cpus": os.cpu_count()}
        cpu["gpu_hits_bit_exact_on_sample"] = (m.match(sample) == hits)
        # GNU grep -E on the agreeing subset (tests/golden/c4_grep_subset.json: signatures
        # whose POSIX-ERE reading matches re.search), fanned over the host cores, against a
        # GPU matcher compiled from the same subset on the same banners
        sub_idx = json.load(open(os.path.join(ROOT, "tests", "golden", "c4_grep_subset.json")))["subset"]
        sub = [pats[i] for i in sub_idx]
        cores = host_cores()
        g_lines = min(n_lines, max(args.gnu_lines // 5, 1000))
        gcut = int(np.flatnonzero(buf == 10)[g_lines - 1]) + 1
        g = gnu_grep(buf[:gcut].tobytes(), sub, cores, "-E")
        if g:
            gm, secs = g
            msub = swarm_amd.Matcher(sub, "regex")
            dg = torch.from_numpy(buf[:gcut].copy()).cuda()
            rg = msub.dev_match(ctx, dg.data_ptr(), dg.numel())
            cpu["gnu_grep"] = {"value": round(g_lines / secs, 1), "unit": "records/s", "cores": cores, "seconds": secs,
                               "signatures": len(sub),
                               "sample": "%d C4 banners x the %d-signature grep-agreeing subset" % (g_lines, len(sub)),
                               "command": "LC_ALL=C grep -a -E -f subset (x%d line-aligned splits)" % cores,
                               "bit_exact_vs_gpu_same_subset": ctx.to_bytes(rg.lines, rg.lines_bytes) == gm}
            msub.close()
            del dg, rg
    out = {
        "metric": METRIC, "value": round(g_rec * args.steps / el, 1), "unit": "records/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el * 1e3 / args.steps, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (nmap-style port banners, ~30 % from known products, SURVEY.md §8(d) C4)",
        "config": {"workload": "C4: %.1fM banners x %d regex signatures per GPU (8-GPU config share)"
                               % (n_lines / 1e6, len(pats)),
                   "generic_regexes_left_out": n_generic,
                   "bytes": int(d.numel()), "automaton_states": m.info()["states"],
                   "compile_s": round(compile_s, 2),
                   "parallelism": ("replicated automata, contiguous input shards, count all-reduce x%d" % world)
                                  if world > 1 else "single GPU"},
        "gbps": round(d.numel() * world * args.steps / el / 1e9, 2),
        "records": {"in": g_rec, "hits": g_hits, "matched": g_matched,
                    "matched_frac": round(g_matched / max(g_rec, 1), 4)},
        "roofline": roofline_of(stats, dominant, "c4", full),
        "cpu_baseline": cpu,
        "kernels": kernel_table(full),
        "kernels_note": "per-kernel table from one fully profiled untimed step; the timed steps record "
                        "HIP events only around the dominant kernel",
    }
    out["kernels_top"] = dict(list(out["kernels"].items())[:8])
    if rank == 0 and emit:
        print(json.dumps(out), flush=True)
    m.close()
    del d, buf, r
    if own:
        ctx.close()
        if world > 1:
            dist.destroy_process_group()
    return out


def field_templates():
    """The template corpus (tests/golden/templates.json, record part) plus tech-detect-style
    templates on httpx -json fields (title / webserver / tech)."""
    import base64
    from swarm_amd import corpus
    d = json.load(open(os.path.join(ROOT, "tests", "golden", "templates.json")))
    T = [dict(t, matchers=[dict(m, patterns=[base64.b64decode(p) for p in m["patterns"]]) for m in t["matchers"]])
         for t in d["templates"]]
    for tech in corpus._TECH:
        T.append({"condition": "or", "matchers": [{"type": "word", "part": "tech", "condition": "or",
                                                   "patterns": [tech.split(b":")[0]]}]})
    for srv in corpus.SERVERS:
        T.append({"condition": "and", "matchers": [
            {"type": "word", "part": "webserver", "patterns": [srv.split(b"/")[0]]},
            {"type": "word", "part": "title", "patterns": [b"Login", b"Admin"], "negative": True}]})
    T.append({"condition": "or", "matchers": [{"type": "regex", "part": "title", "patterns": [rb"(?i)index of /"]}]})
    return T


def bench_fields(args, ctx=None, emit=True):
    """SURVEY.md §8(f) rows 1+3: httpx -json result lines -> field rows (url, title,
    webserver, tech) and nuclei matcher logic (the 1,006 word/regex templates of the
    reference corpus on the record + 31 field templates) per GPU. One step = field
    extraction + template evaluation over the whole batch. ctx given: a sub-leg of the
    default line (returns the leg's dict)."""
    import numpy as np
    import torch

    import swarm_amd
    from swarm_amd import corpus

    own = ctx is None
    if own:
        torch.cuda.set_device(0)
    n_lines = args.fields_lines
    buf = corpus.lines_from_pool(corpus.httpx_json_pool(1 << 14, seed=5), n_lines, seed=6)
    d = torch.from_numpy(buf).cuda()
    if own:
        ctx = swarm_amd.Context(0, torch.cuda.current_stream().cuda_stream)
    keys = [b"url", b"title", b"webserver", b"tech"]
    T = field_templates()
    tm = swarm_amd.Templates(T, keys)
    holder = {}

    def run():
        # one parse of the JSON lines: the field rows feed the template evaluation too
        holder["rows"] = ctx.json_fields(d.data_ptr(), d.numel(), keys)
        return tm.dev_match(ctx, d.data_ptr(), d.numel(), rows=holder["rows"], rows_keys=keys)
    el, full, stats, dominant, r = timed_steps(ctx, run, args)
    R = int(r.in_records)
    cpu = None
    if not args.no_cpu_baseline:
        from oracle import semantics as S
        m_s = 300
        cut = int(np.flatnonzero(buf == 10)[m_s - 1]) + 1
        sample = buf[:cut].tobytes()
        tc = time.perf_counter()
        want = S.template_matches(sample, T, keys)
        rows = S.json_field_rows(sample, keys)
        tc = time.perf_counter() - tc
        cpu = {"value": round(m_s / tc, 1), "unit": "records/s", "cores": 1, "kind": "port",
               "sample": "%d httpx -json lines: oracle field rows + %d templates, 1 thread, %.2f s" % (m_s, len(T), tc),
               "host_cpus": os.cpu_count()}
        cpu["gpu_bit_exact_on_sample"] = (tm.match(sample) == want and
                                          swarm_amd.json_fields(sample, keys)[0] == rows[0])
    out = {
        "metric": METRIC, "value": round(R * args.steps / el, 1), "unit": "records/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el * 1e3 / args.steps, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (httpx -json lines, Go-style escaping; template corpus from the reference)",
        "config": {"workload": "F: %.1fM httpx -json lines -> 4 field keys + %d nuclei templates per GPU"
                               % (n_lines / 1e6, len(T)), "bytes": int(d.numel()), "templates": tm.info()},
        "gbps": round(d.numel() * args.steps / el / 1e9, 2),
        "records": {"in": R, "field_rows": int(holder["rows"].rows), "template_matches": int(r.n)},
        "roofline": roofline_of(stats, dominant, "fields", full),
        "cpu_baseline": cpu,
        "kernels": kernel_table(full),
        "kernels_note": "per-kernel table from one fully profiled untimed step; the timed steps record "
                        "HIP events only around the dominant kernel",
    }
    out["kernels_top"] = dict(list(out["kernels"].items())[:8])
    if emit:
        print(json.dumps(out), flush=True)
    tm.close()
    del d, buf, r, holder
    if own:
        ctx.close()
    return out


def bench_c5(args, world=1, rank=0, dev=None, ctx=None, emit=True):
    """BASELINE.json configs[4] (C5): 1B host:port records (~31 GB) in total, deduped and
    diffed against a prior scan at 90 % overlap; STRONG scaling: the N ranks share the 1B
    records. Records are rendered on the GPU: 64M hosts x 4 open-port slots (ports from 32
    common ones) = 256M distinct combos, 1B draws (~4 copies each).
    N = 1: the shard (in pieces of 50M records) is routed into local byte-range parts of
    < 4 GiB by one partition call that hands each part's parse to its dedup
    (swarm_amd.sharded.dedup_diff_large); the stored prior is kept one aligned part each.
    N > 1: one partition call routes the rank's pieces into N x R byte ranges, one all-to-all
    of the part sizes, R all-to-alls of bytes queued on RCCL's stream, each local part deduped
    as soon as its round arrives (swarm_amd.distributed.dedup_diff_rounds_step); rank
    outputs concatenated in rank order are the global sort -u / comm -13 output. Setup
    (untimed): the prior scan = sort -u of another 1B draw over combos shifted by 10 %,
    routed to its owner ranks and parts by the same splitters (byte quantiles of the prior's
    sampled records, agreed across ranks), and stored.
    --c5-data ips: 10.x.y.z:port records (every record shares '10.', most their first 7
    bytes), the case key0 routing could not divide."""
    import numpy as np
    import torch
    import torch.distributed as dist

    import swarm_amd
    from swarm_amd import corpus, sharded
    from swarm_amd import distributed as D

    dev = dev or torch.device("cuda", 0)
    own = ctx is None
    if own:
        ctx = swarm_amd.Context(dev.index, torch.cuda.current_stream(dev).cuda_stream)
    total = args.c5_records
    per = total // world + (1 if rank < total % world else 0)
    if args.c5_data == "ips":
        # 10.x.y.z:port from an internal-range scan: 15M hosts x 16 open-port slots
        n_hosts = min(args.c5_hosts, 1 << 24) if args.c5_hosts != 64_000_000 else 15_000_000
        K = 16
        pool = corpus.ip_pool_torch(n_hosts + n_hosts // 10 + 1, seed=5, device=dev)
    else:
        n_hosts = args.c5_hosts
        K = 4  # open-port slots per host (ports drawn from 32 common ports)
        pool = corpus.host_pool_torch(n_hosts + n_hosts // 10 + 1, seed=5, device=dev)
    U = n_hosts * K
    t_setup = time.perf_counter()
    prior_raw = corpus.hostport_pieces(pool, per, U // 10, U + U // 10, seed=900 + rank, ports_per_host=K)
    cur = corpus.hostport_pieces(pool, per, 0, U, seed=100 + rank, ports_per_host=K)
    del pool
    cur_bytes = sum(p.numel() for p in cur)
    if world == 1 and args.c5_path == "local":
        parts = sharded.plan_parts(prior_raw, [], args.c5_part_bytes)
        split = sharded.choose_splitters(sharded.sample_records(ctx, prior_raw), parts)
        pu, _, pst = sharded.dedup_diff_large(ctx, prior_raw, (), splitters=split, align_parts=True)
        del prior_raw
        # the stored prior is this path's own part-ordered output: one 16-byte aligned part
        # per local range, read in place by every step (never routed again)
        prior_parts = sharded.stored_parts(pu, pst) if not pst["rerouted_parts"] else None
        prior_store = pu
        rounds = len(split) + 1

        def step():
            if prior_parts is not None:
                return sharded.dedup_diff_large(ctx, cur, (), splitters=split, prior_parts=prior_parts)
            # (pu's '\n' part padding reads as empty lines, which are not records: A7 drops them)
            return sharded.dedup_diff_large(ctx, cur, [pu], splitters=split)
    else:
        # N > 1 (or --c5-path rounds at N = 1: the per-rank compute of the N-GPU step; with a
        # 1-rank process group (--dist-backend nccl) its size exchange and per-round RCCL
        # all-to-alls are issued too, force_exchange)
        force = world == 1 and dist.is_initialized()
        rounds = D.all_max_int(D.plan_rounds(max(cur_bytes, 1), world)) if world > 1 else \
            D.plan_rounds(max(cur_bytes, 1), 8)
        split = D.agree_splitters(ctx, prior_raw, world * rounds)
        prior_parts, prior_store = D.build_prior_rounds(ctx, prior_raw, split, rounds, force_exchange=force)
        del prior_raw

        def step():
            return D.dedup_diff_rounds_step(ctx, cur, prior_parts, split, rounds, force_exchange=force)
    torch.cuda.synchronize()
    t_setup = time.perf_counter() - t_setup
    prior_bytes = int(prior_store.numel())

    holder = {}

    def run():
        u, f, st = step()
        holder["st"], holder["ub"], holder["fb"] = st, int(u.numel()), int(f.numel())
        return None
    el, full, stats, dominant, _ = timed_steps(ctx, run, args, world)
    st, ub, fb = holder["st"], holder["ub"], holder["fb"]
    step_bytes = cur_bytes + prior_bytes + ub + fb
    if world > 1:
        step_bytes = D.all_max_int(step_bytes) * world  # reported as the whole job's (max rank x N)
        tot_in = D.all_max_int(st["in_records"])
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import semantics as S
        m = 2_000_000
        c0 = cur[0][: int(torch.nonzero(cur[0][: 40 * m] == 10)[m - 1].item()) + 1].cpu().numpy().tobytes()
        p0 = prior_store[:40 * m].cpu().numpy().tobytes()
        p0 = p0[: p0.rfind(b"\n") + 1]
        tc = time.perf_counter()
        eu, ef = S.dedup_diff(c0, p0)
        tc = time.perf_counter() - tc
        cpu = {"value": round(m / tc, 1), "unit": "records/s", "cores": 1, "kind": "port",
               "sample": "2M C5 records + a 2M-record slice of the prior; oracle sorted(set())+set difference, "
                         "1 thread, %.2f s" % tc, "host_cpus": os.cpu_count()}
        gu, gf, _ = sharded.dedup_diff_large(ctx, [dev_bytes(c0, dev)], [dev_bytes(p0, dev)], part_bytes=16 << 20)
        cpu["gpu_bit_exact_on_sample"] = (gu.cpu().numpy().tobytes() == eu and gf.cpu().numpy().tobytes() == ef)
        del gu, gf
        # the whole step at full size (untimed): its unique and new outputs against the
        # expectation computed from the drawn combo ids (oracle/c5_check.py: counts, record
        # checksum, strict byte order)
        from oracle import c5_check
        tc = time.perf_counter()
        u_full, f_full, _ = step()
        pool2 = (corpus.ip_pool_torch(n_hosts + n_hosts // 10 + 1, seed=5, device=dev) if args.c5_data == "ips"
                 else corpus.host_pool_torch(n_hosts + n_hosts // 10 + 1, seed=5, device=dev))
        chk = c5_check.check_step(pool2, K, K, corpus.hostport_ids(per, 0, U, 100 + rank, device=dev),
                                  corpus.hostport_ids(per, U // 10, U + U // 10, 900 + rank, device=dev),
                                  u_full, f_full)
        chk["seconds"] = round(time.perf_counter() - tc, 1)
        chk["method"] = ("the full step's outputs parsed back into records vs the drawn (host, port) ids: "
                         "distinct counts, sum of 64-bit record fingerprints, strict byte order")
        cpu["full_size"] = chk
        cpu["full_size_bit_exact"] = chk["full_size_bit_exact"]
        del u_full, f_full, pool2
    out = None
    if rank == 0:
        pb = st["part_bytes"]
        out = {
            "metric": METRIC, "value": round(total * args.steps / el, 1), "unit": "records/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el * 1e3 / args.steps, 4),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (host:port records rendered on the GPU, SURVEY.md §8(d) C5)",
            "config": {"workload": "C5: %dM %s records in total (%.1f GB on rank 0) + prior at 90%% overlap, "
                                   "byte-range sharded over %d GPU(s)" % (
                                       total // 1_000_000, "10.x.y.z:port" if args.c5_data == "ips" else "host:port",
                                       cur_bytes / 1e9, world),
                       "records_total": total, "hosts": n_hosts, "ports_per_host": K,
                       "prior_bytes_rank0": prior_bytes, "local_parts": rounds,
                       "part_balance_max_over_mean": round(max(pb) * len(pb) / max(1, sum(pb)), 3) if pb else None,
                       "rerouted_parts": st["rerouted_parts"],
                       "setup_s": round(t_setup, 1),
                       "parallelism": ("byte-range sharding, %d exchange rounds of all-to-all x%d "
                                       "(backend %s, world size %d)" % (rounds, world, dist.get_backend(),
                                                                        dist.get_world_size()))
                                      if dist.is_initialized() else ("single GPU" if args.c5_path == "local" else
                                                                     "single GPU, the N-rank step's local path (%d "
                                                                     "rounds, no exchange)" % rounds)},
            "gbps": round(step_bytes * args.steps / el / 1e9, 2),
            "hbm_frac_step": round(step_bytes * args.steps / el / 1e9 / (HBM_PEAK_GBS * world), 4),
            "records": {"in_rank0": st["in_records"], "unique_rank0": st["uniq_records"],
                        "new_rank0": st["fresh_records"], "max_part_bytes": st["max_part_bytes"]},
            # the rounds path's traffic from its own PMC passes (profiles/pmc_traffic.json "c5r")
            "roofline": roofline_of(stats, dominant, "c5" if world == 1 and args.c5_path == "local" else "c5r", full),
            "cpu_baseline": cpu,
            "kernels": kernel_table(full),
            "kernels_note": "per-kernel table from one fully profiled untimed step; the timed steps record "
                            "HIP events only around the dominant kernel",
        }
        if world > 1:
            out["records"]["in_max_rank"] = tot_in
            out["records"]["recv_bytes_rank0"] = st.get("recv_bytes")
        out["kernels_top"] = dict(list(out["kernels"].items())[:10])
        if emit:
            print(json.dumps(out), flush=True)
    del cur, prior_parts, prior_store
    if own:
        ctx.close()
    return out


def bench_c1(args, ctx):
    """BASELINE.json configs[0] (C1), the reference's CPU-runnable case: 1M synthetic
    subdomain lines written with the A1 chunk layout into 16 worker chunks (client/swarm:147-148
    readlines keeps each '\n', server/server.py:447 joins them with '\n': a blank line between
    records), the chunk outputs (identity module) merged in A5 key order (server/server.py:
    403-410), sort -u, then the diff against the prior scan. Timed three ways on the same
    bytes: the oracle (1 thread), GNU sort -u --parallel + comm -13 on the merged body, and
    the drop-in completion hook (swarm_amd.hooks.completion_dedup_diff: key order, UTF-8
    check, H2D, GPU dedup+diff, D2H — PCIe inclusive, host buffers in and out)."""
    from swarm_amd import corpus, hooks
    from oracle import semantics as S
    n = args.c1_lines
    sub, ids = corpus.subdomains(n, seed=1234)
    prior = corpus.prior_of(ids).tobytes()
    chunks = S.server_chunks(S.client_readlines(sub.tobytes()), max(1, n // 16))
    objects = {"c1scan/output/chunk_%d.txt" % i: b for i, b in enumerate(chunks)}
    # GPU: the hook, K timed calls after W warmups (host-buffer API)
    for _ in range(max(1, args.warmup)):
        gu, gf = hooks.completion_dedup_diff(objects, "c1scan", prior)
    K = max(1, min(args.steps, 10))
    t0 = time.perf_counter()
    for _ in range(K):
        gu, gf = hooks.completion_dedup_diff(objects, "c1scan", prior)
    tg = (time.perf_counter() - t0) / K
    out = {"value": round(n / tg, 1), "unit": "records/s", "ms_per_step": round(tg * 1e3, 3), "steps": K,
           "config": {"workload": "C1: %dM subdomain lines, A1 layout in %d chunks, A5 merge, sort -u, diff vs the "
                                  "prior scan (90 %% of the unique set)" % (n // 1_000_000, len(chunks)),
                      "chunks": len(chunks), "merged_bytes": sum(len(b) for b in chunks), "prior_bytes": len(prior),
                      "gpu_path": "swarm_amd.hooks.completion_dedup_diff (host buffers, PCIe inclusive)"},
           "records": {"in": n, "unique": gu.count(b"\n"), "new": gf.count(b"\n")}}
    if not args.no_cpu_baseline:
        tc = time.perf_counter()
        merged = S.merge_chunks(objects, "c1scan")
        eu, ef = S.dedup_diff(merged, prior)
        tc = time.perf_counter() - tc
        out["cpu_baseline"] = {"value": round(n / tc, 1), "unit": "records/s", "cores": 1, "kind": "port",
                               "sample": "the whole C1 input: oracle A5 merge + sorted(set()) + set difference, "
                                         "1 thread, %.2f s" % tc, "host_cpus": os.cpu_count(),
                               "gpu_bit_exact": gu == eu and gf == ef}
        if not args.no_gnu:
            out["cpu_baseline"]["gnu_sort_comm"] = gnu_sort_comm(merged, prior, eu, ef, threads=host_cores())
    return out


def bench_c2(args, world, rank, dev, ctx):
    """BASELINE.json configs[1] (C2): 10M synthetic subdomain lines per GPU + the prior scan
    (90 % of the unique set), sort -u + diff, inputs resident in HBM. N > 1: WEAK scaling,
    every rank brings 10M lines drawn from one global universe; records routed by byte range
    (one partition, one all-to-all: dedup_diff_rounds_step with one round) or by hash."""
    import numpy as np
    import torch

    from swarm_amd import corpus

    n_lines = args.lines
    cur_np, ids = corpus.subdomains(n_lines, seed=1234 + rank, universe=n_lines * world)
    cur = torch.from_numpy(cur_np).to(dev)
    prior_np = None
    if world == 1:
        prior_np = corpus.prior_of(ids)
        prior = torch.from_numpy(prior_np).to(dev)
    else:
        from swarm_amd import distributed as D
        u = np.unique(ids)
        cand = torch.from_numpy(corpus._flatten(*corpus.render_names(u[(u % np.uint64(10)) != 0]))).to(dev)
        if args.route == "range":
            # splitters from every rank's prior record samples: rank r owns byte range r of the
            # prior AND of every later scan, so the rank outputs concatenate into global order
            gsplit = D.agree_splitters(ctx, [cand], world)
            prior_parts, prior = D.build_prior_rounds(ctx, [cand], gsplit, 1)
        else:
            prior = D.build_prior_partition(ctx, cand)
        del cand
    torch.cuda.synchronize()
    holder = {}

    def run():
        if world == 1:
            r = ctx.dedup_diff(cur.data_ptr(), cur.numel(), prior.data_ptr(), prior.numel())
            holder.update(R=int(r.in_records), U=int(r.uniq_records), F=int(r.fresh_records), Rp=int(r.prior_records),
                          ub=int(r.uniq_bytes), fb=int(r.fresh_bytes))
            return r
        from swarm_amd import distributed as D
        if args.route == "range":
            u, f, st = D.dedup_diff_rounds_step(ctx, [cur], prior_parts, gsplit, 1)
            holder.update(R=st["in_records"], U=st["uniq_records"], F=st["fresh_records"], Rp=None,
                          ub=int(u.numel()), fb=int(f.numel()))
            return None
        r, recv = D.dedup_diff_step(ctx, cur, prior)
        holder.update(R=int(r.in_records), U=int(r.uniq_records), F=int(r.fresh_records), Rp=int(r.prior_records),
                      ub=int(r.uniq_bytes), fb=int(r.fresh_bytes))
        return r
    elapsed, full, stats, dominant, r = timed_steps(ctx, run, args, world)
    ms_per_step = elapsed * 1e3 / args.steps
    cur_bytes, prior_bytes = int(cur.numel()), int(prior.numel())
    step_bytes = cur_bytes + prior_bytes + holder["ub"] + holder["fb"]
    if world > 1:
        from swarm_amd import distributed as D
        step_bytes = D.all_max_int(step_bytes) * world
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import semantics as S  # CPU baseline leg only
        m = min(args.cpu_sample, n_lines)
        if m < n_lines:
            cut = int(np.flatnonzero(cur_np == 10)[m - 1]) + 1
            cbytes = cur_np[:cut].tobytes()
        else:
            cbytes = cur_np.tobytes()
        pbytes = prior_np.tobytes()
        tc = time.perf_counter()
        eu, ef = S.dedup_diff(cbytes, pbytes)
        tc = time.perf_counter() - tc
        cpu = {"value": round(m / tc, 1), "unit": "records/s", "cores": 1, "kind": "port",
               "sample": "%d C2 lines + full prior (%d B); oracle sorted(set())+set difference, 1 thread, %.2f s"
                         % (m, len(pbytes), tc),
               "host_cpus": os.cpu_count()}
        if m == n_lines:
            cpu["gpu_output_bit_exact"] = (ctx.to_bytes(r.uniq, r.uniq_bytes) == eu and
                                           ctx.to_bytes(r.fresh, r.fresh_bytes) == ef)
            if not args.no_gnu:
                cpu["gnu_sort_comm"] = gnu_sort_comm(cbytes, pbytes, eu, ef, threads=host_cores())
    line = {
        "metric": METRIC, "value": round(n_lines * world * args.steps / elapsed, 1), "unit": "records/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (seeded subdomain corpus, SURVEY.md §8(d) C2)",
        "config": {"workload": "C2: %dM-line subdomain merge + sort -u dedup + new-record diff per GPU"
                               % (n_lines // 1_000_000),
                   "lines_per_gpu": n_lines, "bytes_per_gpu": cur_bytes, "prior_bytes": prior_bytes,
                   "unique_frac": round(holder["U"] / max(holder["R"], 1), 4),
                   "parallelism": ("%s all-to-all x%d (backend %s)" % (
                       "byte-range (global byte order)" if args.route == "range" else "hash-partition", world,
                       args.dist_backend)) if world > 1 else "single GPU"},
        "gbps": round(step_bytes * args.steps / elapsed / 1e9, 2),
        "hbm_frac_step": round(step_bytes * args.steps / elapsed / 1e9 / (HBM_PEAK_GBS * world), 4),
        "records": {"in": holder["R"], "unique": holder["U"], "new": holder["F"], "prior": holder["Rp"]},
        "roofline": roofline_of(stats, dominant, "c2", full),
        "cpu_baseline": cpu,
        "gpu_kernel_ms_per_step": round(sum(v[1] for v in full.values()), 4),
        "kernels": kernel_table(full),
        "kernels_note": "per-kernel table from one fully profiled untimed step; the timed steps record "
                        "HIP events only around the dominant kernel",
        "dedup_path": ctx.last_path()[0],
    }
    line["kernels_top"] = dict(list(line["kernels"].items())[:10])
    del cur, prior, r
    return line


def host_cores() -> int:
    """CPU threads this process may use on the host: the affinity set, capped by the job's
    thread budget (OMP_NUM_THREADS is the GPU box's per-GPU CPU share)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(n, cap) if cap > 0 else n)


def c3_signatures():
    """C3's 2,000 literal signatures: sampled (seed 0) from the nuclei template words of length
    >= 4."""
    import base64
    import random
    sig = json.load(open(os.path.join(ROOT, "tests", "golden", "signatures.json")))
    words = [base64.b64decode(w) for w in sig["words"]]
    return random.Random(0).sample([w for w in words if len(w) >= 4], 2000)


def gnu_grep(data: bytes, pats, cores: int, flag: str = "-F"):
    """`LC_ALL=C grep -a <flag> -f pats` fanned out over `cores` line-aligned splits of data
    (BASELINE.md CPU-baseline plan; outputs concatenated in input order). Returns (matched
    lines, seconds of the grep stage) or None without grep."""
    import shutil
    import subprocess
    import tempfile
    if not shutil.which("grep"):
        return None
    env = dict(os.environ, LC_ALL="C")
    with tempfile.TemporaryDirectory() as d:
        pf = os.path.join(d, "pats")
        with open(pf, "wb") as f:
            f.write(b"".join(s + b"\n" for s in pats if s and b"\n" not in s))
        cuts, n = [0], len(data)
        for k in range(1, cores):
            c = data.find(b"\n", n * k // cores)
            cuts.append(n if c < 0 else c + 1)
        cuts.append(n)
        names = []
        for k in range(cores):
            fn = os.path.join(d, "in%d" % k)
            with open(fn, "wb") as f:
                f.write(data[cuts[k]:cuts[k + 1]])
            names.append(fn)
        t0 = time.perf_counter()
        procs = [subprocess.Popen(["grep", "-a", flag, "-f", pf, fn], env=env, stdout=subprocess.PIPE) for fn in names]
        outs = [p.communicate()[0] for p in procs]
        secs = time.perf_counter() - t0
    return b"".join(outs), round(secs, 3)


def gnu_grep_sort_comm(data: bytes, sigs, prior: bytes, cores: int):
    """The shell restatement of the fused step on the host: `LC_ALL=C grep -a -F -f sigs` fanned
    out over `cores` line-aligned splits (outputs concatenated in input order), then
    `sort -u --parallel=cores`, then `comm -13 prior -` (SURVEY.md §8(d) CPU baselines).
    Returns (matched, uniq, fresh, seconds per stage)."""
    import shutil
    import subprocess
    import tempfile
    if not (shutil.which("grep") and shutil.which("sort") and shutil.which("comm")):
        return None
    env = dict(os.environ, LC_ALL="C")
    with tempfile.TemporaryDirectory() as d:
        pf, pp = os.path.join(d, "sigs"), os.path.join(d, "prior")
        with open(pf, "wb") as f:
            f.write(b"".join(s + b"\n" for s in sigs if s and b"\n" not in s))
        with open(pp, "wb") as f:
            f.write(prior)
        cuts, n = [0], len(data)
        for k in range(1, cores):
            c = data.find(b"\n", n * k // cores)
            cuts.append(n if c < 0 else c + 1)
        cuts.append(n)
        names = []
        for k in range(cores):
            fn = os.path.join(d, "in%d" % k)
            with open(fn, "wb") as f:
                f.write(data[cuts[k]:cuts[k + 1]])
            names.append(fn)
        t0 = time.perf_counter()
        procs = [subprocess.Popen(["grep", "-a", "-F", "-f", pf, fn], env=env, stdout=subprocess.PIPE) for fn in names]
        outs = [p.communicate()[0] for p in procs]
        t1 = time.perf_counter()
        matched = b"".join(outs)
        pm, pu = os.path.join(d, "matched"), os.path.join(d, "uniq")
        with open(pm, "wb") as f:
            f.write(matched)
        t2 = time.perf_counter()
        subprocess.run(["sort", "-u", "--parallel=%d" % cores, "-S", "25%", "-T", d, "-o", pu, pm], env=env, check=True)
        fresh = subprocess.run(["comm", "-13", pp, pu], env=env, check=True, stdout=subprocess.PIPE).stdout
        t3 = time.perf_counter()
        with open(pu, "rb") as f:
            uniq = f.read()
    if uniq.startswith(b"\n"):
        uniq = uniq[1:]
    if fresh.startswith(b"\n"):
        fresh = fresh[1:]
    return matched, uniq, fresh, {"grep": round(t1 - t0, 3), "sort_comm": round(t3 - t2, 3)}


def bench_x1(args, ctx=None, emit=True):
    """The metric's fused step (BASELINE.json "match+dedup+diff"): 10M httpx
    result lines (URLs of subdomains drawn like C2, each URL with a fixed title/server tail)
    -> A3 parse -> A4 match against C3's 2,000 literal signatures -> A7 sort -u of the matched
    lines -> A8 diff against the prior scan's matched set (worker/worker.py:83-98 ->
    server/server.py:399-412 -> README.md:11). One device-resident call per step
    (sg_dev_match_dedup_diff). Returns the result dict (printed as one JSON line if emit)."""
    import numpy as np
    import torch

    import swarm_amd
    from swarm_amd import corpus

    own = ctx is None
    if own:
        torch.cuda.set_device(0)
        ctx = swarm_amd.Context(0, torch.cuda.current_stream().cuda_stream)
    n_lines = args.x1_lines
    sigs = c3_signatures()
    tails = corpus.httpx_tails(sigs)
    buf, ids = corpus.httpx_hosts(n_lines, tails, seed=1234)
    d = torch.from_numpy(buf).cuda()
    m = swarm_amd.Matcher(sigs, "literal")
    # setup (untimed): the prior scan's matched set = sort -u of the matched lines of the
    # prior's URLs (90 % of this scan's distinct URLs), computed by the same library call
    pbuf = corpus.httpx_rows(corpus.prior_ids(ids), tails)
    dp_in = torch.from_numpy(pbuf).cuda()
    r0, _, _ = m.dev_match_dedup_diff(ctx, dp_in.data_ptr(), dp_in.numel())
    d_prior = torch.empty(max(int(r0.uniq_bytes), 1), dtype=torch.uint8, device=d.device)
    if r0.uniq_bytes:
        ctx.memcpy(d_prior.data_ptr(), r0.uniq, int(r0.uniq_bytes))
    n_prior = int(r0.uniq_bytes)
    del dp_in
    holder = {}

    def run():
        # the step: the hit count is not part of the metric's output, so the literal matcher
        # only flags matched records (sg_dev_match_dedup_diff with n_hits NULL)
        r, _, nm = m.dev_match_dedup_diff(ctx, d.data_ptr(), d.numel(), d_prior.data_ptr(), n_prior,
                                          count_hits=False)
        holder["h"] = nm
        return r
    el, full, stats, dominant, r = timed_steps(ctx, run, args)
    nm = holder["h"]
    uniq_step = ctx.to_bytes(r.uniq, r.uniq_bytes)
    fresh_step = ctx.to_bytes(r.fresh, r.fresh_bytes)
    # untimed: the hit count, and the same outputs from the hit-list path
    r2, nh, nm2 = m.dev_match_dedup_diff(ctx, d.data_ptr(), d.numel(), d_prior.data_ptr(), n_prior)
    paths_agree = (nm2 == nm and ctx.to_bytes(r2.uniq, r2.uniq_bytes) == uniq_step and
                   ctx.to_bytes(r2.fresh, r2.fresh_bytes) == fresh_step)
    del uniq_step, fresh_step
    R = int(r.in_records)
    # algorithmic bytes of the step: the match reads the input; dedup+diff
    # read the matched records (in place, no copy) + the prior and write unique + new
    matched_bytes = int(m.dev_match(ctx, d.data_ptr(), d.numel()).lines_bytes)  # untimed
    step_bytes = d.numel() + matched_bytes + n_prior + int(r.uniq_bytes) + int(r.fresh_bytes)
    cpu = None
    if not args.no_cpu_baseline:
        from oracle import semantics as S
        prior_host = ctx.to_bytes(d_prior.data_ptr(), n_prior)
        m_s = 3000
        cut = int(np.flatnonzero(buf == 10)[m_s - 1]) + 1
        sample = buf[:cut].tobytes()
        tc = time.perf_counter()
        eu, ef = S.dedup_diff(S.matched_lines(sample, S.literal_hits(sample, sigs)), prior_host)
        tc = time.perf_counter() - tc
        ds = torch.from_numpy(buf[:cut].copy()).cuda()
        rs, _, _ = m.dev_match_dedup_diff(ctx, ds.data_ptr(), ds.numel(), d_prior.data_ptr(), n_prior,
                                         count_hits=False)
        cpu = {"value": round(m_s / tc, 1), "unit": "records/s", "cores": 1, "kind": "port",
               "sample": "%d X1 lines: oracle `sig in line` + sorted(set()) + set difference vs the prior matched "
                         "set, 1 thread, %.2f s" % (m_s, tc), "host_cpus": os.cpu_count(),
               "gpu_bit_exact_on_sample": (ctx.to_bytes(rs.uniq, rs.uniq_bytes) == eu and
                                           ctx.to_bytes(rs.fresh, rs.fresh_bytes) == ef)}
        cores = host_cores()
        g_lines = min(n_lines, args.gnu_lines)
        gcut = int(np.flatnonzero(buf == 10)[g_lines - 1]) + 1
        gdata = buf[:gcut].tobytes()
        g = gnu_grep_sort_comm(gdata, sigs, prior_host, cores)
        if g:
            gm, gu, gf, secs = g
            dg = torch.from_numpy(buf[:gcut].copy()).cuda()
            rg, _, _ = m.dev_match_dedup_diff(ctx, dg.data_ptr(), dg.numel(), d_prior.data_ptr(), n_prior,
                                             count_hits=False)
            tot = secs["grep"] + secs["sort_comm"]
            cpu["gnu_grep_sort_comm"] = {
                "value": round(g_lines / tot, 1), "unit": "records/s", "cores": cores, "seconds": secs,
                "sample": "%d X1 lines (%d B)" % (g_lines, len(gdata)),
                "command": "LC_ALL=C grep -a -F -f sigs (x%d line-aligned splits) | sort -u --parallel=%d | "
                           "comm -13 prior -" % (cores, cores),
                "bit_exact_vs_gpu": (ctx.to_bytes(rg.uniq, rg.uniq_bytes) == gu and
                                     ctx.to_bytes(rg.fresh, rg.fresh_bytes) == gf)}
    out = {
        "metric": METRIC, "value": round(R * args.steps / el, 1), "unit": "records/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el * 1e3 / args.steps, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (httpx lines: C2-style subdomain URLs + fixed per-URL title/server tails, SURVEY.md "
                "§8(d) C3 signatures)",
        "config": {"workload": "X1: %dM httpx lines -> match 2000 literals -> sort -u matched -> diff vs prior "
                               "matched set, 1 GPU" % (n_lines // 1_000_000),
                   "bytes": int(d.numel()), "prior_bytes": n_prior},
        "gbps": round(step_bytes * args.steps / el / 1e9, 2),
        "hbm_frac_step": round(step_bytes * args.steps / el / 1e9 / HBM_PEAK_GBS, 4),
        "flag_path_equals_hit_list_path": paths_agree,
        "records": {"in": R, "hits": int(nh), "matched": int(nm), "unique_matched": int(r.uniq_records),
                    "new_matched": int(r.fresh_records)},
        "roofline": roofline_of(stats, dominant, "x1", full),
        "cpu_baseline": cpu,
        "kernels": kernel_table(full),
        "dedup_path": ctx.last_path()[0],
    }
    if emit:
        print(json.dumps(out), flush=True)
    if own:
        ctx.close()
    return out


def bench_urls(args, ctx=None, emit=True):
    """C2's dedup+diff on 10M httpx -silent URLs ('https://' + the C2
    subdomain draw), where every record shares its first 8 bytes, so a key0 taken at byte 0
    is one value for the whole input. The pipeline keys from the common prefix (k_lcp) and
    the range routing splits with byte splitters. Bit-exact on a 1M-record sample against the
    oracle; reported as ns/record beside C2's."""
    import numpy as np
    import torch

    import swarm_amd
    from swarm_amd import corpus

    own = ctx is None
    if own:
        torch.cuda.set_device(0)
        ctx = swarm_amd.Context(0, torch.cuda.current_stream().cuda_stream)
    n_lines = args.lines

    def urls(a):
        b = a.tobytes()
        return np.frombuffer(b"https://" + b[:-1].replace(b"\n", b"\nhttps://") + b"\n", dtype=np.uint8)
    sub, ids = corpus.subdomains(n_lines, seed=1234)
    cur_np = urls(sub)
    prior_np = urls(corpus.prior_of(ids))
    del sub
    cur = torch.from_numpy(cur_np).cuda()
    prior = torch.from_numpy(prior_np).cuda()
    run = lambda: ctx.dedup_diff(cur.data_ptr(), cur.numel(), prior.data_ptr(), prior.numel())  # noqa: E731
    el, full, stats, dominant, r = timed_steps(ctx, run, args)
    step_bytes = cur.numel() + prior.numel() + int(r.uniq_bytes) + int(r.fresh_bytes)
    cpu = None
    if not args.no_cpu_baseline:
        from oracle import semantics as S
        m = min(1_000_000, n_lines)
        cut = int(np.flatnonzero(cur_np == 10)[m - 1]) + 1
        cs, ps = cur_np[:cut].tobytes(), prior_np.tobytes()
        tc = time.perf_counter()
        eu, ef = S.dedup_diff(cs, ps)
        tc = time.perf_counter() - tc
        dc = torch.from_numpy(cur_np[:cut].copy()).cuda()
        rs = ctx.dedup_diff(dc.data_ptr(), dc.numel(), prior.data_ptr(), prior.numel())
        cpu = {"value": round(m / tc, 1), "unit": "records/s", "cores": 1, "kind": "port",
               "sample": "%d URL records + full prior; oracle sorted(set())+set difference, 1 thread, %.2f s" % (m, tc),
               "gpu_bit_exact_on_sample": (ctx.to_bytes(rs.uniq, rs.uniq_bytes) == eu and
                                           ctx.to_bytes(rs.fresh, rs.fresh_bytes) == ef)}
    R = int(r.in_records)
    out = {
        "metric": METRIC, "value": round(R * args.steps / el, 1), "unit": "records/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el * 1e3 / args.steps, 4),
        "ns_per_record": round(el * 1e9 / args.steps / max(R, 1), 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (https:// + the C2 subdomain draw)",
        "config": {"workload": "URLs: %dM httpx -silent URLs sort -u + new-record diff, 1 GPU" % (n_lines // 1_000_000),
                   "bytes": int(cur.numel()), "prior_bytes": int(prior.numel())},
        "gbps": round(step_bytes * args.steps / el / 1e9, 2),
        "hbm_frac_step": round(step_bytes * args.steps / el / 1e9 / HBM_PEAK_GBS, 4),
        "records": {"in": R, "unique": int(r.uniq_records), "new": int(r.fresh_records)},
        "roofline": roofline_of(stats, dominant, "urls", full),
        "cpu_baseline": cpu,
        "kernels": kernel_table(full),
        "dedup_path": ctx.last_path()[0],
    }
    if emit:
        print(json.dumps(out), flush=True)
    if own:
        ctx.close()
    return out


def gnu_sort_comm(cur: bytes, prior: bytes, want_uniq: bytes, want_fresh: bytes, threads: int = 16):
    """The shell restatement of A7+A8 timed on the host: LC_ALL=C sort -u --parallel over
    the whole input, then comm -13 against the prior (SURVEY.md §8(d) CPU baseline).
    Inputs are staged in a temp dir first (outside the timing); the empty line that sort -u
    keeps is dropped before the comparison, as A7 defines."""
    import shutil
    import subprocess
    import tempfile
    if not shutil.which("sort") or not shutil.which("comm"):
        return None
    threads = max(1, min(threads, os.cpu_count() or 1))
    env = dict(os.environ, LC_ALL="C")
    with tempfile.TemporaryDirectory() as d:
        pc, pp, pu = os.path.join(d, "cur"), os.path.join(d, "prior"), os.path.join(d, "uniq")
        with open(pc, "wb") as f:
            f.write(cur)
        with open(pp, "wb") as f:
            f.write(prior)
        t = time.perf_counter()
        subprocess.run(["sort", "-u", "--parallel=%d" % threads, "-S", "25%", "-T", d, "-o", pu, pc], env=env,
                       check=True)
        fresh = subprocess.run(["comm", "-13", pp, pu], env=env, check=True, stdout=subprocess.PIPE).stdout
        t = time.perf_counter() - t
        with open(pu, "rb") as f:
            uniq = f.read()
    if uniq.startswith(b"\n"):
        uniq = uniq[1:]
    if fresh.startswith(b"\n"):
        fresh = fresh[1:]
    n = cur.count(b"\n") + (0 if cur.endswith(b"\n") or not cur else 1)
    return {"value": round(n / t, 1), "unit": "records/s", "cores": threads, "seconds": round(t, 2),
            "command": "LC_ALL=C sort -u --parallel=%d | comm -13 prior -" % threads,
            "bit_exact_with_oracle": uniq == want_uniq and fresh == want_fresh}


def dev_bytes(b, dev):
    import numpy as np
    import torch
    return torch.from_numpy(np.frombuffer(b, dtype=np.uint8).copy()).to(dev)


def free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(args, argv) -> int:
    """`--gpus N` (N > 1) without a torch.distributed launcher around us: start N ranks
    ourselves, one process per GPU, before this process touches any GPU (the parent only
    parses arguments), as `torch.distributed.run` on 127.0.0.1 would. Rank 0 prints the
    JSON line; the exit code is the launcher's."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % args.gpus,
           "--master-addr=127.0.0.1", "--master-port=%d" % free_port(), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    env.setdefault("OMP_NUM_THREADS", "4")
    return subprocess.run(cmd, env=env).returncode


def dist_setup(args):
    """(world, rank, local) from the launcher's env; initialises the process group when
    world > 1 and checks it matches --gpus."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("bench.py: WORLD_SIZE=%d but --gpus %d" % (world, args.gpus))
    return world, rank, local


def launcher_check(args):
    """CPU rehearsal of the N-rank launch and the timing protocol (barrier, max over ranks,
    one JSON line from rank 0) with no GPU work: what tests/test_bench_launcher.py runs."""
    import torch
    import torch.distributed as dist
    world, rank, _ = dist_setup(args)
    if world > 1:
        dist.init_process_group("gloo")
        dist.barrier()
    t0 = time.perf_counter()
    x = torch.arange(1 << 16, dtype=torch.int64)
    for _ in range(args.steps):
        x = (x * 3 + rank) % 1000003
    el = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "records/s", "n_gpus": world,
                          "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el * 1e3 / args.steps, 4),
                          "launcher_check": True, "workload": args.workload,
                          "world_size_seen": dist.get_world_size() if world > 1 else 1}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def init_dist(args):
    """(world, rank, local, device): one process per GPU; the process group (RCCL = "nccl",
    or gloo rehearsals) is initialised when world > 1 and must match --gpus."""
    import torch
    import torch.distributed as dist
    world, rank, local = dist_setup(args)
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        local = local % max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(local)
        dist.init_process_group(args.dist_backend)
        if dist.get_world_size() != args.gpus:
            raise SystemExit("bench.py: the process group has %d ranks, --gpus %d" % (dist.get_world_size(), args.gpus))
        world = dist.get_world_size()
    else:
        torch.cuda.set_device(0)
        if args.workload == "c5" and args.c5_path == "rounds" and args.dist_backend:
            # a 1-rank process group: the rounds step issues its collectives at world size 1
            # (on nccl = RCCL, the device-tensor all-to-all path of the N-rank step)
            os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
            dist.init_process_group(args.dist_backend, rank=0, world_size=1,
                                    init_method="tcp://127.0.0.1:%d" % free_port())
    return world, rank, local, torch.device("cuda", local)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--lines", type=int, default=10_000_000, help="C2 / URL lines per GPU")
    ap.add_argument("--workload", choices=["c2", "c3", "c4", "c5", "fields", "x1", "urls"], default=None,
                    help="default: c2 (+ every other config as sub-objects) at --gpus 1, c5 strong scaling at N > 1")
    ap.add_argument("--x1-lines", type=int, default=10_000_000, help="X1 fused-step input lines")
    ap.add_argument("--c1-lines", type=int, default=1_000_000, help="C1 lines")
    ap.add_argument("--c3-lines", type=int, default=50_000_000, help="C3 lines")
    ap.add_argument("--c4-lines", type=int, default=12_500_000, help="C4 banners per GPU")
    ap.add_argument("--c5-records", type=int, default=1_000_000_000, help="C5 records in total (all ranks)")
    ap.add_argument("--fields-lines", type=int, default=4_000_000, help="fields leg httpx -json lines")
    ap.add_argument("--gnu-lines", type=int, default=2_000_000, help="lines of the GNU-tool CPU baseline sample")
    ap.add_argument("--no-x1", action="store_true", help="default run: skip the fused X1 and URL legs")
    ap.add_argument("--no-sub", action="store_true", help="default run: headline only (no c1/c3/c4/c5/fields/x1/urls legs)")
    ap.add_argument("--no-c2-weak", action="store_true", help="N > 1 c5 run: skip the C2 weak-scaling sub-object")
    ap.add_argument("--c5-part-bytes", type=int, default=2 << 30,
                    help="C5 local path: bytes per local part (one library call each; 1.25 x headroom)")
    ap.add_argument("--c5-hosts", type=int, default=64_000_000, help="C5 hosts (x 4 open-port slots = combos)")
    ap.add_argument("--c5-data", choices=["hosts", "ips"], default="hosts",
                    help="C5 records: host:port names, or 10.x.y.z:port (15M hosts x 16 port slots)")
    ap.add_argument("--c5-path", choices=["local", "rounds"], default="local",
                    help="C5 at N = 1: local range parts with the parse handed over (default), or the N-rank "
                         "rounds step without its exchange (per-rank compute model)")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL) for real runs; gloo rehearses N ranks on fewer GPUs")
    ap.add_argument("--route", choices=["range", "hash"], default="range",
                    help="C2 N>1 record routing: byte ranges (outputs in global byte order) or hash parts")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gnu", action="store_true", help="skip the GNU coreutils/grep baselines")
    ap.add_argument("--cpu-sample", type=int, default=10_000_000)
    ap.add_argument("--launcher-check", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.workload is None:
        args.workload = "c2" if args.gpus == 1 else "c5"
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args, sys.argv[1:])
    if args.launcher_check:
        return launcher_check(args)
    if args.workload == "c3":
        bench_c3(args)
        return 0
    if args.workload == "c4":
        bench_c4(args)
        return 0
    if args.workload == "fields":
        bench_fields(args)
        return 0
    if args.workload == "x1":
        bench_x1(args)
        return 0
    if args.workload == "urls":
        bench_urls(args)
        return 0

    import torch
    import torch.distributed as dist

    import swarm_amd

    world, rank, local, dev = init_dist(args)
    ctx = swarm_amd.Context(local, torch.cuda.current_stream(dev).cuda_stream)

    if args.workload == "c5":
        line = bench_c5(args, world, rank, dev, ctx, emit=False)
        torch.cuda.empty_cache()
        if world > 1 and not args.no_c2_weak:
            # the C2 weak-scaling step beside C5's strong scaling (every rank runs it)
            c2 = bench_c2(args, world, rank, dev, ctx)
            if rank == 0:
                line["c2_weak"] = {k: c2[k] for k in SUB_KEYS if k in c2}
        if rank == 0:
            print(json.dumps(line), flush=True)
        ctx.close()
        if dist.is_initialized():
            dist.destroy_process_group()
        return 0

    # c2: the headline (configs[1]); at N = 1 every other config rides along as a sub-object
    line = bench_c2(args, world, rank, dev, ctx)
    torch.cuda.empty_cache()
    if rank == 0 and world == 1 and not args.no_sub:
        if not args.no_x1:
            u_full = sub_leg("urls", lambda: bench_urls(args, ctx=ctx, emit=False))
            if "ns_per_record" in u_full:
                u_full["ns_per_record_vs_c2"] = round(u_full["ns_per_record"] / (line["ms_per_step"] * 1e6 /
                                                                                 args.lines), 3)
            line["urls"] = {k: u_full[k] for k in SUB_KEYS + ("ns_per_record", "ns_per_record_vs_c2", "error")
                            if k in u_full}
            x1 = sub_leg("x1", lambda: bench_x1(args, ctx=ctx, emit=False))
            if "kernels" in x1:
                x1["kernels_top"] = dict(list(x1["kernels"].items())[:10])
            line["fused_x1"] = {k: x1[k] for k in SUB_KEYS + ("error",) if k in x1}
        line["c1"] = sub_leg("c1", lambda: bench_c1(args, ctx))
        line["c3"] = sub_leg("c3", lambda: bench_c3(args, ctx=ctx, emit=False), SUB_KEYS + ("error",))
        # C5 on a context of its own (its slots sized by its own parts, not grown from the
        # legs before it)
        line["c5"] = sub_leg("c5", lambda: bench_c5(args, 1, 0, dev, None, emit=False), SUB_KEYS + ("error",))
        line["c4"] = sub_leg("c4", lambda: bench_c4(args, ctx=ctx, emit=False), SUB_KEYS + ("records", "error"))
        line["fields"] = sub_leg("fields", lambda: bench_fields(args, ctx=ctx, emit=False),
                                 SUB_KEYS + ("records", "error"))
        line["legs"] = legs_summary(line)  # last: survives a truncated tail of the line
    if rank == 0:
        print(json.dumps(line), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main() or 0)
