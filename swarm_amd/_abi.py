"""ctypes binding of libswarmgpu.so (include/swarmgpu.h). No fallback: if the library is
missing or fails to load, importing this module raises."""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libswarmgpu.so")

SG_OK = 0
SG_E_INVAL = 1
SG_E_CAP = 2
SG_E_HIP = 3
SG_E_NOMEM = 4
SG_E_TOO_LARGE = 5
SG_E_UNSUPPORTED = 6
SG_E_STATES = 7
SG_E_NODEV = 8
SG_E_CORRUPT = 9
SG_NOCASE = 1

ERRNAMES = {1: "SG_E_INVAL", 2: "SG_E_CAP", 3: "SG_E_HIP", 4: "SG_E_NOMEM", 5: "SG_E_TOO_LARGE",
            6: "SG_E_UNSUPPORTED", 7: "SG_E_STATES", 8: "SG_E_NODEV", 9: "SG_E_CORRUPT"}

EXPORTS = [
    "sg_last_error", "sg_version", "sg_device_count", "sg_ctx_create", "sg_ctx_destroy",
    "sg_ctx_sync", "sg_ctx_profile", "sg_ctx_profile_only", "sg_ctx_kernel_stat", "sg_ctx_reset_stats", "sg_ctx_memcpy",
    "sg_ctx_last_path", "sg_ctx_last_key_width", "sg_lines",
    "sg_dedup", "sg_dedup_chunks", "sg_diff", "sg_dedup_diff", "sg_dev_dedup_diff",
    "sg_dev_partition", "sg_hash64", "sg_ac_compile", "sg_dfa_compile", "sg_matcher_info",
    "sg_match", "sg_match_lines", "sg_dev_match", "sg_dev_match_dedup_diff", "sg_free",
    "sg_nmap_ports", "sg_dev_nmap_ports", "sg_json_fields", "sg_dev_json_fields",
]


class SGError(RuntimeError):
    def __init__(self, rc: int, msg: str):
        super().__init__("%s: %s" % (ERRNAMES.get(rc, rc), msg))
        self.rc = rc


class DevResult(C.Structure):
    _fields_ = [("uniq", C.c_void_p), ("uniq_bytes", C.c_uint64), ("uniq_records", C.c_uint64),
                ("fresh", C.c_void_p), ("fresh_bytes", C.c_uint64), ("fresh_records", C.c_uint64),
                ("in_records", C.c_uint64), ("prior_records", C.c_uint64)]


class DevHits(C.Structure):
    _fields_ = [("rec_idx", C.c_void_p), ("sig_id", C.c_void_p), ("n_hits", C.c_uint64),
                ("lines", C.c_void_p), ("lines_bytes", C.c_uint64), ("matched_records", C.c_uint64),
                ("in_records", C.c_uint64)]


class DevText(C.Structure):
    _fields_ = [("data", C.c_void_p), ("bytes", C.c_uint64), ("records", C.c_uint64), ("in_records", C.c_uint64)]


class DevRows(C.Structure):
    _fields_ = [("data", C.c_void_p), ("bytes", C.c_uint64), ("rows", C.c_uint64), ("row_rec", C.c_void_p),
                ("row_key", C.c_void_p), ("in_records", C.c_uint64)]


def _load():
    # One HIP runtime per process: torch bundles its own libamdhip64 (soname
    # libamdhip64.so.7, the same soname as /opt/rocm's). Loading torch first makes our
    # NEEDED entry bind to the already-loaded runtime instead of a second copy, so torch
    # tensors, streams and RCCL share the device with our kernels.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError("libswarmgpu.so not built (%s); run `make -C swarm_amd/csrc` or "
                          "__graft_entry__.build()" % LIB_PATH)
    lib = C.CDLL(LIB_PATH)
    P, U8P, SZ, SZP = C.c_void_p, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)
    U64P, U32P = C.POINTER(C.c_uint64), C.POINTER(C.c_uint32)
    sig = {
        "sg_last_error": (C.c_char_p, []),
        "sg_version": (C.c_int, []),
        "sg_device_count": (C.c_int, [C.POINTER(C.c_int)]),
        "sg_ctx_create": (C.c_int, [C.c_int, P, C.POINTER(P)]),
        "sg_ctx_destroy": (C.c_int, [P]),
        "sg_ctx_sync": (C.c_int, [P]),
        "sg_ctx_profile": (C.c_int, [P, C.c_int]),
        "sg_ctx_profile_only": (C.c_int, [P, C.c_char_p]),
        "sg_ctx_kernel_stat": (C.c_int, [P, C.c_int, C.POINTER(C.c_char_p), U64P, C.POINTER(C.c_double),
                                         C.POINTER(C.c_double)]),
        "sg_ctx_reset_stats": (C.c_int, [P]),
        "sg_ctx_memcpy": (C.c_int, [P, P, P, SZ]),
        "sg_ctx_last_path": (C.c_int, [P, C.POINTER(C.c_int), U32P]),
        "sg_ctx_last_key_width": (C.c_int, [P, U32P]),
        "sg_lines": (C.c_int, [U8P, SZ, U64P, SZ, SZP]),
        "sg_dedup": (C.c_int, [U8P, SZ, U8P, SZ, SZP]),
        "sg_dedup_chunks": (C.c_int, [C.POINTER(P), SZP, SZ, U8P, SZ, SZP]),
        "sg_diff": (C.c_int, [U8P, SZ, U8P, SZ, U8P, SZ, SZP]),
        "sg_dedup_diff": (C.c_int, [U8P, SZ, U8P, SZ, U8P, SZ, SZP, U8P, SZ, SZP]),
        "sg_dev_dedup_diff": (C.c_int, [P, P, SZ, P, SZ, C.POINTER(DevResult)]),
        "sg_dev_partition": (C.c_int, [P, P, SZ, C.c_uint32, P, SZ, U64P, U64P]),
        "sg_hash64": (C.c_uint64, [U8P, SZ]),
        "sg_ac_compile": (C.c_int, [U8P, U32P, C.c_uint32, C.c_uint32, C.POINTER(P)]),
        "sg_dfa_compile": (C.c_int, [U8P, U32P, C.c_uint32, C.c_uint32, C.POINTER(P)]),
        "sg_matcher_info": (C.c_int, [P, U64P, U32P, U32P]),
        "sg_match": (C.c_int, [P, U8P, SZ, U64P, U32P, SZ, SZP]),
        "sg_match_lines": (C.c_int, [P, U8P, SZ, U8P, SZ, SZP]),
        "sg_dev_match": (C.c_int, [P, P, P, SZ, C.POINTER(DevHits)]),
        "sg_dev_match_dedup_diff": (C.c_int, [P, P, P, SZ, P, SZ, C.POINTER(DevResult), U64P, U64P]),
        "sg_free": (None, [P]),
        "sg_nmap_ports": (C.c_int, [U8P, SZ, U8P, SZ, SZP]),
        "sg_dev_nmap_ports": (C.c_int, [P, P, SZ, C.POINTER(DevText)]),
        "sg_json_fields": (C.c_int, [U8P, SZ, U8P, U32P, C.c_uint32, U8P, SZ, SZP, U32P, U32P, SZ, SZP]),
        "sg_dev_json_fields": (C.c_int, [P, P, SZ, U8P, U32P, C.c_uint32, C.POINTER(DevRows)]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


lib = _load()


def check(rc: int) -> None:
    if rc != SG_OK:
        raise SGError(rc, lib.sg_last_error().decode(errors="replace"))


class TmMatcher(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("part", C.c_uint32), ("flags", C.c_uint32), ("tmpl", C.c_uint32),
                ("first", C.c_uint32), ("count", C.c_uint32)]


class DevTMatches(C.Structure):
    _fields_ = [("rec_idx", C.c_void_p), ("tmpl_id", C.c_void_p), ("n", C.c_uint64), ("in_records", C.c_uint64)]


SG_TM_WORD, SG_TM_REGEX = 0, 1
SG_TM_AND, SG_TM_NEGATIVE, SG_TM_NOCASE = 1, 2, 4
EXPORTS += ["sg_tmpl_compile", "sg_tmpl_info", "sg_dev_tmpl_eval", "sg_dev_tmpl_eval_rows", "sg_tmpl_eval",
            "sg_tmpl_free"]
for _name, (_res, _args) in {
    "sg_tmpl_compile": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint32), C.c_uint32, C.POINTER(TmMatcher), C.c_uint32,
                                  C.POINTER(C.c_uint32), C.c_uint32, C.c_void_p, C.POINTER(C.c_uint32), C.c_uint32,
                                  C.POINTER(C.c_void_p)]),
    "sg_tmpl_info": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
    "sg_dev_tmpl_eval": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.POINTER(DevTMatches)]),
    "sg_dev_tmpl_eval_rows": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.POINTER(DevRows),
                                        C.POINTER(DevTMatches)]),
    "sg_tmpl_eval": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                               C.c_size_t, C.POINTER(C.c_size_t)]),
    "sg_tmpl_free": (None, [C.c_void_p]),
}.items():
    _f = getattr(lib, _name)
    _f.restype = _res
    _f.argtypes = _args

EXPORTS += ["sg_ingest_open", "sg_ingest_append", "sg_ingest_finish", "sg_ingest_close"]
for _name, (_res, _args) in {
    "sg_ingest_open": (C.c_int, [C.c_void_p, C.c_size_t, C.POINTER(C.c_void_p)]),
    "sg_ingest_append": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t]),
    "sg_ingest_finish": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_uint64)]),
    "sg_ingest_close": (C.c_int, [C.c_void_p]),
}.items():
    _f = getattr(lib, _name)
    _f.restype = _res
    _f.argtypes = _args

EXPORTS += ["sg_dev_partition_range", "sg_dev_key_sample", "sg_dev_partition_bytes", "sg_dev_record_sample",
            "sg_dev_partition_bytes_pieces", "sg_dev_partition_bytes_pieces_a16", "sg_dev_dedup_diff_into",
            "sg_dev_partition_bytes_pieces_spans", "sg_dev_dedup_diff_spans_into",
            "sg_dev_partition_bytes_pieces_rounds", "sg_dev_partition_pieces_count",
            "sg_dev_partition_bytes_pieces_rounds_spans", "sg_dev_rebase_spans", "sg_span_sum"]
for _name, (_res, _args) in {
    "sg_dev_partition_pieces_count": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t), C.c_size_t,
                                                C.POINTER(C.c_uint64)]),
    "sg_dev_partition_bytes_pieces_rounds_spans": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p),
                                                             C.POINTER(C.c_size_t), C.c_size_t, C.c_void_p,
                                                             C.POINTER(C.c_uint32), C.c_uint32, C.c_uint32, C.c_void_p,
                                                             C.c_size_t, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                                             C.c_void_p, C.c_void_p, C.c_size_t,
                                                             C.POINTER(C.c_uint64)]),
    "sg_dev_rebase_spans": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t,
                                      C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.c_uint32, C.POINTER(C.c_uint64)]),
    "sg_dev_partition_bytes_pieces": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t), C.c_size_t,
                                                C.c_void_p, C.POINTER(C.c_uint32), C.c_uint32, C.c_void_p, C.c_size_t,
                                                C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "sg_dev_partition_bytes_pieces_a16": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t),
                                                    C.c_size_t, C.c_void_p, C.POINTER(C.c_uint32), C.c_uint32,
                                                    C.c_void_p, C.c_size_t, C.POINTER(C.c_uint64),
                                                    C.POINTER(C.c_uint64)]),
    "sg_dev_partition_bytes_pieces_rounds": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t),
                                                       C.c_size_t, C.c_void_p, C.POINTER(C.c_uint32), C.c_uint32,
                                                       C.c_uint32, C.c_void_p, C.c_size_t, C.POINTER(C.c_uint64),
                                                       C.POINTER(C.c_uint64)]),
    "sg_dev_dedup_diff_into": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_void_p,
                                         C.c_size_t, C.c_void_p, C.c_size_t, C.POINTER(DevResult)]),
    "sg_dev_partition_bytes_pieces_spans": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t),
                                                      C.c_size_t, C.c_void_p, C.POINTER(C.c_uint32), C.c_uint32,
                                                      C.c_void_p, C.c_size_t, C.POINTER(C.c_uint64),
                                                      C.POINTER(C.c_uint64), C.POINTER(C.c_void_p),
                                                      C.POINTER(C.c_void_p), C.POINTER(C.c_uint64)]),
    "sg_dev_dedup_diff_spans_into": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p,
                                               C.c_size_t, C.c_uint64, C.c_void_p, C.c_size_t, C.c_void_p,
                                               C.c_size_t, C.c_void_p, C.c_size_t, C.POINTER(DevResult)]),
    "sg_span_sum": (C.c_uint64, [C.c_void_p, C.c_void_p, C.c_size_t]),
    "sg_dev_partition_bytes": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.POINTER(C.c_uint32),
                                         C.c_uint32, C.c_void_p, C.c_size_t, C.POINTER(C.c_uint64),
                                         C.POINTER(C.c_uint64)]),
    "sg_dev_record_sample": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_uint32, C.c_void_p,
                                       C.POINTER(C.c_uint32), C.POINTER(C.c_uint64)]),
    "sg_dev_partition_range": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.POINTER(C.c_uint64), C.c_uint32,
                                         C.c_void_p, C.c_size_t, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "sg_dev_key_sample": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_uint32, C.POINTER(C.c_uint64),
                                    C.POINTER(C.c_uint64)]),
}.items():
    _f = getattr(lib, _name)
    _f.restype = _res
    _f.argtypes = _args
