"""ctypes binding of libwost.so (include/wost.h).

The library is the product: there is no CPU fallback. If libwost.so has not
been built this module raises ImportError immediately, and every solve call
fails loudly if no HIP device is present.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_float, c_int32, c_int64, c_uint8, c_uint32, c_uint64, c_void_p

import numpy as np

LIB_PATH = os.environ.get("WOST_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libwost.so")

WOST_OK = 0
WOST_ERR_INVALID_ARG = -1
WOST_ERR_HIP = -2
WOST_ERR_NO_DEVICE = -3
WOST_ERR_UNSUPPORTED = -4
WOST_ERR_OOM = -5
WOST_ERR_COMM = -6

ABI_VERSION = 6   # include/wost.h WOST_ABI_VERSION
WOST_COMM_ID_BYTES = 128
WOST_COMM_SUM, WOST_COMM_MAX = 0, 1
WOST_BLOCK_WALKS = 4096
WOST_MAX_SOURCES = 16   # include/wost.h
WOST_TRIG = {"auto": 0, "exact": 1, "fast": 2}   # include/wost.h wost_trig
WOST_SAMPLER_TABLE_N = 4097
COMPAT = {"reference": 0, "fixed": 1}
SLOT_BOUNDARY, SLOT_SOURCE = 0, 1
GEOM_OPS = {"distance": 0, "isSilhouette": 1, "silhouetteDistance": 2, "rayIntersection": 3,
            "intersectPolylines": 4}
WOST_GEOM_TREE = 256   # wost_geom_op flag: the query through the segment tree (ops 2 and 4)


class WostFactor(ctypes.Structure):
    _fields_ = [("kind", c_int32), ("p", c_float * 8)]


class WostTerm(ctypes.Structure):
    _fields_ = [("coef", c_float), ("first_factor", c_int32), ("n_factors", c_int32)]


class WostField(ctypes.Structure):
    _fields_ = [("terms", POINTER(WostTerm)), ("n_terms", c_int32),
                ("factors", POINTER(WostFactor)), ("n_factors", c_int32), ("flags", c_int32),
                ("grid", POINTER(c_float)), ("n_grid", c_int64)]


class WostPolyline(ctypes.Structure):
    _fields_ = [("xy", POINTER(c_float)), ("n_vertices", c_int32)]


class WostProblem(ctypes.Structure):
    _fields_ = [("dirichlet", WostPolyline), ("neumann", WostPolyline),
                ("boundary", POINTER(WostField)), ("source", POINTER(WostField)),
                ("sigma", POINTER(WostField)), ("alpha", POINTER(WostField)),
                ("compat", c_int32), ("device", c_int32), ("sigma_bar_override", c_double)]


class WostTiming(ctypes.Structure):
    _fields_ = [("walk_kernel_ms", c_double), ("reduce_kernel_ms", c_double), ("total_ms", c_double),
                ("n_launches", c_int32), ("grid_blocks", c_int32), ("total_steps", c_uint64),
                ("total_walks", c_uint64), ("jit", c_int32), ("tree", c_int32),
                ("blocks_per_cu", c_int32), ("block_threads", c_int32), ("chunk0", c_int32), ("chunk", c_int32),
                ("adaptive", c_int32), ("max_walk_steps", c_uint32), ("jit_ms", c_double), ("span_ms", c_double),
                ("tail_ms", c_double), ("last_wave_ms", c_double), ("last_wave_iters", c_uint32),
                ("max_wave_iters", c_uint32), ("precompiled_walks", c_uint64)]


class WostDistTiming(ctypes.Structure):
    _fields_ = [("local", WostTiming), ("walk_begin", c_int64), ("walk_end", c_int64), ("total_steps", c_uint64),
                ("local_ms", c_double), ("agree_ms", c_double), ("gather_ms", c_double), ("merge_ms", c_double)]


DIST_PREPARE = ctypes.CFUNCTYPE(c_int32, c_void_p, c_int64)
DIST_SOLVE_RANGE = ctypes.CFUNCTYPE(c_int32, c_void_p, c_int64, c_int64, POINTER(c_double))
DIST_ALLREDUCE = ctypes.CFUNCTYPE(c_int32, c_void_p, POINTER(c_double), c_int64, c_int32)
DIST_ALLGATHER = ctypes.CFUNCTYPE(c_int32, c_void_p, POINTER(c_double), c_int64, POINTER(c_double))


class WostDistOps(ctypes.Structure):
    """include/wost.h wost_dist_ops: the transport of wost_distributed_run."""
    _fields_ = [("ctx", c_void_p), ("prepare", DIST_PREPARE), ("solve_range", DIST_SOLVE_RANGE),
                ("allreduce", DIST_ALLREDUCE), ("allgather", DIST_ALLGATHER), ("key", POINTER(c_double)),
                ("n_key", c_int32)]


class WostError(RuntimeError):
    """A libwost call failed (HIP error, no device, out of memory)."""


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is not built. Build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "or `make -C dcrmontecarlo_amd/csrc`. There is no CPU fallback.")
    lib = ctypes.CDLL(LIB_PATH)
    H = c_void_p
    sig = {
        "wost_version": (c_int32, []),
        "wost_last_error": (c_char_p, []),
        "wost_device_count": (c_int32, [POINTER(c_int32)]),
        "wost_create": (c_int32, [POINTER(WostProblem), POINTER(c_void_p)]),
        "wost_destroy": (None, [H]),
        "wost_set_field": (c_int32, [H, c_int32, POINTER(WostField)]),
        "wost_get_info": (c_int32, [H, POINTER(c_double), POINTER(c_int32)]),
        "wost_num_blocks": (c_int64, [c_int64, c_int64]),
        # (plain addresses: c_void_p takes a pointer object or an int, and the facade's solve
        # passes the arrays' addresses -- a data_as() pointer costs ~3 us of host time each)
        "wost_solve": (c_int32, [H, c_void_p, c_int64, c_int64, c_int64, c_int64, c_int32, c_float,
                                 c_uint64, c_void_p, c_void_p, c_void_p, c_void_p]),
        "wost_solve_history": (c_int32, [H, POINTER(c_float), c_int64, c_int64, c_int32, c_float, c_uint64,
                                         POINTER(c_double), POINTER(c_float), POINTER(c_uint32), POINTER(c_float)]),
        "wost_prepare_sources": (c_int32, [H, POINTER(POINTER(WostField)), c_int32, c_int64]),
        "wost_set_sources": (c_int32, [H, POINTER(POINTER(WostField)), c_int32]),
        "wost_solve_multi": (c_int32, [H, POINTER(c_float), c_int64, c_int64, c_int64, c_int64, c_int32, c_float,
                                       c_uint64, POINTER(c_double), POINTER(c_double), POINTER(c_float),
                                       POINTER(c_uint32)]),
        "wost_last_timing": (c_int32, [H, POINTER(WostTiming)]),
        "wost_num_sources": (c_int32, [H, POINTER(c_int32)]),
        "wost_solve_range": (c_int32, [H, POINTER(c_float), c_int64, c_int64, c_int64, c_int64, c_int32, c_float,
                                       c_uint64, POINTER(c_double), POINTER(c_double), POINTER(c_float),
                                       POINTER(c_uint32)]),
        "wost_comm_unique_id": (c_int32, [POINTER(c_uint8)]),
        "wost_comm_create": (c_int32, [POINTER(c_uint8), c_int32, c_int32, c_int32, POINTER(c_void_p)]),
        "wost_comm_destroy": (None, [c_void_p]),
        "wost_comm_info": (c_int32, [c_void_p, POINTER(c_int32), POINTER(c_int32), POINTER(c_int32)]),
        "wost_comm_last_error": (c_char_p, []),
        "wost_comm_allgather": (c_int32, [c_void_p, POINTER(c_double), c_int64, POINTER(c_double)]),
        "wost_comm_allreduce": (c_int32, [c_void_p, POINTER(c_double), c_int64, c_int32]),
        "wost_comm_barrier": (c_int32, [c_void_p]),
        "wost_shard_walk_range": (c_int32, [c_int64, c_int32, c_int32, POINTER(c_int64), POINTER(c_int64)]),
        "wost_solve_distributed": (c_int32, [H, c_void_p, POINTER(c_float), c_int64, c_int64, c_int32, c_float,
                                             c_uint64, POINTER(c_double), POINTER(WostDistTiming)]),
        "wost_shard_blocks_max": (c_int64, [c_int64, c_int32]),
        "wost_shard_pack": (c_int32, [POINTER(c_double), c_int64, c_int64, c_int32, c_int32, c_int32,
                                      POINTER(c_double)]),
        "wost_shard_merge": (c_int32, [POINTER(c_double), c_int64, c_int64, c_int32, c_int32, POINTER(c_double)]),
        "wost_distributed_run": (c_int32, [POINTER(WostDistOps), c_int32, c_int32, c_int64, c_int64, c_int32,
                                           POINTER(c_double), POINTER(c_int64), POINTER(c_int64),
                                           POINTER(c_uint64)]),
        "wost_dist_last_phases": (c_int32, [POINTER(c_double)]),
        "wost_dist_solve_key": (c_int32, [c_uint64, c_float, c_int32, POINTER(c_float), c_int64, POINTER(c_double)]),
        "wost_greens_norm": (c_int32, [c_double, POINTER(c_float), c_int64, POINTER(c_float)]),
        "wost_screened_sample_fixed": (c_int32, [POINTER(c_float), POINTER(c_float), c_int64, POINTER(c_float)]),
        "wost_screened_cdf_fixed": (c_int32, [c_double, POINTER(c_double), c_int64, POINTER(c_double)]),
        "wost_set_jit": (c_int32, [H, c_int32]),
        "wost_set_trig": (c_int32, [H, c_int32]),
        "wost_set_fixed_step_check": (c_int32, [H, c_int32]),
        "wost_set_segment_tree": (c_int32, [H, c_int32, c_int32]),
        "wost_set_option": (c_int32, [H, c_char_p, c_double]),
        "wost_get_option": (c_int32, [H, c_char_p, POINTER(c_double)]),
        "wost_options_report": (c_int32, [H, ctypes.c_char_p, c_int64, POINTER(c_int64)]),
        "wost_kernel_source": (c_int32, [POINTER(WostProblem), ctypes.c_char_p, c_int64, POINTER(c_int64)]),
        "wost_kernel_source_sources": (c_int32, [POINTER(WostProblem), POINTER(POINTER(WostField)), c_int32,
                                                 ctypes.c_char_p, c_int64, POINTER(c_int64)]),
        "wost_jit_compile": (c_int32, [ctypes.c_char_p, ctypes.c_char_p, c_int32, POINTER(c_uint8), c_int64,
                                       POINTER(c_int64), POINTER(c_int32)]),
        "wost_eval_field": (c_int32, [H, c_int32, POINTER(c_float), c_int64, POINTER(c_float)]),
        "wost_sampler_table": (c_int32, [H, POINTER(c_float), c_int32]),
        "wost_geometry_query": (c_int32, [c_int32, c_int32, POINTER(WostPolyline), POINTER(c_float),
                                          POINTER(c_float), POINTER(c_float), c_int64, POINTER(c_float),
                                          POINTER(c_uint8)]),
    }
    for name, (res, args) in sig.items():
        # an older build may lack a newer entry point: it loads, and calling the
        # missing one raises AttributeError (the export test checks a fresh build)
        fn = getattr(lib, name, None)
        if fn is None:
            continue
        fn.restype = res
        fn.argtypes = args
    if lib.wost_version() != ABI_VERSION:
        raise ImportError(f"libwost ABI version {lib.wost_version()} != {ABI_VERSION} (rebuild libwost.so)")
    return lib


lib = _load()


def check(rc: int, what: str = "libwost", comm: bool = False):
    if rc == WOST_OK:
        return
    msg = ((lib.wost_comm_last_error() if comm else lib.wost_last_error()) or b"").decode(errors="replace")
    if rc == WOST_ERR_INVALID_ARG:
        raise ValueError(f"{what}: {msg}")
    if rc == WOST_ERR_UNSUPPORTED:
        raise NotImplementedError(f"{what}: {msg}")
    raise WostError(f"{what} failed ({rc}): {msg}")


def options_report(h=None) -> dict:
    """wost_options_report: {"build": "product"|"study", "non_default": {...}} of a handle
    (None: the library's build only)."""
    import json

    n = c_int64(0)
    check(lib.wost_options_report(h, None, 0, ctypes.byref(n)), "wost_options_report")
    buf = ctypes.create_string_buffer(n.value + 1)
    check(lib.wost_options_report(h, buf, n.value + 1, ctypes.byref(n)), "wost_options_report")
    return json.loads(buf.value.decode())


def device_count() -> int:
    n = c_int32(0)
    rc = lib.wost_device_count(ctypes.byref(n))
    return int(n.value) if rc == WOST_OK else 0


def fptr(a: np.ndarray):
    return a.ctypes.data_as(POINTER(c_float)) if a is not None else None


def dptr(a: np.ndarray):
    return a.ctypes.data_as(POINTER(c_double)) if a is not None else None


def addr(a: np.ndarray):
    """The array's data address for a c_void_p argument (None for None)."""
    return a.__array_interface__["data"][0] if a is not None else None


def u32ptr(a: np.ndarray):
    return a.ctypes.data_as(POINTER(c_uint32)) if a is not None else None


def make_polyline(xy: np.ndarray | None):
    """(WostPolyline, keepalive)"""
    if xy is None or len(xy) == 0:
        return WostPolyline(None, 0), None
    a = np.ascontiguousarray(xy, dtype=np.float32).reshape(-1, 2)
    return WostPolyline(fptr(a), a.shape[0]), a


def make_field(field):
    """Field (dcrmontecarlo_amd.fields) -> (WostField, keepalive) or (None, None)."""
    if field is None:
        return None, None
    terms, factors = field.pack()
    T = (WostTerm * max(1, len(terms)))()
    for i, (coef, first, n) in enumerate(terms):
        T[i].coef = np.float32(coef)
        T[i].first_factor = first
        T[i].n_factors = n
    F = (WostFactor * max(1, len(factors)))()
    for i, (kind, p) in enumerate(factors):
        F[i].kind = kind
        for k in range(8):
            F[i].p[k] = np.float32(p[k])
    G = field.grid_values()
    wf = WostField(ctypes.cast(T, POINTER(WostTerm)), len(terms), ctypes.cast(F, POINTER(WostFactor)),
                   len(factors), field.flags, fptr(G) if G.size else None, int(G.size))
    return wf, (T, F, G, wf)


def declared_symbols() -> list[str]:
    """Entry points declared in include/wost.h (for the export check)."""
    import re

    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    hdr = os.path.join(here, "include", "wost.h")
    text = open(hdr).read()
    return sorted(set(re.findall(r"^[A-Za-z_][\w\s\*]*?\b(wost_\w+)\s*\(", text, re.M)))

REC_FLOATS = 8   # include/wost.h WOST_REC_FLOATS
