"""WostSolver_2D on MI355X (reference: solvers/WoStSolver.py:15-353).

Drop-in for the reference class: same constructor arguments, same
``setBoundaryConditions`` / ``setSourceTerm`` / ``solve`` signatures and
defaults, same attributes (``use_delta_tracking``, ``sigma_bar``,
``domain_bounds``, ``sigma_prime``). The walk loop runs in libwost's gfx950
kernel; this class only describes the problem and moves arrays.

Differences a caller sees:

* Coefficient functions become device-evaluable fields
  (:mod:`dcrmontecarlo_amd.fields`): pass fields or numbers directly, or the
  reference's Python callables, which are traced into closed form (exact) or
  tabulated over the domain (approximate, with a warning) by
  :mod:`dcrmontecarlo_amd.trace`.
* Randomness is counter-based: ``solve(..., seed=0)`` is bitwise reproducible
  and independent of the GPU count. Walk ``i`` of point ``p`` uses Philox
  subsequence ``p*nWalks + i``.
* ``solve`` returns a float32 ``[N, 1]`` array (a torch tensor if the points
  were a torch tensor); ``return_stats=True`` adds per-point standard errors
  and mean step counts.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
from dataclasses import dataclass

import numpy as np

from .. import _lib
from ..fields import Field, as_field, const, detach


def _is_torch(a) -> bool:
    return type(a).__module__.startswith("torch")


_TIMING_FIELDS = tuple(k for k, _ in _lib.WostTiming._fields_)


def _points_np(a) -> np.ndarray:
    if _is_torch(a):
        a = a.detach().cpu().numpy()
    p = np.ascontiguousarray(np.asarray(a, dtype=np.float32))
    if p.ndim == 1 and p.shape[0] == 2:
        p = p.reshape(1, 2)
    if p.ndim != 2 or p.shape[1] != 2:
        raise ValueError(f"solvePoints must have shape [N, 2], got {p.shape}")
    return p


def _field_or_none(f, what: str):
    if f is None:
        return None
    try:
        return as_field(f)
    except TypeError as e:
        raise TypeError(f"{what}: {e}") from None


def _bounds_of(dxy: np.ndarray, nxy) -> list:
    allp = dxy if nxy is None else np.concatenate([dxy, nxy])
    return [[float(allp[:, 0].min()), float(allp[:, 0].max())],
            [float(allp[:, 1].min()), float(allp[:, 1].max())]]


@dataclass
class SolveStats:
    """Per-point Monte-Carlo statistics of one solve."""

    mean: np.ndarray        # [N] float64: sum / nWalks
    stderr: np.ndarray      # [N] float64: sample std / sqrt(nWalks)
    mean_steps: np.ndarray  # [N] float64
    walks: int              # walks per point
    total_steps: int
    kernel_ms: float        # walk-kernel time (HIP events)
    total_ms: float         # device time of the whole solve


def stats_from_sums(sums: np.ndarray, n_walks: int, total_steps=None, kernel_ms=0.0, total_ms=0.0) -> SolveStats:
    s, q, st = sums[:, 0], sums[:, 1], sums[:, 2]
    mean = s / n_walks
    var = np.maximum(q / n_walks - mean * mean, 0.0) * (n_walks / max(n_walks - 1, 1))
    return SolveStats(mean=mean, stderr=np.sqrt(var / n_walks), mean_steps=st / n_walks, walks=n_walks,
                      total_steps=int(st.sum()) if total_steps is None else int(total_steps),
                      kernel_ms=float(kernel_ms), total_ms=float(total_ms))


def _problem(dxy, nxy, g, f, sigma, alpha, compat, device, sigma_bar):
    """wost_problem for the given geometry and fields (None = absent; the library
    applies the sigma = 0 / alpha = 1 defaults itself) and the objects to keep alive."""
    keep = []
    dpoly, k1 = _lib.make_polyline(dxy)
    npoly, k2 = _lib.make_polyline(nxy)
    fields = {}
    for name, fld in (("boundary", g), ("source", f), ("sigma", sigma), ("alpha", alpha)):
        wf, k = _lib.make_field(fld)
        fields[name] = ctypes.pointer(wf) if wf is not None else None
        keep.append(k)
    prob = _lib.WostProblem(dpoly, npoly, fields["boundary"], fields["source"], fields["sigma"], fields["alpha"],
                            _lib.COMPAT[compat], int(device), float(sigma_bar) if sigma_bar else 0.0)
    return prob, keep + [k1, k2]


def kernel_source(dirichletBoundary, dirichletBoundaryFunction=None, neumannBoundary=None, source=None,
                  sigma=None, alpha=None, *, sigma_bar: float | None = None, compat: str = "reference",
                  sources=None) -> str:
    """HIP source of the field-specialised walk kernel a WostSolver_2D with these
    arguments would compile (no device needed; wost_kernel_source). sources: the fields
    of a multi-source solve (solve_sources; wost_kernel_source_sources)."""
    dxy = np.asarray(_np(dirichletBoundary.points), dtype=np.float32).reshape(-1, 2)
    nxy = None if neumannBoundary is None else np.asarray(_np(neumannBoundary.points), dtype=np.float32).reshape(-1, 2)
    conv = _Converter(_bounds_of(dxy, nxy))
    g = conv(dirichletBoundaryFunction, "dirichletBoundaryFunction")
    f = conv(source, "source")
    s = conv(sigma, "sigma")
    a = conv(alpha, "alpha", is_alpha=True)
    if a is not None and a.is_constant():
        a = detach(a)
    if compat not in _lib.COMPAT:
        raise ValueError(f"compat must be one of {sorted(_lib.COMPAT)}")
    prob, keep = _problem(dxy, nxy, g, f, s, a, compat, 0, sigma_bar)
    packed = [_lib.make_field(conv(x, "source")) for x in (sources or [])]
    arr = (ctypes.POINTER(_lib.WostField) * max(1, len(packed)))(*[ctypes.pointer(wf) for wf, _ in packed])
    n = ctypes.c_int64(0)
    call = lambda buf, cap: _lib.lib.wost_kernel_source_sources(ctypes.byref(prob), arr, len(packed), buf, cap,
                                                                 ctypes.byref(n))
    _lib.check(call(None, 0), "wost_kernel_source")
    buf = ctypes.create_string_buffer(n.value + 1)
    _lib.check(call(buf, n.value + 1), "wost_kernel_source")
    return buf.value.decode()


class _Converter:
    """Coefficient arguments -> device fields: Fields and numbers as they are,
    Python callables traced into closed form or tabulated over the domain
    (dcrmontecarlo_amd.trace). Records how each one was converted."""

    def __init__(self, bounds, resolution: int = 513, trace: bool = True):
        self.bounds, self.resolution, self.trace = bounds, resolution, trace
        self.log = {}

    def __call__(self, obj, what: str, is_alpha: bool = False):
        if obj is None:
            return None
        from ..trace import field_from_callable

        c = field_from_callable(obj, self.bounds, what=what, is_alpha=is_alpha, resolution=self.resolution,
                                trace_first=self.trace)
        self.log[what] = c
        return c.field


class WostSolver_2D:
    """Walk-on-Stars solver for -div(alpha grad u) + sigma u = f with Dirichlet
    and (optionally) Neumann polyline boundaries, on a HIP device.

    Coefficients (dirichletBoundaryFunction, source, sigma, alpha) may be
    :mod:`dcrmontecarlo_amd.fields` fields, numbers, or the reference's Python
    callables ``fn(point)``: those are traced into closed-form device fields,
    or -- when they use something the tracer cannot express -- tabulated on a
    ``grid_resolution``-node grid over the domain with a warning
    (dcrmontecarlo_amd.trace). ``field_conversions`` records which."""

    def __init__(self, dirichletBoundary, dirichletBoundaryFunction=None, neumannBoundary=None,
                 source=None, sigma=None, alpha=None, *, compat: str = "reference", device: int | None = None,
                 sigma_bar: float | None = None, grid_resolution: int = 513, trace_callables: bool = True):
        self.dirichletBoundary = dirichletBoundary
        self.neumannBoundary = neumannBoundary
        dxy = np.asarray(_np(dirichletBoundary.points), dtype=np.float32).reshape(-1, 2)
        nxy = None if neumannBoundary is None else np.asarray(_np(neumannBoundary.points), dtype=np.float32).reshape(-1, 2)
        # solvers/WoStSolver.py:37-43
        self.domain_bounds = _bounds_of(dxy, nxy)
        self._conv = _Converter(self.domain_bounds, grid_resolution, trace_callables)
        self.field_conversions = self._conv.log
        self.boundaryDirichlet = self._conv(dirichletBoundaryFunction, "dirichletBoundaryFunction")
        self.source = self._conv(source, "source")
        self.use_delta_tracking = sigma is not None or alpha is not None     # :51-64
        self.sigma = self.alpha = None
        if self.use_delta_tracking:
            s = self._conv(sigma, "sigma")
            a = self._conv(alpha, "alpha", is_alpha=True)
            self.sigma = s if s is not None else const(0.0)                    # :55-56
            a = a if a is not None else const(1.0)                             # :57-58
            if a.is_constant():
                a = detach(a)   # autograd of a constant raises -> sigma/alpha (Q9)
            self.alpha = a
        if compat not in _lib.COMPAT:
            raise ValueError(f"compat must be one of {sorted(_lib.COMPAT)}")
        self.compat = compat
        if device is None:
            device = int(os.environ.get("WOST_DEVICE", os.environ.get("LOCAL_RANK", "0")))
        self.device = int(device)

        prob, self._keep = _problem(dxy, nxy, self.boundaryDirichlet, self.source,
                                    self.sigma if sigma is not None else None,
                                    self.alpha if alpha is not None else None, compat, self.device, sigma_bar)
        h = ctypes.c_void_p()
        _lib.check(_lib.lib.wost_create(ctypes.byref(prob), ctypes.byref(h)), "WostSolver_2D")
        self._h = h
        sb = ctypes.c_double(0.0)
        dt = ctypes.c_int32(0)
        _lib.check(_lib.lib.wost_get_info(self._h, ctypes.byref(sb), ctypes.byref(dt)), "wost_get_info")
        self.sigma_bar = float(sb.value) if self.use_delta_tracking else None
        self.last_timing = None
        self.last_point_sums = None   # (sum, sum^2, steps) per point of the last solve

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            _lib.lib.wost_destroy(h)
            self._h = None

    # ---- setters (solvers/WoStSolver.py:141-157) ------------------------------
    # the attribute changes only once libwost has accepted the field, so that it always
    # describes what the device solves
    def setBoundaryConditions(self, boundaryDirichlet):
        g = self._conv(boundaryDirichlet, "boundaryDirichlet")
        wf, keep = _lib.make_field(g)
        _lib.check(_lib.lib.wost_set_field(self._h, _lib.SLOT_BOUNDARY, ctypes.pointer(wf) if wf else None),
                   "setBoundaryConditions")
        self.boundaryDirichlet = g

    def setSourceTerm(self, source):
        f = self._conv(source, "source")
        wf, keep = _lib.make_field(f)
        _lib.check(_lib.lib.wost_set_field(self._h, _lib.SLOT_SOURCE, ctypes.pointer(wf) if wf else None),
                   "setSourceTerm")
        self.source = f

    # ---- sigma' as a callable, like the reference's attribute ----------------
    def sigma_prime(self, point):
        """sigma'(point) evaluated on the device (buildModifiedSigma's closure, :88-127)."""
        p = _points_np(point)
        out = self.eval_field("sigma_prime", p)[:, 0]
        return out[0] if np.asarray(_np(point)).ndim == 1 else out

    def eval_field(self, which: str, points) -> np.ndarray:
        """Device evaluation: which in {g, f, sigma, alpha, sigma_prime} -> [N, 4]
        (value, d/dx, d/dy, Laplacian; sigma_prime: sigma', alpha, sigma, 0)."""
        idx = {"g": 0, "f": 1, "sigma": 2, "alpha": 3, "sigma_prime": 4}[which]
        p = _points_np(points)
        out = np.empty((p.shape[0], 4), np.float32)
        _lib.check(_lib.lib.wost_eval_field(self._h, idx, _lib.fptr(p), p.shape[0], _lib.fptr(out)), "eval_field")
        return out

    def sampler_table(self) -> np.ndarray:
        t = np.empty(_lib.WOST_SAMPLER_TABLE_N, np.float32)
        _lib.check(_lib.lib.wost_sampler_table(self._h, _lib.fptr(t), t.shape[0]), "sampler_table")
        return t

    # ---- the hot path ----------------------------------------------------------
    def solve_blocks(self, solvePoints, nWalks: int, block_begin: int, block_end: int, maxSteps: int = 1000,
                     eps: float = 1e-4, seed: int = 0, walk_values: np.ndarray | None = None,
                     walk_steps: np.ndarray | None = None):
        """Run walk blocks [block_begin, block_end) (WOST_BLOCK_WALKS walks of one point
        each) and return their (sum, sum^2, steps) rows in block order. This is
        the unit of multi-GPU sharding (dcrmontecarlo_amd.distributed)."""
        p = _points_np(solvePoints)
        nb = int(block_end) - int(block_begin)
        bs = np.zeros((max(nb, 0), 3), np.float64)
        _lib.check(_lib.lib.wost_solve(self._h, _lib.fptr(p), p.shape[0], int(nWalks), int(block_begin),
                                       int(block_end), int(maxSteps), float(eps), int(seed) & (2**64 - 1),
                                       _lib.dptr(bs), None, _lib.fptr(walk_values), _lib.u32ptr(walk_steps)),
                   "WostSolver_2D.solve")
        self.last_timing = self.timing()
        return bs

    def solve_range(self, solvePoints, nWalks: int, walk_begin: int, walk_end: int, maxSteps: int = 1000,
                    eps: float = 1e-4, seed: int = 0):
        """Walks [walk_begin, walk_end) of every point (block-aligned ends; wost_solve_range):
        the (sum, sum^2, steps) rows of its blocks, [N, blocks, 3], each equal to the
        corresponding block of the full solve. The unit of dcrmontecarlo_amd.comm's sharding."""
        p = _points_np(solvePoints)
        n = p.shape[0]
        nbr = -(-(int(walk_end) - int(walk_begin)) // _lib.WOST_BLOCK_WALKS)
        ns = ctypes.c_int32(1)
        _lib.check(_lib.lib.wost_num_sources(self._h, ctypes.byref(ns)), "wost_num_sources")
        bs = np.zeros((n, max(nbr, 0), 2 * ns.value + 1), np.float64)
        _lib.check(_lib.lib.wost_solve_range(self._h, _lib.fptr(p), n, int(nWalks), int(walk_begin), int(walk_end),
                                             int(maxSteps), float(eps), int(seed) & (2**64 - 1), _lib.dptr(bs), None,
                                             None, None), "WostSolver_2D.solve_range")
        self.last_timing = self.timing()
        return bs

    def set_jit(self, enable: bool):
        """Use the field-specialised (hiprtc) walk kernel (default) or the precompiled
        kernel that interprets the fields. Both give identical results."""
        _lib.check(_lib.lib.wost_set_jit(self._h, 1 if enable else 0), "wost_set_jit")

    def set_trig(self, mode: str = "auto"):
        """The walk direction's cos/sin (wost_set_trig): "exact" correctly rounded (the
        reference's torch values but for their own ulp errors), "fast" the hardware
        sin/cos, "auto" (default) exact when the Neumann polyline has >= 3 segments."""
        if mode not in _lib.WOST_TRIG:
            raise ValueError(f"trig mode must be one of {sorted(_lib.WOST_TRIG)}, got {mode!r}")
        _lib.check(_lib.lib.wost_set_trig(self._h, _lib.WOST_TRIG[mode]), "wost_set_trig")

    def set_fixed_step_check(self, enable: bool):
        """compat="fixed" delta tracking refuses (ValueError) a solve whose walks would all
        hit maxSteps (~d^2 sigma_bar / 4 steps from Dirichlet distance d at the median
        query point, wost_set_fixed_step_check); False lets such truncated solves run."""
        _lib.check(_lib.lib.wost_set_fixed_step_check(self._h, 1 if enable else 0), "wost_set_fixed_step_check")

    def set_segment_tree(self, min_segments: int = 64, leaf_segments: int = 0):
        """Route the Neumann closest-silhouette and ray queries through the segment
        tree when the Neumann polyline has >= min_segments segments (< 0: never,
        0: always). Results are bit-identical to the full scans."""
        _lib.check(_lib.lib.wost_set_segment_tree(self._h, int(min_segments), int(leaf_segments)),
                   "wost_set_segment_tree")

    def set_option(self, name: str, value):
        """A kernel or launch option of this handle (include/wost.h wost_set_option: the
        walk pools, LDS staging, work-queue chunks, tree hand-outs ...). None of them
        changes a walk's value or step count; unknown names and bad values raise
        ValueError, study-build-only names NotImplementedError."""
        _lib.check(_lib.lib.wost_set_option(self._h, str(name).encode(), float(value)), f"set_option({name!r})")

    def get_option(self, name: str) -> float:
        v = ctypes.c_double(0.0)
        _lib.check(_lib.lib.wost_get_option(self._h, str(name).encode(), ctypes.byref(v)), f"get_option({name!r})")
        return float(v.value)

    def options_report(self) -> dict:
        """{"build": "product"|"study", "non_default": {name: value}} (wost_options_report)."""
        return _lib.options_report(self._h)

    def num_blocks(self, n_points: int, nWalks: int) -> int:
        return int(_lib.lib.wost_num_blocks(int(n_points), int(nWalks)))

    def timing(self) -> dict:
        t = _lib.WostTiming()
        _lib.check(_lib.lib.wost_last_timing(self._h, ctypes.byref(t)), "wost_last_timing")
        return {k: getattr(t, k) for k in _TIMING_FIELDS}

    def solve(self, solvePoints, nWalks=1000, maxSteps=1000, eps=1e-4, return_history=False, *,
              seed: int = 0, return_stats: bool = False):
        """Estimate u at each point (reference: solvers/WoStSolver.py:319-353).

        Returns ``[N, 1]`` float32 (torch tensor if ``solvePoints`` is one). With
        ``return_history=True`` returns ``(u, history)`` with the reference's
        structure (:335-350): per point a list of walk dicts with ``walk_id``,
        ``path`` (each step's point and Dirichlet / Neumann distances),
        ``contributions`` (each step's source sample and contribution, then the
        boundary term) and ``total_contribution`` (the running point total, :308),
        plus this walk's ``value`` and ``steps``. Points are torch tensors when
        ``solvePoints`` is one, numpy arrays otherwise. With ``return_stats=True``
        a :class:`SolveStats` is appended.
        """
        p = _points_np(solvePoints)
        n = p.shape[0]
        nWalks = int(nWalks)
        if nWalks < 1:
            raise ValueError("nWalks must be >= 1")
        sums = np.zeros((n, 3), np.float64)
        if return_history:
            # the recorder keeps maxSteps + 1 records per walk on the host: refuse sizes the
            # host cannot hold before allocating (WOST_HISTORY_MAX_BYTES, default 8 GiB)
            rec_bytes = n * nWalks * (int(maxSteps) + 1) * _lib.REC_FLOATS * 4
            limit = int(os.environ.get("WOST_HISTORY_MAX_BYTES", str(8 << 30)))
            if rec_bytes > limit:
                raise ValueError(f"return_history needs {rec_bytes / 2**30:.1f} GiB of walk records "
                                 f"({n} points x {nWalks} walks x {int(maxSteps) + 1} records); lower maxSteps, "
                                 f"nWalks or the point count, or raise WOST_HISTORY_MAX_BYTES ({limit} bytes)")
            wv = np.empty(n * nWalks, np.float32)
            ws = np.empty(n * nWalks, np.uint32)
            stride = int(maxSteps) + 1
            rec = np.empty((n * nWalks, stride, _lib.REC_FLOATS), np.float32)
            _lib.check(_lib.lib.wost_solve_history(self._h, _lib.fptr(p), n, nWalks, int(maxSteps), float(eps),
                                                   int(seed) & (2**64 - 1), _lib.dptr(sums), _lib.fptr(wv),
                                                   _lib.u32ptr(ws), _lib.fptr(rec)),
                       "WostSolver_2D.solve")
        else:
            nb = self.num_blocks(n, nWalks)
            _lib.check(_lib.lib.wost_solve(self._h, _lib.addr(p), n, nWalks, 0, nb, int(maxSteps), float(eps),
                                           int(seed) & (2**64 - 1), None, _lib.addr(sums), None, None),
                       "WostSolver_2D.solve")
        self.last_timing = self.timing()
        self.last_point_sums = sums
        u = (sums[:, 0] / nWalks).astype(np.float32).reshape(n, 1)
        out = [_like(u, solvePoints)]
        if return_history:
            out.append(_history(rec, wv, ws, n, nWalks, self.neumannBoundary is not None, self.source is not None,
                                _is_torch(solvePoints)))
        if return_stats:
            t = self.last_timing
            out.append(stats_from_sums(sums, nWalks, t["total_steps"], t["walk_kernel_ms"], t["total_ms"]))
        return out[0] if len(out) == 1 else tuple(out)

    def solve_walks(self, solvePoints, nWalks=1000, maxSteps=1000, eps=1e-4, *, seed: int = 0):
        """Per-walk results without the paths: (values float32 [N, nWalks],
        steps uint32 [N, nWalks]) in walk order (walk j of point i has global id
        i * nWalks + j, as in return_history)."""
        p = _points_np(solvePoints)
        n = p.shape[0]
        nWalks = int(nWalks)
        if nWalks < 1:
            raise ValueError("nWalks must be >= 1")
        wv = np.empty(n * nWalks, np.float32)
        ws = np.empty(n * nWalks, np.uint32)
        nb = self.num_blocks(n, nWalks)
        _lib.check(_lib.lib.wost_solve(self._h, _lib.fptr(p), n, nWalks, 0, nb, int(maxSteps), float(eps),
                                       int(seed) & (2**64 - 1), None, None, _lib.fptr(wv), _lib.u32ptr(ws)),
                   "WostSolver_2D.solve_walks")
        self.last_timing = self.timing()
        return wv.reshape(n, nWalks), ws.reshape(n, nWalks)

    # ---- multi-source batching -------------------------------
    def source_fields(self, sources) -> list:
        """The device fields of a list of sources (fields, numbers or callables; None = 0)."""
        srcs = list(sources)
        if not srcs:
            raise ValueError("sources must hold at least one source field")
        return [self._conv(0.0 if f is None else f, f"sources[{k}]") for k, f in enumerate(srcs)]

    @contextlib.contextmanager
    def sources_installed(self, fields):
        """Score up to WOST_MAX_SOURCES source fields per walk (wost_set_sources) inside
        the block; the solver's own (single) source is restored afterwards."""
        if not 1 <= len(fields) <= _lib.WOST_MAX_SOURCES:
            raise ValueError(f"1..{_lib.WOST_MAX_SOURCES} sources per launch, got {len(fields)}")
        packed = [_lib.make_field(f) for f in fields]
        arr = (ctypes.POINTER(_lib.WostField) * len(fields))(*[ctypes.pointer(wf) for wf, _ in packed])
        _lib.check(_lib.lib.wost_set_sources(self._h, arr, len(fields)), "WostSolver_2D.solve_sources")
        try:
            yield len(fields)
        finally:
            wf, keep = _lib.make_field(self.source)
            _lib.check(_lib.lib.wost_set_field(self._h, _lib.SLOT_SOURCE, ctypes.pointer(wf) if wf else None),
                       "WostSolver_2D.solve_sources")

    def prepare_sources(self, sources, n_points: int):
        """Compile (or fetch from the kernel caches) the kernel that solve_sources of
        ``n_points`` points with these ``sources`` launches, without solving or changing the
        handle (wost_prepare_sources). Thread-safe with other prepare_sources calls, also on
        this solver, but not with its solves: a survey prepares every group's kernel from a
        thread pool first, so that their compiles overlap in the compile helper."""
        fields = self.source_fields(sources)
        for c0 in range(0, len(fields), _lib.WOST_MAX_SOURCES):
            chunk = fields[c0:c0 + _lib.WOST_MAX_SOURCES]
            packed = [_lib.make_field(f) for f in chunk]
            arr = (ctypes.POINTER(_lib.WostField) * len(chunk))(*[ctypes.pointer(wf) for wf, _ in packed])
            _lib.check(_lib.lib.wost_prepare_sources(self._h, arr, len(chunk), int(n_points)),
                       "WostSolver_2D.prepare_sources")

    def _solve_sources(self, solvePoints, sources, nWalks, maxSteps, eps, seed, want_walks):
        p = _points_np(solvePoints)
        n = p.shape[0]
        nWalks = int(nWalks)
        if nWalks < 1:
            raise ValueError("nWalks must be >= 1")
        fields = self.source_fields(sources)
        nb = self.num_blocks(n, nWalks)
        sums, vals, steps = [], [], None
        for c0 in range(0, len(fields), _lib.WOST_MAX_SOURCES):
            with self.sources_installed(fields[c0:c0 + _lib.WOST_MAX_SOURCES]) as S:
                s = np.zeros((n, 2 * S + 1), np.float64)
                wv = np.empty(n * nWalks * S, np.float32) if want_walks else None
                ws = np.empty(n * nWalks, np.uint32) if want_walks else None
                _lib.check(_lib.lib.wost_solve_multi(self._h, _lib.fptr(p), n, nWalks, 0, nb, int(maxSteps),
                                                     float(eps), int(seed) & (2**64 - 1), None, _lib.dptr(s),
                                                     _lib.fptr(wv), _lib.u32ptr(ws)), "WostSolver_2D.solve_sources")
                self.last_timing = self.timing()
            sums.append(s)
            if want_walks:
                vals.append(wv.reshape(n, nWalks, S).transpose(2, 0, 1))
                steps = ws.reshape(n, nWalks)
        return sums, vals, steps

    def solve_sources(self, solvePoints, sources, nWalks=1000, maxSteps=1000, eps=1e-4, *, seed: int = 0,
                      return_stats: bool = False):
        """Multi-source batching (beyond the reference, which solves one source per
        solve): u[k] is the solve of this problem with source ``sources[k]``
        (fields, numbers or callables), all scored by the same walks. The walks
        do not depend on f (solvers/WoStSolver.py:242-258), so each u[k] is bit for
        bit ``setSourceTerm(sources[k]); solve(...)`` with the same seed, at about
        the cost of one solve (16 sources per launch; more are batched in groups).
        Returns float32 [S, N]; with ``return_stats`` also a SolveStats whose mean
        and stderr are [S, N]. The solver's own source is restored afterwards."""
        sums, _, _ = self._solve_sources(solvePoints, sources, nWalks, maxSteps, eps, seed, False)
        stats = [st for s in sums for st in _stats_of_multi(s, int(nWalks))]
        u = np.stack([st.mean.astype(np.float32) for st in stats])
        if not return_stats:
            return u
        t = self.last_timing
        return u, SolveStats(mean=np.stack([st.mean for st in stats]), stderr=np.stack([st.stderr for st in stats]),
                             mean_steps=stats[0].mean_steps, walks=stats[0].walks, total_steps=stats[0].total_steps,
                             kernel_ms=t["walk_kernel_ms"], total_ms=t["total_ms"])

    def solve_sources_walks(self, solvePoints, sources, nWalks=1000, maxSteps=1000, eps=1e-4, *, seed: int = 0):
        """Per-walk values of every source, float32 [S, N, nWalks], and the walks'
        step counts, uint32 [N, nWalks] (shared by all sources)."""
        _, vals, steps = self._solve_sources(solvePoints, sources, nWalks, maxSteps, eps, seed, True)
        return np.concatenate(vals, axis=0), steps


def _stats_of_multi(sums: np.ndarray, n_walks: int):
    """SolveStats of each source from [N, 2S+1] wost_solve_multi rows."""
    S = (sums.shape[1] - 1) // 2
    return [stats_from_sums(np.stack([sums[:, 2 * k], sums[:, 2 * k + 1], sums[:, -1]], axis=1), n_walks)
            for k in range(S)]


def _history(rec, wv, ws, n, nWalks, has_neumann, has_source, as_torch):
    """The reference's history_dict (solvers/WoStSolver.py:180-309) from the recorder's
    records (include/wost.h, wost_solve_history)."""
    if as_torch:
        import torch

        pt = lambda x, y: torch.tensor([float(x), float(y)], dtype=torch.float32)
    else:
        pt = lambda x, y: np.array([x, y], np.float32)
    hist = {}
    for i in range(n):
        walks = []
        running = 0.0
        for j in range(nWalks):
            g = i * nWalks + j
            k = int(ws[g])
            r = rec[g]
            path = [{"point": pt(r[s, 0], r[s, 1]), "dirichlet_distance": float(r[s, 2]),
                     "neumann_distance": float(r[s, 3]) if has_neumann else None} for s in range(k)]
            contrib = []
            if has_source:
                contrib = [{"step": s, "type": "source", "point": pt(r[s, 4], r[s, 5]), "contribution": float(r[s, 6])}
                           for s in range(k)]
            contrib.append({"step": k, "type": "boundary", "point": pt(r[k, 0], r[k, 1]),
                            "contribution": float(r[k, 6])})
            running += float(wv[g])
            walks.append({"walk_id": j, "path": path, "contributions": contrib, "total_contribution": running,
                          "value": float(wv[g]), "steps": k})
        hist[i] = walks
    return hist


def _np(a):
    if _is_torch(a):
        return a.detach().cpu().numpy()
    return np.asarray(a)


def _like(u: np.ndarray, ref):
    if _is_torch(ref):
        import torch

        return torch.from_numpy(u)
    return u
