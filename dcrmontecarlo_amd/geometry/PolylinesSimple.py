"""Brute-force polyline queries on the GPU (reference: geometry/PolylinesSimple.py:199-307).

``PolyLinesSimple`` keeps the reference's interface -- ``distance``,
``isSilhouette``, ``silhouetteDistance``, ``rayIntersection``,
``intersectPolylines``, ``crossProduct2D``, ``funcToPolyline`` -- and answers
every query with libwost's gfx950 kernels (``wost_geometry_query``), including
the reference's conventions: the ray "time" is the segment parameter (quirk
Q1), the end vertices are never silhouettes (Q6), and ``funcToPolyline``
starts at x = 0 whatever ``x_min`` says (Q11).

Queries accept one point ``[2]`` (like the reference) or a batch ``[M,2]``
(one kernel launch for all of them). numpy in -> numpy out; torch in -> torch out.
"""
from __future__ import annotations

import numpy as np

from .. import _lib
from .Polylines import PolyLines


def _is_torch(a) -> bool:
    return type(a).__module__.startswith("torch")


def _np32(a) -> np.ndarray:
    if _is_torch(a):
        a = a.detach().cpu().numpy()
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32))


def _out(a, like):
    if _is_torch(like):
        import torch

        return torch.from_numpy(np.ascontiguousarray(a))
    return a


class PolyLinesSimple(PolyLines):
    """Polyline with brute-force (all-segment) queries evaluated on a HIP device."""

    device = 0

    def __init__(self, points):
        super().__init__(points)
        xy = _np32(points)
        if xy.ndim != 2 or xy.shape[1] != 2:
            raise ValueError(f"points must have shape [N, 2], got {xy.shape}")
        self._xy = xy

    # ------------------------------------------------------------------
    def _query(self, op: str, point, direction=None, r=None, tree: bool = False):
        p = _np32(point)
        single = p.ndim == 1
        p = p.reshape(-1, 2)
        n = p.shape[0]
        nv = self._xy.shape[0]
        d = None
        rr = None
        if direction is not None:
            d = np.ascontiguousarray(np.broadcast_to(_np32(direction).reshape(-1, 2), (n, 2)))
        if r is not None:
            rr = np.ascontiguousarray(np.broadcast_to(np.asarray(_np32(r)).reshape(-1), (n,)))
        code = _lib.GEOM_OPS[op] | (_lib.WOST_GEOM_TREE if tree else 0)
        out_f = out_m = None
        if op in ("distance", "silhouetteDistance"):
            out_f = np.empty(n, np.float32)
        elif op == "rayIntersection":
            out_f = np.empty((n, max(nv - 1, 0)), np.float32)
        elif op == "intersectPolylines":
            out_f = np.empty((n, 5), np.float32)
        else:
            out_m = np.empty((n, max(nv - 2, 0)), np.uint8)
        poly, keep = _lib.make_polyline(self._xy)
        rc = _lib.lib.wost_geometry_query(
            int(self.device), code, poly, _lib.fptr(p), _lib.fptr(d), _lib.fptr(rr), n,
            _lib.fptr(out_f), out_m.ctypes.data_as(_lib.POINTER(_lib.c_uint8)) if out_m is not None else None)
        _lib.check(rc, f"PolyLinesSimple.{op}")
        return (out_f if out_m is None else out_m.astype(bool)), single

    # ---- reference API (PolylinesSimple.py:214-307) -------------------
    def distance(self, point):
        """Distance to the polyline (distance_to_polyline_jit, :25-49)."""
        v, single = self._query("distance", point)
        if single:
            return _scalar(v[0]) if _is_torch(point) else np.float32(v[0])
        return _out(v, point)

    def isSilhouette(self, point):
        """Silhouette mask of the interior vertices (is_silhouette_jit, :51-81)."""
        m, single = self._query("isSilhouette", point)
        return _out(m[0] if single else m, point)

    def silhouetteDistance(self, point, *, tree: bool = False):
        """Distance to the nearest silhouette vertex, inf if none (:83-102). ``tree``:
        answered by the walk kernels' segment tree (same bits as the scan)."""
        v, single = self._query("silhouetteDistance", point, tree=tree)
        if single:
            return _scalar(v[0]) if _is_torch(point) else np.float32(v[0])
        return _out(v, point)

    def rayIntersection(self, point, direction):
        """Per-segment hit "times" = segment parameters, inf if missed (:104-132)."""
        t, single = self._query("rayIntersection", point, direction)
        return _out(t[0] if single else t, point)

    def intersectPolylines(self, point, direction, r, *, tree: bool = False):
        """(hit point or point + r*d, normal, found) (intersect_polylines_jit, :134-197).
        ``tree``: answered by the walk kernels' segment tree (same bits as the scan)."""
        o, single = self._query("intersectPolylines", point, direction, r, tree=tree)
        if single:
            return _out(o[0, 0:2].copy(), point), _out(o[0, 2:4].copy(), point), bool(o[0, 4] != 0)
        return _out(o[:, 0:2].copy(), point), _out(o[:, 2:4].copy(), point), _out(o[:, 4] != 0, point)

    def crossProduct2D(self, a, b):
        """a_x b_y - a_y b_x with (N,2)/(2,) broadcasting (cross_product_2d_jit, :13-23)."""
        A, B = _np32(a), _np32(b)
        A2, B2 = np.atleast_2d(A), np.atleast_2d(B)
        A2, B2 = np.broadcast_arrays(A2, B2)
        r = A2[:, 0] * B2[:, 1] - A2[:, 1] * B2[:, 0]
        return _out(r.astype(np.float32), a)

    @staticmethod
    def funcToPolyline(func, x_min: float, x_max: float, resolution: float) -> "PolyLinesSimple":
        """Heightmap -> polyline. Like the reference (:226-240) the samples start at
        x = 0 and x_min is ignored (quirk Q11). ``func`` receives what the reference
        gives it, a float32 torch tensor torch.arange(0, x_max, resolution), when torch
        is importable (the polyline's points are then a torch tensor, as there), and
        the same values as a float32 numpy array otherwise."""
        try:
            import torch
        except ImportError:
            torch = None
        if torch is not None:
            x = torch.arange(0, x_max, resolution)
            y = func(x)
            if not isinstance(y, torch.Tensor):
                y = torch.as_tensor(np.asarray(y, dtype=np.float32))
            return PolyLinesSimple(torch.stack((x, y.to(x.dtype)), dim=-1))
        # ATen's CPU arange: n = ceil((end - start) / step), x_i = start + i * step in double
        n = int(np.ceil((float(x_max) - 0.0) / float(resolution)))
        x = (np.arange(max(n, 0), dtype=np.float64) * float(resolution)).astype(np.float32)
        y = np.asarray(func(x), dtype=np.float32)
        return PolyLinesSimple(np.stack((x, y), axis=-1))


def _scalar(v):
    import torch

    return torch.tensor(float(v), dtype=torch.float32)
