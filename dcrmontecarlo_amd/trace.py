"""Reference-style coefficient callables -> device fields.

The reference takes the Dirichlet data g, the source f, the absorption sigma
and the diffusion alpha as Python callables ``fn(point)`` of one float32
point tensor (solvers/WoStSolver.py:22, :141-157) and calls them inside the
walk loop. A GPU kernel cannot call Python, so a callable becomes a
:class:`~dcrmontecarlo_amd.fields.Field` in one of two ways:

1. **Tracing (exact).** ``fn`` is run on a symbolic point. Arithmetic,
   ``**``, indexing, the torch functions the reference's scenarios use
   (``exp``, ``sin``, ``cos``, ``sigmoid``, ``sqrt``, ``norm``, ``sum``,
   ``abs``, ``where``; ``torch.tensor`` re-wrapping, ``float()``) and
   ``if``/``and``/``or`` on comparisons (every branch is explored; the
   conditions become box / disk indicators) build the closed-form field
   directly. The reference's own scenario callables all trace
   (tests/test_trace.py), e.g. ``torch_smooth_circle`` (utils.py:123-129)
   becomes a radial sigmoid factor.
2. **Tabulation (approximate).** Anything else (``math.*`` on the point,
   data-dependent loops, unsupported functions) is evaluated on a regular
   grid over the domain and interpolated on the device (Catmull-Rom bicubic,
   include/wost.h ``WOST_FK_GRID``). A warning says so.

Every traced field is checked against the callable itself at sample points
before it is used; a mismatch falls back to tabulation. Whether alpha is
differentiable -- the reference's sigma' falls back to sigma/alpha when
autograd raises (solvers/WoStSolver.py:123-127, quirk Q9) -- is decided the
way the reference decides it: by running autograd on the callable.
"""
from __future__ import annotations

import math
import numbers
import struct
import warnings
from dataclasses import dataclass

import numpy as np

from . import fields as F

__all__ = ["Untraceable", "trace", "tabulate", "field_from_callable", "Conversion", "alpha_is_detached"]


class Untraceable(Exception):
    """The callable uses something the tracer cannot express as a field."""


# ---------------------------------------------------------------------------
# symbolic values
# ---------------------------------------------------------------------------
class _Radial:
    """k * (sqrt((x-cx)^2 + (y-cy)^2) - R): a distance to a point, from norm()/sqrt()."""

    __slots__ = ("k", "cx", "cy", "R")

    def __init__(self, k, cx, cy, R):
        self.k, self.cx, self.cy, self.R = float(k), float(cx), float(cy), float(R)


def _is_const(v) -> bool:
    return isinstance(v, float) or (isinstance(v, F.Field) and v.is_constant())


def _const_value(v) -> float:
    if isinstance(v, float):
        return v
    return float(sum(t.coef for t in v.terms))


def _fold(v):
    """Constant fields -> floats (keeps the arithmetic of constants in double)."""
    if isinstance(v, F.Field) and v.is_constant():
        return _const_value(v)
    return v


def _add(a, b):
    if isinstance(a, _Radial) or isinstance(b, _Radial):
        r, c = (a, b) if isinstance(a, _Radial) else (b, a)
        if isinstance(c, _Radial) or not _is_const(c):
            raise Untraceable("sum of a distance and a non-constant term")
        return _Radial(r.k, r.cx, r.cy, r.R - _const_value(c) / r.k) if r.k != 0 else _const_value(c)
    if isinstance(a, float) and isinstance(b, float):
        return a + b
    return _fold(F.as_field(a) + F.as_field(b))


def _mul(a, b):
    if isinstance(a, _Radial) or isinstance(b, _Radial):
        r, c = (a, b) if isinstance(a, _Radial) else (b, a)
        if isinstance(c, _Radial):
            if (r.R == 0 and c.R == 0 and (r.cx, r.cy) == (c.cx, c.cy)):
                return _fold(r.k * c.k * ((F.X - r.cx) ** 2 + (F.Y - r.cy) ** 2))
            raise Untraceable("product of distances")
        if not _is_const(c):
            raise Untraceable("product of a distance and a non-constant term")
        k = _const_value(c)
        return _Radial(r.k * k, r.cx, r.cy, r.R) if k != 0 else 0.0
    if isinstance(a, float) and isinstance(b, float):
        return a * b
    return _fold(F.as_field(a) * F.as_field(b))


def _neg(a):
    return _mul(a, -1.0)


def _div(a, b):
    if not _is_const(b):
        raise Untraceable("division by a non-constant field")
    return _mul(a, 1.0 / _const_value(b))


def _pow(a, e):
    if not _is_const(e):
        raise Untraceable("non-constant exponent")
    e = _const_value(e)
    if _is_const(a):
        return _const_value(a) ** e
    if e == 0.5:
        return _sqrt(a)
    if e != int(e) or e < 0:
        raise Untraceable(f"power {e} of a field")
    e = int(e)
    if isinstance(a, _Radial):
        if e == 2 and a.R == 0:
            return _mul(a, a)
        if e == 1:
            return a
        raise Untraceable("power of a shifted distance")
    return _fold(F.as_field(a) ** e)


def _sqrt(a):
    if _is_const(a):
        return math.sqrt(_const_value(a))
    if isinstance(a, _Radial):
        raise Untraceable("sqrt of a distance")
    poly = a.polynomial()
    if poly is None or any(i + j > 2 for (i, j) in poly) or poly.get((1, 1), 0.0) != 0.0:
        raise Untraceable("sqrt of a field that is not a scaled squared distance")
    A, B = poly.get((2, 0), 0.0), poly.get((0, 2), 0.0)
    if not (A > 0 and abs(A - B) <= 1e-12 * A):
        raise Untraceable("sqrt of a field that is not a scaled squared distance")
    cx, cy = -poly.get((1, 0), 0.0) / (2 * A), -poly.get((0, 1), 0.0) / (2 * A)
    rem = poly.get((0, 0), 0.0) - A * (cx * cx + cy * cy)
    if abs(rem) > 1e-9 * (abs(poly.get((0, 0), 0.0)) + A * (cx * cx + cy * cy) + 1.0):
        raise Untraceable("sqrt of a squared distance plus a constant")
    return _Radial(math.sqrt(A), cx, cy, 0.0)


def _unary(name, a):
    if _is_const(a):
        c = _const_value(a)
        fn = {"exp": math.exp, "sin": math.sin, "cos": math.cos, "sqrt": math.sqrt, "abs": abs,
              "sigmoid": lambda z: 1.0 / (1.0 + math.exp(-z)) if z > -700 else 0.0}[name]
        return fn(c)
    if name == "sqrt":
        return _sqrt(a)
    if name == "abs":
        return _Abs(a)
    if isinstance(a, _Radial):
        if name == "sigmoid" and a.k != 0:
            return F.sigmoid_radial(a.k, (a.cx, a.cy), a.R)
        raise Untraceable(f"{name} of a distance")
    try:
        return _fold({"exp": F.exp, "sin": F.sin, "cos": F.cos, "sigmoid": F.sigmoid}[name](a))
    except (ValueError, TypeError) as e:
        raise Untraceable(f"{name}: {e}") from None


class _Abs:
    """|a X + b| or |a Y + b|: only usable in comparisons (a box condition)."""

    __slots__ = ("inner",)

    def __init__(self, inner):
        self.inner = inner


# ---------------------------------------------------------------------------
# conditions -> indicator fields
# ---------------------------------------------------------------------------
_INF = float("inf")


def _f32(v: float) -> float:
    return float(np.float32(v))


def _below(v: float) -> float:
    """Largest float32 strictly below the float32 value of v."""
    return float(np.nextafter(np.float32(v), np.float32(-np.inf)))


def _above(v: float) -> float:
    return float(np.nextafter(np.float32(v), np.float32(np.inf)))


class _Cond:
    """A comparison of the traced point against a constant. true()/false() give
    the indicator fields of the two outcomes (float32-exact for half-planes)."""

    def __init__(self, true_field: F.Field, false_field: F.Field):
        self._t, self._f = true_field, false_field

    @classmethod
    def __torch_function__(cls, func, types, args=(), kwargs=None):     # torch.where(cond, a, b)
        return _Sym.__torch_function__(func, types, args, kwargs)

    def ind(self, outcome: bool) -> F.Field:
        return self._t if outcome else self._f

    def __bool__(self):
        return _explorer().decide(self)

    def __invert__(self):
        return _Cond(self._f, self._t)


def _half_plane(var: int, op: str, c: float) -> _Cond:
    """x_var op c with op in < <= > >=, as closed boxes in float32."""
    def box(lo, hi):
        b = (lo, hi, -_INF, _INF) if var == 0 else (-_INF, _INF, lo, hi)
        return F.indicator_box(*b)
    c = _f32(c)
    if op == "<":
        return _Cond(box(-_INF, _below(c)), box(c, _INF))
    if op == "<=":
        return _Cond(box(-_INF, c), box(_above(c), _INF))
    if op == ">":
        return _Cond(box(_above(c), _INF), box(-_INF, c))
    return _Cond(box(c, _INF), box(-_INF, _below(c)))


_FLIP = {"<": ">", "<=": ">=", ">": "<", ">=": "<="}


def _compare(a, op: str, b) -> _Cond:
    """a op b for traced scalars a, b."""
    if isinstance(a, _Abs) or isinstance(b, _Abs):
        if isinstance(b, _Abs):
            a, b, op = b, a, _FLIP[op]
        if not _is_const(b):
            raise Untraceable("comparison of |.| with a non-constant")
        inner = a.inner
        poly = inner.polynomial() if isinstance(inner, F.Field) else None
        if poly is None or any(i + j > 1 for (i, j) in poly) or ((1, 0) in poly and (0, 1) in poly):
            raise Untraceable("|.| of a field that is not linear in one coordinate")
        var = 0 if (1, 0) in poly else 1
        s = poly[(1, 0) if var == 0 else (0, 1)]
        c0 = poly.get((0, 0), 0.0)
        m = _const_value(b) / abs(s)
        lo, hi = -c0 / s - m, -c0 / s + m            # |s v + c0| <= b  <=>  lo <= v <= hi
        strict = op in ("<", ">")
        if op in ("<", "<="):
            inside = F.indicator_box(*((_above(lo), _below(hi)) if strict else (_f32(lo), _f32(hi))),
                                     -_INF, _INF) if var == 0 else \
                F.indicator_box(-_INF, _INF, *((_above(lo), _below(hi)) if strict else (_f32(lo), _f32(hi))))
            return _Cond(inside, 1.0 - inside)
        inside = F.indicator_box(*((_f32(lo), _f32(hi)) if strict else (_above(lo), _below(hi))),
                                 -_INF, _INF) if var == 0 else \
            F.indicator_box(-_INF, _INF, *((_f32(lo), _f32(hi)) if strict else (_above(lo), _below(hi))))
        return _Cond(1.0 - inside, inside)
    if _is_const(a) and _is_const(b):
        r = {"<": _const_value(a) < _const_value(b), "<=": _const_value(a) <= _const_value(b),
             ">": _const_value(a) > _const_value(b), ">=": _const_value(a) >= _const_value(b)}[op]
        one, zero = F.const(1.0), F.const(0.0)
        return _Cond(one if r else zero, zero if r else one)
    if _is_const(a):
        a, b, op = b, a, _FLIP[op]
    if not _is_const(b):
        return _compare(_add(a, _neg(b)), op, 0.0)
    c = _const_value(b)
    if isinstance(a, _Radial):                       # k (r - R) op c  <=>  r op' R + c/k
        rr = a.R + c / a.k
        if a.k < 0:
            op = _FLIP[op]
        return _disk_cond(a.cx, a.cy, rr * rr if rr > 0 else -1.0, op, sq_scale=1.0)
    poly = a.polynomial()
    if poly is None:
        raise Untraceable("comparison of a non-polynomial field")
    if all(i + j <= 1 for (i, j) in poly) and not ((1, 0) in poly and (0, 1) in poly):
        if (1, 0) not in poly and (0, 1) not in poly:
            return _compare(_const_value(a), op, c)
        var = 0 if (1, 0) in poly else 1
        s = poly[(1, 0) if var == 0 else (0, 1)]
        t = (c - poly.get((0, 0), 0.0)) / s
        return _half_plane(var, op if s > 0 else _FLIP[op], t)
    A, B = poly.get((2, 0), 0.0), poly.get((0, 2), 0.0)
    if (all(i + j <= 2 for (i, j) in poly) and poly.get((1, 1), 0.0) == 0.0 and A != 0.0
            and abs(A - B) <= 1e-12 * abs(A)):
        cx, cy = -poly.get((1, 0), 0.0) / (2 * A), -poly.get((0, 1), 0.0) / (2 * A)
        rem = poly.get((0, 0), 0.0) - A * (cx * cx + cy * cy)
        r2 = (c - rem) / A                            # A q + rem op c  <=>  q op' (c - rem)/A
        return _disk_cond(cx, cy, r2, op if A > 0 else _FLIP[op], sq_scale=1.0)
    raise Untraceable("comparison that is neither a half-plane nor a disk")


def _disk_cond(cx, cy, r2, op, sq_scale=1.0) -> _Cond:
    """q = (x-cx)^2 + (y-cy)^2 (float32 as the device computes it) op r2."""
    if r2 < 0:
        inside = F.const(0.0)
    else:
        inside = None
    r2f = _f32(r2)
    if op in ("<", "<="):
        lim = r2f if op == "<=" else _below(r2f)
        ind = inside if inside is not None else _disk(cx, cy, lim)
        return _Cond(ind, 1.0 - ind)
    lim = r2f if op == ">" else _below(r2f)           # q > r2  <=>  not (q <= r2)
    ind = inside if inside is not None else _disk(cx, cy, lim)
    return _Cond(1.0 - ind, ind)


def _disk(cx, cy, r2f) -> F.Field:
    return F.Field([F._Term(1.0, (0, 0), [F._Factor(F.FK_IND_DISK, (cx, cy, r2f))])])


# ---------------------------------------------------------------------------
# the symbolic tensor
# ---------------------------------------------------------------------------
def _scalar(o):
    """Operand -> float | Field | _Radial | _Abs | tuple (vector)."""
    if isinstance(o, _Sym):
        return o.v
    if isinstance(o, bool):
        return float(o)
    if isinstance(o, numbers.Real):
        return float(o)
    if isinstance(o, np.ndarray) or isinstance(o, np.generic):
        a = np.asarray(o, dtype=np.float64)
        return float(a) if a.ndim == 0 else tuple(float(v) for v in a.ravel()) if a.ndim == 1 else _bad(o)
    if type(o).__module__.startswith("torch"):
        if o.dim() == 0:
            return float(o.item())
        if o.dim() == 1:
            return tuple(float(v) for v in o.detach().double().tolist())
    if isinstance(o, (list, tuple)):
        return tuple(_scalar(v) for v in o)
    return _bad(o)


def _bad(o):
    raise Untraceable(f"operand of type {type(o).__name__}")


def _lift(fn, a, b=None, nargs=1):
    """Elementwise application with scalar/vector broadcasting."""
    if nargs == 1:
        if isinstance(a, tuple):
            return tuple(fn(v) for v in a)
        return fn(a)
    if isinstance(a, tuple) and isinstance(b, tuple):
        if len(a) != len(b):
            raise Untraceable("vector length mismatch")
        return tuple(fn(x, y) for x, y in zip(a, b))
    if isinstance(a, tuple):
        return tuple(fn(x, b) for x in a)
    if isinstance(b, tuple):
        return tuple(fn(a, y) for y in b)
    return fn(a, b)


def _check_num(v):
    if isinstance(v, _Abs):
        raise Untraceable("|.| used outside a comparison")
    return v


def _sum(v):
    if not isinstance(v, tuple):
        return v
    acc = 0.0
    for e in v:
        acc = _add(acc, _check_num(e))
    return acc


def _norm(v):
    if not isinstance(v, tuple):
        return _unary("abs", v) if _is_const(v) else _sqrt(_mul(v, v))
    return _sqrt(_sum(tuple(_mul(e, e) for e in v)))


_BINOPS = {
    "add": _add, "__add__": _add, "__radd__": lambda a, b: _add(b, a),
    "sub": lambda a, b: _add(a, _neg(b)), "__sub__": lambda a, b: _add(a, _neg(b)),
    "__rsub__": lambda a, b: _add(b, _neg(a)), "rsub": lambda a, b: _add(b, _neg(a)),
    "mul": _mul, "__mul__": _mul, "__rmul__": lambda a, b: _mul(b, a), "multiply": _mul,
    "div": _div, "true_divide": _div, "__truediv__": _div, "__rtruediv__": lambda a, b: _div(b, a),
    "__div__": _div, "divide": _div,
    "pow": _pow, "__pow__": _pow, "__rpow__": lambda a, b: _pow(b, a), "float_power": _pow,
}
_UNOPS = {"exp", "sin", "cos", "sigmoid", "sqrt", "abs", "absolute"}
_CMPOPS = {"lt": "<", "__lt__": "<", "less": "<", "le": "<=", "__le__": "<=", "less_equal": "<=",
           "gt": ">", "__gt__": ">", "greater": ">", "ge": ">=", "__ge__": ">=", "greater_equal": ">="}
_PASSTHRU = {"clone", "detach", "contiguous", "float", "double", "to", "squeeze", "flatten", "reshape", "view",
             "requires_grad_", "__getitem__", "item", "__float__", "cpu"}


class _Sym:
    """A traced value: a scalar (float / Field / distance) or a vector of them."""

    __slots__ = ("v",)

    def __init__(self, v):
        self.v = v

    @classmethod
    def __torch_function__(cls, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        name = getattr(func, "__name__", str(func))
        if name in _BINOPS:
            a, b = _scalar(args[0]), _scalar(args[1])
            return _wrap(_lift(lambda x, y: _BINOPS[name](_check_num(x), _check_num(y)), a, b, nargs=2))
        if name in ("neg", "__neg__", "negative"):
            return _wrap(_lift(lambda x: _neg(_check_num(x)), _scalar(args[0])))
        if name in _UNOPS:
            op = "abs" if name == "absolute" else name
            return _wrap(_lift(lambda x: _unary(op, _check_num(x) if op != "abs" else x), _scalar(args[0])))
        if name in _CMPOPS:
            return _cmp(_scalar(args[0]), _CMPOPS[name], _scalar(args[1]))
        if name in ("norm", "linalg_norm", "vector_norm"):
            p = kwargs.get("p", args[1] if len(args) > 1 else None)
            if p not in (None, "fro", 2, 2.0) or kwargs.get("dim") is not None:
                raise Untraceable(f"norm with p={p}")
            return _wrap(_norm(_scalar(args[0])))
        if name == "sum":
            if kwargs.get("dim") is not None or len(args) > 1:
                raise Untraceable("sum over a dimension")
            return _wrap(_sum(_scalar(args[0])))
        if name in ("square",):
            return _wrap(_lift(lambda x: _mul(x, x), _scalar(args[0])))
        if name == "dot":
            a, b = _scalar(args[0]), _scalar(args[1])
            return _wrap(_sum(_lift(_mul, a, b, nargs=2)))
        if name == "where":
            c, a, b = args[0], _scalar(args[1]), _scalar(args[2])
            if not isinstance(c, _Cond):
                raise Untraceable("where() on a non-condition")
            return _wrap(_lift(lambda x, y: _add(_mul(c.ind(True), x), _mul(c.ind(False), y)), a, b, nargs=2))
        if name == "stack" or name == "cat":
            seq = args[0]
            return _wrap(tuple(_scalar(e) for e in seq))
        if name in _PASSTHRU:
            if name == "__getitem__":
                return args[0][args[1]]
            if name in ("item", "__float__"):
                return args[0].__float__()
            return args[0]
        raise Untraceable(f"torch function {name}")

    # Python operators
    def __add__(self, o): return _wrap(_lift(lambda x, y: _add(_check_num(x), _check_num(y)), self.v, _scalar(o), nargs=2))
    def __radd__(self, o): return _wrap(_lift(lambda x, y: _add(_check_num(y), _check_num(x)), self.v, _scalar(o), nargs=2))
    def __sub__(self, o): return _wrap(_lift(lambda x, y: _add(_check_num(x), _neg(_check_num(y))), self.v, _scalar(o), nargs=2))
    def __rsub__(self, o): return _wrap(_lift(lambda x, y: _add(_check_num(y), _neg(_check_num(x))), self.v, _scalar(o), nargs=2))
    def __mul__(self, o): return _wrap(_lift(lambda x, y: _mul(_check_num(x), _check_num(y)), self.v, _scalar(o), nargs=2))
    def __rmul__(self, o): return _wrap(_lift(lambda x, y: _mul(_check_num(y), _check_num(x)), self.v, _scalar(o), nargs=2))
    def __truediv__(self, o): return _wrap(_lift(lambda x, y: _div(_check_num(x), _check_num(y)), self.v, _scalar(o), nargs=2))
    def __rtruediv__(self, o): return _wrap(_lift(lambda x, y: _div(_check_num(y), _check_num(x)), self.v, _scalar(o), nargs=2))
    def __pow__(self, o): return _wrap(_lift(lambda x, y: _pow(_check_num(x), _check_num(y)), self.v, _scalar(o), nargs=2))
    def __rpow__(self, o): return _wrap(_lift(lambda x, y: _pow(_check_num(y), _check_num(x)), self.v, _scalar(o), nargs=2))
    def __neg__(self): return _wrap(_lift(lambda x: _neg(_check_num(x)), self.v))
    def __pos__(self): return self
    def __abs__(self): return _wrap(_lift(lambda x: _unary("abs", x), self.v))
    def __lt__(self, o): return _cmp(self.v, "<", _scalar(o))
    def __le__(self, o): return _cmp(self.v, "<=", _scalar(o))
    def __gt__(self, o): return _cmp(self.v, ">", _scalar(o))
    def __ge__(self, o): return _cmp(self.v, ">=", _scalar(o))

    def __getitem__(self, i):
        if not isinstance(self.v, tuple):
            if i in (0, -1, Ellipsis) or i == ():
                return self
            raise Untraceable("indexing a scalar")
        if isinstance(i, tuple) and len(i) == 1:
            i = i[0]
        r = self.v[i]
        return _wrap(r)

    def __len__(self):
        if isinstance(self.v, tuple):
            return len(self.v)
        raise TypeError("len() of a scalar")

    def __iter__(self):
        if isinstance(self.v, tuple):
            return iter([_wrap(e) for e in self.v])
        raise TypeError("iteration over a scalar")

    def __bool__(self):
        raise Untraceable("truth value of a field (use a comparison)")

    def __float__(self):
        return _explorer().float_sentinel(self)

    def __int__(self):
        raise Untraceable("int() of a field")

    # tensor-style methods
    def exp(self): return _wrap(_lift(lambda x: _unary("exp", _check_num(x)), self.v))
    def sin(self): return _wrap(_lift(lambda x: _unary("sin", _check_num(x)), self.v))
    def cos(self): return _wrap(_lift(lambda x: _unary("cos", _check_num(x)), self.v))
    def sigmoid(self): return _wrap(_lift(lambda x: _unary("sigmoid", _check_num(x)), self.v))
    def sqrt(self): return _wrap(_lift(lambda x: _unary("sqrt", _check_num(x)), self.v))
    def abs(self): return self.__abs__()
    def square(self): return self * self
    def pow(self, e): return self ** e
    def norm(self, p=None, dim=None, **kw):
        if p not in (None, "fro", 2, 2.0) or dim is not None:
            raise Untraceable(f"norm with p={p}, dim={dim}")
        return _wrap(_norm(self.v))
    def sum(self, dim=None, **kw):
        if dim is not None:
            raise Untraceable("sum over a dimension")
        return _wrap(_sum(self.v))
    def dot(self, o): return _wrap(_sum(_lift(_mul, self.v, _scalar(o), nargs=2)))
    def item(self): return self.__float__()
    def clone(self, *a, **k): return self
    def detach(self): return self
    def float(self): return self
    def to(self, *a, **k): return self
    def requires_grad_(self, *a, **k): return self
    def squeeze(self, *a, **k): return self
    def numel(self): return len(self.v) if isinstance(self.v, tuple) else 1
    def dim(self): return 1 if isinstance(self.v, tuple) else 0

    @property
    def shape(self):
        return (len(self.v),) if isinstance(self.v, tuple) else ()

    @property
    def requires_grad(self):
        return True


def _wrap(v):
    return v if isinstance(v, _Sym) else _Sym(v)


def _cmp(a, op, b):
    if isinstance(a, tuple) or isinstance(b, tuple):
        raise Untraceable("comparison of vectors")
    return _compare(a, op, b)


# ---------------------------------------------------------------------------
# branch exploration and float() sentinels
# ---------------------------------------------------------------------------
# float(sym) must return a Python float: it returns a quiet NaN whose payload
# names the traced value. The payload sits in the top mantissa bits so that it
# survives a float64 -> float32 conversion (torch.tensor(float(...))).
_MAGIC = 0b101101


def _sentinel(i: int) -> float:
    bits = (0x7FF << 52) | (1 << 51) | (_MAGIC << 45) | ((i & 0xFFFF) << 29)
    return struct.unpack("<d", struct.pack("<Q", bits))[0]


def _sentinel_index(v):
    try:
        d = float(v)
    except Exception:
        return None
    if d == d:
        return None
    bits = struct.unpack("<Q", struct.pack("<d", d))[0]
    if (bits >> 45) & 0x3F != _MAGIC:
        return None
    return (bits >> 29) & 0xFFFF


class _Explorer:
    def __init__(self, prefix):
        self.prefix = list(prefix)
        self.taken = []          # (cond, outcome) in the order the callable asked
        self.floats = []         # values passed through float()/torch.tensor()
        self.detached = False

    def decide(self, cond: _Cond) -> bool:
        i = len(self.taken)
        outcome = self.prefix[i] if i < len(self.prefix) else False
        self.taken.append((cond, outcome))
        return outcome

    def float_sentinel(self, sym: _Sym) -> float:
        if isinstance(sym.v, tuple):
            raise Untraceable("float() of a vector")
        self.floats.append(sym)
        self.detached = True
        return _sentinel(len(self.floats) - 1)


_ACTIVE: list = []


def _explorer() -> _Explorer:
    if not _ACTIVE:
        raise Untraceable("traced value used outside trace()")
    return _ACTIVE[-1]


class _TorchPatch:
    """torch.tensor / torch.as_tensor applied to traced values return them
    (marked detached, as the reference's re-wrapping detaches autograd)."""

    def __enter__(self):
        import torch

        self.torch = torch
        self.saved = (torch.tensor, torch.as_tensor)
        orig_tensor, orig_as = self.saved

        def contains_sym(d):
            if isinstance(d, _Sym):
                return True
            if isinstance(d, (list, tuple)):
                return any(contains_sym(e) for e in d)
            return False

        def tensor(data, *a, **k):
            if contains_sym(data):
                _explorer().detached = True
                return data if isinstance(data, _Sym) else _wrap(tuple(_scalar(e) for e in data))
            return orig_tensor(data, *a, **k)

        def as_tensor(data, *a, **k):
            if contains_sym(data):
                return data if isinstance(data, _Sym) else _wrap(tuple(_scalar(e) for e in data))
            return orig_as(data, *a, **k)

        torch.tensor, torch.as_tensor = tensor, as_tensor
        return self

    def __exit__(self, *exc):
        self.torch.tensor, self.torch.as_tensor = self.saved
        return False


def _result_field(out, ex: _Explorer):
    """The callable's return value -> Field (or float)."""
    if isinstance(out, _Sym):
        v = out.v
    else:
        idx = _sentinel_index(out) if not isinstance(out, (F.Field,)) else None
        if idx is not None:
            if idx >= len(ex.floats):
                raise Untraceable("unrecognised NaN result")
            v = ex.floats[idx].v
        elif isinstance(out, F.Field):
            v = out
        else:
            try:
                v = _scalar(out)
            except Untraceable:
                raise Untraceable(f"return value of type {type(out).__name__}") from None
            if isinstance(v, float) and v != v:
                raise Untraceable("NaN result")
    if isinstance(v, tuple):
        if len(v) == 1:
            v = v[0]
        else:
            raise Untraceable("the callable returns a vector")
    if isinstance(v, (_Radial, _Abs)):
        raise Untraceable("the callable returns a bare distance / |.|")
    return v


def trace(fn, max_paths: int = 64) -> F.Field:
    """Run ``fn`` on a symbolic point and return the field it computes
    (all branches of its comparisons combined with indicator factors).
    Raises :class:`Untraceable` when that is not possible."""
    total = F.const(0.0)
    stack = [[]]
    paths = 0
    while stack:
        prefix = stack.pop()
        paths += 1
        if paths > max_paths:
            raise Untraceable(f"more than {max_paths} branch paths")
        ex = _Explorer(prefix)
        _ACTIVE.append(ex)
        try:
            with _TorchPatch():
                point = _Sym((F.X, F.Y))
                try:
                    out = fn(point)
                except Untraceable:
                    raise
                except Exception as e:   # the callable itself failed on the symbolic point
                    raise Untraceable(f"{type(e).__name__}: {e}") from None
            v = _result_field(out, ex)
        finally:
            _ACTIVE.pop()
        for i in range(len(prefix), len(ex.taken)):
            if ex.taken[i][1] is False:
                stack.append([o for _, o in ex.taken[:i]] + [True])
        if _is_const(v) and _const_value(v) == 0.0:
            continue
        term = F.as_field(v)
        for cond, outcome in ex.taken:
            term = term * cond.ind(outcome)
        total = total + term
    return _merge_boxes(total)


def _merge_boxes(field: F.Field) -> F.Field:
    """Intersect the box indicators within each term (a chain of half-plane
    conditions becomes one box factor)."""
    terms = []
    for t in field.terms:
        boxes = [f for f in t.factors if f.kind == F.FK_IND_BOX]
        if len(boxes) < 2:
            terms.append(t)
            continue
        lo_x = max(b.params[0] for b in boxes)
        hi_x = min(b.params[1] for b in boxes)
        lo_y = max(b.params[2] for b in boxes)
        hi_y = min(b.params[3] for b in boxes)
        if lo_x > hi_x or lo_y > hi_y:
            continue                                   # empty region: the term vanishes
        rest = [f for f in t.factors if f.kind != F.FK_IND_BOX]
        terms.append(F._Term(t.coef, t.mono, rest + [F._Factor(F.FK_IND_BOX, (lo_x, hi_x, lo_y, hi_y))]))
    return F.Field(terms, field.flags)


# ---------------------------------------------------------------------------
# validation, tabulation, alpha's autograd behaviour
# ---------------------------------------------------------------------------
def _call_reference_style(fn, p: np.ndarray) -> float:
    import torch

    out = fn(torch.tensor([float(p[0]), float(p[1])], dtype=torch.float32))
    if isinstance(out, torch.Tensor):
        return float(out.detach().reshape(-1)[0]) if out.numel() >= 1 else float("nan")
    return float(out)


def _sample_points(bounds, n: int, seed: int = 7) -> np.ndarray:
    (x0, x1), (y0, y1) = bounds
    rng = np.random.default_rng(seed)
    pts = np.stack([rng.uniform(x0, x1, n), rng.uniform(y0, y1, n)], axis=1)
    corners = np.array([[x0, y0], [x1, y0], [x0, y1], [x1, y1], [(x0 + x1) / 2, (y0 + y1) / 2]])
    return np.concatenate([pts, corners]).astype(np.float32)


def _agrees(field: F.Field, fn, pts: np.ndarray, rtol: float = 1e-4) -> tuple[bool, str]:
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        ref = np.array([_call_reference_style(fn, p) for p in pts], np.float64)
    got = np.asarray(field(pts), np.float64)
    nan_r, nan_g = np.isnan(ref), np.isnan(got)
    if np.any(nan_r != nan_g):
        return False, "NaN pattern differs"
    ok = ~nan_r
    if not ok.any():
        return True, ""
    scale = max(float(np.abs(ref[ok]).max()), 1e-30)
    err = np.abs(got[ok] - ref[ok])
    bad = err > rtol * np.abs(ref[ok]) + 1e-6 * scale
    if bad.any():
        i = int(np.argmax(err))
        return False, f"max deviation {float(err[i]):.3g} at {pts[ok][i].tolist()}"
    return True, ""


def tabulate(fn, bounds, resolution: int = 513, margin: float = 0.02) -> F.Field:
    """Evaluate ``fn`` (reference calling convention) on a regular grid over the
    domain bounds (widened by ``margin`` of the extent on each side) and return
    the interpolating field. ``resolution`` nodes along the longer side, the
    other side with the same spacing (at least 4 nodes)."""
    (x0, x1), (y0, y1) = bounds
    wx, wy = max(x1 - x0, 1e-6), max(y1 - y0, 1e-6)
    x0, x1 = x0 - margin * wx, x1 + margin * wx
    y0, y1 = y0 - margin * wy, y1 + margin * wy
    h = max(x1 - x0, y1 - y0) / (resolution - 1)
    nx = max(4, int(math.ceil((x1 - x0) / h)) + 1)
    ny = max(4, int(math.ceil((y1 - y0) / h)) + 1)
    if nx * ny > F._MAX_GRID_VALUES:
        raise ValueError(f"tabulation grid {nx} x {ny} exceeds {F._MAX_GRID_VALUES} values; lower the resolution")
    xs = x0 + h * np.arange(nx)
    ys = y0 + h * np.arange(ny)
    vals = _tabulate_values(fn, xs, ys)
    return F.tabulated(vals, x0, y0, h, h)


def _tabulate_values(fn, xs, ys) -> np.ndarray:
    import torch

    gx, gy = np.meshgrid(xs.astype(np.float32), ys.astype(np.float32))      # [ny, nx]
    # vectorised attempt: point = [x-row, y-row] (point[0], point[1] elementwise)
    try:
        with torch.no_grad():
            out = fn(torch.stack([torch.from_numpy(gx.ravel()), torch.from_numpy(gy.ravel())]))
        if isinstance(out, torch.Tensor) and out.numel() == gx.size:
            vals = out.detach().to(torch.float32).reshape(gx.shape).numpy().copy()
            rng = np.random.default_rng(3)
            ii = rng.integers(0, gx.size, 16)
            ref = np.array([_call_reference_style(fn, (gx.ravel()[i], gy.ravel()[i])) for i in ii], np.float32)
            if np.allclose(vals.ravel()[ii], ref, rtol=1e-5, atol=1e-6 * max(float(np.abs(ref).max()), 1e-30),
                           equal_nan=True):
                return vals
    except Exception:
        pass
    vals = np.empty(gx.shape, np.float32)
    for j in range(gx.shape[0]):
        for i in range(gx.shape[1]):
            vals[j, i] = _call_reference_style(fn, (gx[j, i], gy[j, i]))
    return vals


def alpha_is_detached(fn, pts: np.ndarray) -> bool:
    """What the reference's sigma' does with this alpha (solvers/WoStSolver.py:80-127):
    alpha_wrapped re-wraps non-tensors and clamps; torchGradient raises when
    the value is not connected to the point, and sigma' then falls back to
    sigma/alpha (Q9). True when that happens at the sample points."""
    import torch

    detached = []
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        for p in pts[:16]:
            q = torch.tensor([float(p[0]), float(p[1])], dtype=torch.float32).requires_grad_(True)
            try:
                r = fn(q)
                if not isinstance(r, torch.Tensor):
                    r = torch.tensor(r, dtype=torch.float32, requires_grad=True)
                r = torch.clamp(r, min=1e-8)
                torch.autograd.grad(r, q, create_graph=True)
                detached.append(False)
            except Exception:
                detached.append(True)
    return sum(detached) * 2 > len(detached)


@dataclass
class Conversion:
    """How a coefficient argument became a device field."""

    field: F.Field
    how: str          # "field" | "constant" | "traced" | "tabulated"
    detail: str = ""


def field_from_callable(obj, bounds, *, what: str = "field", is_alpha: bool = False, resolution: int = 513,
                        trace_first: bool = True) -> Conversion:
    """A coefficient argument of WostSolver_2D (Field, number or callable) -> Conversion."""
    if obj is None:
        return None
    if isinstance(obj, F.Field):
        return Conversion(obj, "field")
    if isinstance(obj, numbers.Real):
        return Conversion(F.const(float(obj)), "constant")
    if not callable(obj):
        raise TypeError(f"{what}: expected a field, a number or a callable, got {type(obj).__name__}")
    pts = _sample_points(bounds, 48)
    reason = "tracing disabled"
    fld = None
    if trace_first:
        try:
            fld = trace(obj)
            ok, why = _agrees(fld, obj, pts)
            if not ok:
                reason = f"traced field disagrees with the callable ({why})"
                fld = None
        except Untraceable as e:
            reason = str(e)
            fld = None
    how = "traced"
    if fld is None:
        warnings.warn(f"{what}: the callable cannot be expressed as a closed-form device field ({reason}); "
                      f"tabulating it on a {resolution}-node grid over the domain (Catmull-Rom interpolation)",
                      RuntimeWarning, stacklevel=3)
        fld = tabulate(obj, bounds, resolution=resolution)
        how = "tabulated"
        reason = f"{reason}; grid {int(fld.terms[0].factors[0].params[4])} x {int(fld.terms[0].factors[0].params[5])}"
    else:
        reason = ""
    if is_alpha and alpha_is_detached(obj, pts):
        fld = F.detach(fld)
    return Conversion(fld, how, reason)
