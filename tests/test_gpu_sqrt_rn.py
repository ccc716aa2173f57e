"""The distances' correctly rounded square root (wost_device.h sqrt_rn: the residual
test without the compiler's scaling and class steps for 2^-96 <= x < inf, sqrtf
under a wave vote otherwise) against IEEE float32 on the host, through the device
distance query (wost_geometry_query, poly_distance).

For the point (0, y) and the segment (-1, 0) -> (1, 0) the kernel's squared
distance is exactly RN(y * y) (projection t = 1/2, closest point (0, 0)), so the
returned distance must be numpy's float32 sqrt of that, bit for bit -- across
zero, denormal squares, the 2^-96 switch point and its neighbours, huge squares
and an overflow to inf, with lanes of both paths in one wave."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _ys():
    rng = np.random.default_rng(5)
    f = np.float32
    edge = [0.0, 1e-45, 1e-40, 1e-30, 2.0 ** -75, 2.0 ** -60, 2.0 ** -49, 2.0 ** -48, 2.0 ** -47, 1.0, 3.0,
            1e10, 1e19, 1.8e19, 1.9e19, 1e20, 3e38]
    near = []
    for b in (2.0 ** -48, 2.0 ** -47.5, 1.0, 2.0 ** 20):   # y with y*y around the switch and elsewhere
        for towards in (np.inf, 0.0):
            x = f(b)
            for _ in range(40):
                near.append(x)
                x = np.nextafter(x, f(towards))
    mags = 10.0 ** rng.uniform(-44, 38, 4000)
    ys = np.concatenate([np.array(edge), np.array(near, dtype=np.float64), mags]).astype(np.float32)
    ys = np.concatenate([ys, -ys[: ys.size // 3]])
    rng.shuffle(ys)
    return ys


def test_distance_sqrt_matches_ieee(gpu_available):
    from dcrmontecarlo_amd.geometry import PolyLinesSimple

    seg = PolyLinesSimple(np.array([[-1.0, 0.0], [1.0, 0.0]], np.float32))
    ys = _ys()
    pts = np.stack([np.zeros_like(ys), ys], axis=1).astype(np.float32)
    got = np.asarray(seg.distance(pts), dtype=np.float32)
    with np.errstate(over="ignore", under="ignore"):
        want = np.sqrt(ys * ys)          # float32 throughout: RN(y^2), then the IEEE square root
    assert want.dtype == np.float32
    diff = got.view(np.uint32) != want.view(np.uint32)
    assert not diff.any(), list(zip(ys[diff][:8], got[diff][:8], want[diff][:8]))
    assert np.isinf(got).any() and (got == 0).any()   # both ends of the slow path were exercised
    with np.errstate(over="ignore", under="ignore"):
        sq = ys * ys
    assert ((sq >= 2.0 ** -96) & np.isfinite(sq)).mean() > 0.3   # and the fast path for many lanes
