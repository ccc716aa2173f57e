"""The reference's scenarios as device-evaluable problems.

Each builder returns a :class:`Scenario` whose fields restate the reference's
Python callables with :mod:`dcrmontecarlo_amd.fields` (tests/golden/fields_*.npz
pins every one of them against the original callable, evaluated by the
reference itself). Geometry and query points follow the reference's
construction (torch.linspace semantics, float32).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field as dc_field

import numpy as np

from . import fields as F
from .fields import X, Y


@dataclass
class Scenario:
    name: str
    dirichlet: np.ndarray                 # [V,2] float32
    neumann: np.ndarray | None            # [V,2] float32 or None
    g: F.Field | None = None
    f: F.Field | None = None
    sigma: F.Field | None = None
    alpha: F.Field | None = None
    points: np.ndarray = dc_field(default_factory=lambda: np.zeros((0, 2), np.float32))
    n_walks: int = 1000
    max_steps: int = 1000
    eps: float = 1e-4
    reference: str = ""

    def solver(self, **kw):
        from .geometry import PolyLinesSimple
        from .solvers import WostSolver_2D

        return WostSolver_2D(PolyLinesSimple(self.dirichlet), self.g,
                             PolyLinesSimple(self.neumann) if self.neumann is not None else None,
                             source=self.f, sigma=self.sigma, alpha=self.alpha, **kw)

    def kernel_source(self, **kw) -> str:
        """Generated source of this scenario's field-specialised walk kernel (host only)."""
        from .geometry import PolyLinesSimple
        from .solvers.WoStSolver import kernel_source

        return kernel_source(PolyLinesSimple(self.dirichlet), self.g,
                             PolyLinesSimple(self.neumann) if self.neumann is not None else None,
                             source=self.f, sigma=self.sigma, alpha=self.alpha, **kw)


def torch_linspace(start: float, end: float, steps: int) -> np.ndarray:
    """torch.linspace in float32 (ATen CPU: first half from start, second half from end)."""
    start, end = np.float32(start), np.float32(end)
    if steps == 1:
        return np.array([start], np.float32)
    step = np.float32((end - start) / np.float32(steps - 1))
    i = np.arange(steps)
    half = steps // 2
    lo = start + step * i.astype(np.float32)
    hi = end - step * (steps - i - 1).astype(np.float32)
    return np.where(i < half, lo, hi).astype(np.float32)


def _square(h: float) -> np.ndarray:
    return np.array([[-h, -h], [h, -h], [h, h], [-h, h], [-h, -h]], np.float32)


def _grid(lo: float, hi: float, n: int) -> np.ndarray:
    g = torch_linspace(lo, hi, n)
    gx, gy = np.meshgrid(g, g, indexing="ij")
    return np.stack([gx.ravel(), gy.ravel()], axis=1).astype(np.float32)


# ---------------------------------------------------------------------------
def laplace_square(n_points: int = 64, n_walks: int = 1000) -> Scenario:
    """C1a: Laplace on the unit square, g = x^2 - y^2 (harmonic, exact solution)."""
    rng = np.random.default_rng(1234)
    pts = rng.uniform(0.1, 0.9, size=(n_points, 2)).astype(np.float32)
    sq = np.array([[0, 0], [1, 0], [1, 1], [0, 1], [0, 0]], np.float32)
    return Scenario("laplace_square", sq, None, g=X**2 - Y**2, points=pts, n_walks=n_walks,
                    max_steps=1000, eps=1e-4, reference="geometry/PolylinesSimple.py:309-316 square; SURVEY 8d C1a")


def manufactured_polynomial(n_walks: int = 150) -> Scenario:
    """C1b: tests/testWoStCorrectness.py:81-142, delta tracking on the square +-1."""
    u = (1 - X**2) * (1 - Y**2)
    D = 2.0 + 0.5 * X + 0.5 * Y                               # :97 (passed as alpha)
    lap_u = -2 * (2 - X**2 - Y**2)                            # :131
    gdg = -X * (1 - Y**2) - Y * (1 - X**2)                    # :133
    absorption = X * Y + 2                                    # :100 (passed as sigma)
    f = -(D * lap_u + gdg) + (2 + X * Y) * u                  # :134-140
    g = (1 - X**2) * (1 - Y**2)                               # :102-104
    pts = _grid(-0.7, 0.7, 4)                                 # create_test_points :144-156
    return Scenario("manufactured_polynomial", _square(1.0), None, g=g, f=f, sigma=absorption, alpha=D,
                    points=pts, n_walks=n_walks, max_steps=800, eps=1e-4,
                    reference="tests/testWoStCorrectness.py:159-196")


def poisson_square(n_points: int = 64, n_walks: int = 10_000) -> Scenario:
    """C2: tests/testWostWithSource.py, f = -4 on the square +-2, g = x^2 + y^2."""
    pts = _grid(-1.8, 1.8, 21)                                # :64-69
    pts = pts[np.sqrt((pts.astype(np.float32) ** 2).sum(1)).astype(np.float32) > np.float32(0.6)]   # :72-73
    f = -4.0 * F.indicator_box(-2.0, 2.0, -2.0, 2.0)          # :51-56
    return Scenario("poisson_square", _square(2.0), None, g=X**2 + Y**2, f=f, points=pts[:n_points],
                    n_walks=n_walks, max_steps=500, eps=1e-4, reference="tests/testWostWithSource.py:82-110")


def _circle(n: int, radius: float) -> np.ndarray:
    th = torch_linspace(0.0, 2 * math.pi, n + 1)
    return np.stack([np.float32(radius) * np.cos(th), np.float32(radius) * np.sin(th)], axis=1).astype(np.float32)


def variable_coefficients(n_points: int = 256, n_walks: int = 100_000) -> Scenario:
    """C3: tests/testWostVariableCoefficients.py, mixed boundary + delta tracking."""
    pi = math.pi
    alpha = F.detach(0.5 + 1.5 * F.exp(-2.0 * (X**2 + Y**2)))                 # :42-49 (torch.tensor(..) => Q9)
    sigma = 0.3 + 0.7 * (1 + F.sin(2 * pi * X) * F.cos(2 * pi * Y))           # :51-57
    g = F.sin(pi * X) * F.sin(pi * Y)                                         # :67-72
    f = F.exp(-(X**2 + Y**2)) * F.sin(pi * X) * F.cos(pi * Y) * F.indicator_disk((0.0, 0.0), 1.5)  # :74-84
    pts = _grid(-1.3, 1.3, 27)                                                # :95-99
    pts = pts[np.sqrt((pts ** 2).sum(1)).astype(np.float32) > np.float32(0.5)]  # :102-103
    return Scenario("variable_coefficients", _square(1.5), _circle(32, 0.4), g=g, f=f, sigma=sigma, alpha=alpha,
                    points=pts[:n_points], n_walks=n_walks, max_steps=1000, eps=1e-4,
                    reference="tests/testWostVariableCoefficients.py:185-264")


def dcr_alpha_geophysical() -> F.Field:
    """conductivity_field, tests/testGeophysicalScenario.py:35-55."""
    bg = 1e2
    return bg + (1e1 - bg) * F.smooth_circle((-20.0, -30.0), 10.0) + (1e3 - bg) * F.smooth_circle((25.0, -40.0), 10.0)


def dcr_source_geophysical() -> F.Field:
    """dcr_current_source, tests/testGeophysicalScenario.py:11-33. Its return value is
    positive_source - negative_sink with negative_sink already negated, so both
    electrodes inject current (quirk Q10, kept)."""
    s = 0.5
    norm = 1.0 / (2 * math.pi * s**2)
    return norm * F.gaussian((-10.0, 0.0), s) + norm * F.gaussian((10.0, 0.0), s)


def dcr_dipole(n_electrodes: int = 48, n_walks: int = 1_000_000, eps: float = 0.9) -> Scenario:
    """C4: testGeophysicalScenario fields on the +-100 box with the top Neumann segment,
    48 surface electrodes x = -70.5 + 3k. eps = 0.9 because the reference's eps = 1.0
    (:149) never starts a walk (dDirichlet is seeded with 1.0, quirk Q12)."""
    h = 100.0
    D = np.array([[-h, -h], [h, -h], [h, h], [-h, h], [-h, -h]], np.float32)   # :88-94
    N = np.array([[-h, h], [h, h]], np.float32)                              # :99-102
    x = (-70.5 + 3.0 * np.arange(n_electrodes)).astype(np.float32)
    pts = np.stack([x, np.zeros_like(x)], axis=1)
    return Scenario("dcr_dipole", D, N, g=F.const(0.0), f=dcr_source_geophysical(), sigma=None,
                    alpha=dcr_alpha_geophysical(), points=pts, n_walks=n_walks, max_steps=500, eps=eps,
                    reference="tests/testGeophysicalScenario.py:77-154")


def dcr_reference_electrodes() -> np.ndarray:
    """create_surface_measurement_grid((-40, 40), 0, 10) (testGeophysicalScenario.py:58-74, 109-113)."""
    x = np.arange(-40.0, 40.0 + 10.0, 10.0).astype(np.float32)
    return np.stack([x, np.zeros_like(x)], axis=1)


def notebook_alpha(air: bool = True) -> F.Field:
    """conductivity_field_torch, tests/testNotebook.ipynb cell 17. ``air=False`` drops
    its air term (alpha = 1e-8 above y = 0): over a topographic Neumann surface that
    rises to y = 3, the term would put surface electrodes in "air"; the zero-flux
    surface already models the air."""
    bg, air_v = 1e-2, 1e-8
    a = (bg + (1e-1 - bg) * F.smooth_circle((-120.0, -80.0), 60.0)
         + (1e-3 - bg) * F.smooth_circle((120.0, -80.0), 60.0))
    return a + (air_v - bg) * F.sigmoid(10000.0 * Y) if air else a


def notebook_source() -> F.Field:
    """dcr_current_source_torch, notebook cell 17 (a proper +/- dipole at x = -+200)."""
    s = 5.0
    norm = 1.0 / (2 * math.pi * s**2)
    return norm * F.gaussian((-200.0, 0.0), s) - norm * F.gaussian((200.0, 0.0), s)


def notebook_dcr(n_walks: int = 250) -> Scenario:
    """Notebook cells 17-19: open U Dirichlet boundary, flat Neumann top, 21 electrodes."""
    D = np.array([[-500.0, 1.0], [-500.0, -1000.0], [500.0, -1000.0], [500.0, 1.0]], np.float32)
    N = np.array([[500.0, 1.0], [-500.0, 1.0]], np.float32)
    x = np.arange(-400.0, 400.0 + 40.0, 40.0).astype(np.float32)
    pts = np.stack([x, np.full_like(x, -0.1)], axis=1).astype(np.float32)
    return Scenario("notebook_dcr", D, N, g=F.const(0.0), f=notebook_source(), sigma=None, alpha=notebook_alpha(),
                    points=pts, n_walks=n_walks, max_steps=500, eps=0.9, reference="tests/testNotebook.ipynb cells 17-19")


def topography(n_segments: int = 10_000) -> np.ndarray:
    """C5 Neumann surface: y = 1 + 2 sin(x/37), x from 500 down to -500."""
    x = np.linspace(500.0, -500.0, n_segments + 1)
    return np.stack([x, 1.0 + 2.0 * np.sin(x / 37.0)], axis=1).astype(np.float32)


def wenner_topography(n_electrodes: int = 256, n_walks: int = 10_000, n_segments: int = 10_000,
                      physical: bool = False) -> Scenario:
    """C5: notebook fields and U boundary with a 10k-segment topographic Neumann surface.
    The literal variant keeps the notebook's conductivity, air term included (the
    parity workload); ``physical=True`` (wenner_topography_physical) drops the air
    term, which is flat at y = 0 while the surface rises to y = 3, so that the
    electrodes sit in the ground and the apparent resistivities mean something."""
    D = np.array([[-500.0, 1.0], [-500.0, -1000.0], [500.0, -1000.0], [500.0, 1.0]], np.float32)
    N = topography(n_segments)
    x = np.linspace(-400.0, 400.0, n_electrodes).astype(np.float32)
    y = (1.0 + 2.0 * np.sin(x.astype(np.float64) / 37.0) - 0.1).astype(np.float32)
    return Scenario("wenner_topography_physical" if physical else "wenner_topography", D, N, g=F.const(0.0),
                    f=notebook_source(), sigma=None, alpha=notebook_alpha(air=not physical),
                    points=np.stack([x, y], axis=1), n_walks=n_walks, max_steps=500, eps=0.9,
                    reference="SURVEY.md 8d C5 (notebook cells 17-18 + synthetic topography)")


def wenner_topography_physical(n_electrodes: int = 256, n_walks: int = 10_000, n_segments: int = 10_000) -> Scenario:
    return wenner_topography(n_electrodes, n_walks, n_segments, physical=True)


ALL = {
    "laplace_square": laplace_square,
    "manufactured_polynomial": manufactured_polynomial,
    "poisson_square": poisson_square,
    "variable_coefficients": variable_coefficients,
    "dcr_dipole": dcr_dipole,
    "notebook_dcr": notebook_dcr,
    "wenner_topography": wenner_topography,
    "wenner_topography_physical": wenner_topography_physical,
}
