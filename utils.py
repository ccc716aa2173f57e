"""Import-path shim for the reference's top-level ``utils`` module (reference utils.py).

* ``torch_smooth_circle`` (:123-129): the field primitive of the DCR scenarios
  (tests/testGeophysicalScenario.py:49-50, notebook cell 17). It evaluates
  sigmoid(-100 (|x - center| - radius)) with the operations the reference uses, so it
  works on torch tensors and is traced into the closed-form ``fields.smooth_circle``
  factor by dcrmontecarlo_amd.trace when a coefficient callable built from it is
  handed to WostSolver_2D.
* ``torchGradient``, ``torchLaplacian``, ``gridSampleMinMax`` (:11-120): the host-side
  autograd helpers the reference builds sigma' and sigma_bar with. The device path
  does not use them (libwost evaluates analytic jets); they are restated
  here with the reference's semantics (the +1e-8 Laplacian offset, the silent
  fallback when a second derivative fails, NaN/inf samples skipped) for scripts that
  call them directly.
* ``plot_walk_history``, ``plot_multiple_walks``, ``plot_walk_statistics``
  (:237-639): visualisation, out of scope. They raise
  NotImplementedError; ``WostSolver_2D.solve(..., return_history=True)`` returns the
  reference's history structure, so the reference's own plotting functions accept it.
"""


def torch_smooth_circle(x, center, radius):
    signed_distance = (x - center).norm() - radius      # < 0 inside the circle
    return (signed_distance * -100).sigmoid()


def torchGradient(function, point):
    """d function / d point by autograd, kept differentiable (create_graph)."""
    import torch

    p = point if point.requires_grad else point.clone().requires_grad_(True)
    value = function(p)
    if value.numel() != 1:
        raise ValueError(f"Function must return a scalar, got tensor with {value.numel()} elements")
    return torch.autograd.grad(value, p, create_graph=True)[0]


def torchLaplacian(function, point):
    """Sum of the second derivatives, starting from 1e-8 (reference :54); if a second
    derivative cannot be taken, the partial sum so far is returned (:60-61)."""
    import torch

    p = point if point.requires_grad else point.clone().requires_grad_(True)
    grad = torchGradient(function, p)
    lap = torch.zeros_like(grad[0]) + 1e-8
    try:
        for i in range(len(grad)):
            lap = lap + torch.autograd.grad(grad[i], p, create_graph=True, retain_graph=True)[0][i]
    except Exception:   # noqa: BLE001 -- the reference's silent fallback
        return lap
    return lap


def gridSampleMinMax(function, domain_bounds, grid_resolution: int = 100):
    """(min, max, min_point, max_point) of function over a torch.linspace grid (ij
    meshgrid, 1-3 dimensions). Points where it fails or is NaN/inf are skipped; as in
    the reference (:111-118) the returned points index the grid by the position among
    the kept values."""
    import torch

    axes = [torch.linspace(b[0], b[1], grid_resolution) for b in domain_bounds]
    if not 1 <= len(axes) <= 3:
        raise ValueError(f"Grid sampling for {len(axes)}D not implemented. Maximum supported dimension is 3.")
    mesh = torch.meshgrid(*axes, indexing="ij") if len(axes) > 1 else (axes[0],)
    pts = torch.stack([m.flatten() for m in mesh], dim=1)
    vals = []
    for p in pts:
        try:
            v = function(p)
            if torch.isnan(torch.as_tensor(v)) or torch.isinf(torch.as_tensor(v)):
                continue
            vals.append(v.item() if hasattr(v, "item") else float(v))
        except Exception:   # noqa: BLE001
            continue
    if not vals:
        raise ValueError("Function could not be evaluated at any grid points")
    t = torch.tensor(vals)
    i, j = int(torch.argmin(t)), int(torch.argmax(t))
    return t[i].item(), t[j].item(), pts[i], pts[j]


def _plot_out_of_scope(name):
    def f(*args, **kwargs):
        raise NotImplementedError(
            f"utils.{name} (reference utils.py:237-639) is visualisation, outside this build's scope; "
            "WostSolver_2D.solve(..., return_history=True) returns the reference's history structure, "
            "so the reference's own plotting functions can draw it")
    f.__name__ = name
    return f


plot_walk_history = _plot_out_of_scope("plot_walk_history")
plot_multiple_walks = _plot_out_of_scope("plot_multiple_walks")
plot_walk_statistics = _plot_out_of_scope("plot_walk_statistics")

__all__ = ["torch_smooth_circle", "torchGradient", "torchLaplacian", "gridSampleMinMax", "plot_walk_history",
           "plot_multiple_walks", "plot_walk_statistics"]
