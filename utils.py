"""Import-path shim for the reference's top-level ``utils`` module: the one helper its
scenario scripts import, ``torch_smooth_circle`` (reference utils.py:123-129), used by
tests/testGeophysicalScenario.py:49-50 and notebook cell 17.

It evaluates sigmoid(-100 (|x - center| - radius)) with the operations the reference
uses (norm, sigmoid), so it works on torch tensors and is traced into the closed-form
``fields.smooth_circle`` factor by dcrmontecarlo_amd.trace when a coefficient callable
built from it is handed to WostSolver_2D. For a field object directly, use
``dcrmontecarlo_amd.fields.smooth_circle(center, radius)``."""


def torch_smooth_circle(x, center, radius):
    signed_distance = (x - center).norm() - radius      # < 0 inside the circle
    return (signed_distance * -100).sigmoid()


__all__ = ["torch_smooth_circle"]
