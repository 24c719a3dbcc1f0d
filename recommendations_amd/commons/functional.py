"""Drop-in for commons/functional.py."""
from ..kernels import CapGradientsFn


def cap_gradients(x):
    """Identity forward; backward g / (||g||_2 + 1e-6) (commons/functional.py:4-28), on the GPU."""
    return CapGradientsFn.apply(x)
