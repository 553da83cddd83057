"""Fused op library: every op dispatches to the HIP kernels in ``_C`` for GPU tensors and to a
plain-torch reference (the numerics oracle) on CPU."""
from . import activations, attention, cross_entropy, norms, rng
from .optim import FusedAdamW

__all__ = ["activations", "attention", "cross_entropy", "norms", "rng", "FusedAdamW"]
