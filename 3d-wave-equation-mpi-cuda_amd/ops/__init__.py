"""Kernel-level ops: ``kernels`` (HIP, device tensors) and ``reference`` (plain PyTorch)."""
from . import kernels, reference  # noqa: F401
