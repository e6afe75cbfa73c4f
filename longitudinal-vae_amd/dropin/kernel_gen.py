"""kernel_gen.py surface (reference kernel_gen.py:9-310): the additive-kernel builders, returning
lvae_amd kernel modules whose Grams run in the HIP library (gpytorch batch semantics)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from lvae_amd.kernels import generate_kernel, generate_kernel_approx, generate_kernel_batched  # noqa: E402,F401

__all__ = ["generate_kernel", "generate_kernel_approx", "generate_kernel_batched"]
