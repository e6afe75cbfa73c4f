"""GP_model.py surface (reference GP_model.py:7-236): kernel modules, Likelihoods and the batched
builder, backed by lvae_amd."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from lvae_amd.kernels import (AdditiveKernel, BinKernel, CatKernel, ProductKernel, RbfKernel,  # noqa: E402,F401
                              ScaleKernel, generate_kernel_batched)
from lvae_amd.likelihoods import GaussianLikelihood  # noqa: E402


class Likelihoods(GaussianLikelihood):
    """Likelihoods(latent_dim, noise, constrain=True) (GP_model.py:7-29): per-dim Gaussian noise
    [latent_dim] with the same softplus parametrisation."""

    def __init__(self, latent_dim, noise, constrain=True):
        super().__init__(latent_dim, float(noise), constrain=constrain)


__all__ = ["Likelihoods", "BinKernel", "CatKernel", "RbfKernel", "ScaleKernel", "AdditiveKernel", "ProductKernel",
           "generate_kernel_batched"]
