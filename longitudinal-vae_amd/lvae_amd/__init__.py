"""lvae_amd -- MI355X-native hot path of the Longitudinal-VAE (SidRama/Longitudinal-VAE).

The GP-prior ELBO term (additive-kernel Gram, blocked Cholesky / inverse, KL reductions, the
Hensman SVI bound and its natural-gradient update) runs in hand-written HIP kernels for gfx950
behind the C ABI of include/lvae_hip.h; the conv encoder/decoder runs on PyTorch-ROCm.
"""
import os

# MIOpen's Winograd solvers, which it picks for the ConvVAE's 3x3 conv and 4x4 transposed conv at the bench's
# 4096 images, put the transposed conv's input gradient 4.3e-2 (max-norm) from fp64, against 5.8e-7 with them
# off (scripts/deconv_check.py; +0.3 ms a step): off unless LVAE_MIOPEN_WINOGRAD=1 (read by MIOpen when it first
# picks a solver, so this import must come before the first convolution).
if os.environ.get("LVAE_MIOPEN_WINOGRAD", "0") != "1":
    os.environ.setdefault("MIOPEN_DEBUG_CONV_WINOGRAD", "0")

from . import _lib  # noqa: F401,E402
from .kernels import (AdditiveKernel, BinKernel, CatKernel, LinearKernel, PeriodicKernel,  # noqa: F401
                      ProductKernel, RbfKernel, ScaleKernel, generate_kernel, generate_kernel_approx,
                      generate_kernel_batched, kernel_spec_and_params)
from .likelihoods import GaussianLikelihood  # noqa: F401
from .elbo import (HensmanPrior, KL_closed, KL_closed_batched, check_pending, kl_closed_prefactor,  # noqa: F401
                   minibatch_KLD_upper_bound, minibatch_KLD_upper_bound_iter, natural_gradient_update,
                   set_sync_checks)
from .predict import batch_predict_varying_T  # noqa: F401
from .gpapprox import deviance_upper_bound, elbo, spd_inverse, validation_dubo  # noqa: F401

__version__ = "0.1.0"
