"""lvae_amd -- MI355X-native hot path of the Longitudinal-VAE (SidRama/Longitudinal-VAE).

The GP-prior ELBO term (additive-kernel Gram, blocked Cholesky / inverse, KL reductions, the
Hensman SVI bound and its natural-gradient update) runs in hand-written HIP kernels for gfx950
behind the C ABI of include/lvae_hip.h; the conv encoder/decoder runs on PyTorch-ROCm.
"""
from . import _lib  # noqa: F401
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
