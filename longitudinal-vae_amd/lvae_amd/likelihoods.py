"""Gaussian likelihood with the two access conventions the reference's ELBO code uses:
``likelihood.noise`` (KL_closed, elbo_functions.py:23) and ``likelihood.noise_covar.noise``
(elbo_functions.py:62,116,174 -- shape [L, 1] for a batched likelihood, as gpytorch's
GaussianLikelihood(batch_shape=[L]) in LVAE.py:183-188).  Positivity as GP_model.Likelihoods
(GP_model.py:7-29): noise = exp(m + softplus(raw - m)), m = -16.
"""
import math

import torch
import torch.nn.functional as F
from torch import nn

MIN_LOG = -16.0


class _NoiseCovar:
    def __init__(self, owner):
        self._owner = owner

    @property
    def noise(self):
        n = self._owner.noise
        return n.unsqueeze(-1) if self._owner.batched else n


class GaussianLikelihood(nn.Module):
    def __init__(self, latent_dim=1, noise=1.0, batched=None, constrain=True):
        super().__init__()
        self.latent_dim = latent_dim
        self.batched = (latent_dim > 1) if batched is None else batched
        raw = math.log(noise - math.exp(MIN_LOG))
        self._log_noise = nn.Parameter(torch.full((latent_dim,), raw, dtype=torch.float64), requires_grad=constrain)
        self.register_buffer("min_log_noise", torch.full((1,), MIN_LOG, dtype=torch.float64))
        self.noise_covar = _NoiseCovar(self)

    @property
    def noise(self):
        r = self._log_noise
        if r.is_cuda and r.dtype == torch.float64 and r.dim() == 1 and r.is_contiguous() and self.min_log_noise.is_cuda:
            from .kernels import _ParamPackFn  # (glue.hip: one launch each way)
            return _ParamPackFn.apply(([0], [self.min_log_noise], r.shape[0], 1), r).reshape(-1)
        return torch.exp(self.min_log_noise + F.softplus(self._log_noise - self.min_log_noise))

    @noise.setter
    def noise(self, value):
        with torch.no_grad():
            if isinstance(value, (int, float)):  # a device fill: no host copy, so graph-capturable
                self._log_noise.fill_(math.log(value - math.exp(MIN_LOG)))
                return
            v = torch.as_tensor(value, dtype=torch.float64, device=self._log_noise.device)
            self._log_noise.copy_(torch.log(v - math.exp(MIN_LOG)).expand_as(self._log_noise))


Likelihoods = GaussianLikelihood
