"""Full-batch GP-approximation bounds of one latent dim: ``elbo`` (elbo_functions.py:36-84),
``deviance_upper_bound`` (DUBO, elbo_functions.py:86-142) and the all-dims ``validation_dubo``
(validation.py:8-68).  Same signatures and values as the reference.

The additive-kernel Grams and every SPD factorisation (K0zz, the per-subject B_p, the M x M
Woodbury matrix W) run in the HIP library: Grams through the differentiable ``covar_module(x1,
x2).evaluate()``, the factorisations through ``spd_inverse`` (lvae_spd_inv_small_f64, one
workgroup per matrix, returning A^-1 and log|A|).  The remaining M x M / T x M products are plain
library GEMMs (rocBLAS via torch.matmul); autograd composes the gradients (d A^-1 = -A^-1 dA A^-1,
d log|A| = tr(A^-1 dA)).
"""
import math

import torch

from . import _lib
from .elbo import _check_info


class _SpdInvFn(torch.autograd.Function):
    """(A^-1, log|A|) of a batch of SPD matrices [..., n, n], n <= 128 (HIP, fp64)."""

    @staticmethod
    def forward(ctx, A):
        lib = _lib.lib()
        n = A.shape[-1]
        lead = A.shape[:-2]
        Ab = A.detach().to(torch.float64).reshape(-1, n, n).contiguous()
        b = Ab.shape[0]
        Ai = torch.empty_like(Ab)
        ld = torch.empty(b, dtype=torch.float64, device=A.device)
        info = torch.empty(b, dtype=torch.int32, device=A.device)
        rc = lib.lvae_spd_inv_small_f64(n, b, _lib.ptr(Ab), n * n, _lib.ptr(Ai), n * n, _lib.ptr(ld), _lib.ptr(info),
                                        _lib.stream_ptr())
        _lib.check(rc, "spd_inv_small")
        _check_info(info, "cholesky")
        Ai = Ai.reshape(A.shape)
        ctx.save_for_backward(Ai)
        return Ai, ld.reshape(lead)

    @staticmethod
    def backward(ctx, g_inv, g_ld):
        (Ai,) = ctx.saved_tensors
        dA = torch.zeros_like(Ai)
        if g_inv is not None:
            dA = dA - Ai @ g_inv @ Ai
        if g_ld is not None:
            dA = dA + g_ld[..., None, None] * Ai
        return dA


def spd_inverse(A):
    """(A^-1, log|A|) for SPD A [..., n, n] (n <= 128), differentiable."""
    return _SpdInvFn.apply(A)


def _common(covar_module0, covar_module1, likelihood, train_xt, z, P, T, eps):
    dt = torch.float64
    M = z.shape[-2]
    x = train_xt.to(dt)
    x_st = x.reshape(P, T, x.shape[-1])
    K0xz = covar_module0(x, z).evaluate()
    K0zz = covar_module0(z, z).evaluate() + eps * torch.eye(M, dtype=dt, device=x.device)
    iK, ldK = spd_inverse(K0zz)
    K0_st = covar_module0(x_st, x_st).evaluate()
    B_st = covar_module1(x_st, x_st).evaluate() + torch.eye(T, dtype=dt, device=x.device) * \
        likelihood.noise_covar.noise.reshape(-1)[0]
    iB, ldB = spd_inverse(B_st)
    iBK = iB @ K0xz.reshape(P, T, M)
    Q = K0xz.transpose(-1, -2) @ iBK.reshape(P * T, M)
    W = K0zz + Q
    W = 0.5 * (W + W.transpose(-1, -2))
    iW, ldW = spd_inverse(W)
    logdet = -ldK + ldB.sum() + ldW
    tr = (iB * K0_st).sum() - (Q * iK).sum()
    return dict(K0xz=K0xz, iB=iB, iBK=iBK, iW=iW, logdet=logdet, tr=tr, M=M)


def _quad(c, y, P, T):
    y_st = y.reshape(P, T, 1)
    iBy = c["iB"] @ y_st
    q1 = (y_st * iBy).sum()
    p = c["K0xz"].transpose(-1, -2) @ iBy.reshape(P * T)
    return q1 - p @ (c["iW"] @ p)


def elbo(covar_module0, covar_module1, likelihood, train_xt, train_yt, z, P, T, eps):
    """log N(y | 0, K0xz K0zz^-1 K0zx + B) - 1/2 tr(...) of one latent dim (elbo_functions.py:36-84)."""
    c = _common(covar_module0, covar_module1, likelihood, train_xt, z, P, T, eps)
    y = train_yt.to(torch.float64)
    loglike = -0.5 * T * P * math.log(2 * math.pi) - 0.5 * (c["logdet"] + _quad(c, y, P, T))
    return loglike - 0.5 * c["tr"]


def deviance_upper_bound(covar_module0, covar_module1, likelihood, train_xt, m, log_v, z, P, T, eps):
    """DUBO of one latent dim from the variational mean / log-variance (elbo_functions.py:86-142)."""
    c = _common(covar_module0, covar_module1, likelihood, train_xt, z, P, T, eps)
    m = m.to(torch.float64)
    log_v = log_v.to(torch.float64)
    v = torch.exp(log_v)
    v_st = v.reshape(P, T)
    tr_iB_D = (torch.diagonal(c["iB"], dim1=-2, dim2=-1) * v_st).sum()
    Dh = (c["iBK"] * torch.sqrt(v_st)[:, :, None]).reshape(P * T, c["M"])
    tr2 = (c["iW"] * (Dh.transpose(0, 1) @ Dh)).sum()
    return 0.5 * ((tr_iB_D - tr2) + _quad(c, m, P, T) - P * T + c["logdet"] - log_v.sum() + c["tr"])


def validation_dubo(latent_dim, covar_module0, covar_module1, likelihood, train_xt, m, log_v, z, P, T, eps):
    """Sum over the latent dims of the DUBO with batched kernels (validation.py:8-68); m / log_v
    [N, L], z [L, M, Q].  Returns a [1] tensor like the reference."""
    from .kernels import kernel_spec_and_params
    spec0, p0 = kernel_spec_and_params(covar_module0)
    spec1, p1 = kernel_spec_and_params(covar_module1)
    L = int(latent_dim)
    nz = likelihood.noise_covar.noise.reshape(-1)
    total = torch.zeros(1, dtype=torch.float64, device=m.device)
    for i in range(L):
        k0 = _Fixed(spec0, p0[i:i + 1])
        k1 = _Fixed(spec1, p1[i:i + 1])
        lik = _Noise(nz[i if nz.numel() > 1 else 0])
        total = total + deviance_upper_bound(k0, k1, lik, train_xt, m[:, i], log_v[:, i], z[i], P, T, eps)
    return total


class _Lazy:
    def __init__(self, t):
        self.t = t

    def evaluate(self):
        return self.t


class _Fixed:
    """One latent dim's slice of a batched kernel (spec + [1, P] params)."""

    def __init__(self, spec, params):
        self.spec, self.params = spec, params

    def __call__(self, x1, x2):
        from .kernels import gram
        return _Lazy(gram(self.spec, self.params, x1, x2).reshape(*torch.broadcast_shapes(x1.shape[:-2], x2.shape[:-2]),
                                                                  x1.shape[-2], x2.shape[-2]))


class _Noise:
    def __init__(self, v):
        import types
        self.noise_covar = types.SimpleNamespace(noise=v.reshape(1))
