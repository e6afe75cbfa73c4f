"""GP-prior KL / ELBO terms with the reference's call surface (elbo_functions.py:8-307).

Each function takes the same arguments as its reference twin and returns autograd-attached
tensors; the arithmetic runs in the HIP library through a ``torch.autograd.Function`` whose
backward is the analytic adjoint (also HIP).  No PyTorch / CPU fallback exists.
"""
import torch

from . import _lib
from .kernels import kernel_spec_and_params

# Numerical failures (non-PD pivots) come back in a device ``info`` array.  With sync checks on
# (default, like torch.cholesky) every call synchronises and raises; benchmarks turn them off and
# call ``check_pending()`` once at the end.
_SYNC_CHECKS = True
_PENDING = []


def set_sync_checks(on):
    global _SYNC_CHECKS
    _SYNC_CHECKS = bool(on)


def _check_info(info, what):
    if _SYNC_CHECKS:
        bad = info.nonzero()
        if bad.numel():
            l = int(bad[0, 0])
            raise torch.linalg.LinAlgError(
                f"{what}: latent dim {l}: the leading minor of order {int(info[l])} is not positive-definite")
    else:
        _PENDING.append((info, what))


def check_pending():
    global _PENDING
    pend, _PENDING = _PENDING, []
    for info, what in pend:
        bad = info.nonzero()
        if bad.numel():
            l = int(bad[0, 0])
            raise torch.linalg.LinAlgError(f"{what}: latent dim {l}: leading minor {int(info[l])} not PD")


# ------------------------------------------------------------------------------------------
# Regime B: exact KL (elbo_functions.py:8-34), batched over latent dims
# ------------------------------------------------------------------------------------------
class _KLClosedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, params, noise, mu, logv, x, spec):
        lib = _lib.lib()
        n, L = mu.shape
        dev = mu.device
        x64 = x.detach().to(torch.float64).contiguous()
        p = params.detach().to(torch.float64).contiguous()
        nz = noise.detach().to(torch.float64).reshape(L).contiguous()
        mu64 = mu.detach().to(torch.float64).contiguous()
        lv64 = logv.detach().to(torch.float64).contiguous()
        ws = torch.empty(int(lib.lvae_kl_closed_workspace_size(n, L)), dtype=torch.uint8, device=dev)
        kl = torch.empty(L, dtype=torch.float64, device=dev)
        info = torch.empty(L, dtype=torch.int32, device=dev)
        rc = lib.lvae_kl_closed_fwd_f32(spec, _lib.ptr(x64), x64.shape[1], n, L, _lib.ptr(p), _lib.ptr(nz),
                                        _lib.ptr(mu64), _lib.ptr(lv64), L, _lib.ptr(kl), _lib.ptr(info),
                                        _lib.ptr(ws), 1, _lib.stream_ptr())
        _lib.check(rc, "kl_closed_fwd")
        _check_info(info, "KL_closed cholesky")
        ctx.save_for_backward(p, mu64, lv64, x64, ws)
        ctx.spec = spec
        ctx.in_dtypes = (params.dtype, noise.dtype, noise.shape, mu.dtype, logv.dtype)
        return kl

    @staticmethod
    def backward(ctx, gkl):
        lib = _lib.lib()
        p, mu64, lv64, x64, ws = ctx.saved_tensors
        n, L = mu64.shape
        g = gkl.detach().to(torch.float64).reshape(L).contiguous()
        dmu = torch.empty_like(mu64)
        dlv = torch.empty_like(lv64)
        dp = torch.empty_like(p)
        dnz = torch.empty(L, dtype=torch.float64, device=p.device)
        rc = lib.lvae_kl_closed_bwd_f32(ctx.spec, _lib.ptr(x64), x64.shape[1], n, L, _lib.ptr(p), _lib.ptr(mu64),
                                        _lib.ptr(lv64), L, _lib.ptr(g), _lib.ptr(dmu), _lib.ptr(dlv), _lib.ptr(dp),
                                        _lib.ptr(dnz), _lib.ptr(ws), _lib.stream_ptr())
        _lib.check(rc, "kl_closed_bwd")
        pd, nd, nshape, md, ld = ctx.in_dtypes
        return dp.to(pd), dnz.to(nd).reshape(nshape), dmu.to(md), dlv.to(ld), None, None


def _stack_modules(covar_modules):
    """One spec + [L, P] params from a batched module or a list of per-dim modules."""
    if isinstance(covar_modules, (list, tuple, torch.nn.ModuleList)):
        specs, ps = zip(*[kernel_spec_and_params(k) for k in covar_modules])
        return specs[0], torch.cat(ps, 0)
    return kernel_spec_and_params(covar_modules)


def _noise_vector(likelihoods, L):
    if isinstance(likelihoods, (list, tuple, torch.nn.ModuleList)):
        return torch.cat([lk.noise.reshape(-1) for lk in likelihoods]).reshape(L)
    nz = likelihoods.noise.reshape(-1)
    return nz.expand(L) if nz.numel() == 1 else nz


def KL_closed_batched(covar_modules, train_x, likelihoods, mu, log_var):
    """Per-dim exact KLs [L] for mu / log_var [N, L] (one batched HIP pass for all dims)."""
    spec, params = _stack_modules(covar_modules)
    L = mu.shape[1]
    if params.shape[0] != L:
        raise ValueError(f"kernel batch {params.shape[0]} != latent dims {L}")
    noise = _noise_vector(likelihoods, L).to(params.device)
    return _KLClosedFn.apply(params, noise, mu, log_var, train_x, spec)


def KL_closed(covar_module, train_x, likelihoods, data, mu, log_var):
    """Closed-form KL for one latent dim (elbo_functions.py:8-34); ``data`` only gives N."""
    n = data.shape[0]
    return KL_closed_batched(covar_module, train_x[:n], likelihoods, mu.reshape(n, 1), log_var.reshape(n, 1))[0]
