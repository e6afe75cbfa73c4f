"""Additive GP kernels with the reference's module surface (GP_model.py:31-236; kernel_gen.py:9-310).

Modules keep GP_model's class and parameter names (``_log_scale``, ``_log_lengthscale``, the
``min_log_*`` buffers, positivity ``exp(m + softplus(raw - m))``, m = -16) so state dicts carry over,
and the gpytorch call convention the reference's ELBO code relies on: ``k(x1, x2).evaluate()``
returns the dense Gram, batched right-aligned over ``batch_shape=[latent_dim]``.

The arithmetic never runs in PyTorch: a kernel compiles itself into an ``lvae_kernel_spec``
(component list) plus a ``[L, P]`` parameter matrix, and the Gram / its adjoint run in the HIP
library (``lvae_gram_f64`` / ``lvae_gram_bwd_f64``).  The ELBO functions consume the spec directly.
"""
import ctypes
import math

import torch
import torch.nn.functional as F
from torch import nn

from . import _lib

MIN_LOG = -16.0


def _positive(raw, min_log):
    return torch.exp(min_log + F.softplus(raw - min_log))


def _raw_from(value, min_log):
    return math.log(value - math.exp(min_log))


# ------------------------------------------------------------------------------------------
# factor kernels (no scale)
# ------------------------------------------------------------------------------------------
class _Factor(nn.Module):
    kind = None

    def factors(self):
        """[(kind, dim, module)] -- flattened product factors."""
        return [(self.kind, self.dim, self)]

    def factor_params(self):
        return []

    def factor_raw(self):
        """[(raw parameter, min_log buffer)] in factor_params order"""
        return []

    def forward(self, x1, x2):
        return Gram(_Scaled(self, None), x1, x2)


class BinKernel(_Factor):
    """1[x1_d + x2_d == 2] (GP_model.py:31-41; kernel_spec.py:9-23)."""
    kind = "bin"

    def __init__(self, dim):
        super().__init__()
        self.dim = dim


class CatKernel(_Factor):
    """1[x1_d == x2_d] (GP_model.py:43-53; kernel_spec.py:26-32)."""
    kind = "cat"

    def __init__(self, dim):
        super().__init__()
        self.dim = dim


class RbfKernel(_Factor):
    """exp(-(x1_d - x2_d)^2 / (2 l^2)), one lengthscale per latent dim (GP_model.py:55-85;
    init 2.5 as kernel_spec.py:58-69)."""
    kind = "rbf"

    def __init__(self, dim, latent_dim=1, lengthscale=2.5):
        super().__init__()
        self.dim = dim
        self.latent_dim = latent_dim
        self._log_lengthscale = nn.Parameter(torch.full((latent_dim,), _raw_from(lengthscale, MIN_LOG), dtype=torch.float64))
        self.register_buffer("min_log_lengthscale", torch.full((1,), MIN_LOG, dtype=torch.float64))

    @property
    def lengthscale(self):
        return _positive(self._log_lengthscale, self.min_log_lengthscale)

    @lengthscale.setter
    def lengthscale(self, value):
        with torch.no_grad():
            self._log_lengthscale.copy_(torch.log(torch.as_tensor(value, dtype=self._log_lengthscale.dtype)
                                                  - math.exp(MIN_LOG)))

    def factor_params(self):
        return [self.lengthscale]

    def factor_raw(self):
        return [(self._log_lengthscale, self.min_log_lengthscale)]


class PeriodicKernel(_Factor):
    """exp(-2 sin^2(pi |x1_d - x2_d| / p) / l^2).  EXTENSION (BASELINE config 5): not in the
    reference; parity unpinned."""
    kind = "per"

    def __init__(self, dim, latent_dim=1, lengthscale=1.0, period=4.0):
        super().__init__()
        self.dim = dim
        self.latent_dim = latent_dim
        self._log_lengthscale = nn.Parameter(torch.full((latent_dim,), _raw_from(lengthscale, MIN_LOG), dtype=torch.float64))
        self._log_period = nn.Parameter(torch.full((latent_dim,), _raw_from(period, MIN_LOG), dtype=torch.float64))
        self.register_buffer("min_log_lengthscale", torch.full((1,), MIN_LOG, dtype=torch.float64))

    @property
    def lengthscale(self):
        return _positive(self._log_lengthscale, self.min_log_lengthscale)

    @property
    def period(self):
        return _positive(self._log_period, self.min_log_lengthscale)

    def factor_params(self):
        return [self.lengthscale, self.period]

    def factor_raw(self):
        return [(self._log_lengthscale, self.min_log_lengthscale), (self._log_period, self.min_log_lengthscale)]


class LinearKernel(_Factor):
    """x1_d * x2_d (its variance is the enclosing ScaleKernel).  EXTENSION, parity unpinned."""
    kind = "lin"

    def __init__(self, dim):
        super().__init__()
        self.dim = dim


class ProductKernel(nn.Module):
    """k1 * k2 (GP_model.py:133-144)."""

    def __init__(self, kernel1, kernel2):
        super().__init__()
        self.k1 = kernel1
        self.k2 = kernel2

    def factors(self):
        return self.k1.factors() + self.k2.factors()

    def forward(self, x1, x2):
        return Gram(_Scaled(self, None), x1, x2)


class ScaleKernel(nn.Module):
    """s * k, one scale per latent dim, init ln 2 (GP_model.py:87-117)."""

    def __init__(self, kernel, latent_dim=1, scale=math.log(2)):
        super().__init__()
        self.latent_dim = latent_dim
        self.kernel = kernel
        self._log_scale = nn.Parameter(torch.full((latent_dim,), _raw_from(scale, MIN_LOG), dtype=torch.float64))
        self.register_buffer("min_log_scale", torch.full((1,), MIN_LOG, dtype=torch.float64))

    @property
    def scale(self):
        return _positive(self._log_scale, self.min_log_scale)

    @scale.setter
    def scale(self, value):
        with torch.no_grad():
            self._log_scale.copy_(torch.log(torch.as_tensor(value, dtype=self._log_scale.dtype)
                                            - math.exp(MIN_LOG)))

    def components(self):
        """[(factors, [param tensors])] for this single component."""
        facs = self.kernel.factors()
        params = [self.scale]
        for _, _, mod in facs:
            params += mod.factor_params()
        return [([(k, d) for k, d, _ in facs], params)]

    def raw_components(self):
        """[(factors, [(raw, min_log)])]: the same parameters, unconstrained"""
        facs = self.kernel.factors()
        refs = [(self._log_scale, self.min_log_scale)]
        for _, _, mod in facs:
            refs += mod.factor_raw()
        return [([(k, d) for k, d, _ in facs], refs)]

    def forward(self, x1, x2):
        return Gram(AdditiveKernel([self]), x1, x2)


class _Scaled:
    """An unscaled factor / product viewed as a one-component kernel with unit scale."""

    def __init__(self, mod, _):
        self.mod = mod

    def components(self):
        facs = self.mod.factors()
        one = None
        params = []
        for _, _, m in facs:
            params += m.factor_params()
        ld = params[0].shape[0] if params else 1
        dev = params[0].device if params else None
        one = torch.ones(ld, dtype=torch.float64, device=dev)
        return [([(k, d) for k, d, _ in facs], [one] + params)]

    def raw_components(self):
        refs = [None]  # the unit scale
        for _, _, m in self.mod.factors():
            refs += m.factor_raw()
        return [([(k, d) for k, d, _ in self.mod.factors()], refs)]

    @property
    def latent_dim(self):
        return getattr(self.mod, "latent_dim", 1)


class AdditiveKernel(nn.Module):
    """sum of ScaleKernels (GP_model.py:119-131)."""

    def __init__(self, kernels):
        super().__init__()
        self.kernels = nn.ModuleList(kernels)

    @property
    def latent_dim(self):
        return self.kernels[0].latent_dim if len(self.kernels) else 1

    def components(self):
        out = []
        for k in self.kernels:
            out += k.components()
        return out

    def raw_components(self):
        out = []
        for k in self.kernels:
            out += k.raw_components()
        return out

    def spec(self):
        comps = self.components()
        return _lib.make_spec([c for c, _ in comps])

    def param_matrix(self):
        """[L, P] constrained parameters (differentiable wrt the raw parameters)."""
        cols = []
        for _, ps in self.components():
            cols += ps
        return torch.stack([c.to(torch.float64) for c in cols], dim=-1)

    def forward(self, x1, x2):
        return Gram(self, x1, x2)

    def __add__(self, other):
        return AdditiveKernel(list(self.kernels) + list(other.kernels))


class _ParamPackFn(torch.autograd.Function):
    """[L, P] = exp(m + softplus(raw - m)) of the raw [L] fp64 tensors into their columns (1 elsewhere), one
    HIP launch each way (glue.hip) instead of the stack / transform / transpose chain."""

    @staticmethod
    def forward(ctx, meta, *raws):
        lib = _lib.lib()
        cols, mlogs, L, P = meta
        n = len(raws)
        out = torch.empty(L, P, dtype=torch.float64, device=raws[0].device)
        ca = (ctypes.c_int32 * n)(*cols)
        ra = (ctypes.c_void_p * n)(*[r.data_ptr() for r in raws])
        ma = (ctypes.c_void_p * n)(*[m.data_ptr() for m in mlogs])
        _lib.check(lib.lvae_param_pack_fwd_f64(n, L, P, ca, ra, ma, _lib.ptr(out), _lib.stream_ptr()), "param_pack_fwd")
        ctx.meta = meta
        ctx.save_for_backward(*raws)
        return out

    @staticmethod
    def backward(ctx, g):
        lib = _lib.lib()
        raws = ctx.saved_tensors
        cols, mlogs, L, P = ctx.meta
        n = len(raws)
        g = g.to(torch.float64)
        grad = torch.empty(n, L, dtype=torch.float64, device=g.device)
        ca = (ctypes.c_int32 * n)(*cols)
        ra = (ctypes.c_void_p * n)(*[r.data_ptr() for r in raws])
        ma = (ctypes.c_void_p * n)(*[m.data_ptr() for m in mlogs])
        _lib.check(lib.lvae_param_pack_bwd_f64(n, L, P, ca, ra, ma, _lib.ptr(g), g.stride(0), g.stride(1),
                                               _lib.ptr(grad), _lib.stream_ptr()), "param_pack_bwd")
        return (None,) + tuple(grad[k] for k in range(n))


def kernel_spec_and_params(kernel):
    """(KernelSpec, [L, P] parameter matrix) of an AdditiveKernel / ScaleKernel.

    The positivity transform exp(m + softplus(raw - m)) runs ONCE on the stacked raw parameters
    (a handful of kernels forward and backward) instead of once per parameter tensor: the step is
    launch-bound at the Hensman sizes, where the per-parameter form cost ~40 launches."""
    comps = kernel.raw_components()
    spec = _lib.make_spec([c for c, _ in comps])
    refs = [r for _, rs in comps for r in rs]
    raws = [r for r in refs if r is not None]
    if not raws:
        return spec, torch.ones(1, len(refs), dtype=torch.float64)
    L = raws[0][0].shape[0]
    if (len(raws) <= 64 and len(refs) <= 64 and
            all(r.is_cuda and r.dtype == torch.float64 and r.dim() == 1 and r.shape[0] == L and r.is_contiguous()
                and m.is_cuda and m.dtype == torch.float64 for r, m in raws)):
        cols = [j for j, r in enumerate(refs) if r is not None]
        meta = (cols, [m for _, m in raws], L, len(refs))
        return spec, _ParamPackFn.apply(meta, *[r for r, _ in raws])  # (glue.hip: one launch each way)
    R = torch.stack([r[0] for r in raws], 0).to(torch.float64)          # [P', L]
    m = torch.cat([r[1] for r in raws]).to(torch.float64).unsqueeze(1)  # [P', 1]
    C = torch.exp(m + F.softplus(R - m))
    if len(raws) == len(refs):
        return spec, C.t()
    one = torch.ones(L, dtype=torch.float64, device=R.device)
    cols, j = [], 0
    for r in refs:
        if r is None:
            cols.append(one)
        else:
            cols.append(C[j])
            j += 1
    return spec, torch.stack(cols, dim=-1)


# ------------------------------------------------------------------------------------------
# lazy Gram with gpytorch batch semantics, evaluated by the HIP library
# ------------------------------------------------------------------------------------------
class Gram:
    """``covar_module(x1, x2)``: ``.evaluate()`` gives the dense fp64 Gram.

    Batch rule (gpytorch, right-aligned ``batch_shape=[L]``): with L > 1 the output batch shape is
    broadcast(x1.shape[:-2], x2.shape[:-2], [L]); with L == 1 (a per-dim kernel) the parameters are
    scalars and the output batch shape is broadcast(x1.shape[:-2], x2.shape[:-2])."""

    def __init__(self, kernel, x1, x2):
        self.kernel, self.x1, self.x2 = kernel, x1, x2

    def evaluate(self):
        spec, params = kernel_spec_and_params(self.kernel)
        return gram(spec, params, self.x1, self.x2)

    to_dense = evaluate


def gram(spec, params, x1, x2, diag=None):
    """Dense Gram (+ diag[l] on the diagonal) through the HIP library, differentiable wrt params/diag."""
    return _GramFn.apply(params, diag, x1, x2, spec)


def _batch_layout(params, x1, x2):
    L = params.shape[0]
    b1, b2 = x1.shape[:-2], x2.shape[:-2]
    if L > 1:
        bshape = torch.broadcast_shapes(b1, b2, (L,))
    else:
        bshape = torch.broadcast_shapes(b1, b2)
    lead = bshape[:-1] if (L > 1) else bshape
    nb = int(torch.tensor(lead).prod().item()) if len(lead) else 1
    return bshape, nb, L


def _expand(x, bshape, nb, L, batched):
    full = tuple(bshape) + tuple(x.shape[-2:])
    xe = x.to(torch.float64).expand(full)
    if batched:
        xe = xe.reshape((nb, L) + tuple(x.shape[-2:]))
    else:
        xe = xe.reshape((nb, 1) + tuple(x.shape[-2:]))
    if xe.stride(-1) != 1:
        xe = xe.contiguous()
    return xe


class _GramFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, params, diag, x1, x2, spec):
        lib = _lib.lib()
        bshape, nb, L = _batch_layout(params, x1, x2)
        batched = L > 1
        x1e = _expand(x1.detach(), bshape, nb, L, batched)
        x2e = _expand(x2.detach(), bshape, nb, L, batched)
        n1, n2 = x1.shape[-2], x2.shape[-2]
        p = params.detach().contiguous()
        out = torch.empty((nb, L, n1, n2), dtype=torch.float64, device=x1.device)
        dg = None if diag is None else diag.detach().reshape(L).to(torch.float64).contiguous()
        rc = lib.lvae_gram_f64(spec, _lib.xview(x1e, x1e.stride(0), x1e.stride(1)),
                               _lib.xview(x2e, x2e.stride(0), x2e.stride(1)), nb, L, n1, n2, _lib.ptr(p),
                               _lib.ptr(dg), _lib.ptr(out), out.stride(0), out.stride(1), out.stride(2),
                               _lib.stream_ptr())
        _lib.check(rc, "gram")
        ctx.save_for_backward(p, x1e, x2e)
        ctx.spec, ctx.nb, ctx.L, ctx.has_diag = spec, nb, L, diag is not None
        ctx.diag_shape = None if diag is None else diag.shape
        return out.reshape(tuple(bshape) + (n1, n2))

    @staticmethod
    def backward(ctx, g):
        lib = _lib.lib()
        p, x1e, x2e = ctx.saved_tensors
        nb, L = ctx.nb, ctx.L
        n1, n2 = x1e.shape[-2], x2e.shape[-2]
        G = g.reshape(nb, L, n1, n2).to(torch.float64).contiguous()
        dp = torch.zeros_like(p)
        dd = torch.zeros(L, dtype=torch.float64, device=p.device) if ctx.has_diag else None
        ws = torch.empty(int(lib.lvae_gram_bwd_workspace_size(nb, L, n1, n2)), dtype=torch.uint8, device=p.device)
        rc = lib.lvae_gram_bwd_f64(ctx.spec, _lib.xview(x1e, x1e.stride(0), x1e.stride(1)),
                                   _lib.xview(x2e, x2e.stride(0), x2e.stride(1)), nb, L, n1, n2, _lib.ptr(p),
                                   _lib.ptr(G), G.stride(0), G.stride(1), G.stride(2), _lib.ptr(dp), _lib.ptr(dd),
                                   _lib.ptr(ws), _lib.stream_ptr())
        _lib.check(rc, "gram_bwd")
        ddiag = None if dd is None else dd.reshape(ctx.diag_shape)
        return dp, ddiag, None, None, None


# ------------------------------------------------------------------------------------------
# builders from the config lists
# ------------------------------------------------------------------------------------------
def _masked(factor, idx, missing, covariate_missing_val):
    if idx in missing:
        dm = covariate_missing_val[missing.index(idx)]
        return ProductKernel(factor, BinKernel(dm["mask"]))
    return factor


def generate_kernel_batched(latent_dim, cat_kernel, bin_kernel, sqexp_kernel, cat_int_kernel, bin_int_kernel,
                            covariate_missing_val, id_covariate):
    """(non-id, id) AdditiveKernels batched over latent_dim (GP_model.py:146-236 component order;
    kernel_gen.py:199-310 is the gpytorch twin -- its non-id Cat branch NameError at :242 is not
    reproduced)."""
    missing = [d["covariate"] for d in covariate_missing_val]
    k0, k1 = [], []
    L = latent_dim
    m = lambda f, i: _masked(f, i, missing, covariate_missing_val)
    for idx in cat_kernel:
        (k1 if idx == id_covariate else k0).append(ScaleKernel(m(CatKernel(idx), idx), L))
    for idx in sqexp_kernel:
        k0.append(ScaleKernel(m(RbfKernel(idx, L), idx), L))
    for idx in bin_kernel:
        k0.append(ScaleKernel(m(BinKernel(idx), idx), L))
    for di in cat_int_kernel:
        c, x = di["cat_covariate"], di["cont_covariate"]
        comp = ScaleKernel(ProductKernel(m(CatKernel(c), c), m(RbfKernel(x, L), x)), L)
        (k1 if c == id_covariate else k0).append(comp)
    for di in bin_int_kernel:
        b, x = di["bin_covariate"], di["cont_covariate"]
        k0.append(ScaleKernel(ProductKernel(m(BinKernel(b), b), m(RbfKernel(x, L), x)), L))
    return AdditiveKernel(k0), AdditiveKernel(k1)


def generate_kernel(cat_kernel, bin_kernel, sqexp_kernel, cat_int_kernel, bin_int_kernel, covariate_missing_val,
                    latent_dim=1):
    """The full additive kernel (kernel_gen.py:9-94 component order), one module; latent_dim > 1
    batches the L per-dim kernels of the reference's closed-form path into one module."""
    missing = [d["covariate"] for d in covariate_missing_val]
    L = latent_dim
    m = lambda f, i: _masked(f, i, missing, covariate_missing_val)
    ks = []
    for idx in cat_kernel:
        ks.append(ScaleKernel(m(CatKernel(idx), idx), L))
    for idx in sqexp_kernel:
        ks.append(ScaleKernel(m(RbfKernel(idx, L), idx), L))
    for idx in bin_kernel:
        ks.append(ScaleKernel(m(BinKernel(idx), idx), L))
    for di in cat_int_kernel:
        c, x = di["cat_covariate"], di["cont_covariate"]
        ks.append(ScaleKernel(ProductKernel(m(CatKernel(c), c), m(RbfKernel(x, L), x)), L))
    for di in bin_int_kernel:
        b, x = di["bin_covariate"], di["cont_covariate"]
        ks.append(ScaleKernel(ProductKernel(m(BinKernel(b), b), m(RbfKernel(x, L), x)), L))
    return AdditiveKernel(ks)


def generate_kernel_approx(cat_kernel, bin_kernel, sqexp_kernel, cat_int_kernel, bin_int_kernel,
                           covariate_missing_val, id_covariate):
    """Per-dim (non-id, id) pair (kernel_gen.py:97-197)."""
    return generate_kernel_batched(1, cat_kernel, bin_kernel, sqexp_kernel, cat_int_kernel, bin_int_kernel,
                                   covariate_missing_val, id_covariate)
