"""GP-prior KL / ELBO terms with the reference's call surface (elbo_functions.py:8-307).

Each function takes the same arguments as its reference twin and returns autograd-attached
tensors; the arithmetic runs in the HIP library through a ``torch.autograd.Function`` whose
backward is the analytic adjoint (also HIP).  No PyTorch / CPU fallback exists.
"""
import contextlib
import os

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


def take_pending():
    """The deferred info checks recorded since the last check (and forget them) -- a captured graph
    keeps these: its replays rewrite the same info tensors (steps.GraphedStep)."""
    global _PENDING
    pend, _PENDING = _PENDING, []
    return pend


def check_pending(pend=None):
    for info, what in (take_pending() if pend is None else pend):
        bad = info.nonzero()
        if bad.numel():
            l = int(bad[0, 0])
            raise torch.linalg.LinAlgError(f"{what}: latent dim {l}: leading minor {int(info[l])} not PD")


# ------------------------------------------------------------------------------------------
# Regime B: exact KL (elbo_functions.py:8-34), batched over latent dims
# ------------------------------------------------------------------------------------------
# The factor's host-side enqueue (Gram, then per block column of the blocked Cholesky ~8 HIP calls across
# two streams: ~1-2 ms of host time) runs on a worker thread (ctypes releases the GIL), so that the caller's
# thread goes on enqueueing the ConvVAE meanwhile -- at a few latent dims per GPU the step is otherwise
# host-bound.  Not under graph capture.  LVAE_ASYNC_FACTOR=0 enqueues in the caller's thread.
_ASYNC_FACTOR = os.environ.get("LVAE_ASYNC_FACTOR", "1") != "0"
_FACTOR_POOL = None


def _factor_pool():
    global _FACTOR_POOL
    if _FACTOR_POOL is None:
        from concurrent.futures import ThreadPoolExecutor
        _FACTOR_POOL = ThreadPoolExecutor(max_workers=1, thread_name_prefix="lvae-factor")
    return _FACTOR_POOL


class KLFactor:
    """K^-1 and log|K| of the L covariances, computed ahead of (mu, logvar) on a caller stream
    (lvae_kl_closed_factor_f32): kl_closed_prefactor launches it, KL_closed_batched(..., factor=)
    waits for it and finishes with lvae_kl_closed_reduce_f32.  Single use: the reduce writes the B
    planes over the factor's Gram buffer and the backward writes S over its Y^T planes, so a second
    KL_closed_batched(..., factor=) on the same factor would read overwritten operands -- it raises."""

    def __init__(self, spec, params, noise, x, stream):
        lib = _lib.lib()
        self.spec, self.params, self.noise = spec, params, noise
        L = params.shape[0]
        n = x.shape[0]
        dev = params.device
        main = torch.cuda.current_stream(dev)
        stream.wait_stream(main)
        with torch.cuda.stream(stream):
            self.x64 = x.detach().to(torch.float64).contiguous()
            self.p = params.detach().to(torch.float64).contiguous()
            self.nz = noise.detach().to(torch.float64).reshape(L).contiguous()
            self.ws = torch.empty(int(lib.lvae_kl_closed_workspace_size(n, L)), dtype=torch.uint8, device=dev)
            self.info = torch.empty(L, dtype=torch.int32, device=dev)
        args = (spec, _lib.ptr(self.x64), self.x64.shape[1], n, L, _lib.ptr(self.p), _lib.ptr(self.nz),
                _lib.ptr(self.info), _lib.ptr(self.ws), _lib.ctypes.c_void_p(stream.cuda_stream))
        self._fut = None
        if _ASYNC_FACTOR and not torch.cuda.is_current_stream_capturing():
            dix = dev.index if dev.index is not None else torch.cuda.current_device()

            def enqueue():
                torch.cuda.set_device(dix)  # (the worker thread's HIP device: the library keys its side stream on it)
                return lib.lvae_kl_closed_factor_f32(*args)
            self._fut = _factor_pool().submit(enqueue)
        else:
            _lib.check(lib.lvae_kl_closed_factor_f32(*args), "kl_closed_factor")
        self.stream = stream
        self.n, self.L = n, L
        self.consumed = False

    def wait_enqueued(self):
        """Block until the factor's launches are all enqueued (call before enqueueing anything else on its
        stream, so that nothing lands between them)."""
        if self._fut is not None:
            rc = self._fut.result()
            self._fut = None
            _lib.check(rc, "kl_closed_factor")

    def join(self):
        """Make the current stream wait for the factorisation (and own its buffers)."""
        self.wait_enqueued()
        cur = torch.cuda.current_stream(self.ws.device)
        cur.wait_stream(self.stream)
        for t in (self.ws, self.info, self.x64, self.p, self.nz):
            t.record_stream(cur)


def kl_closed_prefactor(covar_modules, train_x, likelihoods, L, stream):
    """Launch the (mu, logvar)-independent part of KL_closed_batched -- the Gram and its blocked
    Cholesky inverse -- on ``stream`` now; pass the result as KL_closed_batched(..., factor=)."""
    spec, params = _stack_modules(covar_modules)
    if params.shape[0] != L:
        raise ValueError(f"kernel batch {params.shape[0]} != latent dims {L}")
    noise = _noise_vector(likelihoods, L).to(params.device)
    return KLFactor(spec, params, noise, train_x, stream)


class _KLState:
    """What the hyper-parameter half of the backward needs from the forward (filled by _KLClosedFn)."""
    ws = p = x64 = spec = None
    n = L = 0


_refine_log = None  # a list while kl_closed_refine_log() is active


@contextlib.contextmanager
def kl_closed_refine_log():
    """Yields a list that gets, per KL_closed forward inside the block, the fp64 diag(K^-1) refinement's
    gate (kl_refine.hip): (est [L] fp64 = (sum of the scales + noise) max (K^-1)_ii, the proxy of the fp32 inverse's
    diagonal error; flag [L] int32, 1 where diag K^-1 was refined in fp64).  Device tensors, filled in
    stream order."""
    global _refine_log
    prev, _refine_log = _refine_log, []
    try:
        yield _refine_log
    finally:
        _refine_log = prev


_hyper_log = None  # a list while kl_closed_hyper_log() is active


@contextlib.contextmanager
def kl_closed_hyper_log():
    """Yields a list that gets, per KL_closed forward inside the block, the device int32 [1]: 1 when the
    backward's hyper-parameter half takes the binned route (kl_hyper.hip: no S GEMM), 0 for the S GEMM +
    Gram adjoint (lvae_kl_closed_hyper_state)."""
    global _hyper_log
    prev, _hyper_log = _hyper_log, []
    try:
        yield _hyper_log
    finally:
        _hyper_log = prev


def _log_refine(lib, ws, n, L, dev):
    est = torch.zeros(L, dtype=torch.float64, device=dev)
    flag = torch.zeros(L, dtype=torch.int32, device=dev)
    _lib.check(lib.lvae_kl_closed_refine_state(n, L, _lib.ptr(ws), _lib.ptr(est), _lib.ptr(flag), _lib.stream_ptr()),
               "kl_closed_refine_state")
    _refine_log.append((est, flag))


class _KLHyperFn(torch.autograd.Function):
    """A zero-valued [L] term carrying d kl / d (params, noise) (lvae_kl_closed_bwd_hyper_f32: the S GEMM
    and the Gram adjoint, ~all of the KL backward's time) as a node of its own.  Created before the
    (mu, logvar) node, it runs after it in the backward (autograd runs later-created ready nodes first),
    so the encoder's backward gets d kl / d (mu, logvar) from the cheap elementwise half and runs on its
    stream beside this one's GEMMs."""

    @staticmethod
    def forward(ctx, params, noise, state, L):
        ctx.state = state
        ctx.in_dtypes = (params.dtype, noise.dtype, noise.shape)
        return torch.zeros(L, dtype=torch.float64, device=params.device)

    @staticmethod
    def backward(ctx, gkl):
        lib = _lib.lib()
        st = ctx.state
        if st.ws is None:
            raise RuntimeError("KL_closed: the hyper-parameter backward ran twice (its workspace is released "
                               "after the first; use retain_graph only for the (mu, logvar) half)")
        g = gkl.detach().to(torch.float64).reshape(st.L).contiguous()
        dp = torch.empty_like(st.p)
        dnz = torch.empty(st.L, dtype=torch.float64, device=st.p.device)
        rc = lib.lvae_kl_closed_bwd_hyper_f32(st.spec, _lib.ptr(st.x64), st.x64.shape[1], st.n, st.L, _lib.ptr(st.p),
                                              _lib.ptr(g), _lib.ptr(dp), _lib.ptr(dnz), _lib.ptr(st.ws),
                                              _lib.stream_ptr())
        _lib.check(rc, "kl_closed_bwd_hyper")
        # the backward consumed the workspace (S over the Y^T planes): release it now rather than with the
        # graph (GBs at the headline shape); the stream order keeps it alive for the kernels just queued
        st.ws = st.p = st.x64 = None
        pd, nd, nshape = ctx.in_dtypes
        return dp.to(pd), dnz.to(nd).reshape(nshape), None, None


class _KLClosedFn(torch.autograd.Function):
    """kl [L] from (mu, logvar) (and the detached hyper-parameters); backward: d kl / d (mu, logvar)
    only (lvae_kl_closed_bwd_latent_f32), the hyper-parameter half is _KLHyperFn's."""

    @staticmethod
    def forward(ctx, params, noise, mu, logv, x, spec, factor, state, need_bwd):
        lib = _lib.lib()
        n, L = mu.shape
        dev = mu.device
        mu64 = mu.detach().to(torch.float64).contiguous()
        lv64 = logv.detach().to(torch.float64).contiguous()
        kl = torch.empty(L, dtype=torch.float64, device=dev)
        if factor is not None:
            if factor.n != n or factor.L != L:
                raise ValueError(f"factor is for n={factor.n}, L={factor.L}; got n={n}, L={L}")
            factor.join()
            x64, p, ws, info = factor.x64, factor.p, factor.ws, factor.info
            rc = lib.lvae_kl_closed_reduce_f32(spec, _lib.ptr(x64), x64.shape[1], n, L, _lib.ptr(p), _lib.ptr(factor.nz),
                                               _lib.ptr(mu64), _lib.ptr(lv64), L, _lib.ptr(kl), _lib.ptr(ws),
                                               need_bwd, _lib.stream_ptr())
            _lib.check(rc, "kl_closed_reduce")
        else:
            x64 = x.detach().to(torch.float64).contiguous()
            p = params.detach().to(torch.float64).contiguous()
            nz = noise.detach().to(torch.float64).reshape(L).contiguous()
            ws = torch.empty(int(lib.lvae_kl_closed_workspace_size(n, L)), dtype=torch.uint8, device=dev)
            info = torch.empty(L, dtype=torch.int32, device=dev)
            rc = lib.lvae_kl_closed_fwd_f32(spec, _lib.ptr(x64), x64.shape[1], n, L, _lib.ptr(p), _lib.ptr(nz),
                                            _lib.ptr(mu64), _lib.ptr(lv64), L, _lib.ptr(kl), _lib.ptr(info),
                                            _lib.ptr(ws), need_bwd, _lib.stream_ptr())
            _lib.check(rc, "kl_closed_fwd")
        _check_info(info, "KL_closed cholesky")
        if _refine_log is not None:
            _log_refine(lib, ws, n, L, dev)
        if _hyper_log is not None:
            on = torch.zeros(1, dtype=torch.int32, device=dev)
            _lib.check(lib.lvae_kl_closed_hyper_state(n, L, _lib.ptr(ws), _lib.ptr(on), _lib.stream_ptr()),
                       "kl_closed_hyper_state")
            _hyper_log.append(on)
        state.ws, state.p, state.x64, state.spec, state.n, state.L = ws, p, x64, spec, n, L
        ctx.save_for_backward(lv64, ws)
        ctx.in_dtypes = (mu.dtype, logv.dtype)
        return kl

    @staticmethod
    def backward(ctx, gkl):
        lib = _lib.lib()
        lv64, ws = ctx.saved_tensors
        n, L = lv64.shape
        g = gkl.detach().to(torch.float64).reshape(L).contiguous()
        dmu = torch.empty_like(lv64)
        dlv = torch.empty_like(lv64)
        rc = lib.lvae_kl_closed_bwd_latent_f32(n, L, _lib.ptr(lv64), L, _lib.ptr(g), _lib.ptr(dmu), _lib.ptr(dlv),
                                               _lib.ptr(ws), _lib.stream_ptr())
        _lib.check(rc, "kl_closed_bwd_latent")
        md, ld = ctx.in_dtypes
        return None, None, dmu.to(md), dlv.to(ld), None, None, None, None, None


def _kl_closed_apply(params, noise, mu, log_var, train_x, spec, factor):
    L = mu.shape[1]
    need_bwd = int(torch.is_grad_enabled() and any(t.requires_grad for t in (params, noise, mu, log_var)))
    state = _KLState()
    hyper = None
    if torch.is_grad_enabled() and (params.requires_grad or noise.requires_grad):
        hyper = _KLHyperFn.apply(params, noise, state, L)  # (first: its node runs after the (mu, logvar) one)
    kl = _KLClosedFn.apply(params.detach(), noise.detach(), mu, log_var, train_x, spec, factor, state, need_bwd)
    return kl if hyper is None else kl + hyper


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


def KL_closed_batched(covar_modules, train_x, likelihoods, mu, log_var, factor=None):
    """Per-dim exact KLs [L] for mu / log_var [N, L] (one batched HIP pass for all dims).
    ``factor``: a kl_closed_prefactor result for the same modules / covariates, whose Gram and
    inverse were launched ahead (its hyperparameters are the ones differentiated)."""
    L = mu.shape[1]
    if factor is not None:
        if factor.consumed:
            raise RuntimeError("KL_closed_batched: this KLFactor was already used (one reduce per factor: "
                               "launch a new kl_closed_prefactor for each step)")
        factor.consumed = True
        return _kl_closed_apply(factor.params, factor.noise, mu, log_var, train_x, factor.spec, factor)
    spec, params = _stack_modules(covar_modules)
    if params.shape[0] != L:
        raise ValueError(f"kernel batch {params.shape[0]} != latent dims {L}")
    noise = _noise_vector(likelihoods, L).to(params.device)
    return _kl_closed_apply(params, noise, mu, log_var, train_x, spec, None)


def KL_closed(covar_module, train_x, likelihoods, data, mu, log_var):
    """Closed-form KL for one latent dim (elbo_functions.py:8-34); ``data`` only gives N."""
    n = data.shape[0]
    return KL_closed_batched(covar_module, train_x[:n], likelihoods, mu.reshape(n, 1), log_var.reshape(n, 1))[0]


# ------------------------------------------------------------------------------------------
# Regime A: Hensman mini-batch KL upper bound (elbo_functions.py:144-216), fp64
# ------------------------------------------------------------------------------------------
class _HensmanPre:
    """The fp64 operands, workspace and outputs of one Hensman forward, and (launch) its part 1 -- the
    Grams, inverses and products that need neither mu nor logv (lvae_hensman_fwd_part_f64)."""

    def __init__(self, params0, params1, noise, m, H, x, z, spec0, spec1, dims, want_ng, dev):
        lib = _lib.lib()
        f64 = lambda t: t.detach().to(torch.float64).contiguous()
        self.p0, self.p1, self.nz = f64(params0), f64(params1), f64(noise).reshape(-1)
        self.m64, self.H64, self.x64, self.z64 = f64(m), f64(H), f64(x), f64(z)
        L, M = dims.L, dims.M
        self.ws = torch.empty(int(lib.lvae_hensman_workspace_size(dims)), dtype=torch.uint8, device=dev)
        self.kld = torch.empty((), dtype=torch.float64, device=dev)
        self.gm = torch.empty(L, M, 1, dtype=torch.float64, device=dev) if want_ng else None
        self.gH = torch.empty(L, M, M, dtype=torch.float64, device=dev) if want_ng else None
        self.info = torch.empty(L, dtype=torch.int32, device=dev)
        self.spec0, self.spec1, self.dims = spec0, spec1, dims

    def run(self, part, mu64=None, lv64=None):
        rc = _lib.lib().lvae_hensman_fwd_part_f64(
            part, self.spec0, self.spec1, self.dims, _lib.ptr(self.x64), _lib.ptr(self.z64), _lib.ptr(self.m64),
            _lib.ptr(self.H64), _lib.ptr(mu64), _lib.ptr(lv64), _lib.ptr(self.p0), _lib.ptr(self.p1),
            _lib.ptr(self.nz), _lib.ptr(self.kld), _lib.ptr(self.gm), _lib.ptr(self.gH), _lib.ptr(self.info),
            _lib.ptr(self.ws), _lib.stream_ptr())
        _lib.check(rc, "hensman_fwd")


class HensmanPrior:
    """minibatch_KLD_upper_bound's (mu, logv)-independent part -- the Grams, the K0zz / B_p / H inverses
    and the products of elbo_functions.py:171-186, 208-214 that do not read the batch's latents --
    launched now, on ``stream`` (default: the current stream; the hyper-parameter transforms always run
    on the current stream, so their backward stays there), so that the ConvVAE can run beside it; pass it
    as minibatch_KLD_upper_bound(..., prior=) (single use; that call joins the current stream to it)."""

    def __init__(self, covar_module0, covar_module1, likelihood, latent_dim, m, H, train_xt, z, P_tot, P_batch, T,
                 natural_gradient, eps, ng_prior_share=1.0, stream=None):
        a = _hensman_args(covar_module0, covar_module1, likelihood, latent_dim, H, train_xt, z, P_tot, P_batch, T,
                          natural_gradient, eps, ng_prior_share)
        self.params0, self.params1, self.noise, self.zz, self.spec0, self.spec1, self.dims = a
        self.m, self.H, self.x = m, H, train_xt
        self.want_ng = bool(natural_gradient)
        self.stream = stream
        if stream is not None:
            stream.wait_stream(torch.cuda.current_stream(train_xt.device))
        with torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext():
            self.pre = _HensmanPre(self.params0, self.params1, self.noise, m, H, train_xt, self.zz, self.spec0,
                                   self.spec1, self.dims, self.want_ng, train_xt.device)
            self.pre.run(1)
        self.consumed = False

    def join(self):
        """Make the current stream wait for part 1 (and own its buffers)."""
        if self.stream is None:
            return
        cur = torch.cuda.current_stream(self.pre.ws.device)
        cur.wait_stream(self.stream)
        pre = self.pre
        for t in (pre.p0, pre.p1, pre.nz, pre.m64, pre.H64, pre.x64, pre.z64, pre.ws, pre.kld, pre.gm, pre.gH,
                  pre.info):
            if t is not None:
                t.record_stream(cur)


class _HensmanFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, params0, params1, noise, mu, logv, m, H, x, z, spec0, spec1, dims, want_ng, pre=None):
        dev = mu.device
        f64 = lambda t: t.detach().to(torch.float64).contiguous()
        mu64, lv64 = f64(mu), f64(logv)
        L, M = dims.L, dims.M
        if pre is None:
            pre = _HensmanPre(params0, params1, noise, m, H, x, z, spec0, spec1, dims, want_ng, dev)
            pre.run(0, mu64, lv64)
        else:  # part 1 ran ahead (HensmanPrior)
            pre.run(2, mu64, lv64)
        lib = _lib.lib()
        p0, p1, nz, m64, H64, x64, z64, ws = pre.p0, pre.p1, pre.nz, pre.m64, pre.H64, pre.x64, pre.z64, pre.ws
        kld, gm, gH, info = pre.kld, pre.gm, pre.gH, pre.info
        _check_info(info, "minibatch_KLD_upper_bound cholesky (10000+col: K0zz, 20000+col: B_st, 30000+col: H)")
        ctx.save_for_backward(p0, p1, nz, mu64, lv64, m64, H64, x64, z64, ws)
        ctx.spec0, ctx.spec1, ctx.dims = spec0, spec1, dims
        ctx.dtypes = (params0.dtype, params1.dtype, noise.dtype, noise.shape, mu.dtype, logv.dtype, m.dtype, H.dtype)
        if want_ng:
            # H^-1 stays in the workspace: the natural-gradient update reuses it while H is unchanged
            off = int(lib.lvae_hensman_iH_offset(dims))
            gH._lvae_iH = (ws[off:off + L * M * M * 8].view(torch.float64).view(L, M, M), H, H._version)
            ctx.mark_non_differentiable(gm, gH)
            return kld, gm, gH
        return kld, None, None

    @staticmethod
    def backward(ctx, gkld, _gm=None, _gH=None):
        lib = _lib.lib()
        p0, p1, nz, mu64, lv64, m64, H64, x64, z64, ws = ctx.saved_tensors
        d = ctx.dims
        g = gkld.detach().to(torch.float64).reshape(1).contiguous()
        dmu, dlv = torch.empty_like(mu64), torch.empty_like(lv64)
        dp0, dp1 = torch.empty_like(p0), torch.empty_like(p1)
        dnz = torch.empty_like(nz)
        adam = not d.natural_gradient
        dm = torch.empty_like(m64) if adam else None
        dH = torch.empty_like(H64) if adam else None
        rc = lib.lvae_hensman_bwd_f64(ctx.spec0, ctx.spec1, d, _lib.ptr(x64), _lib.ptr(z64), _lib.ptr(m64),
                                      _lib.ptr(H64), _lib.ptr(mu64), _lib.ptr(lv64), _lib.ptr(p0), _lib.ptr(p1),
                                      _lib.ptr(nz), _lib.ptr(g), _lib.ptr(dmu), _lib.ptr(dlv), _lib.ptr(dp0),
                                      _lib.ptr(dp1), _lib.ptr(dnz), _lib.ptr(dm), _lib.ptr(dH), _lib.ptr(ws),
                                      _lib.stream_ptr())
        _lib.check(rc, "hensman_bwd")
        t0, t1, tn, nshape, tmu, tlv, tm, tH = ctx.dtypes
        return (dp0.to(t0), dp1.to(t1), dnz.to(tn).reshape(nshape), dmu.to(tmu), dlv.to(tlv),
                None if dm is None else dm.to(tm), None if dH is None else dH.to(tH),
                None, None, None, None, None, None, None)


def minibatch_KLD_upper_bound(covar_module0, covar_module1, likelihood, latent_dim, m, H, train_xt, mu, log_v, z,
                              P_tot, P_batch, T, natural_gradient, eps, ng_prior_share=1.0, prior=None):
    """Unbiased mini-batch estimate of the KL upper bound and (natural_gradient) its natural-gradient
    directions wrt (m, H) -- same signature and return as elbo_functions.py:144-216.

    ng_prior_share (extension): weight of the data-independent part of grad_m / grad_H; 1/world
    under data parallelism so that the SUM over ranks equals the union batch's directions.
    prior (extension): a HensmanPrior of the same arguments, launched ahead (its part 1 is not redone)."""
    if prior is not None:
        if prior.consumed:
            raise RuntimeError("minibatch_KLD_upper_bound: this HensmanPrior was already used")
        prior.consumed = True
        prior.join()
        return _HensmanFn.apply(prior.params0, prior.params1, prior.noise, mu, log_v, prior.m, prior.H, prior.x,
                                prior.zz, prior.spec0, prior.spec1, prior.dims, prior.want_ng, prior.pre)
    a = _hensman_args(covar_module0, covar_module1, likelihood, latent_dim, H, train_xt, z, P_tot, P_batch, T,
                      natural_gradient, eps, ng_prior_share)
    params0, params1, noise, zz, spec0, spec1, dims = a
    return _HensmanFn.apply(params0, params1, noise, mu, log_v, m, H, train_xt, zz, spec0, spec1, dims,
                            bool(natural_gradient))


def _hensman_args(covar_module0, covar_module1, likelihood, latent_dim, H, train_xt, z, P_tot, P_batch, T,
                  natural_gradient, eps, ng_prior_share):
    spec0, params0 = kernel_spec_and_params(covar_module0)
    spec1, params1 = kernel_spec_and_params(covar_module1)
    L, M = latent_dim, H.shape[-1]
    if params0.shape[0] == 1 and L > 1:
        params0 = params0.expand(L, -1)
    if params1.shape[0] == 1 and L > 1:
        params1 = params1.expand(L, -1)
    noise = likelihood.noise_covar.noise.reshape(-1)
    if noise.numel() == 1 and L > 1:
        noise = noise.expand(L)
    Q = train_xt.shape[-1]
    if train_xt.shape[0] != P_batch * T:
        raise ValueError(f"train_xt has {train_xt.shape[0]} rows, expected P_batch*T = {P_batch * T}")
    zz = z if z.dim() == 3 else z.unsqueeze(0).expand(L, -1, -1)
    dims = _lib.HensmanDims(L, M, int(P_batch), int(T), int(Q), float(P_tot), float(eps), int(bool(natural_gradient)),
                            float(ng_prior_share))
    return params0, params1, noise, zz, spec0, spec1, dims


def _subject_layout(ids):
    """Host-side layout of a varying-length batch: subjects in torch.unique (sorted) order, each
    padded to the longest subject.  Returns (gather [P_b*T_max] row indices, valid mask, seg_len
    [P_b], T_max).  Padding slots point at the subject's first row and are masked out."""
    ids_c = ids.detach().to("cpu", torch.float64)
    subjects = torch.unique(ids_c)
    rows = [torch.nonzero(ids_c == s_, as_tuple=False).reshape(-1) for s_ in subjects]
    T_max = max(int(r.numel()) for r in rows)
    gather = torch.empty(len(rows), T_max, dtype=torch.int64)
    valid = torch.zeros(len(rows), T_max, dtype=torch.bool)
    for p, r in enumerate(rows):
        gather[p, :r.numel()] = r
        gather[p, r.numel():] = r[0]
        valid[p, :r.numel()] = True
    seg = torch.tensor([int(r.numel()) for r in rows], dtype=torch.int32)
    return gather.reshape(-1), valid.reshape(-1), seg, T_max


def minibatch_KLD_upper_bound_iter(covar_module0, covar_module1, likelihood, latent_dim, m, H, train_xt, mu, log_v,
                                   z, P, P_in_current_batch, N, natural_gradient, id_covariate, eps,
                                   ng_prior_share=1.0):
    """The Hensman bound for subjects of varying length (elbo_functions.py:219-307), same signature.

    The reference loops over the batch's subjects in Python; here the batch is laid out once as
    [P_b, T_max] (subject-sorted, as torch.unique orders them) and the whole bound runs in the
    same HIP kernels as minibatch_KLD_upper_bound with the padding rows masked out
    (lvae_hensman_dims.seg_len).  Gradients flow back to the caller's mu / log_v rows."""
    spec0, params0 = kernel_spec_and_params(covar_module0)
    spec1, params1 = kernel_spec_and_params(covar_module1)
    L, M = latent_dim, H.shape[-1]
    if params0.shape[0] == 1 and L > 1:
        params0 = params0.expand(L, -1)
    if params1.shape[0] == 1 and L > 1:
        params1 = params1.expand(L, -1)
    noise = likelihood.noise_covar.noise.reshape(-1)
    if noise.numel() == 1 and L > 1:
        noise = noise.expand(L)
    dev = mu.device
    gather, valid, seg, T_max = _subject_layout(train_xt[:, id_covariate])
    P_b = int(seg.numel())
    gather_d = gather.to(dev)
    keep = valid.to(dev, mu.dtype).unsqueeze(1)
    x_pad = train_xt.detach()[gather_d]
    mu_pad = mu[gather_d] * keep
    lv_pad = log_v[gather_d] * keep.to(log_v.dtype)
    seg_d = seg.to(dev)
    zz = z if z.dim() == 3 else z.unsqueeze(0).expand(L, -1, -1)
    # scale P / P_in_current_batch (elbo_functions.py:298) with P_b padded subjects: P_tot' = P P_b / P_in
    p_tot = float(P) * P_b / float(P_in_current_batch)
    dims = _lib.HensmanDims(L, M, P_b, int(T_max), int(train_xt.shape[-1]), p_tot, float(eps),
                            int(bool(natural_gradient)), float(ng_prior_share), seg_d.data_ptr(), float(N))
    dims.keepalive = seg_d  # the device seg_len array lives as long as the dims (saved for backward)
    kld, gm, gH = _HensmanFn.apply(params0, params1, noise, mu_pad, lv_pad, m, H, x_pad, zz, spec0, spec1, dims,
                                   bool(natural_gradient))
    return kld, gm, gH


def natural_gradient_update_(m, H, grad_m, grad_H, natural_gradient_lr):
    """natural_gradient_update IN PLACE on m [L, M, 1] / H [L, M, M] (fp64, contiguous, on the device): the
    library updates the buffers it reads (lvae_natgrad_update_f64 reads m and H before writing them), no
    clones and no copies back.  Returns False (nothing done) when m / H do not qualify."""
    if not (m.dtype == H.dtype == torch.float64 and m.is_contiguous() and H.is_contiguous() and m.is_cuda):
        return False
    lib = _lib.lib()
    L, M = H.shape[0], H.shape[-1]
    gm = grad_m.detach().to(torch.float64).contiguous()
    gH = grad_H.detach().to(torch.float64).contiguous()
    ws = torch.empty(int(lib.lvae_natgrad_workspace_size(L, M)), dtype=torch.uint8, device=H.device)
    info = torch.empty(L, dtype=torch.int32, device=H.device)
    iH = None
    cached = getattr(grad_H, "_lvae_iH", None)
    if cached is not None and cached[1] is H and cached[1]._version == cached[2]:
        iH = cached[0]
    with torch.no_grad():
        rc = lib.lvae_natgrad_update_f64(L, M, _lib.ptr(m.detach()), _lib.ptr(H.detach()), _lib.ptr(gm), _lib.ptr(gH),
                                         float(natural_gradient_lr), _lib.ptr(iH), _lib.ptr(info), _lib.ptr(ws),
                                         _lib.stream_ptr())
    _lib.check(rc, "natgrad_update")
    # the raw-pointer write is invisible to autograd's version counters: bump them, so that saved-tensor checks
    # and the iH cache (keyed on H._version) see the new (m, H)
    from torch.autograd.graph import increment_version
    increment_version(m)
    increment_version(H)
    _check_info(info, "natural-gradient update cholesky")  # (any failure: no dim was updated, natgrad_commit_kernel)
    return True


def natural_gradient_update(m, H, grad_m, grad_H, natural_gradient_lr):
    """training.py:129-135 on the device: returns the updated (m, H) (new tensors, detached)."""
    lib = _lib.lib()
    L, M = H.shape[0], H.shape[-1]
    m2 = m.detach().to(torch.float64).contiguous().clone()
    H2 = H.detach().to(torch.float64).contiguous().clone()
    gm = grad_m.detach().to(torch.float64).contiguous()
    gH = grad_H.detach().to(torch.float64).contiguous()
    ws = torch.empty(int(lib.lvae_natgrad_workspace_size(L, M)), dtype=torch.uint8, device=H.device)
    info = torch.empty(L, dtype=torch.int32, device=H.device)
    # H^-1 from the forward that produced grad_H, if H is still the very tensor (same version) it saw
    iH = None
    cached = getattr(grad_H, "_lvae_iH", None)
    if cached is not None and cached[1] is H and cached[1]._version == cached[2]:
        iH = cached[0]
    rc = lib.lvae_natgrad_update_f64(L, M, _lib.ptr(m2), _lib.ptr(H2), _lib.ptr(gm), _lib.ptr(gH),
                                     float(natural_gradient_lr), _lib.ptr(iH), _lib.ptr(info), _lib.ptr(ws),
                                     _lib.stream_ptr())
    _lib.check(rc, "natgrad_update")
    _check_info(info, "natural-gradient update cholesky")
    return m2.reshape(m.shape), H2
