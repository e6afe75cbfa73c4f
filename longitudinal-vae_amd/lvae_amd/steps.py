"""One optimisation step of each training driver, as tensors-in / tensors-out (no host syncs).

ClosedStep   : standard_training with type_KL='closed' (training.py:484-592)
HensmanStep  : hensman_training batch body incl. the natural-gradient update (training.py:91-135)
GraphedStep  : either step replayed as HIP graphs (torch.cuda.CUDAGraph is a hipGraph on ROCm)

Both steps return detached device scalars; callers read them when they choose (the reference's
per-step ``.item()`` calls, training.py:137-140, are the sync points this removes).  Gradients are
reset to None (``optimiser.zero_grad()``'s default, as training.py:93 calls it): backward then
assigns each gradient instead of filling it with zeros and adding, two kernels less per parameter.  Each step is
split into ``forward_backward`` (everything up to the gradients) and ``apply`` (optimiser + state
updates) so that a data-parallel all-reduce can sit between two captured graphs.
"""
import contextlib
import os

import torch

from .elbo import (KL_closed_batched, kl_closed_prefactor, minibatch_KLD_upper_bound, natural_gradient_update,
                   natural_gradient_update_, take_pending)


# LVAE_BWD_ON_CALLER=0: the closed steps' backward on autograd's per-device worker thread (torch's default) instead
# of the calling thread.  On the caller the step's host side is shorter: at one W = 8 rank's share, whose step the
# host's enqueue paces, 3.52-3.54 vs 3.71-3.76 ms (profiles/r6_bwd_thread_ab.txt)
_BWD_ON_CALLER = os.environ.get("LVAE_BWD_ON_CALLER", "1") != "0"


def bwd_thread_ctx():
    """The context the closed steps run their backward passes in (see _BWD_ON_CALLER)."""
    return torch.autograd.set_multithreading_enabled(False) if _BWD_ON_CALLER else contextlib.nullcontext()


def _graph_vae_default():
    # opt-in (LVAE_GRAPH_VAE=1): measured SLOWER on ROCm 7 -- the ConvVAE's graph replays on its stream held
    # back the other streams' kernels (rank share of 8 GPUs 3.8 -> 10.9 ms per step, headline 11.7 -> 16.6 ms)
    import os
    return os.environ.get("LVAE_GRAPH_VAE", "0") == "1"


class ClosedStep:
    def __init__(self, vae, kernel, likelihood, optimiser, weight=0.15, loss_function="mse",
                 constrain_scales=True, grad_hook=None, vae_stream_priority=-1, graph_vae=None):
        self.vae, self.kernel, self.lik, self.opt = vae, kernel, likelihood, optimiser
        # the ConvVAE as replayed graphs (GraphedConvVAE; opt-in, see _graph_vae_default)
        from .vae import GraphedConvVAE
        self.gvae = GraphedConvVAE(vae) if (_graph_vae_default() if graph_vae is None else graph_vae) else None
        self.weight, self.loss_function, self.constrain_scales = weight, loss_function, constrain_scales
        self.grad_hook = grad_hook  # e.g. the data-parallel all-reduce
        # The ConvVAE's stream is created with a high priority by default: its kernels are small and
        # would otherwise queue behind the KL's grids of thousands of LDS-heavy workgroups (one per CU)
        # until those drain, which put the encoder backward at the end of the step.
        self.vae_stream_priority = vae_stream_priority

    def _stream(self, name, device):
        s = getattr(self, name, None)
        if s is None or s.device != device:
            s = torch.cuda.Stream(device=device, priority=self.vae_stream_priority)
            setattr(self, name, s)
        return s

    def forward_backward(self, img, mask, X, eps=None):
        with bwd_thread_ctx():
            return self._forward_backward(img, mask, X, eps)

    def _forward_backward(self, img, mask, X, eps=None):
        self.opt.zero_grad(set_to_none=True)
        if img.is_cuda:
            # The Gram and its inverse need only the covariates and hyperparameters: they are
            # enqueued first, on the caller's stream, and the whole ConvVAE runs on one second stream
            # beside them -- the encoder (its (mu, logvar) join the KL through an event), then the
            # decoder and recon loss, which do not depend on the KL at all.  Autograd runs each
            # backward op on its forward's stream: the decoder backward beside the KL reduce, the
            # encoder backward (once d kl / d (mu, logvar) is out: elbo._KLClosedFn) beside the KL's
            # hyper-parameter half (S GEMM + Gram adjoint, elbo._KLHyperFn).  (Two extra streams at
            # most: the box exposes 4 hardware queues, and the inverse keeps one side stream of its own.)
            main = torch.cuda.current_stream(img.device)
            capturing = torch.cuda.is_current_stream_capturing()  # (an outer graph capture: the ConvVAE eager)
            vst = self._stream("_vae_stream", img.device)
            vst.wait_stream(main)  # the previous step's updates, before the factorisation is queued
            factor = kl_closed_prefactor(self.kernel, X, self.lik, self.vae.latent_dim, main)
            enc_done = torch.cuda.Event()
            mse_mode = self.loss_function == "mse"
            with torch.cuda.stream(vst):
                gv = None if capturing else self.gvae
                if gv is not None:
                    mu, log_var = gv.encode(img, mask)
                else:
                    mu, log_var = self.vae.encode(img)
                enc_done.record(vst)
                z = self.vae.sample_latent(mu, log_var, eps)
                # The decoder and the recon loss run from a detached copy of z, and their backward is enqueued
                # right here -- before the host waits for the factorisation's enqueue (~250 launches from the
                # worker thread) and enqueues the KL -- so the decoder backward runs beside the Cholesky instead
                # of behind the KL's host work.  Its dLoss/dz joins the KL's d/d(mu, logvar) in ONE encoder
                # backward below (the same sums as the single backward over both loss terms).
                zd = z.detach().requires_grad_()
                if gv is not None:
                    recon_loss, nll_loss = gv.decode_loss(zd, img, mask)
                else:
                    recon = self.vae.decode(zd)
                    mse, nll = self.vae.loss_function(recon, img, mask)
                    recon_loss, nll_loss = mse.sum(), nll.sum()
                rec_term = recon_loss if mse_mode else nll_loss
                rec_term.backward()
            factor.wait_enqueued()  # (its launches on `main` all precede the wait below)
            main.wait_event(enc_done)
            mu.record_stream(main)
            log_var.record_stream(main)
            kl = KL_closed_batched(self.kernel, X, self.lik, mu, log_var, factor=factor)
            L = mu.shape[1]
            if mse_mode:
                gp = kl.sum() / L
                gp_term = self.weight * gp
            else:
                gp = kl.sum()
                gp_term = gp
            # The encoder backward from dLoss/dz (the decoder's) and the KL term, called on the ConvVAE's stream
            # (the KL's backward kernels run on their forward's stream; the encoder's join them through the
            # d/d(mu, logvar) events of elbo._KLClosedFn).
            with torch.cuda.stream(vst):
                torch.autograd.backward([z, gp_term], [zd.grad, None])
            main.wait_stream(vst)
            for t in (recon_loss, nll_loss, rec_term):
                t.record_stream(main)
            net = rec_term.detach() + gp_term.detach()
            return net, recon_loss.detach().clone(), nll_loss.detach().clone(), gp.detach()
        else:
            recon, mu, log_var = self.vae(img, eps)
            mse, nll = self.vae.loss_function(recon, img, mask)
            recon_loss, nll_loss = mse.sum(), nll.sum()
            kl = KL_closed_batched(self.kernel, X, self.lik, mu, log_var)
        L = mu.shape[1]
        if self.loss_function == "mse":
            gp = kl.sum() / L
            net = recon_loss + self.weight * gp
        else:
            gp = kl.sum()
            net = nll_loss + gp
        net.backward()
        return net.detach(), recon_loss.detach(), nll_loss.detach(), gp.detach()

    def communicate(self):
        if self.grad_hook is not None:
            self.grad_hook()

    def apply(self):
        self.opt.step()
        if self.constrain_scales:
            self.lik.noise = 1.0

    def __call__(self, img, mask, X, eps=None):
        out = self.forward_backward(img, mask, X, eps)
        self.communicate()
        self.apply()
        return out


class _StepTermsFn(torch.autograd.Function):
    """(net, rec, nll, kld') of the Hensman step from (mse [B], nll [B], kld) in one launch each way
    (glue.hip: lvae_step_terms_fwd / _bwd) instead of the sums, scalings and their backward ops."""

    @staticmethod
    def forward(ctx, mse, nll, kld, c, ks, w, use_nll):
        from . import _lib
        lib = _lib.lib()
        dev = mse.device
        m, n, k = mse.contiguous(), nll.contiguous(), kld.detach().to(torch.float64).contiguous()
        rec, nl = torch.empty((), device=dev), torch.empty((), device=dev)
        net, kd = torch.empty((), dtype=torch.float64, device=dev), torch.empty((), dtype=torch.float64, device=dev)
        _lib.check(lib.lvae_step_terms_fwd(_lib.ptr(m), _lib.ptr(n), m.numel(), _lib.ptr(k), float(c), float(ks),
                                           float(w), int(use_nll), _lib.ptr(rec), _lib.ptr(nl), _lib.ptr(net),
                                           _lib.ptr(kd), _lib.stream_ptr()), "step_terms_fwd")
        ctx.set_materialize_grads(False)
        ctx.meta = (float(c), float(ks), float(w), int(use_nll), m.numel(), kld.shape, kld.dtype)
        return net, rec, nl, kd

    @staticmethod
    def backward(ctx, g_net, g_rec, g_nl, g_kd):
        from . import _lib
        lib = _lib.lib()
        c, ks, w, use_nll, B, kshape, kdtype = ctx.meta
        dev = next(g for g in (g_net, g_rec, g_nl, g_kd) if g is not None).device
        f64 = lambda g: None if g is None else g.detach().to(torch.float64).contiguous()
        f32 = lambda g: None if g is None else g.detach().to(torch.float32).contiguous()
        gn, gr, gl, gk = f64(g_net), f32(g_rec), f32(g_nl), f64(g_kd)
        g_mse, g_nll = torch.empty((), device=dev), torch.empty((), device=dev)
        g_kld = torch.empty((), dtype=torch.float64, device=dev)
        _lib.check(lib.lvae_step_terms_bwd(_lib.ptr(gn), _lib.ptr(gr), _lib.ptr(gl), _lib.ptr(gk), c, ks, w, use_nll,
                                           _lib.ptr(g_mse), _lib.ptr(g_nll), _lib.ptr(g_kld), _lib.stream_ptr()),
                   "step_terms_bwd")
        return (g_mse.expand(B), g_nll.expand(B), g_kld.reshape(kshape).to(kdtype), None, None, None, None)


class HensmanStep:
    """hensman_training batch body (training.py:91-135), loss 'mse' or 'nll'.

    State: the inducing posterior (m [L,M,1], H [L,M,M]) lives here and is updated IN PLACE by the
    natural-gradient step (training.py:129-135) when natural_gradient is on (so a captured graph
    replays it); otherwise m and H are leaf tensors the optimiser owns (H enters as H H^T,
    training.py:108).
    Data parallel: pass ``world`` and a ``grad_hook`` (all-reduce of the Adam gradients) and
    ``ng_reduce`` (SUM all-reduce of the natural-gradient directions, see lvae_hensman_dims)."""

    def __init__(self, vae, k0, k1, likelihood, optimiser, m, H, z, P_tot, T, weight=0.15, loss_function="mse",
                 natural_gradient=True, natural_gradient_lr=0.01, eps=1e-6, world=1, grad_hook=None,
                 ng_reduce=None):
        self.vae, self.k0, self.k1, self.lik, self.opt = vae, k0, k1, likelihood, optimiser
        self.m, self.H, self.z = m, H, z
        self.P_tot, self.T = P_tot, T
        self.weight, self.loss_function = weight, loss_function
        self.ng, self.ng_lr, self.eps = natural_gradient, natural_gradient_lr, eps
        self.world, self.grad_hook, self.ng_reduce = world, grad_hook, ng_reduce
        self._gm = self._gH = None

    def forward_backward(self, img, mask, X, eps=None):
        self.opt.zero_grad(set_to_none=True)
        # (one stream: HensmanPrior on a second stream beside the ConvVAE forward measured slower in the
        # graphed step, 1.37-1.39 vs 1.34 ms)
        recon, mu, log_var = self.vae(img, eps)
        mse, nll = self.vae.loss_function(recon, img, mask)
        L = mu.shape[1]
        P_b = X.shape[0] // self.T
        PSD_H = self.H if self.ng else self.H @ self.H.transpose(-1, -2)
        kld, gm, gH = minibatch_KLD_upper_bound(self.k0, self.k1, self.lik, L, self.m, PSD_H, X, mu, log_var,
                                                self.z, self.P_tot, P_b, self.T, self.ng, self.eps,
                                                ng_prior_share=1.0 / self.world)
        mse_loss = self.loss_function == "mse"
        if mse.is_cuda and mse.dtype == nll.dtype == torch.float32 and kld.numel() == 1:
            # (glue.hip: the sums, scalings and their backward in one launch each way)
            net, recon_loss, nll_loss, kld = _StepTermsFn.apply(mse, nll, kld, self.P_tot / P_b,
                                                                1.0 / L if mse_loss else 1.0, self.weight,
                                                                not mse_loss)
        else:
            recon_loss = mse.sum() * self.P_tot / P_b
            nll_loss = nll.sum() * self.P_tot / P_b
            if mse_loss:
                kld = kld / L
                net = recon_loss + self.weight * kld
            else:
                net = nll_loss + kld
        net.backward()
        self._gm, self._gH = gm, gH
        return net.detach(), recon_loss.detach(), nll_loss.detach(), kld.detach()

    def communicate(self):
        if self.grad_hook is not None:
            self.grad_hook()
        if self.ng and self.ng_reduce is not None:
            self.ng_reduce([self._gm, self._gH])

    def apply(self):
        self.opt.step()
        if self.ng:
            # (fp64 state: updated in place by the library, no clones / copies back)
            if not natural_gradient_update_(self.m, self.H, self._gm, self._gH, self.ng_lr):
                m2, H2 = natural_gradient_update(self.m, self.H, self._gm, self._gH, self.ng_lr)
                with torch.no_grad():
                    self.m.copy_(m2.reshape(self.m.shape).to(self.m.dtype))
                    self.H.copy_(H2.to(self.H.dtype))

    def __call__(self, img, mask, X, eps=None):
        out = self.forward_backward(img, mask, X, eps)
        self.communicate()
        self.apply()
        return out


def _comm_capturable():
    """RCCL collectives captured into the step's graph (one replay per step): opt-in, LVAE_GRAPH_COMM=1 with an
    RCCL ("nccl") default process group.  Measured (r6): it matches the eager step (test_rccl_world1_graphed_hensman
    _two_graphs[True]) and 100 back-to-back replays leave every info word clean (scripts/dp_replay_diag.py), but a
    process that had replayed the two-graph form first and then the captured form aborted in its final
    synchronise (profiles/r6_capture_comm_abort.log, cause not found) -- so the default stays two graphs around
    the eager collectives, which the driver's multi-GPU run cannot lose to an abort."""
    import os
    import torch.distributed as dist
    if os.environ.get("LVAE_GRAPH_COMM", "0") != "1":
        return False
    return dist.is_available() and dist.is_initialized() and dist.get_backend() == "nccl"


class GraphedStep:
    """A ClosedStep / HensmanStep replayed as HIP graphs.

    ``inputs`` are static device tensors (img, mask, X, eps) the caller refills in place between
    replays (e.g. ``index_select(..., out=)`` of the next batch).  With no communication the whole
    step is one graph; with a ``grad_hook`` / ``ng_reduce`` (data parallel) the step is two graphs around the
    eager collectives, or (``capture_comm``, opt-in LVAE_GRAPH_COMM=1 over RCCL) one graph with the collectives
    captured.  The optimiser must be capturable (torch.optim.Adam(...,
    capturable=True)); numerical-failure checks are deferred (set_sync_checks(False)) and
    ``check()`` reads the captured info arrays, which every replay rewrites.  shared_pool: capture the
    second graph into the first one's memory pool (diagnostics, scripts/dp_replay_diag.py)."""

    def __init__(self, step, inputs, warmup=3, shared_pool=False, capture_comm=None):
        self.step, self.inputs = step, inputs
        if getattr(step, "gvae", None) is not None:
            step.gvae = None  # (the whole step is one graph here: no graphed ConvVAE parts inside the capture)
        comm = getattr(step, "grad_hook", None) is not None or getattr(step, "ng_reduce", None) is not None
        if capture_comm is None:
            capture_comm = _comm_capturable()
        if comm and capture_comm:
            comm = False  # the collectives are captured into the one graph with the rest of the step
        self.stream = torch.cuda.Stream()
        self.stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.stream):  # warm-up: allocations, MIOpen / hipBLASLt plans, side streams
            for _ in range(warmup):
                step(*inputs)
        torch.cuda.current_stream().wait_stream(self.stream)
        torch.cuda.synchronize()
        take_pending()
        self.g1 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.g1, stream=self.stream):
            self.out = step.forward_backward(*inputs)
            if not comm:
                step.communicate()  # (no-op without hooks; RCCL collectives captured as graph nodes otherwise)
                step.apply()
        self.g2 = None
        if comm:
            self.g2 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.g2, stream=self.stream, pool=self.g1.pool() if shared_pool else None):
                step.apply()
        self.pending = take_pending()
        self.comm = comm

    def __call__(self):
        self.g1.replay()
        if self.comm:
            self.step.communicate()
            self.g2.replay()
        return self.out

    def check(self):
        from .elbo import check_pending
        check_pending(self.pending)
