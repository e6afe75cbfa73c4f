"""Multi-GPU forms of the two training steps: one process per GPU, torch.distributed over RCCL
(backend "nccl" is RCCL on ROCm).  The reference has no distributed code; both
forms below reproduce the single-process step of the union exactly.

Regime A (Hensman SVI, training.py:90-140): data parallel over subject mini-batches.  Each rank
takes P_b subjects of one global permutation; Adam gradients are AVERAGED (each rank's bound is
scaled by P_tot / P_b, so the mean equals the union batch's P_tot / (W P_b) scaling) and the
natural-gradient directions SUMMED with ng_prior_share = 1/W (HensmanStep + GradAllReduce).

Regime B (exact KL, training.py:484-592): the L latent GPs are independent given (mu, logvar), so
the KL shards over latent dims with no approximation (LatentShardedClosedStep):
  * images are split over ranks (rows [r N/W, (r+1) N/W)); each rank runs the ConvVAE on its rows;
  * one all-gather assembles (mu, logvar) [N, L] on every rank (N L 8 B: 0.5 MB at C3);
  * rank r computes the exact KL of its dims [r L/W, (r+1) L/W) over all N observations, forward
    and backward (the N x N Gram / Cholesky inverse / S GEMM never leave the GPU);
  * one SUM all-reduce of d loss / d(mu, logvar) [N, 2L] returns every rank its rows' gradient
    (each entry has exactly one non-zero contributor, so the sum is exact);
  * the encoder / decoder backward runs on the local rows, and one flat SUM all-reduce carries the
    network gradients (a sum over image shards: the loss is a sum over images) together with the
    kernel / likelihood gradients (non-zero only in the owner's rows), so every rank applies the
    identical Adam update and the replicas stay bit-identical.
"""
import torch
import torch.distributed as dist
from torch._utils import _flatten_dense_tensors, _unflatten_dense_tensors


class GradAllReduce:
    """Average (or sum) the .grad of `params` over the process group (between backward and step)."""

    def __init__(self, params, world=None, group=None, average=True):
        self.params = [p for p in params if p.requires_grad]
        self.group = group
        self.world = world or dist.get_world_size(group)
        self.average = average

    def __call__(self):
        by_dtype = {}
        for p in self.params:
            if p.grad is None:
                p.grad = torch.zeros_like(p)
            by_dtype.setdefault((p.grad.dtype, p.grad.device), []).append(p.grad)
        for grads in by_dtype.values():
            flat = _flatten_dense_tensors(grads)
            dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group)
            if self.average:
                flat.div_(self.world)
            for g, r in zip(grads, _unflatten_dense_tensors(flat, grads)):
                g.copy_(r)


def allreduce_tensors(tensors, average=True, group=None):
    """In-place SUM (or mean) all-reduce of a list of same-dtype tensors in one flat bucket."""
    if not tensors:
        return
    flat = _flatten_dense_tensors(tensors)
    dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    if average:
        flat.div_(dist.get_world_size(group))
    for t, r in zip(tensors, _unflatten_dense_tensors(flat, tensors)):
        t.copy_(r)


def shard_bounds(n, world, rank):
    """[lo, hi) of rank's contiguous share of n items (the first n % world ranks take one more)."""
    q, r = divmod(n, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def _hip_kl(spec, params, noise, mu, logv, x):
    from .elbo import _kl_closed_apply
    return _kl_closed_apply(params, noise, mu, logv, x, spec, None)


class LatentShardedClosedStep:
    """standard_training's exact-KL step (training.py:484-592) with the latent dims sharded over the
    process group (see the module docstring).  Same arguments and return as steps.ClosedStep except
    that ``img`` / ``mask`` / ``eps`` are this rank's rows (shard_bounds(N, world, rank)) while ``X``
    holds all N covariate rows.  Returns (net, recon, nll, gp) of the WHOLE batch on every rank.

    kl_fn(spec, params [Lr, P], noise [Lr], mu [N, Lr], logv [N, Lr], X) -> per-dim KL [Lr] is the
    exact-KL engine: the HIP library by default (tests substitute the CPU oracle to exercise the
    collectives on gloo).

    On the GPU with the HIP engine the step keeps ClosedStep's overlap (steps.py) around the
    collectives:
      caller stream : the factor of the rank's dims (Gram + potrf + trtri) FIRST, before the encoder;
                      then the KL reduce once the gathered (mu, logvar) are in; the (mu, logvar) half of
                      the KL backward (elementwise); then the hyper-parameter half (S GEMM + Gram adjoint)
      ConvVAE stream: encoder; the all-gather of (mu, logvar); decoder + recon loss + their backward;
                      then the SUM all-reduce of d loss / d(mu, logvar) and the encoder backward -- beside
                      the S GEMM on the caller's stream
    and the flat gradient all-reduce + Adam after both.

    sim_world (rehearsal, one process, no process group): run rank 0's share of a world of sim_world
    ranks with the collectives replaced by local stand-ins (the all-gather tiles this rank's rows, the
    all-reduces are identities) -- the per-rank compute of the W-GPU step, timed on one GPU (bench.py
    --rank-share); its numbers are not the union step's."""

    def __init__(self, vae, kernel, likelihood, optimiser, weight=0.15, loss_function="mse", constrain_scales=True,
                 group=None, kl_fn=None, sim_world=None, vae_stream_priority=-1, graph_vae=None):
        self.vae, self.kernel, self.lik, self.opt = vae, kernel, likelihood, optimiser
        self.weight, self.loss_function, self.constrain_scales = weight, loss_function, constrain_scales
        self.group = group
        self.sim = sim_world is not None
        self.world = int(sim_world) if self.sim else dist.get_world_size(group)
        self.rank = 0 if self.sim else dist.get_rank(group)
        self.hip = kl_fn is None
        self.kl_fn = kl_fn or _hip_kl
        self.params = [p for p in list(vae.parameters()) + list(kernel.parameters()) + list(likelihood.parameters())
                       if p.requires_grad]
        self.hyper_params = [p for p in list(kernel.parameters()) + list(likelihood.parameters()) if p.requires_grad]
        self.vae_stream_priority = vae_stream_priority
        from .steps import _graph_vae_default
        from .vae import GraphedConvVAE
        self.gvae = GraphedConvVAE(vae) if (_graph_vae_default() if graph_vae is None else graph_vae) else None

    # -- the collectives (or their single-process stand-ins) -----------------------------------
    def _all_gather(self, loc, N):
        if self.sim:
            return loc.repeat(self.world, 1)
        if dist.get_backend(self.group) == "nccl":
            full = torch.empty(N, loc.shape[1], dtype=loc.dtype, device=loc.device)
            dist.all_gather_into_tensor(full, loc, group=self.group)
            return full
        parts = [torch.empty_like(loc) for _ in range(self.world)]  # gloo (CPU tests, rehearsals): list form
        dist.all_gather(parts, loc, group=self.group)
        return torch.cat(parts, 0)

    def _all_reduce(self, t):
        if not self.sim:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)

    def _grad_all_reduce(self):
        if not self.sim:
            GradAllReduce(self.params, self.world, self.group, average=False)()

    def _stream(self, device):
        s = getattr(self, "_vae_stream", None)
        if s is None or s.device != device:
            s = self._vae_stream = torch.cuda.Stream(device=device, priority=self.vae_stream_priority)
        return s

    def _finish(self, recon_loss, nll_loss, gp_loc, L):
        self._grad_all_reduce()  # network gradients (sum over image shards) + kernel / likelihood (owner rows)
        self.opt.step()
        if self.constrain_scales:
            self.lik.noise = 1.0
        terms = torch.stack([recon_loss.detach().to(torch.float64), nll_loss.detach().to(torch.float64),
                             gp_loc.detach()])
        self._all_reduce(terms)  # whole-batch loss terms
        rl, nl, gp = terms[0], terms[1], terms[2]
        if self.loss_function == "mse":
            gp = gp / L
            net = rl + self.weight * gp
        else:
            net = nl + gp
        return net, rl, nl, gp

    def __call__(self, img, mask, X, eps=None):
        from .steps import bwd_thread_ctx
        if img.is_cuda and self.hip:
            with bwd_thread_ctx():
                return self._step_overlapped(img, mask, X, eps)
        return self._step_plain(img, mask, X, eps)

    def _step_overlapped(self, img, mask, X, eps):
        from .elbo import KLFactor, _noise_vector
        from .kernels import kernel_spec_and_params
        W, r = self.world, self.rank
        self.opt.zero_grad(set_to_none=True)
        main = torch.cuda.current_stream(img.device)
        capturing = torch.cuda.is_current_stream_capturing()  # (an outer graph capture: the ConvVAE eager)
        vst = self._stream(img.device)
        vst.wait_stream(main)  # the previous step's updates
        L = self.vae.latent_dim
        N = X.shape[0]
        n_loc = img.shape[0]
        if n_loc * W != N:  # (checked before the factor's enqueue is handed to its worker thread)
            raise ValueError(f"rank rows {n_loc} x world {W} != N = {N} (equal image shards required)")
        d0, d1 = shard_bounds(L, W, r)
        own = d1 > d0
        factor = None
        if own:  # Gram + potrf + trtri of the rank's dims: covariates and hyper-parameters only
            spec, params = kernel_spec_and_params(self.kernel)
            noise = _noise_vector(self.lik, L).to(params.device)
            factor = KLFactor(spec, params[d0:d1], noise[d0:d1], X, main)
        try:
            return self._step_overlapped_rest(img, mask, X, eps, main, vst, capturing, L, N, n_loc, d0, d1, own,
                                              factor)
        finally:
            if factor is not None:
                factor.wait_enqueued()  # (a no-op once waited: never leave the worker enqueueing into freed buffers)

    def _step_overlapped_rest(self, img, mask, X, eps, main, vst, capturing, L, N, n_loc, d0, d1, own, factor):
        from .elbo import KL_closed_batched
        r = self.rank
        gathered = torch.cuda.Event()
        with torch.cuda.stream(vst):
            gv = None if capturing else self.gvae
            mu, log_var = gv.encode(img, mask) if gv is not None else self.vae.encode(img)
            z = self.vae.sample_latent(mu, log_var, eps)
            full = self._all_gather(torch.cat([mu.detach(), log_var.detach()], 1).contiguous(), N)
            gathered.record(vst)
            z_d = z.detach().requires_grad_()
            if gv is not None:
                recon_loss, nll_loss = gv.decode_loss(z_d, img, mask)
            else:
                recon = self.vae.decode(z_d)
                mse, nll = self.vae.loss_function(recon, img, mask)
                recon_loss, nll_loss = mse.sum(), nll.sum()
            (recon_loss if self.loss_function == "mse" else nll_loss).backward()  # decoder + d/dz
            recon_loss, nll_loss = recon_loss.detach().clone(), nll_loss.detach().clone()
        if factor is not None:
            factor.wait_enqueued()  # (its launches on `main` all precede the wait below)
        main.wait_event(gathered)
        full.record_stream(main)
        coef = self.weight / L if self.loss_function == "mse" else 1.0
        gmv = torch.zeros(N, 2 * L, dtype=full.dtype, device=full.device)
        gp_loc = torch.zeros((), dtype=torch.float64, device=full.device)
        tail = None
        if own:
            mu_own = full[:, d0:d1].to(torch.float64).requires_grad_()
            lv_own = full[:, L + d0:L + d1].to(torch.float64).requires_grad_()
            kl = KL_closed_batched(None, X, None, mu_own, lv_own, factor=factor)  # the reduce
            gp_loc = kl.sum()
            tail = coef * gp_loc
            # the (mu, logvar) half first (elementwise, from K^-1 mu and diag K^-1) ...
            torch.autograd.backward(tail, inputs=[mu_own, lv_own], retain_graph=bool(self.hyper_params))
            gmv[:, d0:d1] = mu_own.grad.to(gmv.dtype)
            gmv[:, L + d0:L + d1] = lv_own.grad.to(gmv.dtype)
        vst.wait_stream(main)
        gmv.record_stream(vst)
        # ... then the hyper-parameter half (S GEMM + Gram adjoint: a few launches) is ENQUEUED first, so that
        # the GPU starts it while the host is still issuing the encoder backward's ~40 small kernels ...
        if own and self.hyper_params:
            torch.autograd.backward(tail, inputs=self.hyper_params)
        with torch.cuda.stream(vst):
            # ... and the all-reduce and the encoder backward run on the ConvVAE stream beside it
            self._all_reduce(gmv)
            g_loc = gmv[r * n_loc:(r + 1) * n_loc]
            gz = z_d.grad
            ((z * gz).sum() + (mu * g_loc[:, :L]).sum() + (log_var * g_loc[:, L:]).sum()).backward()
        main.wait_stream(vst)
        for t in (recon_loss, nll_loss):
            t.record_stream(main)
        return self._finish(recon_loss, nll_loss, gp_loc, L)

    def _step_plain(self, img, mask, X, eps=None):
        from .elbo import _noise_vector
        from .kernels import kernel_spec_and_params
        W, r = self.world, self.rank
        self.opt.zero_grad(set_to_none=False)
        mu, log_var = self.vae.encode(img)
        z = self.vae.sample_latent(mu, log_var, eps)
        recon = self.vae.decode(z)
        mse, nll = self.vae.loss_function(recon, img, mask)
        recon_loss, nll_loss = mse.sum(), nll.sum()
        n_loc, L = mu.shape
        N = X.shape[0]
        if n_loc * W != N:
            raise ValueError(f"rank rows {n_loc} x world {W} != N = {N} (equal image shards required)")
        # (mu, logvar) of all N rows on every rank: one all-gather of [N/W, 2L]
        full = self._all_gather(torch.cat([mu.detach(), log_var.detach()], 1).contiguous(), N)
        d0, d1 = shard_bounds(L, W, r)
        coef = self.weight / L if self.loss_function == "mse" else 1.0
        gmv = torch.zeros(N, 2 * L, dtype=full.dtype, device=full.device)
        gp_loc = torch.zeros((), dtype=torch.float64, device=full.device)
        if d1 > d0:
            spec, params = kernel_spec_and_params(self.kernel)
            noise = _noise_vector(self.lik, L).to(params.device)
            mu_own = full[:, d0:d1].to(torch.float64).requires_grad_()
            lv_own = full[:, L + d0:L + d1].to(torch.float64).requires_grad_()
            kl = self.kl_fn(spec, params[d0:d1], noise[d0:d1], mu_own, lv_own, X)
            gp_loc = kl.sum()
            (coef * gp_loc).backward()  # kernel / noise grads of the owned rows; d/d(mu, logv) of owned dims
            gmv[:, d0:d1] = mu_own.grad.to(gmv.dtype)
            gmv[:, L + d0:L + d1] = lv_own.grad.to(gmv.dtype)
        # every rank's rows of d loss / d(mu, logvar): one SUM all-reduce (one contributor per entry)
        self._all_reduce(gmv)
        g_loc = gmv[r * n_loc:(r + 1) * n_loc]
        main = recon_loss if self.loss_function == "mse" else nll_loss
        (main + (mu * g_loc[:, :L]).sum() + (log_var * g_loc[:, L:]).sum()).backward()
        return self._finish(recon_loss, nll_loss, gp_loc, L)
