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
    and backward (the N x N Gram / sweep / S GEMM never leave the GPU);
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
    collectives on gloo)."""

    def __init__(self, vae, kernel, likelihood, optimiser, weight=0.15, loss_function="mse", constrain_scales=True,
                 group=None, kl_fn=None):
        self.vae, self.kernel, self.lik, self.opt = vae, kernel, likelihood, optimiser
        self.weight, self.loss_function, self.constrain_scales = weight, loss_function, constrain_scales
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.kl_fn = kl_fn or _hip_kl
        self.params = [p for p in list(vae.parameters()) + list(kernel.parameters()) + list(likelihood.parameters())
                       if p.requires_grad]

    def __call__(self, img, mask, X, eps=None):
        from .elbo import _noise_vector
        from .kernels import kernel_spec_and_params
        W, r = self.world, self.rank
        self.opt.zero_grad(set_to_none=False)
        mu, log_var = self.vae.encode(img)
        z = self.vae.sample_latent(mu, log_var, eps)
        side = None
        if img.is_cuda:
            # decoder + recon loss + their backward (decoder / likelihood-scale gradients and dLoss/dz)
            # on a second stream, beside the all-gather, the KL and the (mu, logvar) all-reduce below
            mainst = torch.cuda.current_stream(img.device)
            side = getattr(self, "_dec_stream", None)
            if side is None or side.device != img.device:
                side = self._dec_stream = torch.cuda.Stream(device=img.device)
            z_d = z.detach().requires_grad_()
            side.wait_stream(mainst)
            with torch.cuda.stream(side):
                recon = self.vae.decode(z_d)
                mse, nll = self.vae.loss_function(recon, img, mask)
                recon_loss, nll_loss = mse.sum(), nll.sum()
                (recon_loss if self.loss_function == "mse" else nll_loss).backward()
        else:
            recon = self.vae.decode(z)
            mse, nll = self.vae.loss_function(recon, img, mask)
            recon_loss, nll_loss = mse.sum(), nll.sum()
        n_loc, L = mu.shape
        N = X.shape[0]
        if n_loc * W != N:
            raise ValueError(f"rank rows {n_loc} x world {W} != N = {N} (equal image shards required)")
        # (mu, logvar) of all N rows on every rank: one all-gather of [N/W, 2L]
        loc = torch.cat([mu.detach(), log_var.detach()], 1).contiguous()
        if dist.get_backend(self.group) == "nccl":
            full = torch.empty(N, 2 * L, dtype=loc.dtype, device=loc.device)
            dist.all_gather_into_tensor(full, loc, group=self.group)
        else:  # gloo (CPU tests, multi-rank rehearsals on one GPU): list form
            parts = [torch.empty_like(loc) for _ in range(W)]
            dist.all_gather(parts, loc, group=self.group)
            full = torch.cat(parts, 0)
        d0, d1 = shard_bounds(L, W, r)
        coef = self.weight / L if self.loss_function == "mse" else 1.0
        gmv = torch.zeros(N, 2 * L, dtype=loc.dtype, device=loc.device)
        gp_loc = torch.zeros((), dtype=torch.float64, device=loc.device)
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
        dist.all_reduce(gmv, op=dist.ReduceOp.SUM, group=self.group)
        g_loc = gmv[r * n_loc:(r + 1) * n_loc]
        if side is not None:
            mainst.wait_stream(side)
            gz = z_d.grad
            for t in (recon_loss, nll_loss, gz):
                t.record_stream(mainst)
            ((z * gz).sum() + (mu * g_loc[:, :L]).sum() + (log_var * g_loc[:, L:]).sum()).backward()
        else:
            main = recon_loss if self.loss_function == "mse" else nll_loss
            (main + (mu * g_loc[:, :L]).sum() + (log_var * g_loc[:, L:]).sum()).backward()
        # network gradients (sum over image shards) + kernel / likelihood gradients (owner rows only)
        GradAllReduce(self.params, W, self.group, average=False)()
        self.opt.step()
        if self.constrain_scales:
            self.lik.noise = 1.0
        # whole-batch loss terms
        terms = torch.stack([recon_loss.detach().to(torch.float64), nll_loss.detach().to(torch.float64),
                             gp_loc.detach()])
        dist.all_reduce(terms, op=dist.ReduceOp.SUM, group=self.group)
        rl, nl, gp = terms[0], terms[1], terms[2]
        if self.loss_function == "mse":
            gp = gp / L
            net = rl + self.weight * gp
        else:
            net = nl + gp
        return net, rl, nl, gp
