"""One optimisation step of each training driver, as tensors-in / tensors-out (no host syncs).

closed_step   : standard_training with type_KL='closed' (training.py:484-592)
hensman_step  : hensman_training batch body incl. the natural-gradient update (training.py:91-135)
Both return detached device scalars; callers read them when they choose (the reference's
per-step ``.item()`` calls, training.py:137-140, are the sync points this removes).
"""
import torch

from .elbo import KL_closed_batched, minibatch_KLD_upper_bound, natural_gradient_update


class ClosedStep:
    def __init__(self, vae, kernel, likelihood, optimiser, weight=0.15, loss_function="mse",
                 constrain_scales=True, grad_hook=None):
        self.vae, self.kernel, self.lik, self.opt = vae, kernel, likelihood, optimiser
        self.weight, self.loss_function, self.constrain_scales = weight, loss_function, constrain_scales
        self.grad_hook = grad_hook  # e.g. the data-parallel all-reduce

    def __call__(self, img, mask, X, eps=None):
        self.opt.zero_grad(set_to_none=False)
        recon, mu, log_var = self.vae(img, eps)
        mse, nll = self.vae.loss_function(recon, img, mask)
        recon_loss, nll_loss = mse.sum(), nll.sum()
        L = mu.shape[1]
        kl = KL_closed_batched(self.kernel, X, self.lik, mu, log_var)
        if self.loss_function == "mse":
            gp = kl.sum() / L
            net = recon_loss + self.weight * gp
        else:
            gp = kl.sum()
            net = nll_loss + gp
        net.backward()
        if self.grad_hook is not None:
            self.grad_hook()
        self.opt.step()
        if self.constrain_scales:
            self.lik.noise = 1.0
        return net.detach(), recon_loss.detach(), nll_loss.detach(), gp.detach()


class HensmanStep:
    """hensman_training batch body (training.py:91-135), loss 'mse' or 'nll'.

    State: the inducing posterior (m [L,M,1], H [L,M,M]) lives here and is updated in place by the
    natural-gradient step (training.py:129-135) when natural_gradient is on; otherwise m and H are
    leaf tensors the optimiser owns (H enters as H H^T, training.py:108).
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

    def __call__(self, img, mask, X, eps=None):
        self.opt.zero_grad(set_to_none=False)
        recon, mu, log_var = self.vae(img, eps)
        mse, nll = self.vae.loss_function(recon, img, mask)
        recon_loss, nll_loss = mse.sum(), nll.sum()
        L = mu.shape[1]
        P_b = X.shape[0] // self.T
        PSD_H = self.H if self.ng else self.H @ self.H.transpose(-1, -2)
        kld, gm, gH = minibatch_KLD_upper_bound(self.k0, self.k1, self.lik, L, self.m, PSD_H, X, mu, log_var,
                                                self.z, self.P_tot, P_b, self.T, self.ng, self.eps,
                                                ng_prior_share=1.0 / self.world)
        recon_loss = recon_loss * self.P_tot / P_b
        nll_loss = nll_loss * self.P_tot / P_b
        if self.loss_function == "mse":
            kld = kld / L
            net = recon_loss + self.weight * kld
        else:
            net = nll_loss + kld
        net.backward()
        if self.grad_hook is not None:
            self.grad_hook()
        self.opt.step()
        if self.ng:
            if self.ng_reduce is not None:
                self.ng_reduce([gm, gH])
            self.m, self.H = natural_gradient_update(self.m, self.H, gm, gH, self.ng_lr)
        return net.detach(), recon_loss.detach(), nll_loss.detach(), kld.detach()
