"""One optimisation step of each training driver, as tensors-in / tensors-out (no host syncs).

closed_step   : standard_training with type_KL='closed' (training.py:484-592)
hensman_step  : hensman_training batch body incl. the natural-gradient update (training.py:91-135)
Both return detached device scalars; callers read them when they choose (the reference's
per-step ``.item()`` calls, training.py:137-140, are the sync points this removes).
"""
import torch

from .elbo import KL_closed_batched


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
