"""Generate golden input/output vectors by running the REFERENCE code (/root/reference).

Test infrastructure only.  Runs in the build container (where /root/reference exists); the
GPU box never runs it -- it only reads the committed ``*.npz`` fixtures this script writes.

The reference is imported read-only with the harness shims SURVEY.md §8(c) lists:
  * ``torchvision`` stub (``transforms`` is only used for dataset construction),
  * ``torch.solve`` (removed in torch 2.x; used at elbo_functions.py:75,129),
  * ``np.Inf`` (training.py:82),
  * ``Sampler.__init__`` accepting the data_source argument utils.py:46 passes (torch 2.x),
  * kernel adapter: GP_model.py kernels left-align their ``[L]`` parameters while gpytorch
    (the path LVAE.py really runs, kernel_gen.py:199-310) right-aligns ``batch_shape=[L]``;
    for 4-D inputs the adapter evaluates ``k(a.T01, b.T01).T01`` which is the gpytorch
    semantics ``elbo_functions.py:173-174`` rely on,
  * likelihood stub exposing ``.noise`` and ``.noise_covar.noise``.

Every fixture holds inputs and expected outputs only (data, not reference source).

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py
"""
import math
import os
import sys
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def _install_shims():
    import torch
    tv = types.ModuleType("torchvision")
    tv.transforms = types.SimpleNamespace(ToTensor=lambda: None)
    sys.modules.setdefault("torchvision", tv)
    sys.modules.setdefault("torchvision.transforms", tv.transforms)
    torch.solve = lambda B, A: (torch.linalg.solve(A, B), None)  # present-but-raising in torch 2.x
    # utils.py:46 passes data_source to Sampler.__init__, which torch 2.x rejects
    torch.utils.data.sampler.Sampler.__init__ = lambda self, data_source=None: None
    if not hasattr(np, "Inf"):
        np.Inf = np.inf
    sys.dont_write_bytecode = True
    if REF not in sys.path:
        sys.path.insert(0, REF)


_install_shims()
import torch  # noqa: E402
from torch import nn  # noqa: E402

import GP_model as R  # noqa: E402  (reference)
import elbo_functions as EF  # noqa: E402  (reference)
import VAE as RV  # noqa: E402  (reference)

torch.set_default_dtype(torch.float64)


# ----------------------------------------------------------------------------------------------
# adapters
# ----------------------------------------------------------------------------------------------
class _Lazy:
    def __init__(self, t):
        self.t = t

    def evaluate(self):
        return self.t


class KernelAdapter(nn.Module):
    """gpytorch call convention over a GP_model kernel (see module docstring)."""

    def __init__(self, k):
        super().__init__()
        self.k = k

    def forward(self, a, b):
        if a.dim() == 4:
            return _Lazy(self.k(a.transpose(0, 1), b.transpose(0, 1)).transpose(0, 1))
        return _Lazy(self.k(a, b))


class LikStub:
    def __init__(self, noise):
        self.noise = noise
        self.noise_covar = types.SimpleNamespace(noise=noise)

    def eval(self):
        return self

    def train(self, mode=True):
        return self


# ----------------------------------------------------------------------------------------------
# synthetic Health-MNIST covariates (Health_MNIST_generate.py:89-154)
# columns: time_age, disease_time, subject, gender, disease, location  (dataset_def.py:213)
# ----------------------------------------------------------------------------------------------
def covariates(P, T, seed):
    rng = np.random.default_rng(seed)
    sick = rng.binomial(1, 0.5, size=P)
    loc = rng.binomial(1, 0.5, size=P)
    X = np.zeros((P * T, 6))
    for p in range(P):
        for t in range(T):
            r = p * T + t
            X[r, 0] = t
            X[r, 1] = (t - 9) if sick[p] else 0.0
            X[r, 2] = p
            X[r, 3] = 0.0 if p < P // 2 else 1.0
            X[r, 4] = sick[p]
            X[r, 5] = loc[p]
    return X


# sample config (config/LVAE_config_sample.txt:40-45)
CFG = dict(cat_kernel=[2], bin_kernel=[], sqexp_kernel=[0],
           cat_int_kernel=[{'cont_covariate': 0, 'cat_covariate': 2},
                           {'cont_covariate': 0, 'cat_covariate': 3},
                           {'cont_covariate': 1, 'cat_covariate': 4}],
           bin_int_kernel=[], covariate_missing_val=[], id_covariate=2)


# a config exercising every builder branch the sample config leaves out (GP_model.py:146-236):
# bin_kernel, bin_int_kernel and covariate_missing_val mask products on a Cat, an Rbf (also inside
# the interaction kernels) and the Cat of an id-free Cat x Rbf.  Columns 6 / 7 are the masks of
# time_age / gender (covariates_missing below).
VAR_CFG = dict(cat_kernel=[2, 3], bin_kernel=[5], sqexp_kernel=[0],
               cat_int_kernel=[{'cont_covariate': 0, 'cat_covariate': 2},
                               {'cont_covariate': 1, 'cat_covariate': 4}],
               bin_int_kernel=[{'cont_covariate': 0, 'bin_covariate': 4}],
               covariate_missing_val=[{'covariate': 0, 'mask': 6}, {'covariate': 3, 'mask': 7}], id_covariate=2)


def covariates_missing(P, T, seed):
    """covariates() plus mask columns 6 (time_age observed, per row) and 7 (gender observed, per
    subject); a missing value is stored as 0 (dataset_def.py:213 fills NaN with 0)."""
    rng = np.random.default_rng(seed + 1000)
    X = covariates(P, T, seed)
    m_age = rng.binomial(1, 0.8, size=P * T).astype(np.float64)
    m_gen = np.repeat(rng.binomial(1, 0.85, size=P).astype(np.float64), T)
    X[:, 0] *= m_age
    X[:, 3] *= m_gen
    return np.concatenate([X, m_age[:, None], m_gen[:, None]], 1)


def full_kernel_ref(L):
    """The non-split additive kernel in kernel_gen.generate_kernel order (kernel_gen.py:28-92),
    built from the reference's own gpytorch-free GP_model classes."""
    ks = [R.ScaleKernel(R.CatKernel(2), L),
          R.ScaleKernel(R.RbfKernel(0, L), L),
          R.ScaleKernel(R.ProductKernel(R.CatKernel(2), R.RbfKernel(0, L)), L),
          R.ScaleKernel(R.ProductKernel(R.CatKernel(3), R.RbfKernel(0, L)), L),
          R.ScaleKernel(R.ProductKernel(R.CatKernel(4), R.RbfKernel(1, L)), L)]
    return R.AdditiveKernel(ks)


def randomise(module, rng, lo_s=0.3, hi_s=1.5, lo_l=1.0, hi_l=4.0):
    """Set every scale / lengthscale to a random constrained value (per latent dim)."""
    for name, p in module.named_parameters():
        n = p.numel()
        if name.endswith("_log_scale"):
            v = torch.tensor(rng.uniform(lo_s, hi_s, n))
        elif name.endswith("_log_lengthscale"):
            v = torch.tensor(rng.uniform(lo_l, hi_l, n))
        else:
            continue
        with torch.no_grad():
            p.copy_(torch.log(v - math.exp(-16.0)))


def raw_params(module):
    """Raw parameters in module traversal order, as (names, [L] arrays)."""
    names, vals = [], []
    for name, p in module.named_parameters():
        names.append(name)
        vals.append(p.detach().numpy().copy())
    return names, vals


def raw_grads(module):
    return [(p.grad.detach().numpy().copy() if p.grad is not None else np.zeros(p.shape))
            for _, p in module.named_parameters()]


def save(name, **arrs):
    path = os.path.join(OUT, name)
    np.savez_compressed(path, **{k: np.asarray(v) for k, v in arrs.items()})
    print("wrote", path, sum(np.asarray(v).nbytes for v in arrs.values()), "bytes")


# ----------------------------------------------------------------------------------------------
# 1. KL_closed (elbo_functions.py:8-34), per latent dim, value + autograd grads
# ----------------------------------------------------------------------------------------------
def gen_kl_closed(P, T, L, seed, noise, store_gram, variants=False):
    rng = np.random.default_rng(seed)
    X = covariates_missing(P, T, seed) if variants else covariates(P, T, seed)
    N = P * T
    mu = rng.standard_normal((N, L))
    logv = 0.1 * rng.standard_normal((N, L))
    out = dict(X=X, mu=mu, logv=logv, noise=np.full(L, noise), P=P, T=T, L=L)
    kls, dmus, dlogvs, draws, grams, rawvals = [], [], [], [], [], []
    for l in range(L):
        if variants:  # the per-dim kernel as (non-id components, id components) of the builder
            c = dict(VAR_CFG)
            k0, k1 = R.generate_kernel_batched(1, c['cat_kernel'], c['bin_kernel'], c['sqexp_kernel'],
                                               c['cat_int_kernel'], c['bin_int_kernel'],
                                               c['covariate_missing_val'], c['id_covariate'])
            k = R.AdditiveKernel(list(k0.kernels) + list(k1.kernels))
        else:
            k = full_kernel_ref(1)
        randomise(k, rng)
        names, vals = raw_params(k)
        rawvals.append(np.concatenate(vals))
        x = torch.tensor(X)
        m_ = torch.tensor(mu[:, l], requires_grad=True)
        lv_ = torch.tensor(logv[:, l], requires_grad=True)
        lik = LikStub(torch.tensor([noise]))
        kl = EF.KL_closed(KernelAdapter(k), x, lik, x, m_, lv_)
        kl.backward()
        kls.append(kl.item())
        dmus.append(m_.grad.numpy().copy())
        dlogvs.append(lv_.grad.numpy().copy())
        draws.append(np.concatenate(raw_grads(k)))
        if store_gram:
            with torch.no_grad():
                grams.append(k(x, x).numpy().copy())
    out.update(kl=np.array(kls), dmu=np.stack(dmus, 1), dlogv=np.stack(dlogvs, 1),
               raw=np.stack(rawvals), draw=np.stack(draws), param_names=np.array(names))
    if store_gram:
        out["gram"] = np.stack(grams)
    return out


# ----------------------------------------------------------------------------------------------
# 2. minibatch_KLD_upper_bound (elbo_functions.py:144-216) + _iter (219-307)
# ----------------------------------------------------------------------------------------------
def batched_kernels(L, cfg=None):
    c = cfg or CFG
    return R.generate_kernel_batched(L, c['cat_kernel'], c['bin_kernel'], c['sqexp_kernel'],
                                     c['cat_int_kernel'], c['bin_int_kernel'],
                                     c['covariate_missing_val'], c['id_covariate'])


def gen_hensman(P_tot, T, L, M, P_b, seed, natural_gradient, benign=False, noise=1.0, variants=False):
    rng = np.random.default_rng(seed)
    X = covariates_missing(P_tot, T, seed) if variants else covariates(P_tot, T, seed)
    N = P_tot * T
    k0, k1 = batched_kernels(L, VAR_CFG if variants else None)
    randomise(k0, rng)
    randomise(k1, rng)
    perm = rng.permutation(P_tot)[:P_b]
    idx = np.concatenate([np.arange(T * s, T * (s + 1)) for s in perm])
    xb = X[idx]
    half = M // 2
    zrows = np.concatenate([np.arange(0, half), np.arange(N // 2, N // 2 + half)])
    Z = np.stack([X[zrows]] * L)
    B = P_b * T
    mu = rng.standard_normal((B, L))
    logv = 0.1 * rng.standard_normal((B, L))
    if benign:
        m = np.zeros((L, M, 1))
        with torch.no_grad():
            H = KernelAdapter(k0)(torch.tensor(Z), torch.tensor(Z)).evaluate().numpy().copy()
        H = H + 1e-6 * np.eye(M)
    else:
        m = rng.standard_normal((L, M, 1))
        Hr = rng.standard_normal((L, M, M)) / 10
        H = Hr @ np.transpose(Hr, (0, 2, 1))
    noise_v = np.full((L, 1), noise)
    out = dict(X_all=X, idx=idx, Z=Z, mu=mu, logv=logv, m=m, H=H, noise=noise_v, P_tot=P_tot,
               P_b=P_b, T=T, L=L, M=M, natural_gradient=int(natural_gradient), eps=1e-6)
    if variants:  # the Grams of the call convention elbo_functions.py:171-174 (right-aligned batch)
        with torch.no_grad():
            xs = torch.tensor(xb).reshape(P_b, 1, T, -1).expand(P_b, L, T, xb.shape[1])
            out.update(K0xz=KernelAdapter(k0)(torch.tensor(xb), torch.tensor(Z)).evaluate().numpy().copy(),
                       K0zz=KernelAdapter(k0)(torch.tensor(Z), torch.tensor(Z)).evaluate().numpy().copy(),
                       K1_st=KernelAdapter(k1)(xs, xs).evaluate().numpy().copy())
    n0, v0 = raw_params(k0)
    n1, v1 = raw_params(k1)
    out.update(raw0=np.stack(v0, 0), raw1=np.stack(v1, 0), names0=np.array(n0), names1=np.array(n1))

    def run(iter_variant):
        for p in list(k0.parameters()) + list(k1.parameters()):
            p.grad = None
        mu_t = torch.tensor(mu, requires_grad=True)
        lv_t = torch.tensor(logv, requires_grad=True)
        m_t = torch.tensor(m, requires_grad=not natural_gradient)
        H_t = torch.tensor(H, requires_grad=not natural_gradient)
        lik = LikStub(torch.tensor(noise_v))
        if iter_variant:
            kld, gm, gH = EF.minibatch_KLD_upper_bound_iter(
                KernelAdapter(k0), KernelAdapter(k1), lik, L, m_t, H_t,
                torch.tensor(xb), mu_t, lv_t, torch.tensor(Z), P_tot, P_b, P_tot * T, natural_gradient, 2, 1e-6)
        else:
            kld, gm, gH = EF.minibatch_KLD_upper_bound(
                KernelAdapter(k0), KernelAdapter(k1), lik, L, m_t, H_t, torch.tensor(xb), mu_t, lv_t,
                torch.tensor(Z), P_tot, P_b, T, natural_gradient, 1e-6)
        kld.sum().backward()
        res = dict(kld=kld.detach().numpy().reshape(-1)[0], dmu=mu_t.grad.numpy().copy(),
                   dlogv=lv_t.grad.numpy().copy(), draw0=np.stack(raw_grads(k0)),
                   draw1=np.stack(raw_grads(k1)))
        if natural_gradient:
            res["grad_m"] = gm.detach().numpy().copy()
            res["grad_H"] = gH.detach().numpy().copy()
        else:
            res["dm"] = m_t.grad.numpy().copy()
            res["dH"] = H_t.grad.numpy().copy()
        return res

    r = run(False)
    out.update(r)
    r_it = run(True)
    out["kld_iter"] = r_it["kld"]
    if natural_gradient:
        out["grad_m_iter"] = r_it["grad_m"]
        out["grad_H_iter"] = r_it["grad_H"]
    return out


def varying_batch(X, T, subjects, lengths, rng):
    """Rows of the given subjects, each keeping a sorted random subset of its T time points;
    subjects appear in the given (unsorted) order, rows subject-contiguous."""
    rows = []
    for s, n in zip(subjects, lengths):
        keep = np.sort(rng.choice(T, size=n, replace=False))
        rows.append(T * s + keep)
    return np.concatenate(rows)


def gen_hensman_iter(P_tot, T, L, M, seed, lengths, natural_gradient):
    """minibatch_KLD_upper_bound_iter (elbo_functions.py:219-307) on subjects of varying length."""
    rng = np.random.default_rng(seed)
    X = covariates(P_tot, T, seed)
    k0, k1 = batched_kernels(L)
    randomise(k0, rng)
    randomise(k1, rng)
    subjects = rng.permutation(P_tot)[:len(lengths)]
    idx = varying_batch(X, T, subjects, lengths, rng)
    xb = X[idx]
    N_tot = int(sum(lengths)) * P_tot // len(lengths) + 3  # any N: enters as -L N / 2
    half = M // 2
    zrows = np.concatenate([np.arange(0, half), np.arange(P_tot * T // 2, P_tot * T // 2 + half)])
    Z = np.stack([X[zrows]] * L)
    B = len(idx)
    mu = rng.standard_normal((B, L))
    logv = 0.1 * rng.standard_normal((B, L))
    m = rng.standard_normal((L, M, 1))
    Hr = rng.standard_normal((L, M, M)) / 10
    H = Hr @ np.transpose(Hr, (0, 2, 1)) + 0.05 * np.eye(M)
    noise_v = np.full((L, 1), 0.9)
    out = dict(X_all=X, idx=idx, Z=Z, mu=mu, logv=logv, m=m, H=H, noise=noise_v, P_tot=P_tot,
               P_in_batch=len(lengths), N=N_tot, T=T, L=L, M=M, natural_gradient=int(natural_gradient),
               eps=1e-6, id_covariate=2, lengths=np.array(lengths))
    n0, v0 = raw_params(k0)
    n1, v1 = raw_params(k1)
    out.update(raw0=np.stack(v0, 0), raw1=np.stack(v1, 0))
    mu_t = torch.tensor(mu, requires_grad=True)
    lv_t = torch.tensor(logv, requires_grad=True)
    m_t = torch.tensor(m, requires_grad=not natural_gradient)
    H_t = torch.tensor(H, requires_grad=not natural_gradient)
    kld, gm, gH = EF.minibatch_KLD_upper_bound_iter(
        KernelAdapter(k0), KernelAdapter(k1), LikStub(torch.tensor(noise_v)), L, m_t, H_t, torch.tensor(xb),
        mu_t, lv_t, torch.tensor(Z), P_tot, len(lengths), N_tot, natural_gradient, 2, 1e-6)
    kld.sum().backward()
    out.update(kld=kld.detach().numpy().reshape(-1)[0], dmu=mu_t.grad.numpy().copy(),
               dlogv=lv_t.grad.numpy().copy(), draw0=np.stack(raw_grads(k0)), draw1=np.stack(raw_grads(k1)))
    if natural_gradient:
        out.update(grad_m=gm.detach().numpy().copy(), grad_H=gH.detach().numpy().copy())
    else:
        out.update(dm=m_t.grad.numpy().copy(), dH=H_t.grad.numpy().copy())
    return out


def gen_predict(P, T, L, M, seed, pred_lengths, test_subjects, test_lengths):
    """utils.batch_predict_varying_T (utils.py:115-211): GP posterior mean of the latents at the
    test covariates given the (varying-length) prediction set and its encoder means."""
    import utils as RU  # noqa: E402  (reference)
    rng = np.random.default_rng(seed)
    X = covariates(P, T, seed)
    k0, k1 = batched_kernels(L)
    randomise(k0, rng)
    randomise(k1, rng)
    pidx = varying_batch(X, T, np.arange(P), pred_lengths, rng)
    tidx = varying_batch(X, T, np.asarray(test_subjects), test_lengths, rng)
    half = M // 2
    zrows = np.concatenate([np.arange(0, half), np.arange(P * T // 2, P * T // 2 + half)])
    Z = np.stack([X[zrows]] * L)
    mu = rng.standard_normal((len(pidx), L))
    noise_v = np.full((L, 1), 1.1)
    with torch.no_grad():
        zp = RU.batch_predict_varying_T(L, KernelAdapter(k0), KernelAdapter(k1), LikStub(torch.tensor(noise_v)),
                                        torch.tensor(X[pidx]), torch.tensor(X[tidx]), torch.tensor(mu),
                                        torch.tensor(Z), 2, 1e-6)
    n0, v0 = raw_params(k0)
    n1, v1 = raw_params(k1)
    return dict(X_all=X, pidx=pidx, tidx=tidx, Z=Z, mu=mu, noise=noise_v, L=L, M=M, eps=1e-6, id_covariate=2,
                raw0=np.stack(v0, 0), raw1=np.stack(v1, 0), Z_pred=zp.numpy().copy())


# ----------------------------------------------------------------------------------------------
# 3. per-dim GPapprox: elbo (36-84) and deviance_upper_bound (86-142)
# ----------------------------------------------------------------------------------------------
def gen_gpapprox(P, T, M, seed, noise=1.0):
    rng = np.random.default_rng(seed)
    X = covariates(P, T, seed)
    N = P * T
    k0, k1 = batched_kernels(1)
    randomise(k0, rng)
    randomise(k1, rng)
    half = M // 2
    zrows = np.concatenate([np.arange(0, half), np.arange(N // 2, N // 2 + half)])
    Z = X[zrows]
    y = rng.standard_normal(N)
    mu = rng.standard_normal(N)
    logv = 0.1 * rng.standard_normal(N)
    lik = LikStub(torch.tensor([noise]))
    out = dict(X=X, Z=Z, y=y, mu=mu, logv=logv, noise=noise, P=P, T=T, M=M, eps=1e-6)
    n0, v0 = raw_params(k0)
    n1, v1 = raw_params(k1)
    out.update(raw0=np.stack(v0), raw1=np.stack(v1))

    K2 = KernelAdapter  # 2-D / 3-D inputs with [1] params broadcast identically either way

    # elbo
    for p in list(k0.parameters()) + list(k1.parameters()):
        p.grad = None
    y_t = torch.tensor(y, requires_grad=True)
    el = EF.elbo(K2(k0), K2(k1), lik, torch.tensor(X), y_t, torch.tensor(Z), P, T, 1e-6)
    el = el.reshape(-1)[0]
    el.backward()
    out.update(elbo=el.item(), elbo_dy=y_t.grad.numpy().copy(),
               elbo_draw0=np.stack(raw_grads(k0)), elbo_draw1=np.stack(raw_grads(k1)))
    # dubo
    for p in list(k0.parameters()) + list(k1.parameters()):
        p.grad = None
    mu_t = torch.tensor(mu, requires_grad=True)
    lv_t = torch.tensor(logv, requires_grad=True)
    du = EF.deviance_upper_bound(K2(k0), K2(k1), lik, torch.tensor(X), mu_t, lv_t, torch.tensor(Z),
                                 P, T, 1e-6)
    du = du.reshape(-1)[0]
    du.backward()
    out.update(dubo=du.item(), dubo_dmu=mu_t.grad.numpy().copy(), dubo_dlogv=lv_t.grad.numpy().copy(),
               dubo_draw0=np.stack(raw_grads(k0)), dubo_draw1=np.stack(raw_grads(k1)))
    return out


# ----------------------------------------------------------------------------------------------
# 4. ConvVAE (VAE.py:16-162): weights from a numpy formula (regenerable), fp64
# ----------------------------------------------------------------------------------------------
def vae_weights(model, seed):
    rng = np.random.default_rng(seed)
    sd = {}
    for name, p in model.state_dict().items():
        if name == "min_log_vy":
            sd[name] = p.clone()
        elif name == "_log_vy":
            sd[name] = torch.tensor(0.1 * rng.standard_normal(p.shape))
        else:
            fan = p[0].numel() if p.dim() > 1 else p.numel()
            sd[name] = torch.tensor(rng.standard_normal(p.shape) / math.sqrt(max(fan, 1)))
    return sd


def gen_vae(L, B, seed):
    rng = np.random.default_rng(seed)
    model = RV.ConvVAE(L, 1296, vy_init=1.0, p_input=0.0, p=0.0).double()
    model.load_state_dict(vae_weights(model, seed))
    model.eval()
    x = rng.uniform(0, 1, (B, 1, 36, 36))
    mask = rng.binomial(1, 0.75, (B, 1, 36, 36)).astype(np.float64)
    eps = rng.standard_normal((B, L))
    xt = torch.tensor(x)
    mu, logv = model.encode(xt)
    z = mu + torch.tensor(eps) * torch.exp(0.5 * logv)
    recon = model.decode(z)
    mse, nll = model.loss_function(recon, xt, torch.tensor(mask))
    loss = mse.sum() + nll.sum() + (mu ** 2).sum() + logv.sum()
    loss.backward()
    grads = {("g_" + n): p.grad.numpy().copy() for n, p in model.named_parameters()
             if n in ("conv1.weight", "fc1.bias", "fc211.weight", "deconv2.weight", "_log_vy")}
    return dict(x=x, mask=mask, eps=eps, L=L, seed=seed, mu=mu.detach().numpy(),
                logv=logv.detach().numpy(), recon=recon.detach().numpy().reshape(B, -1)[:, ::7],
                mse=mse.detach().numpy(), nll=nll.detach().numpy(), loss=loss.item(), **grads)


# ----------------------------------------------------------------------------------------------
# 5. data ingest: HealthMNISTDatasetConv (dataset_def.py:172-219) on a tiny CSV trio written in
#    Health_MNIST_generate.py's format (fixture files committed under tests/golden/hmnist_tiny/)
# ----------------------------------------------------------------------------------------------
def gen_hmnist_tiny(seed):
    sys.path.insert(0, os.path.join(os.path.dirname(OUT), "..", "longitudinal-vae_amd"))
    from lvae_amd.data import write_health_mnist_csv  # our writer (format under test)
    import dataset_def as RD  # noqa: E402  (reference)
    rng = np.random.default_rng(seed)
    P, T = 3, 4
    N = P * T
    pixels = rng.integers(0, 256, size=(N, 1296))
    mask = rng.binomial(1, 0.75, size=(N, 1296))
    labels = np.zeros((N, 8))
    for r in range(N):
        p, t = divmod(r, T)
        sick = p % 2
        labels[r] = [p, 5, 0.0, sick, (t - 2) if sick else np.nan, p >= 1, t, (p + 1) % 2]
    d = os.path.join(OUT, "hmnist_tiny")
    os.makedirs(d, exist_ok=True)
    fd, fl, fm = write_health_mnist_csv(d, pixels, mask, labels, prefix="tiny")
    ds = RD.HealthMNISTDatasetConv(csv_file_data=fd, csv_file_label=fl, mask_file=fm, root_dir=d, transform=None)
    items = [ds[i] for i in range(len(ds))]
    return dict(files=np.array([fd, fl, fm]), digit=np.stack([it["digit"] for it in items]),
                label=np.stack([it["label"].numpy() for it in items]), mask=np.stack([it["mask"] for it in items]),
                n=len(ds))


# ----------------------------------------------------------------------------------------------
# 6. samplers (utils.py:40-113) under np.random.seed: the row orders the reference draws
# ----------------------------------------------------------------------------------------------
class _ListDS:
    def __init__(self, labels):
        self.labels = labels

    def __len__(self):
        return len(self.labels)

    def __getitem__(self, i):
        return {"label": torch.tensor(self.labels[i])}


def gen_samplers(seed):
    import utils as RU  # noqa: E402  (reference)
    from torch.utils.data.sampler import BatchSampler
    P, T, P_b = 11, 4, 3
    ds = _ListDS(np.zeros((P * T, 6)))
    np.random.seed(seed)
    ss = RU.SubjectSampler(ds, P, T)
    epochs = [np.array(list(iter(ss))) for _ in range(3)]
    batches = [np.array(b) for b in BatchSampler(ss, P_b * T, drop_last=False)]
    # varying length: subject ids in contiguous runs of lengths 1..5
    lengths = [3, 1, 5, 2, 4, 3, 2]
    ids = np.concatenate([np.full(n, 10 + i) for i, n in enumerate(lengths)]).astype(np.float64)
    lab = np.zeros((len(ids), 6))
    lab[:, 2] = ids
    vds = _ListDS(lab)
    np.random.seed(seed + 1)
    vs = RU.VaryingLengthSubjectSampler(vds, 2)
    v_pairs = [np.array(list(iter(vs))) for _ in range(2)]
    v_batches = [np.array(b) for b in RU.VaryingLengthBatchSampler(vs, 3)]
    return dict(P=P, T=T, P_b=P_b, seed=seed, epochs=np.stack(epochs), batch_lens=np.array([len(b) for b in batches]),
                batches=np.concatenate(batches), v_ids=ids, v_pairs=np.stack(v_pairs),
                v_batch_lens=np.array([len(b) for b in v_batches]), v_batches=np.concatenate(v_batches))


# ----------------------------------------------------------------------------------------------
# 7. two epochs of training.hensman_training (training.py:15-237), natural gradient, loss 'mse',
#    driven with an injected subject order (np.random.seed before the call: SubjectSampler's
#    np.random.shuffle is the only consumer of that state) and injected reparametrisation noise
#    (a ConvVAE subclass whose sample_latent reads a fixed eps queue instead of torch.randn_like).
#    Per step the harness records the batch's subject ids and the KL bound (a recording wrapper
#    around training.minibatch_KLD_upper_bound) and the recon / nll sums (loss_function wrapper).
# ----------------------------------------------------------------------------------------------
def gen_hensman_training(P, T, L, M, P_b, seed, epochs=2):
    import training as RT  # noqa: E402  (reference)
    rng = np.random.default_rng(seed)
    X = covariates(P, T, seed)
    N = P * T
    pix = rng.integers(0, 256, size=(N, 1, 36, 36)).astype(np.uint8)
    msk = rng.binomial(1, 0.75, size=(N, 1, 36, 36)).astype(np.uint8)
    n_batches = (N + P_b * T - 1) // (P_b * T)
    EPS = rng.standard_normal((epochs * n_batches, P_b * T, L))

    class DS(torch.utils.data.Dataset):
        def __len__(self):
            return N

        def __getitem__(self, i):
            return {"idx": i, "digit": torch.tensor(pix[i] / 255.0), "label": torch.tensor(X[i]),
                    "mask": torch.tensor(msk[i].astype(np.float64))}

    rec = {"ids": [], "kld": [], "recon": [], "nll": []}

    class VAE(RV.ConvVAE):
        step = 0

        def sample_latent(self, mu, log_var):
            e = torch.tensor(EPS[VAE.step][:mu.shape[0]])
            VAE.step += 1
            return mu + e * torch.exp(0.5 * log_var)

        def loss_function(self, recon_x, x, mask):
            out = super().loss_function(recon_x, x, mask)
            rec["recon"].append(out[0].sum().item())
            rec["nll"].append(out[1].sum().item())
            return out

    model = VAE(L, 1296, vy_init=1.0, p_input=0.0, p=0.0).double()
    model.load_state_dict(vae_weights(model, seed))
    k0, k1 = batched_kernels(L)
    randomise(k0, rng)
    randomise(k1, rng)
    half = M // 2
    zrows = np.concatenate([np.arange(0, half), np.arange(N // 2, N // 2 + half)])
    Z = np.stack([X[zrows]] * L)
    m0 = rng.standard_normal((L, M, 1))
    Hr = rng.standard_normal((L, M, M)) / 10
    H0 = Hr @ np.transpose(Hr, (0, 2, 1))
    n0, v0 = raw_params(k0)
    n1, v1 = raw_params(k1)
    vae0 = {k: v.numpy().copy() for k, v in model.state_dict().items()}
    opt = torch.optim.Adam([{"params": k0.parameters()}, {"params": k1.parameters()},
                            {"params": model.parameters()}], lr=1e-3)
    orig = RT.minibatch_KLD_upper_bound

    def recording(*a, **kw):
        out = orig(*a, **kw)
        rec["ids"].append(a[6][:, 2].numpy().copy())
        rec["kld"].append(out[0].item())
        return out

    RT.minibatch_KLD_upper_bound = recording
    try:
        np.random.seed(seed)
        res = RT.hensman_training(model, "conv", epochs, DS(), opt, "GPapprox_closed", 1, L, KernelAdapter(k0),
                                  KernelAdapter(k1), LikStub(torch.ones(L, 1)), torch.tensor(m0), torch.tensor(H0),
                                  torch.tensor(Z), P, T, False, 6, 0.15, 2, "mse", natural_gradient=True,
                                  natural_gradient_lr=0.01, subjects_per_batch=P_b, eps=1e-6)
    finally:
        RT.minibatch_KLD_upper_bound = orig
    _, net_arr, nll_arr, recon_arr, kld_arr, m_fin, H_fin, _ = res
    np.random.seed(seed)
    perms = []
    for _ in range(epochs):
        r = np.arange(P)
        np.random.shuffle(r)
        perms.append(r)
    ids = np.concatenate(rec["ids"])
    assert np.array_equal(ids[::T].astype(np.int64), np.concatenate(perms)), "subject order != seeded shuffles"
    fin = {("vae_" + k): v.detach().numpy().copy() for k, v in model.named_parameters()
           if k in ("conv1.weight", "fc211.bias", "deconv2.weight", "_log_vy")}
    fin["vae_fc1_rowsum"] = model.fc1.weight.detach().sum(1).numpy().copy()
    return dict(P=P, T=T, L=L, M=M, P_b=P_b, seed=seed, epochs=epochs, X=X, pix=pix, msk=msk, eps=EPS, Z=Z,
                m0=m0, H0=H0, raw0=np.stack(v0, 0), raw1=np.stack(v1, 0), perms=np.stack(perms),
                step_kld=np.array(rec["kld"]), step_recon=np.array(rec["recon"]), step_nll=np.array(rec["nll"]),
                epoch_net=net_arr, epoch_recon=recon_arr, epoch_nll=nll_arr, epoch_kld=kld_arr,
                m_final=m_fin.numpy().copy(), H_final=H_fin.numpy().copy(),
                raw0_final=np.stack(raw_params(k0)[1], 0), raw1_final=np.stack(raw_params(k1)[1], 0), **fin)


# ----------------------------------------------------------------------------------------------
# 8. epochs of training.standard_training with type_KL='closed' (training.py:431-592): full batch,
#    per-dim kernels and likelihoods, constrain_scales.  The reference samples the latent twice
#    per step (the forward's draw feeds the decoder; the num_samples loop's draw is unused for
#    'closed'), so the eps queue holds two entries per step and the decoder uses the first.
# ----------------------------------------------------------------------------------------------
def gen_standard_training(P, T, L, seed, epochs=3):
    import training as RT  # noqa: E402  (reference)
    rng = np.random.default_rng(seed)
    X = covariates(P, T, seed)
    N = P * T
    pix = rng.integers(0, 256, size=(N, 1, 36, 36)).astype(np.uint8)
    msk = rng.binomial(1, 0.75, size=(N, 1, 36, 36)).astype(np.uint8)
    EPS = rng.standard_normal((2 * epochs, N, L))

    class DS(torch.utils.data.Dataset):
        def __len__(self):
            return N

        def __getitem__(self, i):
            return {"idx": i, "digit": torch.tensor(pix[i] / 255.0), "label": torch.tensor(X[i]),
                    "mask": torch.tensor(msk[i].astype(np.float64))}

    class VAE(RV.ConvVAE):
        calls = 0

        def sample_latent(self, mu, log_var):
            e = torch.tensor(EPS[VAE.calls])
            VAE.calls += 1
            return mu + e * torch.exp(0.5 * log_var)

    model = VAE(L, 1296, vy_init=1.0, p_input=0.0, p=0.0).double()
    model.load_state_dict(vae_weights(model, seed))
    kernels = []
    for _ in range(L):
        k = full_kernel_ref(1)
        randomise(k, rng)
        kernels.append(k)
    raw_init = np.stack([np.concatenate(raw_params(k)[1]) for k in kernels])
    liks = [LikStub(torch.tensor([1.0])) for _ in range(L)]
    groups = [{"params": k.parameters()} for k in kernels] + [{"params": model.parameters()}]
    opt = torch.optim.Adam(groups, lr=1e-3)
    res = RT.standard_training(model, "conv", epochs, DS(), opt, "closed", 1, L,
                               [[KernelAdapter(k) for k in kernels]], liks, None, 2, P, T, 6, 0.15, True, "mse")
    _, net_arr, nll_arr, recon_arr, gp_arr = res
    fin = {("vae_" + k): v.detach().numpy().copy() for k, v in model.named_parameters()
           if k in ("conv1.weight", "fc211.bias", "deconv2.weight", "_log_vy")}
    fin["vae_fc1_rowsum"] = model.fc1.weight.detach().sum(1).numpy().copy()
    return dict(P=P, T=T, L=L, seed=seed, epochs=epochs, X=X, pix=pix, msk=msk, eps=EPS, raw=raw_init,
                step_net=net_arr, step_recon=recon_arr, step_nll=nll_arr, step_gp=gp_arr,
                raw_final=np.stack([np.concatenate(raw_params(k)[1]) for k in kernels]), **fin)


def main(only=None):
    jobs = {
        "kernel_variants_kl.npz": lambda: gen_kl_closed(P=5, T=16, L=2, seed=12, noise=0.9, store_gram=True,
                                                        variants=True),
        "kernel_variants_hensman.npz": lambda: gen_hensman(P_tot=24, T=16, L=3, M=40, P_b=4, seed=13,
                                                           natural_gradient=True, variants=True),
        "samplers.npz": lambda: gen_samplers(seed=14),
        "hensman_training_2ep.npz": lambda: gen_hensman_training(P=8, T=16, L=2, M=20, P_b=3, seed=15),
        "standard_training_closed.npz": lambda: gen_standard_training(P=4, T=16, L=2, seed=16),
    }
    if only:
        for name in only:
            save(name, **jobs[name]())
        return
    save("kl_closed_n64.npz", **gen_kl_closed(P=4, T=16, L=2, seed=0, noise=1.0, store_gram=True))
    save("kl_closed_n256.npz", **gen_kl_closed(P=16, T=16, L=2, seed=1, noise=1.0, store_gram=False))
    save("kl_closed_n96_noise.npz", **gen_kl_closed(P=6, T=16, L=1, seed=2, noise=0.7, store_gram=False))
    save("hensman_ng.npz", **gen_hensman(P_tot=32, T=16, L=4, M=60, P_b=5, seed=3, natural_gradient=True))
    save("hensman_ng_benign.npz", **gen_hensman(P_tot=32, T=16, L=4, M=60, P_b=5, seed=4,
                                                natural_gradient=True, benign=True))
    save("hensman_adam.npz", **gen_hensman(P_tot=32, T=16, L=3, M=40, P_b=4, seed=5,
                                           natural_gradient=False, noise=0.8))
    save("gpapprox.npz", **gen_gpapprox(P=16, T=16, M=40, seed=6))
    save("convvae.npz", **gen_vae(L=4, B=6, seed=7))
    save("hensman_iter_ng.npz", **gen_hensman_iter(P_tot=24, T=16, L=3, M=40, seed=8,
                                                   lengths=[16, 11, 7, 14, 9], natural_gradient=True))
    save("hensman_iter_adam.npz", **gen_hensman_iter(P_tot=24, T=16, L=2, M=40, seed=9,
                                                     lengths=[5, 16, 12], natural_gradient=False))
    save("hmnist_tiny.npz", **gen_hmnist_tiny(seed=11))
    save("predict_varying.npz", **gen_predict(P=12, T=16, L=3, M=40, seed=10,
                                              pred_lengths=[16, 9, 12, 16, 5, 14, 16, 8, 11, 16, 13, 7],
                                              test_subjects=[3, 0, 7, 10], test_lengths=[6, 4, 10, 3]))


    for name, job in jobs.items():
        save(name, **job())


if __name__ == "__main__":
    main(sys.argv[1:])
