"""GP posterior prediction of the latents (utils.py:115-211 batch_predict_varying_T), the step
MSE_test_GPapprox (model_test.py:85-143) runs after training.  Same signature and return value;
the computation is one batched HIP pass (lvae_predict_f64) instead of the reference's per-subject
Python loops and its removed ``torch.solve``.
"""
import torch

from . import _lib
from .elbo import _check_info, _noise_vector, _stack_modules, _subject_layout


def batch_predict_varying_T(latent_dim, covar_module0, covar_module1, likelihoods, prediction_x, test_x, mu,
                            zt_list, id_covariate, eps):
    """Z_pred [N_test, L]: posterior mean of the L latent GPs at ``test_x`` given the encoder means
    ``mu`` [N_pred, L] at ``prediction_x`` (subjects of any length).  ``covar_module0/1`` are
    batched modules or per-dim lists, ``zt_list`` the inducing points [L, M, Q] (or a per-dim
    list of [M, Q])."""
    lib = _lib.lib()
    L = int(latent_dim)
    spec0, params0 = _stack_modules(covar_module0)
    spec1, params1 = _stack_modules(covar_module1)
    if params0.shape[0] == 1 and L > 1:
        params0 = params0.expand(L, -1)
    if params1.shape[0] == 1 and L > 1:
        params1 = params1.expand(L, -1)
    for mod in (covar_module0, covar_module1, likelihoods):
        for m_ in (mod if isinstance(mod, (list, tuple, torch.nn.ModuleList)) else [mod]):
            if hasattr(m_, "eval"):
                m_.eval()
    dev = mu.device
    f64 = lambda t: t.detach().to(dev, torch.float64).contiguous()
    if isinstance(zt_list, (list, tuple)):
        z = torch.stack([f64(zi) for zi in zt_list])
    else:
        z = f64(zt_list)
        if z.dim() == 2:
            z = z.unsqueeze(0).expand(L, -1, -1).contiguous()
    M, Q = z.shape[1], z.shape[2]
    noise = f64(_noise_vector(likelihoods, L)).reshape(L)
    gather, valid, seg, T = _subject_layout(prediction_x[:, id_covariate])
    P = int(seg.numel())
    pred_ids = torch.unique(prediction_x[:, id_covariate].detach().to("cpu", torch.float64))
    test_ids = torch.unique(test_x[:, id_covariate].detach().to("cpu", torch.float64))
    include = torch.isin(pred_ids, test_ids).to(torch.int32)
    g = gather.to(dev)
    x_pad = f64(prediction_x)[g].contiguous()
    mu_pad = (f64(mu)[g] * valid.to(dev, torch.float64).unsqueeze(1)).contiguous()
    tx = f64(test_x)
    Nt = int(tx.shape[0])
    seg_d, inc_d = seg.to(dev), include.to(dev)
    p0, p1 = f64(params0), f64(params1)
    out = torch.empty(Nt, L, dtype=torch.float64, device=dev)
    info = torch.empty(L, dtype=torch.int32, device=dev)
    ws = torch.empty(int(lib.lvae_predict_workspace_size(L, M, P, T, Nt)), dtype=torch.uint8, device=dev)
    rc = lib.lvae_predict_f64(spec0, spec1, L, M, Q, P, T, _lib.ptr(seg_d), _lib.ptr(inc_d), _lib.ptr(x_pad),
                              _lib.ptr(mu_pad), _lib.ptr(z), Nt, _lib.ptr(tx), _lib.ptr(p0), _lib.ptr(p1),
                              _lib.ptr(noise), float(eps), _lib.ptr(out), _lib.ptr(info), _lib.ptr(ws),
                              _lib.stream_ptr())
    _lib.check(rc, "predict")
    _check_info(info, "batch_predict_varying_T cholesky (10000+col: K0zz, 20000+col: B_st, 30000+col: H)")
    return out
