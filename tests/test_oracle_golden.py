"""The CPU oracle (oracle/lvae_oracle.py) against golden vectors from the reference itself."""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import lvae_oracle as O

CFG = dict(cat_kernel=[2], bin_kernel=[], sqexp_kernel=[0],
           cat_int_kernel=[{'cont_covariate': 0, 'cat_covariate': 2},
                           {'cont_covariate': 0, 'cat_covariate': 3},
                           {'cont_covariate': 1, 'cat_covariate': 4}],
           bin_int_kernel=[], covariate_missing_val=[])


def rel(a, b):
    if isinstance(a, torch.Tensor):
        a = a.detach().cpu().numpy()
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-300)


def spec_full():
    return O.spec_full(**CFG)


def spec_split():
    return O.spec_split(**CFG, id_covariate=2)


@pytest.mark.parametrize("name", ["kl_closed_n64.npz", "kl_closed_n256.npz", "kl_closed_n96_noise.npz"])
def test_kl_closed(name):
    g = golden(name)
    spec = spec_full()
    assert O.n_params(spec) == g["raw"].shape[1]
    X = torch.tensor(g["X"])
    for l in range(int(g["L"])):
        raw = torch.tensor(g["raw"][l], requires_grad=True)
        mu = torch.tensor(g["mu"][:, l], requires_grad=True)
        lv = torch.tensor(g["logv"][:, l], requires_grad=True)
        kl = O.kl_closed(spec, O.constrain(raw), X, float(g["noise"][l]), mu, lv)
        kl.backward()
        assert rel(kl.item(), g["kl"][l]) < 1e-12
        assert rel(mu.grad, g["dmu"][:, l]) < 1e-10
        assert rel(lv.grad, g["dlogv"][:, l]) < 1e-10
        assert rel(raw.grad, g["draw"][l]) < 1e-9
        if "gram" in g.files:
            with torch.no_grad():
                K = O.gram(spec, O.constrain(raw), X, X)
            assert rel(K, g["gram"][l]) < 1e-14


@pytest.mark.parametrize("name", ["hensman_ng.npz", "hensman_ng_benign.npz", "hensman_adam.npz"])
def test_hensman(name):
    g = golden(name)
    s0, s1 = spec_split()
    ng = bool(g["natural_gradient"])
    raw0 = torch.tensor(g["raw0"].T.copy(), requires_grad=True)  # [L, P0]
    raw1 = torch.tensor(g["raw1"].T.copy(), requires_grad=True)
    X = torch.tensor(g["X_all"][g["idx"]])
    mu = torch.tensor(g["mu"], requires_grad=True)
    lv = torch.tensor(g["logv"], requires_grad=True)
    m = torch.tensor(g["m"], requires_grad=not ng)
    H = torch.tensor(g["H"], requires_grad=not ng)
    kld, gm, gH = O.hensman_kld(s0, O.constrain(raw0), s1, O.constrain(raw1), torch.tensor(g["noise"]), m, H,
                                X, mu, lv, torch.tensor(g["Z"]), int(g["P_tot"]), int(g["P_b"]), int(g["T"]),
                                ng, float(g["eps"]))
    kld.backward()
    assert rel(kld.item(), g["kld"]) < 1e-10
    assert rel(mu.grad, g["dmu"]) < 1e-8
    assert rel(lv.grad, g["dlogv"]) < 1e-8
    assert rel(raw0.grad.T, g["draw0"]) < 1e-6
    assert rel(raw1.grad.T, g["draw1"]) < 1e-6
    if ng:
        assert rel(gm, g["grad_m"]) < 1e-6
        assert rel(gH, g["grad_H"]) < 1e-6
    else:
        assert rel(m.grad, g["dm"]) < 1e-8
        assert rel(H.grad, g["dH"]) < 1e-8


def test_gpapprox():
    g = golden("gpapprox.npz")
    s0, s1 = spec_split()
    args = lambda r0, r1: (s0, O.constrain(r0), s1, O.constrain(r1), float(g["noise"]))
    X, Z = torch.tensor(g["X"]), torch.tensor(g["Z"])
    P, T = int(g["P"]), int(g["T"])
    r0 = torch.tensor(g["raw0"][:, 0], requires_grad=True)
    r1 = torch.tensor(g["raw1"][:, 0], requires_grad=True)
    y = torch.tensor(g["y"], requires_grad=True)
    el = O.gpapprox_elbo(*args(r0, r1), X, y, Z, P, T, float(g["eps"]))
    el.backward()
    assert rel(el.item(), g["elbo"]) < 1e-10
    assert rel(y.grad, g["elbo_dy"]) < 1e-8
    assert rel(r0.grad, g["elbo_draw0"][:, 0]) < 1e-6
    assert rel(r1.grad, g["elbo_draw1"][:, 0]) < 1e-6
    r0 = torch.tensor(g["raw0"][:, 0], requires_grad=True)
    r1 = torch.tensor(g["raw1"][:, 0], requires_grad=True)
    mu = torch.tensor(g["mu"], requires_grad=True)
    lv = torch.tensor(g["logv"], requires_grad=True)
    du = O.deviance_upper_bound(*args(r0, r1), X, mu, lv, Z, P, T, float(g["eps"]))
    du.backward()
    assert rel(du.item(), g["dubo"]) < 1e-10
    assert rel(mu.grad, g["dubo_dmu"]) < 1e-8
    assert rel(lv.grad, g["dubo_dlogv"]) < 1e-8
    assert rel(r0.grad, g["dubo_draw0"][:, 0]) < 1e-6
    assert rel(r1.grad, g["dubo_draw1"][:, 0]) < 1e-6


def test_convvae():
    g = golden("convvae.npz")
    L = int(g["L"])
    model = O.ConvVAE(L).double()
    model.load_state_dict(O.vae_weights(model, int(g["seed"])))
    x = torch.tensor(g["x"])
    mu, lv = model.encode(x)
    z = mu + torch.tensor(g["eps"]) * torch.exp(0.5 * lv)
    recon = model.decode(z)
    mse, nll = model.loss_function(recon, x, torch.tensor(g["mask"]))
    loss = mse.sum() + nll.sum() + (mu ** 2).sum() + lv.sum()
    loss.backward()
    assert rel(mu.detach(), g["mu"]) < 1e-12
    assert rel(lv.detach(), g["logv"]) < 1e-12
    assert rel(recon.detach().reshape(x.shape[0], -1)[:, ::7], g["recon"]) < 1e-12
    assert rel(mse.detach(), g["mse"]) < 1e-12
    assert rel(nll.detach(), g["nll"]) < 1e-12
    named = dict(model.named_parameters())
    for k in g.files:
        if k.startswith("g_"):
            assert rel(named[k[2:]].grad, g[k]) < 1e-10, k


@pytest.mark.parametrize("name", ["hensman_iter_ng.npz", "hensman_iter_adam.npz"])
def test_hensman_iter_varying_T(name):
    """minibatch_KLD_upper_bound_iter (elbo_functions.py:219-307) on subjects of varying length."""
    g = golden(name)
    s0, s1 = spec_split()
    ng = bool(g["natural_gradient"])
    raw0 = torch.tensor(g["raw0"].T.copy(), requires_grad=True)
    raw1 = torch.tensor(g["raw1"].T.copy(), requires_grad=True)
    X = torch.tensor(g["X_all"][g["idx"]])
    mu = torch.tensor(g["mu"], requires_grad=True)
    lv = torch.tensor(g["logv"], requires_grad=True)
    m = torch.tensor(g["m"], requires_grad=not ng)
    H = torch.tensor(g["H"], requires_grad=not ng)
    kld, gm, gH = O.hensman_kld_iter(s0, O.constrain(raw0), s1, O.constrain(raw1), torch.tensor(g["noise"]), m, H,
                                     X, mu, lv, torch.tensor(g["Z"]), int(g["P_tot"]), int(g["P_in_batch"]),
                                     int(g["N"]), ng, int(g["id_covariate"]), float(g["eps"]))
    kld.backward()
    assert rel(kld.item(), g["kld"]) < 1e-10
    assert rel(mu.grad, g["dmu"]) < 1e-8
    assert rel(lv.grad, g["dlogv"]) < 1e-8
    assert rel(raw0.grad.T, g["draw0"]) < 1e-6
    assert rel(raw1.grad.T, g["draw1"]) < 1e-6
    if ng:
        assert rel(gm, g["grad_m"]) < 1e-6
        assert rel(gH, g["grad_H"]) < 1e-6
    else:
        assert rel(m.grad, g["dm"]) < 1e-8
        assert rel(H.grad, g["dH"]) < 1e-8


def test_batch_predict_varying_T():
    """utils.batch_predict_varying_T (utils.py:115-211)."""
    g = golden("predict_varying.npz")
    s0, s1 = spec_split()
    X = g["X_all"]
    zp = O.batch_predict_varying_T(s0, O.constrain(torch.tensor(g["raw0"].T.copy())), s1,
                                   O.constrain(torch.tensor(g["raw1"].T.copy())), torch.tensor(g["noise"]),
                                   torch.tensor(X[g["pidx"]]), torch.tensor(X[g["tidx"]]), torch.tensor(g["mu"]),
                                   torch.tensor(g["Z"]), int(g["id_covariate"]), float(g["eps"]))
    assert zp.shape == g["Z_pred"].shape
    assert rel(zp, g["Z_pred"]) < 1e-9
