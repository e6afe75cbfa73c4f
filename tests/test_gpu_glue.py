"""The glue launches (glue.hip) against the PyTorch formulas they replace, fp64 on the CPU as the reference:
ConvVAE.loss_function (VAE.py:144-162), sample_latent (VAE.py:132-136) and the kernels' positivity
transform exp(m + softplus(raw - m)) (GP_model.py:31-144), values and gradients."""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = a.detach().cpu().double()
    b = b.detach().cpu().double()
    return float((a - b).abs().max() / max(float(b.abs().max()), 1e-300))


def _loss_ref(r, x, m, lv):
    d = lv.numel()
    se = (r.reshape(-1, d) - x.reshape(-1, d)) ** 2 * m.reshape(-1, d)
    msum = m.reshape(-1, d).sum(1)
    msum = torch.where(msum == 0, torch.ones_like(msum), msum)
    return se.sum(1) / msum, (se / (2 * torch.exp(lv)) + 0.5 * (math.log(2 * math.pi) + lv)).sum(1)


@pytest.mark.parametrize("B", [1, 67, 300])
def test_vae_loss_fused(hip, B):
    """Per-image masked MSE / NLL and d recon, d log_vy: ragged image counts (the backward's 64-image
    chunks), one image with an all-zero mask (msum -> 1), weights on both outputs."""
    from lvae_amd.vae import ConvVAE
    torch.manual_seed(B)
    vae = ConvVAE(2, 1296).cuda()
    with torch.no_grad():
        vae._log_vy.copy_(0.3 * torch.randn(1296))
    r = torch.rand(B, 1, 36, 36, device="cuda", requires_grad=True)
    x = torch.rand(B, 1, 36, 36, device="cuda")
    m = (torch.rand(B, 1, 36, 36, device="cuda") > 0.2).float()
    m[0] = 0.0
    mse, nll = vae.loss_function(r, x, m)
    w1, w2 = torch.rand(B, device="cuda"), torch.rand(B, device="cuda")
    ((mse * w1).sum() + (nll * w2).sum()).backward()
    r64 = r.detach().cpu().double().requires_grad_()
    lv64 = vae._log_vy.detach().cpu().double().requires_grad_()
    mse_r, nll_r = _loss_ref(r64, x.cpu().double(), m.cpu().double(), lv64)
    ((mse_r * w1.cpu().double()).sum() + (nll_r * w2.cpu().double()).sum()).backward()
    errs = dict(mse=rel(mse, mse_r), nll=rel(nll, nll_r), dr=rel(r.grad, r64.grad), dlv=rel(vae._log_vy.grad, lv64.grad))
    print(B, errs)
    for k, e in errs.items():
        assert e < 2e-5, (k, e)
    # the reduction-only use (the steps' mse.sum() / nll.sum(): the backward sees stride-0 gradients)
    r.grad = None
    vae._log_vy.grad = None
    mse, nll = vae.loss_function(r, x, m)
    (mse.sum() + 0.5 * nll.sum()).backward()
    r64.grad = None
    lv64.grad = None
    mse_r, nll_r = _loss_ref(r64, x.cpu().double(), m.cpu().double(), lv64)
    (mse_r.sum() + 0.5 * nll_r.sum()).backward()
    assert rel(r.grad, r64.grad) < 2e-5 and rel(vae._log_vy.grad, lv64.grad) < 2e-5


def test_reparam_fused(hip):
    from lvae_amd.vae import ConvVAE
    vae = ConvVAE(16, 1296).cuda()
    torch.manual_seed(3)
    mu = torch.randn(1000, 16, device="cuda", requires_grad=True)
    lv = torch.randn(1000, 16, device="cuda", requires_grad=True)
    eps = torch.randn(1000, 16, device="cuda")
    z = vae.sample_latent(mu, lv, eps)
    g = torch.randn_like(z)
    (z * g).sum().backward()
    mu64, lv64 = mu.detach().cpu().double().requires_grad_(), lv.detach().cpu().double().requires_grad_()
    z64 = mu64 + eps.cpu().double() * torch.exp(0.5 * lv64)
    (z64 * g.cpu().double()).sum().backward()
    assert rel(z, z64) < 1e-6 and rel(mu.grad, mu64.grad) < 1e-6 and rel(lv.grad, lv64.grad) < 1e-6


def test_param_pack_fused(hip):
    """kernel_spec_and_params through the fused launch (fp64 CUDA raws) against the stacked PyTorch
    transform (the same module on the CPU): the [L, P] matrix to fp64 rounding, the raw gradients to
    1e-13, one raw parameter on softplus' linear branch."""
    import lvae_amd as la
    from lvae_amd.kernels import kernel_spec_and_params
    CFG = dict(cat_kernel=[2], bin_kernel=[], sqexp_kernel=[0],
               cat_int_kernel=[{'cont_covariate': 0, 'cat_covariate': 2},
                               {'cont_covariate': 0, 'cat_covariate': 3},
                               {'cont_covariate': 1, 'cat_covariate': 4}],
               bin_int_kernel=[], covariate_missing_val=[])
    for L in (1, 16):
        k = la.generate_kernel(**CFG, latent_dim=L).double()
        rng = np.random.default_rng(L)
        with torch.no_grad():
            for p in k.parameters():
                p.copy_(torch.as_tensor(rng.normal(0.0, 1.5, p.shape)))
            next(iter(k.parameters()))[0] = 30.0  # softplus' linear branch
        kc = la.generate_kernel(**CFG, latent_dim=L).double()
        kc.load_state_dict(k.state_dict())
        kg = k.cuda()
        spec_g, Pg = kernel_spec_and_params(kg)
        spec_c, Pc = kernel_spec_and_params(kc)
        assert Pg.shape == Pc.shape and Pg.is_contiguous()
        assert rel(Pg, Pc) < 1e-15
        W = torch.randn(Pc.shape, dtype=torch.float64)
        (Pg * W.cuda()).sum().backward()
        (Pc * W).sum().backward()
        for (n, pg), (_, pc) in zip(kg.named_parameters(), kc.named_parameters()):
            assert rel(pg.grad, pc.grad) < 1e-13, n


@pytest.mark.parametrize("B,fin,fout,relu", [(4096, 2592, 300, True), (67, 300, 2592, True), (130, 30, 16, False),
                                             (1, 300, 30, True)])
def test_linear_act_fused(hip, B, fin, fout, relu):
    """The fc layers' fused bias + ReLU (VAE.py:44-75; glue.hip bias_act): values and the input / weight /
    bias gradients against fp64 PyTorch; ragged row counts for the 64-row partial chunks."""
    from lvae_amd.vae import linear_act
    torch.manual_seed(B + fout)
    fc = torch.nn.Linear(fin, fout).cuda()
    x = torch.randn(B, fin, device="cuda", requires_grad=True)
    y = linear_act(fc, x, relu)
    g = torch.randn_like(y)
    (y * g).sum().backward()
    x64 = x.detach().cpu().double().requires_grad_()
    w64 = fc.weight.detach().cpu().double().requires_grad_()
    b64 = fc.bias.detach().cpu().double().requires_grad_()
    y64 = x64 @ w64.t() + b64
    if relu:
        y64 = torch.relu(y64)
    (y64 * g.cpu().double()).sum().backward()
    errs = dict(y=rel(y, y64), dx=rel(x.grad, x64.grad), dw=rel(fc.weight.grad, w64.grad), db=rel(fc.bias.grad, b64.grad))
    print(B, fin, fout, relu, errs)
    for k, e in errs.items():
        assert e < 1e-4, (k, e)


def test_linear_act_fused_nan(hip):
    """A NaN pre-activation stays NaN through the fused bias + ReLU, and its gradient passes like
    torch.relu / threshold_backward (fmaxf had mapped it to 0, hiding a diverging layer)."""
    from lvae_amd.vae import linear_act
    torch.manual_seed(0)
    fc = torch.nn.Linear(8, 5).cuda()
    x = torch.randn(3, 8, device="cuda")
    x[1, 2] = float("nan")
    x.requires_grad_()
    y = linear_act(fc, x, True)
    xr = x.detach().clone().requires_grad_()
    yr = torch.relu(torch.nn.functional.linear(xr, fc.weight.detach(), fc.bias.detach()))
    assert torch.equal(torch.isnan(y), torch.isnan(yr)) and bool(torch.isnan(y[1]).all())
    g = torch.ones_like(y)
    (y * g).sum().backward()
    (yr * g).sum().backward()
    assert torch.equal(torch.isnan(x.grad), torch.isnan(xr.grad))


@pytest.mark.parametrize("N", [4096, 37, 1, 2049, 2050])
def test_deconv_relu_fused(hip, N):
    """The decoder's relu(ConvTranspose2d(32, 16, 4, 2, 1)) (VAE.py:73, 122): one direct HIP pass each way
    (vae_ops.hip deconv4s2_relu: the 1 / 3 images-per-block forward grids, the 2 / 4 / 8 images-per-block backward
    with ragged last blocks).
    The output against fp64, and the input / weight / bias gradients against fp64 through the same ReLU mask
    (y > 0 of the GPU forward: at 21M outputs a few pre-activations sit within rounding of 0, where a flipped mask
    is a tie-break, not an error).  MIOpen's Winograd solvers, off by default since r5, had put dx 4.3e-2 from
    fp64 at N = 4096 (scripts/deconv_check.py)."""
    from lvae_amd.vae import deconv_relu
    torch.manual_seed(N)
    dc = torch.nn.ConvTranspose2d(32, 16, kernel_size=4, stride=2, padding=1).cuda()
    x = torch.randn(N, 32, 9, 9, device="cuda", requires_grad=True)
    g = torch.randn(N, 16, 18, 18, device="cuda")
    y = deconv_relu(dc, x)
    (y * g).sum().backward()
    x64 = x.detach().cpu().double().requires_grad_()
    dc64 = torch.nn.ConvTranspose2d(32, 16, kernel_size=4, stride=2, padding=1).double()
    with torch.no_grad():
        dc64.weight.copy_(dc.weight.double().cpu())
        dc64.bias.copy_(dc.bias.double().cpu())
    pre = dc64(x64)
    mask = (y.detach().cpu() > 0).double()
    e_y = rel(y, torch.relu(pre))
    (pre * mask * g.cpu().double()).sum().backward()
    errs = dict(y=e_y, dx=rel(x.grad, x64.grad), dw=rel(dc.weight.grad, dc64.weight.grad),
                db=rel(dc.bias.grad, dc64.bias.grad))
    print(N, errs)
    for k, e in errs.items():
        assert e < 1e-5, (k, e)


def test_deconv4s2_relu_abi(hip):
    """lvae_deconv4s2_relu_fwd / _bwd_f32 directly: -3 for the shapes they do not take, and the backward's
    zero-image call writes zero weight / bias gradients."""
    from lvae_amd import _lib
    x = torch.randn(2, 32, 9, 9, device="cuda")
    w = torch.randn(32, 16, 4, 4, device="cuda")
    b = torch.randn(16, device="cuda")
    y = torch.empty(2, 16, 18, 18, device="cuda")
    assert hip.lvae_deconv4s2_relu_fwd_f32(_lib.ptr(x), _lib.ptr(w), _lib.ptr(b), 2, 16, 16, 9, 9, _lib.ptr(y),
                                           _lib.stream_ptr()) == -3
    assert hip.lvae_deconv4s2_relu_fwd_f32(_lib.ptr(x), _lib.ptr(w), _lib.ptr(b), 2, 32, 16, 8, 8, _lib.ptr(y),
                                           _lib.stream_ptr()) == -3
    dw = torch.full_like(w, float("nan"))
    db = torch.full_like(b, float("nan"))
    ws = torch.empty(16, device="cuda")
    assert hip.lvae_deconv4s2_relu_bwd_f32(_lib.ptr(y), _lib.ptr(y), _lib.ptr(x), _lib.ptr(w), 0, 32, 16, 9, 9,
                                           _lib.ptr(x), _lib.ptr(dw), _lib.ptr(db), _lib.ptr(ws),
                                           _lib.stream_ptr()) == 0
    torch.cuda.synchronize()
    assert float(dw.abs().max()) == 0.0 and float(db.abs().max()) == 0.0
