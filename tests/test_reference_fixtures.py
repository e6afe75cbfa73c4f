"""Oracle and host logic against the round-2 reference fixtures (tests/golden/gen_golden.py):

* kernel_variants_{kl,hensman}.npz -- the builder branches the sample config leaves out
  (bin_kernel, bin_int_kernel, covariate_missing_val mask products; GP_model.py:146-236);
* samplers.npz -- SubjectSampler / BatchSampler / VaryingLength* row orders under np.random.seed
  (utils.py:40-113): bit-exact;
* hensman_training_2ep.npz -- two epochs of the reference's training.hensman_training
  (training.py:15-140) with an injected subject order and reparametrisation noise: per-step KL
  bound / recon sums, per-epoch averages and the final (m, H), kernel and network parameters;
* standard_training_closed.npz -- three full-batch epochs of training.standard_training with
  type_KL='closed' (training.py:431-592): per-step net / recon / GP loss, final parameters.
"""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import lvae_oracle as O

VAR_CFG = dict(cat_kernel=[2, 3], bin_kernel=[5], sqexp_kernel=[0],
               cat_int_kernel=[{'cont_covariate': 0, 'cat_covariate': 2},
                               {'cont_covariate': 1, 'cat_covariate': 4}],
               bin_int_kernel=[{'cont_covariate': 0, 'bin_covariate': 4}],
               covariate_missing_val=[{'covariate': 0, 'mask': 6}, {'covariate': 3, 'mask': 7}])
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


# ------------------------------------------------------------------------------------------
# kernel builder variants
# ------------------------------------------------------------------------------------------
def test_variant_fixture_exercises_every_branch():
    s0, s1 = O.spec_split(**VAR_CFG, id_covariate=2)
    kinds = [[f[0] for f in c] for c in s0 + s1]
    assert ["bin", "bin"] not in kinds and any(k == ["bin"] for k in kinds)       # bin_kernel
    assert any(k[:2] == ["bin", "rbf"] or k[:3] == ["bin", "rbf", "bin"] for k in kinds)  # bin_int
    assert any(k == ["cat", "bin"] for k in kinds)                               # masked cat
    assert any(k == ["rbf", "bin"] for k in kinds)                               # masked rbf
    g = golden("kernel_variants_hensman.npz")
    assert O.n_params(s0) == g["raw0"].shape[0] and O.n_params(s1) == g["raw1"].shape[0]


def test_builder_variants_match_reference_order():
    """lvae_amd.generate_kernel_batched: the same components, factors and parameter order as the
    reference builder (whose parameter names the fixture holds)."""
    import lvae_amd as la
    g = golden("kernel_variants_hensman.npz")
    k0, k1 = la.generate_kernel_batched(3, **VAR_CFG, id_covariate=2)
    s0, s1 = O.spec_split(**VAR_CFG, id_covariate=2)
    assert [c for c, _ in k0.components()] == [list(c) for c in s0]
    assert [c for c, _ in k1.components()] == [list(c) for c in s1]
    ours = [n.split(".")[-1] for n, _ in k0.named_parameters()] + [n.split(".")[-1] for n, _ in k1.named_parameters()]
    ref = [str(n).split(".")[-1] for n in g["names0"]] + [str(n).split(".")[-1] for n in g["names1"]]
    assert ours == ref


def test_kernel_variants_kl_oracle():
    g = golden("kernel_variants_kl.npz")
    s0, s1 = O.spec_split(**VAR_CFG, id_covariate=2)
    spec = s0 + s1  # the fixture's per-dim kernel: non-id components, then id components
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
        with torch.no_grad():
            assert rel(O.gram(spec, O.constrain(raw), X, X), g["gram"][l]) < 1e-14


def test_kernel_variants_hensman_oracle():
    g = golden("kernel_variants_hensman.npz")
    s0, s1 = O.spec_split(**VAR_CFG, id_covariate=2)
    raw0 = torch.tensor(g["raw0"].T.copy(), requires_grad=True)
    raw1 = torch.tensor(g["raw1"].T.copy(), requires_grad=True)
    X = torch.tensor(g["X_all"][g["idx"]])
    Z = torch.tensor(g["Z"])
    mu = torch.tensor(g["mu"], requires_grad=True)
    lv = torch.tensor(g["logv"], requires_grad=True)
    kld, gm, gH = O.hensman_kld(s0, O.constrain(raw0), s1, O.constrain(raw1), torch.tensor(g["noise"]),
                                torch.tensor(g["m"]), torch.tensor(g["H"]), X, mu, lv, Z, int(g["P_tot"]),
                                int(g["P_b"]), int(g["T"]), True, float(g["eps"]))
    kld.backward()
    assert rel(kld.item(), g["kld"]) < 1e-10
    assert rel(mu.grad, g["dmu"]) < 1e-8
    assert rel(lv.grad, g["dlogv"]) < 1e-8
    assert rel(raw0.grad.T, g["draw0"]) < 1e-6
    assert rel(raw1.grad.T, g["draw1"]) < 1e-5
    assert rel(gm, g["grad_m"]) < 1e-6
    with torch.no_grad():
        P_b, T, L = int(g["P_b"]), int(g["T"]), int(g["L"])
        p0, p1 = O.constrain(raw0), O.constrain(raw1)
        assert rel(O.gram(s0, p0, X, Z), g["K0xz"]) < 1e-14
        assert rel(O.gram(s0, p0, Z, Z), g["K0zz"]) < 1e-14
        xs = X.reshape(P_b, 1, T, -1).expand(P_b, L, T, X.shape[1])
        assert rel(O.gram(s1, p1, xs, xs), g["K1_st"]) < 1e-14


# ------------------------------------------------------------------------------------------
# samplers (bit-exact under np.random.seed)
# ------------------------------------------------------------------------------------------
class _Labels:
    def __init__(self, labels):
        self.labels = torch.tensor(labels)

    def __len__(self):
        return len(self.labels)


def test_subject_sampler_matches_reference():
    from torch.utils.data.sampler import BatchSampler
    from dropin.utils import SubjectSampler
    g = golden("samplers.npz")
    P, T, P_b = int(g["P"]), int(g["T"]), int(g["P_b"])
    np.random.seed(int(g["seed"]))
    ss = SubjectSampler(_Labels(np.zeros((P * T, 6))), P, T)
    for e in range(g["epochs"].shape[0]):
        assert np.array_equal(np.array(list(iter(ss))), g["epochs"][e])
    batches = [np.array(b) for b in BatchSampler(ss, P_b * T, drop_last=False)]
    assert [len(b) for b in batches] == g["batch_lens"].tolist()
    assert np.array_equal(np.concatenate(batches), g["batches"])


def test_varying_length_samplers_match_reference():
    from dropin.utils import VaryingLengthBatchSampler, VaryingLengthSubjectSampler
    g = golden("samplers.npz")
    lab = np.zeros((len(g["v_ids"]), 6))
    lab[:, 2] = g["v_ids"]
    np.random.seed(int(g["seed"]) + 1)
    vs = VaryingLengthSubjectSampler(_Labels(lab), 2)
    for e in range(g["v_pairs"].shape[0]):
        assert np.array_equal(np.array(list(iter(vs))), g["v_pairs"][e])
    batches = [np.array(b) for b in VaryingLengthBatchSampler(vs, 3)]
    assert [len(b) for b in batches] == g["v_batch_lens"].tolist()
    assert np.array_equal(np.concatenate(batches), g["v_batches"])


def test_hensman_batches_follow_batch_sampler():
    """samplers.hensman_batches (the index arithmetic the GPU loader uses) = BatchSampler over the
    same subject order, including the short last batch (drop_last=False)."""
    from lvae_amd.samplers import hensman_batches
    g = golden("samplers.npz")
    T, P_b = int(g["T"]), int(g["P_b"])
    perm = g["epochs"][0][::T] // T
    ours = [b.numpy() for b in hensman_batches(perm, P_b, T)]
    ref = np.split(g["epochs"][0], np.cumsum([P_b * T] * ((len(perm) - 1) // P_b)))
    assert len(ours) == len(ref) and all(np.array_equal(a, b) for a, b in zip(ours, ref))


# ------------------------------------------------------------------------------------------
# two epochs of hensman_training: the oracle step composition (training.py:90-140)
# ------------------------------------------------------------------------------------------
def training_inputs(g):
    P, T, L = int(g["P"]), int(g["T"]), int(g["L"])
    img = torch.tensor(g["pix"].astype(np.float64) / 255.0)
    mask = torch.tensor(g["msk"].astype(np.float64))
    return P, T, L, img, mask, torch.tensor(g["X"])


def test_hensman_training_two_epochs_oracle():
    from lvae_amd.samplers import hensman_batches
    g = golden("hensman_training_2ep.npz")
    P, T, L, img, mask, X = training_inputs(g)
    P_b = int(g["P_b"])
    s0, s1 = O.spec_split(**CFG, id_covariate=2)
    vae = O.ConvVAE(L).double()
    vae.load_state_dict(O.vae_weights(vae, int(g["seed"])))
    raw0 = torch.tensor(g["raw0"].T.copy(), requires_grad=True)
    raw1 = torch.tensor(g["raw1"].T.copy(), requires_grad=True)
    opt = torch.optim.Adam([raw0, raw1] + list(vae.parameters()), lr=1e-3)
    m, H, Z = torch.tensor(g["m0"]), torch.tensor(g["H0"]), torch.tensor(g["Z"])
    step = 0
    for e in range(int(g["epochs"])):
        for rows in hensman_batches(g["perms"][e], P_b, T):
            eps = torch.tensor(g["eps"][step][:len(rows)])
            loss, recon, kld, m, H = O.hensman_step(vae, s0, raw0, s1, raw1, torch.ones(L), m, H, img[rows],
                                                    mask[rows], X[rows], Z, eps, P, T, 0.15, 0.01, opt=opt)
            pb = len(rows) // T
            assert rel(kld * L, g["step_kld"][step]) < 1e-9, step
            assert rel(recon * pb / P, g["step_recon"][step]) < 1e-10, step
            step += 1
    assert step == len(g["step_kld"])
    assert rel(m, g["m_final"]) < 1e-7
    assert rel(H, g["H_final"]) < 1e-7
    assert rel(raw0.T, g["raw0_final"]) < 1e-9
    assert rel(raw1.T, g["raw1_final"]) < 1e-9
    sd = dict(vae.named_parameters())
    for k in ("conv1.weight", "fc211.bias", "deconv2.weight", "_log_vy"):
        assert rel(sd[k], g["vae_" + k]) < 1e-9, k
    assert rel(sd["fc1.weight"].sum(1), g["vae_fc1_rowsum"]) < 1e-9


# ------------------------------------------------------------------------------------------
# three epochs of standard_training, type_KL='closed' (training.py:431-592): oracle closed step
# ------------------------------------------------------------------------------------------
def test_standard_training_closed_oracle():
    g = golden("standard_training_closed.npz")
    P, T, L, img, mask, X = training_inputs(g)
    spec = O.spec_full(**CFG)
    vae = O.ConvVAE(L).double()
    vae.load_state_dict(O.vae_weights(vae, int(g["seed"])))
    raw = torch.tensor(g["raw"], requires_grad=True)
    opt = torch.optim.Adam([raw] + list(vae.parameters()), lr=1e-3)
    for s in range(int(g["epochs"])):
        eps = torch.tensor(g["eps"][2 * s])   # the forward's draw (see gen_standard_training)
        net, recon, gp = O.closed_step(vae, spec, raw, torch.ones(L), img, mask, X, eps, 0.15, opt=opt)
        assert rel(net, g["step_net"][s]) < 1e-10, s
        assert rel(recon, g["step_recon"][s]) < 1e-10, s
        assert rel(gp, g["step_gp"][s]) < 1e-10, s
    assert rel(raw, g["raw_final"]) < 1e-9
    sd = dict(vae.named_parameters())
    for k in ("conv1.weight", "fc211.bias", "deconv2.weight", "_log_vy"):
        assert rel(sd[k], g["vae_" + k]) < 1e-9, k
    assert rel(sd["fc1.weight"].sum(1), g["vae_fc1_rowsum"]) < 1e-9
