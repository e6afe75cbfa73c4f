"""Data ingest: the device-preloaded HealthMNISTDatasetConv against the
reference dataset's items on a CSV trio in Health_MNIST_generate.py's format (tests/golden/
hmnist_tiny/, expected items in hmnist_tiny.npz from gen_golden.py), and the batch loader against
the samplers' index order.  Bit-exact: uint8 pixels / masks, fp32 labels."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, golden


def _ds(device="cpu"):
    from lvae_amd.data import HealthMNISTDatasetConv
    g = golden("hmnist_tiny.npz")
    fd, fl, fm = [str(x) for x in g["files"]]
    return g, HealthMNISTDatasetConv(fd, fl, fm, os.path.join(GOLDEN, "hmnist_tiny"), transform=None, device=device)


def test_items_match_reference():
    g, ds = _ds()
    assert len(ds) == int(g["n"])
    for i in range(len(ds)):
        it = ds[i]
        assert it["idx"] == i
        assert np.array_equal(it["digit"], g["digit"][i])
        assert it["digit"].dtype == np.uint8 and it["digit"].shape == (36, 36, 1)
        assert np.array_equal(it["label"].numpy(), g["label"][i])     # NaN disease_time -> 0
        assert np.array_equal(it["mask"].numpy(), g["mask"][i])


def test_device_batch_equals_collated_items():
    g, ds = _ds()
    idx = [5, 0, 11, 7]
    b = ds.batch(idx)
    assert b["digit"].dtype == torch.float32 and tuple(b["digit"].shape) == (4, 1, 36, 36)
    ref = torch.tensor(g["digit"][idx]).permute(0, 3, 1, 2).to(torch.float32) / 255.0   # ToTensor of uint8
    assert torch.equal(b["digit"], ref)
    assert torch.equal(b["label"], torch.tensor(g["label"][idx]))
    assert torch.equal(b["mask"], torch.tensor(g["mask"][idx]))


def test_loader_follows_subject_batches():
    from lvae_amd.data import DeviceBatchLoader
    from lvae_amd.samplers import SubjectSampler, hensman_batches
    g, ds = _ds()
    P, T, P_b = 3, 4, 2
    perm = SubjectSampler(P, T, seed=0).permutation()
    batches = [b for b in hensman_batches(perm, P_b, T)]
    out = list(DeviceBatchLoader(ds, batches))
    assert len(out) == 2
    for b, idx in zip(out, batches):
        assert torch.equal(b["idx"], idx)
        subj = b["label"][:, 2].to(torch.int64)
        # each batch holds whole subjects, rows contiguous per subject, in the permutation order
        assert torch.equal(subj, torch.as_tensor(np.repeat(perm[:P_b] if b is out[0] else perm[P_b:], T)))


@pytest.mark.gpu
def test_device_resident_ingest_on_gpu():
    """The point of the device-preloaded dataset: CSVs parsed once into HBM,
    batches are device gathers in the sampler's order -- bit-exact vs the reference's items."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from lvae_amd.data import DeviceBatchLoader
    from lvae_amd.samplers import SubjectSampler, hensman_batches
    g, ds = _ds(device="cuda")
    assert ds.pixels.is_cuda and ds.masks.is_cuda and ds.labels.is_cuda
    perm = SubjectSampler(3, 4, seed=1).permutation()
    batches = hensman_batches(perm, 2, 4)
    for b, idx in zip(DeviceBatchLoader(ds, batches), batches):
        assert b["digit"].is_cuda and b["label"].is_cuda and b["mask"].is_cuda
        i = idx.numpy()
        ref = torch.tensor(g["digit"][i]).permute(0, 3, 1, 2).to(torch.float32) / 255.0
        assert torch.equal(b["digit"].cpu(), ref)
        assert torch.equal(b["label"].cpu(), torch.tensor(g["label"][i]))
        assert torch.equal(b["mask"].cpu(), torch.tensor(g["mask"][i]))
