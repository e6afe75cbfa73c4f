"""Synthetic Health-MNIST-shaped inputs (no network: the MNIST jpgs are unavailable offline).

Covariate rules follow Health_MNIST_generate.py:89-154 and the label permutation of
dataset_def.py:210-213 -- columns (time_age, disease_time, subject, gender, disease, location),
NaN -> 0; subject-contiguous rows (T per subject), as the Hensman reshape [P_b, T, Q] requires
(elbo_functions.py:168).
"""
import numpy as np
import torch


def health_mnist_covariates(P, T, seed=0):
    rng = np.random.default_rng(seed)
    sick = rng.binomial(1, 0.5, size=P)
    loc = rng.binomial(1, 0.5, size=P)
    p = np.repeat(np.arange(P), T)
    t = np.tile(np.arange(T), P)
    X = np.zeros((P * T, 6))
    X[:, 0] = t
    X[:, 1] = np.where(sick[p] == 1, t - 9, 0.0)
    X[:, 2] = p
    X[:, 3] = (p >= P // 2).astype(np.float64)
    X[:, 4] = sick[p]
    X[:, 5] = loc[p]
    return X


def health_mnist_batch(P, T, seed=0, device="cpu", dtype=torch.float32):
    """(images [N,1,36,36] uniform [0,1), mask [N,1,36,36] Bernoulli(0.75), covariates [N,6] f64)."""
    g = torch.Generator().manual_seed(seed)
    N = P * T
    img = torch.rand(N, 1, 36, 36, generator=g, dtype=dtype)
    mask = (torch.rand(N, 1, 36, 36, generator=g) < 0.75).to(dtype)
    X = torch.tensor(health_mnist_covariates(P, T, seed), dtype=torch.float64)
    return img.to(device), mask.to(device), X.to(device)


# ------------------------------------------------------------------------------------------
# On-disk Health-MNIST: the CSV trio Health_MNIST_generate.py:40-72
# writes -- pixels (1296 "%d" columns per row), mask (same shape, 0 = missing), labels (header
# row; columns subject, digit, angle, disease, disease_time, gender, time_age, location).
# ------------------------------------------------------------------------------------------
LABEL_COLUMNS = [6, 4, 0, 5, 3, 7]  # -> time_age, disease_time, subject, gender, disease, location (dataset_def.py:213)


class HealthMNISTDatasetConv:
    """HealthMNISTDatasetConv (dataset_def.py:172-219), preloaded once into device tensors.

    The reference reads one row per item through pandas ``iloc`` inside DataLoader workers; a
    3 ms GPU step cannot wait for that.  Here the three CSVs are parsed once (pandas' C parser),
    kept on ``device`` as uint8 pixels / uint8 mask / fp32 labels, and a batch is one device
    gather (``batch(idx)``).  ``ds[i]`` keeps the reference's per-item dict for compatibility:
    {'digit': ToTensor-equivalent [1,36,36] fp32 (or the raw [36,36,1] uint8 when transform is
    None), 'label': [6] fp32 (NaN -> 0), 'idx': i, 'mask': [1,1296] uint8}."""

    def __init__(self, csv_file_data, csv_file_label, mask_file, root_dir, transform=None, device="cpu"):
        import os

        import pandas as pd
        data = pd.read_csv(os.path.join(root_dir, csv_file_data), header=None).to_numpy(dtype=np.uint8)
        mask = pd.read_csv(os.path.join(root_dir, mask_file), header=None).to_numpy(dtype=np.uint8)
        lab = pd.read_csv(os.path.join(root_dir, csv_file_label), header=0).to_numpy(dtype=np.float64)
        lab = np.nan_to_num(lab[:, LABEL_COLUMNS]).astype(np.float32)
        if data.shape[1] != 1296 or mask.shape != data.shape or lab.shape[0] != data.shape[0]:
            raise ValueError(f"Health-MNIST CSVs disagree: data {data.shape}, mask {mask.shape}, labels {lab.shape}")
        self.transform = transform
        self.device = torch.device(device)
        self.pixels = torch.from_numpy(data).to(self.device)   # [N, 1296] uint8
        self.masks = torch.from_numpy(mask).to(self.device)    # [N, 1296] uint8
        self.labels = torch.from_numpy(lab).to(self.device)    # [N, 6] fp32
        # ToTensor's uint8 / 255 as a 256-entry table computed on the host: a device fp32 division
        # need not round like the host's, a table gather is bit-exact
        self.lut = (torch.arange(256, dtype=torch.float32) / 255.0).to(self.device)

    def __len__(self):
        return self.pixels.shape[0]

    def __getitem__(self, key):
        if isinstance(key, slice):
            return [self._item(i) for i in range(*key.indices(len(self)))]
        if isinstance(key, (int, np.integer)):
            return self._item(int(key))
        raise TypeError

    def _item(self, i):
        raw = self.pixels[i].reshape(36, 36, 1)
        digit = raw.cpu().numpy() if self.transform is None else self.transform(raw.cpu().numpy())
        return {"digit": digit, "label": self.labels[i], "idx": i, "mask": self.masks[i].reshape(1, 1296)}

    def batch(self, idx):
        """Device batch for row indices ``idx``: digit [B,1,36,36] fp32 (= ToTensor: uint8 / 255),
        label [B,6] fp32, mask [B,1,1296] uint8 (as the default collate of the reference items)."""
        idx = torch.as_tensor(idx, dtype=torch.int64, device=self.device)
        digit = self.lut[self.pixels.index_select(0, idx).to(torch.int64)].reshape(-1, 1, 36, 36)
        return {"digit": digit, "label": self.labels.index_select(0, idx), "idx": idx,
                "mask": self.masks.index_select(0, idx).reshape(-1, 1, 1296)}


class DeviceBatchLoader:
    """Iterates device batches of a preloaded dataset in the order of a batch sampler (any
    iterable of index lists, e.g. BatchSampler(SubjectSampler, P_b*T) or varying_length_batches):
    the HensmanDataLoader (utils.py:24-38) replacement, without worker processes."""

    def __init__(self, dataset, batch_sampler):
        self.dataset, self.batch_sampler = dataset, batch_sampler

    def __len__(self):
        return len(self.batch_sampler)

    def __iter__(self):
        for idx in self.batch_sampler:
            yield self.dataset.batch(idx)


def write_health_mnist_csv(root_dir, pixels, mask, labels, prefix="hmnist"):
    """Write the CSV trio in Health_MNIST_generate.py's format (test / synthetic-data helper):
    pixels, mask [N,1296] ints; labels [N,8] in the generator's column order."""
    import os
    np.savetxt(os.path.join(root_dir, f"{prefix}_data.csv"), pixels, fmt="%d", delimiter=",")
    np.savetxt(os.path.join(root_dir, f"{prefix}_mask.csv"), mask, fmt="%d", delimiter=",")
    with open(os.path.join(root_dir, f"{prefix}_labels.csv"), "w") as f:
        f.write("subject,digit,angle,disease,disease_time,gender,time_age,location\n")
        for row in labels:
            f.write(",".join("" if (isinstance(v, float) and np.isnan(v)) else repr(float(v)) for v in row) + "\n")
    return f"{prefix}_data.csv", f"{prefix}_labels.csv", f"{prefix}_mask.csv"
