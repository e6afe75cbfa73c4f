"""Subject-contiguous batching (utils.py:40-113; training.py:70-75), as index arithmetic.

A Hensman batch is P_b whole subjects: a shuffled subject order, each subject's T rows kept
contiguous, cut into batches of P_b*T rows (BatchSampler(SubjectSampler, P_b*T, drop_last=False)).
The reference draws the order with np.random.shuffle on NumPy's global legacy state (utils.py:53,
76).  seed=None keeps exactly that (so np.random.seed(s) reproduces the reference's orders bit for
bit, tests/golden/samplers.npz); an explicit seed gives a private generator, so data-parallel
ranks agree on the order without touching global state.
"""
import numpy as np
import torch


def _shuffler(seed):
    """In-place shuffle: NumPy's global legacy np.random.shuffle (the reference's) for seed=None."""
    if seed is None:
        return np.random.shuffle
    return np.random.default_rng(seed).shuffle


class SubjectSampler:
    """Row indices of the shuffled subject order (utils.py:40-59)."""

    def __init__(self, P, T, seed=None):
        self.P, self.T = P, T
        self.shuffle = _shuffler(seed)

    def permutation(self):
        r = np.arange(self.P)
        self.shuffle(r)
        return r

    def __iter__(self):
        r = self.permutation()
        return iter((r[:, None] * self.T + np.arange(self.T)[None, :]).reshape(-1).tolist())

    def __len__(self):
        return self.P * self.T


def subject_rows(subjects, T):
    """[subjects] -> contiguous row indices (subject-major, time-minor)."""
    s = torch.as_tensor(subjects, dtype=torch.int64)
    return (s[:, None] * T + torch.arange(T, dtype=torch.int64, device=s.device)[None, :]).reshape(-1)


def check_same_permutation(perm, group=None):
    """Raise if the ranks of an initialised process group hold different subject orders (a sampler
    built without a seed draws from each process's own NumPy global state): one MIN / MAX all-reduce
    of a checksum of the order.  A collective: every rank of the group calls it, once per run (the
    distributed drivers do, right after building the sampler), not per epoch."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return
    p = np.asarray(perm, dtype=np.int64)
    w = (np.arange(len(p), dtype=np.int64) * 2654435761) % 2147483647 + 1
    h = int(((p + 1) * w).sum() % 2305843009213693951)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else "cpu"
    t = torch.tensor([h, -h], dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    if int(t[0]) != h or int(t[1]) != -h:
        raise ValueError("hensman_batches: ranks hold different subject orders -- build the SubjectSampler "
                         "with the same explicit seed on every rank (or broadcast rank 0's permutation)")


def hensman_batches(perm, P_b, T, rank=0, world=1, check=False, group=None):
    """Batches of one epoch for one rank: the global batch of world*P_b consecutive subjects of the
    permutation is split into contiguous per-rank slices of P_b subjects (the last global batch may be
    short, as with drop_last=False; ranks whose slice is empty get no batch in that step).  A pure index
    utility by default; check=True (world > 1, inside an initialised process group) first compares the
    ranks' orders with check_same_permutation -- a collective every rank must reach -- since different
    orders would silently give overlapping / missing subjects."""
    if world > 1 and check:
        check_same_permutation(perm, group)
    perm = np.asarray(perm)
    G = world * P_b
    out = []
    for g0 in range(0, len(perm), G):
        sl = perm[g0 + rank * P_b: min(g0 + (rank + 1) * P_b, g0 + G, len(perm))]
        out.append(subject_rows(sl, T) if len(sl) else None)
    return out


class VaryingLengthSubjectSampler:
    """(row, subject) pairs in shuffled subject order for subjects of varying length (utils.py:61-87).
    As the reference: subject s (in order of first appearance of its id) spans rows from its first
    occurrence to the next subject's first occurrence (contiguous runs in Health-MNIST files)."""

    def __init__(self, subject_ids, seed=None):
        ids = np.asarray(subject_ids).astype(np.int64)
        _, first = np.unique(ids, return_index=True)
        self.start = np.sort(first)
        self.end = np.r_[self.start[1:], len(ids)]
        self.P = len(self.start)
        self.shuffle = _shuffler(seed)

    def __iter__(self):
        r = np.arange(self.P)
        self.shuffle(r)
        for s in r:
            for i in range(self.start[s], self.end[s]):
                yield i, s

    def __len__(self):
        return self.P


def varying_length_batches(sampler, subjects_per_batch):
    """VaryingLengthBatchSampler (utils.py:89-113): batches of `subjects_per_batch` whole subjects."""
    batch, subj = [], set()
    for idx, s in sampler:
        if s not in subj:
            if len(subj) == subjects_per_batch:
                yield batch
                batch, subj = [], set()
            subj.add(s)
        batch.append(idx)
    yield batch
