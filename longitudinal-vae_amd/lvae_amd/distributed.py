"""Data parallelism over subject mini-batches: one process per GPU, torch.distributed over RCCL
(backend "nccl" is RCCL on ROCm), one flat SUM all-reduce per step and dtype bucket.

The reference has no distributed code; this is the multi-GPU form of its
mini-batch estimators: the Hensman bound scales each rank's subject sums by P_tot / P_b, so the
average over ranks equals the bound of the union batch.
"""
import torch
import torch.distributed as dist
from torch._utils import _flatten_dense_tensors, _unflatten_dense_tensors


class GradAllReduce:
    """Average the .grad of `params` over the process group (call between backward and step)."""

    def __init__(self, params, world=None, group=None):
        self.params = [p for p in params if p.requires_grad]
        self.group = group
        self.world = world or dist.get_world_size(group)

    def __call__(self):
        by_dtype = {}
        for p in self.params:
            if p.grad is None:
                p.grad = torch.zeros_like(p)
            by_dtype.setdefault((p.grad.dtype, p.grad.device), []).append(p.grad)
        for grads in by_dtype.values():
            flat = _flatten_dense_tensors(grads)
            dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group)
            flat.div_(self.world)
            for g, r in zip(grads, _unflatten_dense_tensors(flat, grads)):
                g.copy_(r)


def allreduce_tensors(tensors, average=True, group=None):
    """In-place SUM (or mean) all-reduce of a list of same-dtype tensors in one flat bucket."""
    if not tensors:
        return
    flat = _flatten_dense_tensors(tensors)
    dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    if average:
        flat.div_(dist.get_world_size(group))
    for t, r in zip(tensors, _unflatten_dense_tensors(flat, tensors)):
        t.copy_(r)
