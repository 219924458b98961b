"""Data parallelism for the fused step: one process per GPU, one collective per
step.

The reference is single-device (learning.py:74,360).  Segments are independent,
so the batch shards naturally: every rank runs the full step on
its own b segments, then the flat fp32 gradient buffer (all 1.95 M parameters,
7.4 MiB) is SUMMED with ONE all-reduce -- RCCL over xGMI with the "nccl"
backend on ROCm, gloo on CPU for tests -- and every rank applies the identical
global-norm clip + SGD (clip after the reduce, learning.py:161).  Each rank
normalises its loss by the GLOBAL batch size (FusedStep(..., loss_batch=B)):
loss_r = (em_r + off_r + kl_r) / B_global with kl_r using the rank's B_r in the
prior term (B_r / N) and the global N, so sum_r loss_r is exactly the
reference's (em + off + kl) / batch_sizes[0] on the concatenated batch
(learning.py:155-157), for any split, unequal or empty shards included.

``shard_global_batch`` implements the straggler-free partition of §8e: sort
the global batch by length (desc) and deal rows round-robin, so every rank gets
a length-sorted shard with nearly the same T_max and frame count.
"""
import torch
import torch.distributed as dist


def world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def make_allreduce(group=None):
    """Returns f(flat_grad) that sums the flat gradient buffer over the ranks
    in place (each rank's gradient is already scaled by 1 / B_global)."""

    def allreduce(g):
        if dist.get_world_size(group) > 1:
            dist.all_reduce(g, op=dist.ReduceOp.SUM, group=group)

    return allreduce


def attach(step, group=None):
    """Make a FusedStep data-parallel: gradients are summed before clip+SGD."""
    step.allreduce = make_allreduce(group)
    return step


def broadcast_parameters(step, src=0, group=None):
    """Start every rank from rank `src`'s weights (one broadcast of the flat buffer)."""
    dist.broadcast(step.flat.flat, src=src, group=group)


def shard_global_batch(lengths, rank, world_size):
    """Indices (into a list of segments) that rank `rank` trains on: sort by
    length desc, deal round-robin.  Returns a list sorted by length desc."""
    order = sorted(range(len(lengths)), key=lambda i: -int(lengths[i]))
    return order[rank::world_size]
