"""Data parallelism for the fused step: one process per GPU, one collective per
step.

The reference is single-device (learning.py:74,360).  Segments are independent,
so the batch shards naturally: every rank runs the full step on
its own b segments, then the flat fp32 gradient buffer (all 1.95 M parameters,
7.4 MiB) is averaged with ONE all-reduce -- RCCL over xGMI with the "nccl"
backend on ROCm, gloo on CPU for tests -- and every rank applies the identical
global-norm clip + SGD.  With equal per-rank batch sizes the averaged gradient
equals the gradient of the reference loss on the concatenated global batch
(loss_r = (em_r + off_r + kl_r) / B_r, kl_r with the per-rank B_r and the global
N).

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
    """Returns f(flat_grad) that averages the flat gradient buffer in place."""
    backend = dist.get_backend(group)

    def allreduce(g):
        ws = dist.get_world_size(group)
        if ws == 1:
            return
        if backend == "nccl":
            dist.all_reduce(g, op=dist.ReduceOp.AVG, group=group)
        else:
            dist.all_reduce(g, op=dist.ReduceOp.SUM, group=group)
            g.div_(ws)

    return allreduce


def attach(step, group=None):
    """Make a FusedStep data-parallel: gradients are averaged before clip+SGD."""
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
