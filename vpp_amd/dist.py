"""Multi-GPU plumbing of the path: one process per GPU, tuples sharded by
contiguous global index ranges, tables replicated, and exactly one collective -- the sum of
the per-rule hit counters (the statscollector path) over RCCL (backend "nccl") on GPUs, or
gloo in the CPU tests.

The classify path itself has no exchange: every tuple's verdict depends only on the tuple
and the replicated tables, and shards are generated on their own device from
(seed, global index).
"""
import os

import torch
import torch.distributed as dist


def env():
    """(rank, world size, local rank) from the torchrun environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard(rank, world, n_per_rank):
    """Global tuple-index range [base, base + n) of a rank (weak scaling: fixed per rank)."""
    if not 0 <= rank < world:
        raise ValueError("rank %d outside world of %d" % (rank, world))
    return rank * n_per_rank, n_per_rank


def shard_strong(rank, world, n_total):
    """Global index range of a rank when the total is fixed (strong scaling)."""
    if not 0 <= rank < world:
        raise ValueError("rank %d outside world of %d" % (rank, world))
    per = (n_total + world - 1) // world
    lo = min(rank * per, n_total)
    return lo, min(per, n_total - lo)


def allreduce_counters(counters, group=None):
    """Sum the per-rule u64 hit counters (int64 tensor, one entry per counter slot) over all
    ranks in place: ncclAllReduce(ncclUint64 sum) on GPUs. The slot layout is identical on
    every rank because every rank compiles the same committed ACLs."""
    if counters.dtype != torch.int64:
        raise TypeError("counters must be int64 (u64 slots)")
    if dist.is_initialized():
        dist.all_reduce(counters, op=dist.ReduceOp.SUM, group=group)
    return counters


def sum_over_ranks(value, device):
    """Sum of an integer over all ranks (tuples of the whole job)."""
    if not dist.is_initialized():
        return int(value)
    t = torch.tensor([int(value)], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())


def max_over_ranks(value, device):
    """Max of a float over all ranks (the bench's wall time)."""
    if not dist.is_initialized():
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_objects(obj):
    """Every rank's (picklable) object, in rank order, on every rank (a list of one without a
    process group): the per-rank self-checks of the bench line."""
    if not dist.is_initialized():
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out
