"""Multi-GPU plumbing of the topic-routing engine (one process per GPU).

The hot path shards by publish topic: every GPU holds a full replica of the
trie image (10M filters are ~1 GB of HBM of the 288 GB) and matches its own
topic batches, so the data path needs NO collective (SURVEY.md §8(e),
"replicated").  torch.distributed (RCCL on ROCm, gloo on CPU) is used only
for the control plane around a measured region: a barrier, and the max of
the per-rank step times.

The sharded-filter mode of config C4 (filters partitioned by root level,
per-shard match lists exchanged over xGMI with RCCL) lives in shard.py.
"""
import os
import time


def env_rank():
    """(rank, world, local_rank) from the torchrun environment"""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", 0)))


def topic_stream(rank: int) -> int:
    """independent synthetic topic stream per rank (weak scaling)"""
    return rank


def batch_slice(n: int, world: int, rank: int):
    """[lo, hi) of rank's contiguous slice of an n-topic batch (strong
    scaling: SURVEY §8(d) C3 splits one batch 1/2/4/8 ways)"""
    return (n * rank) // world, (n * (rank + 1)) // world


def timed_region(step, steps: int, sync, group=None):
    """Run `steps` calls of step() bracketed by barrier + device sync on both
    sides; returns the MAX over ranks of the wall time (seconds)."""
    import torch
    import torch.distributed as dist
    dist_on = dist.is_available() and dist.is_initialized()
    if dist_on:
        dist.barrier(group=group)
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    if dist_on:
        dist.barrier(group=group)
    dt = time.perf_counter() - t0
    if dist_on:
        dev = torch.device("cuda", torch.cuda.current_device()) \
            if dist.get_backend(group) == "nccl" else torch.device("cpu")
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        dt = float(t.item())
    return dt


def all_true(flag, group=None) -> bool:
    """AND of a per-rank boolean over the ranks (None counts as false)"""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return bool(flag)
    dev = torch.device("cuda", torch.cuda.current_device()) \
        if dist.get_backend(group) == "nccl" else torch.device("cpu")
    t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(int(t.item()))
