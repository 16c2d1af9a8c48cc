"""Data-parallel plumbing: one process per GPU, torch.distributed over RCCL ("nccl" on ROCm).

SURVEY.md §8(e): pure data parallel. Rank r trains on samples [r*n, (r+1)*n) of the global batch,
weights are replicated, BatchNorm uses each rank's LOCAL batch statistics (the reference has no
SyncBN, so this equals running the reference on each shard), and the only exchange is one
all-reduce of the weight gradients per step.

Why one flat all-reduce after backward (not per-bucket overlap): the reference shares the hourglass,
residual4, lin and head modules across all stacks (try_with_torch.py:268,286-297), so every one of
those gradients becomes final only when the backward of stack 0 has run — i.e. at the very end of
backward; the stem is also last. There is nothing left to overlap. The whole gradient is one flat
fp32 buffer (7.65 MB for the primary model, 1.91 M params), so the collective is a handful of
bucket-sized ring all-reduces over xGMI; the loss gradient is pre-scaled by 1/world so SUM == mean.
"""
import os

import torch
import torch.distributed as dist

BUCKET_BYTES = 8 << 20  # xGMI ring: a few MB per call amortises the per-call latency


def world_info():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init_from_env(backend=None):
    """Initialise the default process group from torchrun's env (no-op for world size 1)."""
    rank, world, local = world_info()
    if world == 1 or (dist.is_available() and dist.is_initialized()):
        return rank, world, local
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    kw = {}
    if backend == "nccl":
        torch.cuda.set_device(local)
        kw["device_id"] = torch.device("cuda", local)
    dist.init_process_group(backend, **kw)
    return rank, world, local


def shard_bounds(global_batch, rank, world):
    """Sample range of this rank: [rank*n, (rank+1)*n) with n = global_batch // world."""
    if global_batch % world:
        raise ValueError(f"global batch {global_batch} not divisible by world size {world}")
    n = global_batch // world
    return rank * n, (rank + 1) * n


def broadcast_flat(flat, src=0, group=None):
    """Make every rank start from rank src's weights (seeded init is identical anyway)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.broadcast(flat, src=src, group=group)


def allreduce_flat(flat, group=None, bucket_bytes=BUCKET_BYTES):
    """SUM all-reduce of a contiguous fp32 buffer in fixed-size buckets (in place)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return flat
    per = max(1, bucket_bytes // flat.element_size())
    for off in range(0, flat.numel(), per):
        dist.all_reduce(flat[off:off + per], op=dist.ReduceOp.SUM, group=group)
    return flat
