"""Data-parallel path on CPU with gloo, world_size 2 (SURVEY.md §8(e) parity pin).

Each rank computes the reference-semantics gradient of its own shard (the CPU oracle stands in for
the HIP engine here — gloo has no GPU), scaled by 1/world at the loss exactly as the Trainer does,
flattens it with the Trainer's FlatParams layout and runs dp.allreduce_flat. The result must equal
the mean over shards of the per-shard gradients computed in one process, and every rank must hold
the same buffer. BN statistics stay local to each shard.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle.hourglass_oracle import OracleModel, stack_mse
from progressive_process_for_human_pose_estimation_amd import dp
from progressive_process_for_human_pose_estimation_amd.data import gaussian_targets, synthetic_images
from progressive_process_for_human_pose_estimation_amd.trainer import FlatParams

WORLD = 2
GLOBAL_BATCH = 4
CFG = dict(nStack=2, nFeats=64, nOutChannels=17)


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def shard_grad(rank, world, scale):
    torch.manual_seed(0)
    m = OracleModel(**CFG)
    fp = FlatParams(m)
    # 128x128: innermost level 2x2 -> well-conditioned train-mode BN per shard (a 1x1 innermost
    # level with 2 samples makes the reference itself chaotic, see test_gpu_parity.MODEL_CASES)
    x = synthetic_images(GLOBAL_BATCH, 128, 128)
    t = gaussian_targets(GLOBAL_BATCH, 17, 32)[0]
    lo, hi = dp.shard_bounds(GLOBAL_BATCH, rank, world)
    (stack_mse(m(x[lo:hi]), t[lo:hi]) * scale).backward()
    for p in fp.params:
        if p.grad is not None:
            fp.grad_views[id(p)].copy_(p.grad)
    return fp


def worker(rank, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(WORLD), LOCAL_RANK=str(rank))
    torch.set_num_threads(2)
    dp.init_from_env(backend="gloo")
    fp = shard_grad(rank, WORLD, 1.0 / WORLD)
    dp.broadcast_flat(fp.flat)
    dp.allreduce_flat(fp.grad, bucket_bytes=1 << 16)  # many buckets
    out[rank] = fp.grad.clone()
    dist.destroy_process_group()


def test_shard_bounds():
    assert dp.shard_bounds(64, 1, 2) == (32, 64)
    with pytest.raises(ValueError):
        dp.shard_bounds(10, 0, 3)


def test_gloo_allreduce_equals_mean_of_shard_grads():
    port = free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=worker, args=(r, port, out)) for r in range(WORLD)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
        assert p.exitcode == 0
    torch.set_num_threads(2)  # same intra-op reduction order as the workers
    expect = sum(shard_grad(r, WORLD, 1.0).grad for r in range(WORLD)) / WORLD
    for r in range(WORLD):
        torch.testing.assert_close(out[r], expect, rtol=1e-4, atol=1e-6)
    assert torch.equal(out[0], out[1])
