"""Data-parallel path on CPU with gloo, world_size 2 (SURVEY.md §8(e) parity pin).

Each rank computes the reference-semantics gradient of its own shard (the CPU oracle stands in for
the HIP engine here — gloo on the CPU has no GPU), scaled by 1/world at the loss exactly as the
Trainer's MSE kernel does, places it in the Trainer's flat layout (FlatParams with the ENGINE
model's grad-ready groups: [trunk | stem | never-grad tail]) and reduces it with dp.GradSync
segment by segment in grad-ready order, as Trainer.step does. The result must equal the mean over
shards of the per-shard gradients computed in one process, every rank must hold the same buffer,
and the never-grad tail must stay untouched. BN statistics stay local to each shard.

The launcher test runs `bench.py --gpus 2 --dry-run`: bench.py starts the two ranks itself
(torch.distributed.run child), and rank 0's JSON line must report n_gpus = 2.
"""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import progressive_process_for_human_pose_estimation_amd as P
from oracle.hourglass_oracle import OracleModel, stack_mse
from progressive_process_for_human_pose_estimation_amd import dp
from progressive_process_for_human_pose_estimation_amd.data import gaussian_targets, synthetic_images
from progressive_process_for_human_pose_estimation_amd.trainer import FlatParams, param_layout

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORLD = 2
GLOBAL_BATCH = 4
CFG = dict(nStack=2, nFeats=64, nOutChannels=17)


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def engine_layout():
    return param_layout(P.creatModel(**CFG))


def shard_grad(rank, world, scale):
    torch.manual_seed(0)
    m = OracleModel(**CFG)
    fp = FlatParams(m, layout=engine_layout())
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
    sync = dp.GradSync(fp.grad, fp.segments, bucket_bytes=1 << 16)  # many buckets
    for i in range(len(fp.segments)):  # trunk at the stem barrier, then the stem
        sync.launch(i)
    out[rank] = (fp.grad.clone(), sync.wait())
    dist.destroy_process_group()


def test_shard_bounds():
    assert dp.shard_bounds(64, 1, 2) == (32, 64)
    with pytest.raises(ValueError):
        dp.shard_bounds(10, 0, 3)


def test_never_grad_parameters_match_reference_semantics():
    """The engine's never-grad list == the parameters whose .grad stays None after a backward of
    the CPU restatement (conv4 of every square ResidualBlock, try_with_torch.py:193,205-208)."""
    groups, frozen = param_layout(P.creatModel())
    assert len(frozen) == 12 and all(k.endswith(("conv4.weight", "conv4.bias")) for k in frozen)
    assert [len(g) for g in groups] == [70, 42]
    assert all(k.startswith(("conv1.", "residual1.", "residual2.", "residual3.")) for k in groups[1])
    torch.manual_seed(0)
    m = OracleModel(**CFG)
    x = synthetic_images(2, 64, 64)
    stack_mse(m(x), gaussian_targets(2, 17, 16)[0]).backward()
    none = sorted(k for k, p in m.named_parameters() if p.grad is None)
    assert none == sorted(engine_layout()[1])


def test_flat_layout_is_grad_ready_order():
    torch.manual_seed(0)
    model = P.creatModel(**CFG)
    ref = {k: v.clone() for k, v in model.state_dict().items()}
    fp = FlatParams(model)
    (t0, t1), (s0, s1) = fp.segments
    assert t0 == 0 and t1 == s0 and s1 == fp.active < fp.numel
    named = dict(model.named_parameters())
    assert fp.offsets[id(named["hourglass1.residual_block.conv1.weight"])][0] < t1
    assert s0 <= fp.offsets[id(named["residual1.conv1.weight"])][0] < s1
    assert fp.offsets[id(named["hourglass1.residual_block.conv4.weight"])][0] >= fp.active
    # the parameters became views with unchanged values: the state_dict is still drop-in
    for k, v in model.state_dict().items():
        assert torch.equal(v, ref[k]), k


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
    fps = [shard_grad(r, WORLD, 1.0) for r in range(WORLD)]
    expect = sum(f.grad for f in fps) / WORLD
    active = fps[0].active
    for r in range(WORLD):
        got, launched = out[r]
        assert launched == [0, 1]
        torch.testing.assert_close(got, expect, rtol=1e-4, atol=1e-6)
        assert (got[active:] == 0).all()  # the never-grad tail is neither written nor reduced
    assert torch.equal(out[0][0], out[1][0])


def test_bench_launcher_starts_two_ranks():
    """`bench.py --gpus 2` without WORLD_SIZE launches the ranks itself; --dry-run keeps it off
    the GPU (gloo, flat-gradient all-reduce of the real layout)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--dry-run", "--steps", "2"], capture_output=True, text=True, timeout=300,
                       env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "dp2"
    assert rec["allreduce_ok"] is True and rec["dry_run"] is True
    # the multi-rank line explains itself: bytes / buckets reduced, each rank's step time and the
    # all-reduce time the overlap did not hide (gloo on the CPU: all of it)
    c = rec["comm"]
    assert c["bytes_reduced_per_step"] == 4 * rec["config"]["active_params"]
    assert c["buckets_per_step"] >= c["segments"] == len(rec["config"]["segments"]) == 2
    assert len(c["per_rank_ms_per_step"]) == 2 and all(v > 0 for v in c["per_rank_ms_per_step"])
    assert c["probe_steps"] == 2 and c["allreduce_ms_per_step_max"] > 0
    assert c["exposed_allreduce_ms_per_step_max"] == c["allreduce_ms_per_step_max"]
