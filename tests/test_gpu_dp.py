"""GPU tests of the data-parallel Trainer path (trainer.py + dp.GradSync), SURVEY.md §8(e).

* The overlapped schedule — one hipGraph per grad-ready segment, cut at the stem's grad barrier,
  the trunk's all-reduce launched between the two replays on a side stream — replays bit for bit
  like the single-graph step and like eager execution.
* Two ranks on the one GPU of the test box (gloo process group over CUDA tensors: RCCL refuses two
  ranks on one device) drive the REAL Trainer: the 1/W-scaled MSE kernel, the side-stream
  all-reduce per segment, Adam on the active prefix. The reduced gradient must equal the mean of
  the per-shard gradients of single-rank Trainers, and the ranks must end with identical weights.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import progressive_process_for_human_pose_estimation_amd as P
from progressive_process_for_human_pose_estimation_amd.data import gaussian_targets, synthetic_images
from progressive_process_for_human_pose_estimation_amd.trainer import Trainer

pytestmark = pytest.mark.gpu
DEV = "cuda"
WORLD = 2


def shard(rank, n=2, res=128):
    return (synthetic_images(n, res, res, seed=100 + rank),
            gaussian_targets(n, 17, res // 4, seed=200 + rank)[0])


def snapshot(m, tr, losses):
    torch.cuda.synchronize()
    return (losses, torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu(),
            {k: b.clone().cpu() for k, b in m.named_buffers()}, tr.fp.grad.clone().cpu())


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_overlap_split_graph_bitwise_equals_single_graph(dtype):
    x, t = (v.to(DEV) for v in shard(0))
    res = []
    for use_graph, overlap in ((True, False), (True, True), (False, True)):
        torch.manual_seed(0)
        m = P.creatModel(nStack=2).to(DEV)
        tr = Trainer(m, lr=1e-4, dtype=dtype, use_graph=use_graph, overlap=overlap)
        losses = [float(tr.step(x, t)) for _ in range(3)]
        if use_graph and overlap:
            assert tr.graphs is not None and len(tr.graphs) == 2 and tr.graph is None
        res.append(snapshot(m, tr, losses))
    for other in res[1:]:
        assert other[0] == res[0][0]
        assert torch.equal(other[1], res[0][1])
        assert torch.equal(other[3], res[0][3])
        for k in res[0][2]:
            assert torch.equal(other[2][k], res[0][2][k]), k


def test_never_grad_tail_untouched_by_adam():
    """conv4 of square blocks gets no gradient, no Adam update and no optimizer state (as
    torch.optim.Adam skips parameters whose grad is None), even with weight decay."""
    x, t = (v.to(DEV) for v in shard(0))
    torch.manual_seed(0)
    m = P.creatModel(nStack=2).to(DEV)
    before = m.hourglass1.residual_block.conv4.weight.detach().clone()
    tr = Trainer(m, lr=1e-3, weight_decay=0.1, dtype=torch.float32, use_graph=False)
    for _ in range(2):
        tr.step(x, t)
    torch.cuda.synchronize()
    assert torch.equal(m.hourglass1.residual_block.conv4.weight, before)
    assert (tr.fp.grad[tr.fp.active:] == 0).all()
    sd = tr.optimizer_state_dict()
    assert len(sd["state"]) == len(tr.fp.active_ids) < len(tr.fp.params)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, port, use_graph, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(WORLD), LOCAL_RANK="0")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    x, t = (v.to(DEV) for v in shard(rank))
    torch.manual_seed(0)
    m = P.creatModel(nStack=2).to(DEV)
    tr = Trainer(m, lr=1e-4, dtype=torch.float32, use_graph=use_graph)
    assert tr.world == WORLD and tr.overlap
    loss = float(tr.step(x, t))
    out[rank] = (loss, tr.fp.grad.clone().cpu(),
                 torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu())
    dist.destroy_process_group()


@pytest.mark.parametrize("use_graph", [False, True])
def test_two_rank_trainer_matches_mean_of_shard_grads(use_graph):
    # per-shard gradients of single-rank Trainers (world 1: no scaling, no collective)
    ref = []
    for r in range(WORLD):
        x, t = (v.to(DEV) for v in shard(r))
        torch.manual_seed(0)
        m = P.creatModel(nStack=2).to(DEV)
        tr = Trainer(m, lr=1e-4, dtype=torch.float32, use_graph=False)
        tr.step(x, t)
        torch.cuda.synchronize()
        ref.append(tr.fp.grad.clone().cpu())
        active = tr.fp.active
    expect = (ref[0] + ref[1]) / WORLD
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_worker, args=(r, port, use_graph, out)) for r in range(WORLD)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
        assert p.exitcode == 0
    for r in range(WORLD):
        loss, grad, params = out[r]
        torch.testing.assert_close(grad, expect, rtol=1e-6, atol=1e-9)
        assert (grad[active:] == 0).all()
    assert torch.equal(out[0][1], out[1][1])
    assert torch.equal(out[0][2], out[1][2])  # replicas stay identical after Adam


def _rccl_worker(port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                      LOCAL_RANK="0", HSA_ENABLE_IPC_MODE_LEGACY="0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    x, t = (v.to(DEV) for v in shard(0))
    res = []
    for use_graph in (True, False):
        torch.manual_seed(0)
        m = P.creatModel(nStack=2).to(DEV)
        tr = Trainer(m, lr=1e-4, dtype=torch.bfloat16, use_graph=use_graph, overlap=True)
        assert tr.sync.grouped and tr.sync.stream is not None
        losses = [float(tr.step(x, t)) for _ in range(3)]
        if use_graph:
            assert tr.graphs is not None and len(tr.graphs) == 2
        res.append(snapshot(m, tr, losses))
    dist.destroy_process_group()
    out[0] = res


def test_rccl_world1_overlap_schedule_bitwise():
    """The multi-GPU step's RCCL branch on the box's one GPU: a 1-rank `nccl` process group makes
    GradSync issue the real RCCL all-reduces on its side stream, between the split hipGraphs
    (trunk segment overlapped with the stem's backward). The result must be bit-identical to the
    Trainer without any process group (a 1-rank SUM all-reduce is the identity)."""
    x, t = (v.to(DEV) for v in shard(0))
    torch.manual_seed(0)
    m = P.creatModel(nStack=2).to(DEV)
    tr = Trainer(m, lr=1e-4, dtype=torch.bfloat16, use_graph=True)
    assert not tr.sync.grouped
    ref = snapshot(m, tr, [float(tr.step(x, t)) for _ in range(3)])
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    p = mp.get_context("spawn").Process(target=_rccl_worker, args=(port, out))
    p.start()
    p.join(240)
    assert p.exitcode == 0
    for got in out[0]:
        assert got[0] == ref[0]
        assert torch.equal(got[1], ref[1])
        assert torch.equal(got[3], ref[3])
        for k in ref[2]:
            assert torch.equal(got[2][k], ref[2][k]), k
