"""GPU tests of the fused training step (trainer.py): per-stack MSE kernel, Adam kernel, hipGraph
replay, against the reference loop try_with_torch.py:330-344 (model(x) -> 4x nn.MSELoss -> backward
-> torch.optim.Adam(lr)). 128x128 inputs keep train-mode BN well conditioned (2x2 innermost)."""
import copy

import pytest
import torch
import torch.nn as nn

import progressive_process_for_human_pose_estimation_amd as P
from progressive_process_for_human_pose_estimation_amd import hgk as H
from progressive_process_for_human_pose_estimation_amd.data import gaussian_targets, synthetic_images
from progressive_process_for_human_pose_estimation_amd.trainer import Trainer

pytestmark = pytest.mark.gpu
DEV = "cuda"


def batch(n=2, res=128, k=17):
    return synthetic_images(n, res, res).to(DEV), gaussian_targets(n, k, res // 4)[0].to(DEV)


def test_mse_kernel_matches_torch():
    L = H.load_library()
    o = torch.randn(2, 17, 32, 32, device=DEV)
    t = torch.rand(2, 17, 32, 32, device=DEV)
    part = torch.empty(1024, device=DEV)
    grad = torch.empty_like(o)
    loss = torch.zeros(1, device=DEV)
    rows = H.ctypes.c_int(0)
    s = H.stream_handle()
    H.check(L.hgk_mse_fwd_bwd(s, o.data_ptr(), t.data_ptr(), o.numel(), part.data_ptr(),
                              H.ctypes.byref(rows), grad.data_ptr(), 0.5))
    H.check(L.hgk_mse_finalize(s, part.data_ptr(), rows.value, o.numel(), loss.data_ptr(), 0))
    oo = o.clone().requires_grad_(True)
    ref = nn.functional.mse_loss(oo, t)
    (ref * 0.5).backward()
    torch.testing.assert_close(loss[0], ref.detach(), rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(grad, oo.grad, rtol=1e-6, atol=1e-9)


def test_adam_kernel_matches_torch_adam():
    L = H.load_library()
    p = torch.randn(10000, device=DEV)
    p_ref = p.clone().requires_grad_(True)
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    state = torch.zeros(4, device=DEV)
    opt = torch.optim.Adam([p_ref], lr=1e-3)
    for step in range(3):
        g = torch.randn(10000, device=DEV)
        H.check(L.hgk_adam_step(H.stream_handle(), p.data_ptr(), g.data_ptr(), m.data_ptr(),
                                v.data_ptr(), p.numel(), 1e-3, 0.9, 0.999, 1e-8, 0.0,
                                state.data_ptr()))
        p_ref.grad = g.clone()
        opt.step()
    torch.testing.assert_close(p, p_ref.detach(), rtol=1e-6, atol=1e-7)
    assert float(state[0]) == 3.0


def test_trainer_step_matches_reference_loop():
    """fp32 fused step == autograd through the drop-in model + nn.MSELoss + torch Adam."""
    x, t = batch()
    torch.manual_seed(0)
    ref = P.creatModel(nStack=2).to(DEV)
    model = copy.deepcopy(ref)
    opt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    outs = ref(x)
    loss_ref = sum(nn.functional.mse_loss(o, t) for o in outs)
    opt.zero_grad()
    loss_ref.backward()
    opt.step()
    tr = Trainer(model, lr=1e-3, dtype=torch.float32, use_graph=False)
    loss = tr.step(x, t)
    torch.cuda.synchronize()
    assert abs(float(loss.detach()) - float(loss_ref.detach())) < 1e-5 * float(loss_ref.detach())
    for (k, a), (_, b) in zip(model.named_parameters(), ref.named_parameters()):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=2e-6, msg=k)
    for (k, a), (_, b) in zip(model.named_buffers(), ref.named_buffers()):
        torch.testing.assert_close(a.float(), b.float(), rtol=1e-4, atol=1e-5, msg=k)


def test_graph_replay_bitwise_equals_eager():
    """Deterministic kernels (no float atomics): replaying the captured step reproduces eager
    execution bit for bit."""
    x, t = batch()
    res = []
    for use_graph in (False, True):
        torch.manual_seed(0)
        m = P.creatModel(nStack=2).to(DEV)
        tr = Trainer(m, lr=1e-4, dtype=torch.bfloat16, use_graph=use_graph)
        losses = [float(tr.step(x, t)) for _ in range(3)]
        torch.cuda.synchronize()
        res.append((losses, torch.cat([p.detach().reshape(-1) for p in m.parameters()]).clone(),
                    {k: b.clone() for k, b in m.named_buffers()}))
    assert res[0][0] == res[1][0]
    assert torch.equal(res[0][1], res[1][1])
    for k in res[0][2]:
        assert torch.equal(res[0][2][k], res[1][2][k]), k


def test_bf16_training_reduces_loss():
    x, t = batch(n=4)
    torch.manual_seed(0)
    m = P.creatModel(nStack=2).to(DEV)
    tr = Trainer(m, lr=2e-4, dtype=torch.bfloat16, use_graph=True)
    losses = [float(tr.step(x, t)) for _ in range(15)]
    assert losses[-1] < 0.7 * losses[0], losses
    # state_dict stays drop-in after flattening the parameters into one buffer
    sd = m.state_dict()
    assert len(sd) == 199 and all(torch.isfinite(v.float()).all() for v in sd.values())


@pytest.mark.parametrize("use_graph", [False, True])
def test_branch_parallel_schedule_is_bitwise_identical(use_graph, routes):
    """Hourglass up-branches on side streams (Ctx.enable_branches): the shared-weight
    read-modify-writes are ordered by per-resource events in host issue order, so losses,
    weights and BN running statistics equal the single-stream schedule bit for bit. (The branch
    schedule replaces the twin chains, so the single-stream reference runs without them too.)"""
    routes(twin="0")
    x, t = batch(n=2)
    res = []
    for branches in (False, True):
        torch.manual_seed(0)
        m = P.creatModel(nStack=2).to(DEV)
        tr = Trainer(m, lr=1e-4, dtype=torch.bfloat16, use_graph=use_graph, branches=branches)
        losses = [float(tr.step(x, t)) for _ in range(3)]
        torch.cuda.synchronize()
        res.append((losses, torch.cat([p.detach().reshape(-1) for p in m.parameters()]).clone(),
                    {k: b.clone() for k, b in m.named_buffers()}))
    assert res[0][0] == res[1][0]
    assert torch.equal(res[0][1], res[1][1])
    for k in res[0][2]:
        assert torch.equal(res[0][2][k], res[1][2][k]), k


@pytest.mark.parametrize("use_graph", [False, True])
def test_num_batches_tracked_counts_every_use(use_graph):
    """BN num_batches_tracked (one flat counter buffer in the Trainer) advances by the module's
    uses per step, every step, like PyTorch's per-call increment (try_with_torch.py:217,286)."""
    x, t = batch()
    torch.manual_seed(0)
    ref = P.creatModel(nStack=2).to(DEV)
    with torch.no_grad():
        ref.train()(x)  # one forward: every BN's per-step use count
    per_step = {k: int(b) for k, b in ref.named_buffers() if k.endswith("num_batches_tracked")}
    torch.manual_seed(0)
    m = P.creatModel(nStack=2).to(DEV)
    tr = Trainer(m, lr=1e-4, dtype=torch.bfloat16, use_graph=use_graph)
    for _ in range(3):
        tr.step(x, t)
    torch.cuda.synchronize()
    got = {k: int(b) for k, b in m.named_buffers() if k.endswith("num_batches_tracked")}
    assert got == {k: 3 * v for k, v in per_step.items()}
    assert len(m.state_dict()) == 199


def test_checkpoint_roundtrip_and_reference_adam_format(tmp_path):
    """Trainer checkpoints in the reference's layout (try_with_torch.py:361-367): a torch Adam
    loads the 'optimizer' entry, and a fresh Trainer restored from the file continues exactly."""
    from progressive_process_for_human_pose_estimation_amd.trainer import load_matching
    x, t = batch()
    torch.manual_seed(0)
    m = P.creatModel(nStack=2).to(DEV)
    tr = Trainer(m, lr=1e-4, dtype=torch.bfloat16, use_graph=True)
    for _ in range(2):
        tr.step(x, t)
    path = tmp_path / "params.pkl"
    torch.save(tr.checkpoint(epoch=3, loss=[0.5, 0.4]), path)
    state = torch.load(path, weights_only=True)
    assert set(state) == {"epoch", "state_dict", "optimizer", "loss"}
    # the reference's own optimizer accepts it
    ref = P.creatModel(nStack=2)
    opt = torch.optim.Adam(ref.parameters(), lr=1e-5)
    opt.load_state_dict(state["optimizer"])
    assert float(opt.state[next(iter(ref.parameters()))]["step"]) == 2.0
    # restore into a fresh trainer; both continue identically
    torch.manual_seed(1)
    m2 = P.creatModel(nStack=2).to(DEV)
    tr2 = Trainer(m2, lr=1e-5, dtype=torch.bfloat16, use_graph=True)
    epoch, loss = tr2.load_checkpoint(state)
    assert epoch == 3 and loss == [0.5, 0.4] and tr2.lr == 1e-4
    a = float(tr.step(x, t))
    b = float(tr2.step(x, t))
    torch.cuda.synchronize()
    assert a == b
    for (k, p1), (_, p2) in zip(m.named_parameters(), m2.named_parameters()):
        assert torch.equal(p1, p2), k
    # fine-tune load: a 17-output checkpoint into an 18-output model keeps the matching keys
    m3 = P.creatModel(nStack=2, nOutChannels=18)
    taken = load_matching(m3, state["state_dict"])
    assert "conv2.weight" not in taken and "residual1.conv1.weight" in taken


def test_short_training_pckh_matches_cpu_restatement():
    """SURVEY §8(d) PCKh gate (ii): a short synthetic-target training run (1 stack, 128², N=4,
    fixed batch, 80 Adam steps at lr 1e-3, sum of per-stack MSE) through the fused Trainer (HIP
    engine + HIP Adam, fp32) and through the CPU restatement (oracle + torch Adam) from the same
    seeded weights; PCKh@0.5 (train.py:759-791 on the HIP kernel, head box 4x4 heatmap px ->
    1.7 px threshold) of the two trained models must agree within 0.2."""
    import numpy as np
    from oracle.data_oracle import pckh
    from oracle.hourglass_oracle import OracleModel, stack_mse
    from progressive_process_for_human_pose_estimation_amd.data import synthetic_images
    from progressive_process_for_human_pose_estimation_amd.targets import PCKh
    N, R, J, steps = 4, 128, 16, 80
    h = R // 4
    x = synthetic_images(N, R, R, seed=7)
    rng = np.random.default_rng(3)
    yy, xx = np.mgrid[0:h, 0:h]
    tgt = np.zeros((N, J + 1, h, h), np.float32)
    lab = np.zeros((N, h, h), np.int32)
    for n in range(N):
        for j in range(J):
            py, px = rng.integers(2, h - 2, size=2)
            tgt[n, j + 1] = np.exp(-((yy - py) ** 2 + (xx - px) ** 2) / 2.0)
            lab[n, py, px] = j + 1
    rect = np.tile(np.array([0.0, 0.0, 4.0, 4.0]), (N, 1))
    t = torch.from_numpy(tgt)

    torch.manual_seed(0)
    m = P.creatModel(nStack=1).to(DEV)
    tr = Trainer(m, lr=1e-3, dtype=torch.float32, use_graph=False)
    for _ in range(steps):
        tr.step(x.to(DEV), t.to(DEV))
    with torch.no_grad():
        hm_build = m.train()(x.to(DEV))[-1].cpu()
    acc_build = float(np.nanmean(PCKh()(hm_build, torch.from_numpy(lab), rect)[0][:, 10]))

    torch.set_num_threads(16)
    torch.manual_seed(0)
    o = OracleModel(nStack=1)
    opt = torch.optim.Adam(o.parameters(), lr=1e-3)
    for _ in range(steps):
        loss = stack_mse(o(x), t)
        opt.zero_grad()
        loss.backward()
        opt.step()
    with torch.no_grad():
        hm_cpu = o(x)[-1].numpy()
    acc_cpu = float(np.nanmean(pckh(hm_cpu, lab, rect)[0][:, 10]))
    print(f"PCKh@0.5 after {steps} steps: build {acc_build:.3f}, CPU restatement {acc_cpu:.3f}")
    assert np.isfinite(acc_build) and np.isfinite(acc_cpu)
    assert abs(acc_build - acc_cpu) <= 0.2, (acc_build, acc_cpu)
    # and both actually learned the batch (measured: build 0.969, CPU restatement 0.953)
    assert min(acc_build, acc_cpu) >= 0.8, (acc_build, acc_cpu)


def test_eager_step_frees_activations_without_cyclic_gc():
    """Engine activations form no reference cycles: with the cyclic GC off, the device memory an
    eager Trainer step allocates is back with the caching allocator once the step returns (a
    conv output that referred to itself through Act.producer was freed only by gc)."""
    import gc
    x, t = batch()
    tr = Trainer(P.creatModel(nStack=2).to(DEV), dtype=torch.bfloat16, use_graph=False)
    tr.step(x, t)
    torch.cuda.synchronize()
    gc.collect()
    gc.disable()
    try:
        base = torch.cuda.memory_allocated()
        for _ in range(3):
            tr.step(x, t)
        torch.cuda.synchronize()
        assert torch.cuda.memory_allocated() == base
    finally:
        gc.enable()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_fused_mse_heads_match_the_per_head_path(dtype):
    """Trainer.fused_mse (hgk_mse_heads_nhwc: every head's MSE in one launch on the NHWC heads) vs
    the per-head NCHW path (nhwc_to_nchw + hgk_mse_fwd_bwd + nchw_to_nhwc): the gradients — hence
    every parameter gradient — bit for bit, the loss to fp32 summation order."""
    x, t = batch(n=4)
    res = []
    for fused in (True, False):
        torch.manual_seed(0)
        m = P.creatModel(nStack=4).to(DEV)
        tr = Trainer(m, lr=1e-4, dtype=dtype, use_graph=False)
        tr.fused_mse = fused
        tr.step(x, t)   # the grads stay in tr.fp.grad (Adam reads them)
        torch.cuda.synchronize()
        res.append((float(tr.loss), tr.fp.grad.clone()))
    (l1, g1), (l0, g0) = res
    assert torch.equal(g1, g0)
    assert abs(l1 - l0) <= 1e-6 * abs(l0), (l1, l0)
