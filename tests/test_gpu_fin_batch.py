"""Several BatchNorms' finalizes in one launch (hgk_bn_finalize_multi / hgk_bn_bwd_finalize_multi,
engine route fin_batch): per BN exactly the single-BN launch's result, bitwise — forward stat
[4][C] + running-statistics record with wave- and workgroup-merged jobs of different channel
counts mixed in one launch (and more jobs than one launch holds), backward coefficients and the
accumulated dgamma / dbeta — and whole training steps (hourglass_compare: bn4 + projection BN per
block; the primary 4-stack model) bitwise with the route on and off."""
import pytest
import torch
import torch.nn.functional as F

from progressive_process_for_human_pose_estimation_amd import engine as E
from progressive_process_for_human_pose_estimation_amd import hgk as H
from progressive_process_for_human_pose_estimation_amd.data import gaussian_targets, synthetic_images

pytestmark = pytest.mark.gpu
DEV = "cuda"

# (M, C, affine)
FWD = [(131072, 256, True), (2048, 128, True), (32768, 256, False), (512, 256, True),
       (8192, 64, True), (131072, 128, True), (600, 64, True), (65536, 256, True),
       (4096, 256, True), (16384, 128, False)]


def _stats(L, st, M, C, g):
    x = (torch.randn(M, C, device=DEV, generator=g) * 1.7 + 0.4).to(torch.bfloat16)
    part = torch.empty(min(2048, (M + 7) // 8 + 1) * 3 * C, device=DEV)
    rows = H.ctypes.c_int(0)
    H.check(L.hgk_bn_stats(st, H.BF16, x.data_ptr(), M, C, part.data_ptr(), H.ctypes.byref(rows)))
    return x, part, rows.value


def test_finalize_multi_bitwise_single():
    L = H.load_library()
    st = H.stream_handle()
    g = torch.Generator(device=DEV).manual_seed(3)
    jobs, refs, keep = [], [], []
    for M, C, affine in FWD:
        x, part, rows = _stats(L, st, M, C, g)
        gamma = torch.rand(C, device=DEV, generator=g) + 0.5 if affine else None
        beta = torch.randn(C, device=DEV, generator=g) if affine else None
        rec0, stat0 = torch.empty(2, C, device=DEV, dtype=torch.float64), torch.empty(4, C, device=DEV)
        seg = (H.BnSeg * 1)(H.BnSeg(part.data_ptr(), rows, M, rec0.data_ptr(), stat0.data_ptr()))
        H.check(L.hgk_bn_finalize_deferred(st, seg, 1, C, H.ptr(gamma), H.ptr(beta), 1e-5))
        rec1 = torch.full((2, C), float("nan"), device=DEV, dtype=torch.float64)
        stat1 = torch.full((4, C), float("nan"), device=DEV)
        jobs.append(H.BnFinJob(part.data_ptr(), rows, M, C, H.ptr(gamma), H.ptr(beta), 1e-5,
                               rec1.data_ptr(), stat1.data_ptr()))
        refs.append((rec0, stat0, rec1, stat1, rows))
        keep.append((x, part, gamma, beta))
    assert any(r[4] > 256 for r in refs) and any(r[4] <= 256 for r in refs)
    H.check(L.hgk_bn_finalize_multi(st, (H.BnFinJob * len(jobs))(*jobs), len(jobs)))
    torch.cuda.synchronize()
    for i, (rec0, stat0, rec1, stat1, _) in enumerate(refs):
        assert torch.equal(rec0, rec1), i
        assert torch.equal(stat0, stat1), i


def test_bwd_finalize_multi_bitwise_single():
    L = H.load_library()
    st = H.stream_handle()
    g = torch.Generator(device=DEV).manual_seed(4)
    jobs, refs, keep = [], [], []
    for M, C in [(131072, 256), (32768, 128), (65536, 256)]:
        dA = torch.randn(M, C, device=DEV, generator=g).to(torch.bfloat16)
        y = (torch.randn(M, C, device=DEV, generator=g) + 0.2).to(torch.bfloat16)
        sc = torch.rand(C, device=DEV, generator=g) + 0.5
        sh = torch.randn(C, device=DEV, generator=g) * 0.2
        mu = torch.randn(C, device=DEV, generator=g) * 0.1
        iv = torch.rand(C, device=DEV, generator=g) + 0.5
        part = torch.empty(min(2048, (M + 7) // 8 + 1) * 2 * C, device=DEV)
        rows = H.ctypes.c_int(0)
        H.check(L.hgk_bn_bwd_reduce(st, H.BF16, dA.data_ptr(), y.data_ptr(), M, C, sc.data_ptr(),
                                    sh.data_ptr(), 1, mu.data_ptr(), iv.data_ptr(), part.data_ptr(),
                                    H.ctypes.byref(rows)))
        rows = rows.value
        assert rows >= L.hgk_bn_bwd_finalize_multi_min_rows()
        d0 = [torch.randn(C, device=DEV, generator=g) for _ in range(2)]
        out = []
        for multi in (False, True):
            dg, db, coef = d0[0].clone(), d0[1].clone(), torch.full((4, C), float("nan"), device=DEV)
            out.append((dg, db, coef))
            if not multi:
                H.check(L.hgk_bn_bwd_finalize(st, part.data_ptr(), rows, M, C, sc.data_ptr(), mu.data_ptr(),
                                              iv.data_ptr(), 1, dg.data_ptr(), db.data_ptr(), coef.data_ptr(),
                                              None))
            else:
                jobs.append(H.BnbFinJob(part.data_ptr(), rows, M, C, sc.data_ptr(), mu.data_ptr(),
                                        iv.data_ptr(), 1, dg.data_ptr(), db.data_ptr(), coef.data_ptr()))
        refs.append(out)
        keep.append((dA, y, sc, sh, mu, iv, part))
    H.check(L.hgk_bn_bwd_finalize_multi(st, (H.BnbFinJob * len(jobs))(*jobs), len(jobs)))
    torch.cuda.synchronize()
    for i, (a, b) in enumerate(refs):
        for t0, t1 in zip(a, b):
            assert torch.equal(t0, t1), i


def _step(build, x, t, dtype, batch):
    with E.routing(fin_batch=batch):
        torch.manual_seed(0)
        m = build().to(DEV).set_engine_dtype(dtype).set_graph_mode(False).train()
        outs = m(x)
        sum(F.mse_loss(o, t) for o in outs).backward()
        torch.cuda.synchronize()
        return (torch.stack([o.detach() for o in outs]).cpu(),
                [None if p.grad is None else p.grad.cpu() for p in m.parameters()],
                {k: v.detach().cpu() for k, v in m.named_buffers()})


@pytest.mark.parametrize("model", ["hourglass_compare", "primary"])
def test_step_bitwise_with_batched_finalizes(model, monkeypatch):
    from progressive_process_for_human_pose_estimation_amd.presets import hourglass_compare as HC
    import progressive_process_for_human_pose_estimation_amd as P
    build = HC.creatModel if model == "hourglass_compare" else P.creatModel
    x = synthetic_images(4, 256, 256, seed=41).to(DEV)
    t = gaussian_targets(4, 16 if model == "hourglass_compare" else 17, 64, seed=42)[0].to(DEV)
    counts = []
    orig = E.Ctx.finish_forward

    def spy(self):
        orig(self)
        counts.append(self.n_fin_batched)
    monkeypatch.setattr(E.Ctx, "finish_forward", spy)
    on = _step(build, x, t, torch.bfloat16, True)
    n_on = sum(counts)
    off = _step(build, x, t, torch.bfloat16, False)
    assert n_on > 0 and sum(counts) == n_on
    assert torch.equal(on[0], off[0])
    for a, b in zip(on[1], off[1]):
        assert (a is None) == (b is None) and (a is None or torch.equal(a, b))
    for k in on[2]:
        assert torch.equal(on[2][k], off[2][k]), k


def _grads_eval(build, x, loss_fn, on):
    with E.routing(pair_blocks=on):
        torch.manual_seed(0)
        m = build().to(DEV).set_engine_dtype(torch.float32).set_graph_mode(False).eval()
        outs = m(x)
        loss_fn(outs).backward()
        torch.cuda.synchronize()
        return [o.detach().cpu() for o in outs], [None if p.grad is None else p.grad.cpu() for p in m.parameters()]


def _check_pairing(build, x, loss_fn):
    """route pair_blocks (independent unshared blocks interleaved op by op, their lazy finalizes
    batched): train-mode forward (outputs, BN running statistics) BITWISE the sequential order;
    the backward sums the shared input's gradient contributions in another order, so gradients
    are compared where they are well conditioned — eval mode, fp32 — to 1e-4 relative"""
    res = []
    for on in (True, False):
        with E.routing(pair_blocks=on):
            torch.manual_seed(0)
            m = build().to(DEV).set_engine_dtype(torch.bfloat16).set_graph_mode(False).train()
            with torch.no_grad():
                outs = m(x)
            torch.cuda.synchronize()
            res.append(([o.cpu() for o in outs], {k: v.detach().cpu() for k, v in m.named_buffers()}))
    for a, b in zip(res[0][0], res[1][0]):
        assert torch.equal(a, b)
    for k in res[0][1]:
        assert torch.equal(res[0][1][k], res[1][1][k]), k
    (o1, g1), (o0, g0) = _grads_eval(build, x, loss_fn, True), _grads_eval(build, x, loss_fn, False)
    for a, b in zip(o1, o0):
        assert torch.equal(a, b)
    for a, b in zip(g1, g0):
        assert (a is None) == (b is None)
        if a is not None:
            assert (a - b).abs().max().item() <= 1e-4 * b.abs().max().item() + 1e-7


def test_hourglass_compare_interleaved_block_pairs():
    from progressive_process_for_human_pose_estimation_amd.presets import hourglass_compare as HC
    x = synthetic_images(2, 256, 256, seed=43).to(DEV)
    t = gaussian_targets(2, 16, 64, seed=44)[0].to(DEV)
    _check_pairing(HC.creatModel, x, lambda outs: sum(F.mse_loss(o, t) for o in outs))


def test_trainpy_interleaved_block_pairs():
    from progressive_process_for_human_pose_estimation_amd.presets import train as TP
    x = synthetic_images(2, 256, 256, seed=45).to(DEV)
    _check_pairing(TP.creatModel, x, lambda outs: sum((o * o).mean() for o in outs))
