"""A BN pair whose outputs are summed (hourglass_compare's block output, hourglass_compare.py:
437-440): hgk_bn_apply2_add must be BITWISE hgk_bn_apply x2 + hgk_add + hgk_bn_stats (the sum's
statistics partials), hgk_bn_bwd_reduce2 bitwise two hgk_bn_bwd_reduce calls, and the engine's
fused block output (Ctx.bn_add, the default) bitwise the unfused one (engine route bn_add=0) over a
whole hourglass_compare training step: heatmaps, every gradient, BN running statistics."""
import pytest
import torch
import torch.nn.functional as F

from progressive_process_for_human_pose_estimation_amd import engine as E
from progressive_process_for_human_pose_estimation_amd import hgk as H
from progressive_process_for_human_pose_estimation_amd.data import gaussian_targets, synthetic_images

pytestmark = pytest.mark.gpu
DEV = "cuda"
DT = {torch.bfloat16: H.BF16, torch.float32: H.F32}


def _side(g, M, C, dtype, relu):
    y = (torch.randn(M, C, device=DEV, generator=g) * 2 + 0.3).to(dtype)
    sc = torch.rand(C, device=DEV, generator=g) + 0.5
    sh = torch.randn(C, device=DEV, generator=g) * 0.2
    mu = torch.randn(C, device=DEV, generator=g) * 0.1
    iv = torch.rand(C, device=DEV, generator=g) + 0.5
    return y, sc, sh, mu, iv, relu


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("M,C", [(131072, 256), (2048, 256), (520, 128), (32, 256)])
def test_bn_apply2_add_bitwise(dtype, M, C):
    L = H.load_library()
    st = H.stream_handle()
    g = torch.Generator(device=DEV).manual_seed(M + C)
    a = _side(g, M, C, dtype, 0)
    b = _side(g, M, C, dtype, 1)
    dt = DT[dtype]
    # reference: the separate passes
    ta, tb, ref = (torch.empty(M, C, device=DEV, dtype=dtype) for _ in range(3))
    for (y, sc, sh, _, _, relu), t in ((a, ta), (b, tb)):
        H.check(L.hgk_bn_apply(st, dt, y.data_ptr(), M, C, sc.data_ptr(), sh.data_ptr(), relu, t.data_ptr()))
    H.check(L.hgk_add(st, dt, ta.data_ptr(), tb.data_ptr(), ref.data_ptr(), ref.numel(), 0))
    cap = min(2048, (M + 7) // 8 + 1)
    p_ref = torch.full((cap * 3 * C,), float("nan"), device=DEV)
    rows_ref = H.ctypes.c_int(0)
    H.check(L.hgk_bn_stats(st, dt, ref.data_ptr(), M, C, p_ref.data_ptr(), H.ctypes.byref(rows_ref)))
    # fused
    out = torch.empty(M, C, device=DEV, dtype=dtype)
    part = torch.full((cap * 3 * C,), float("nan"), device=DEV)
    rows = H.ctypes.c_int(0)
    sa = H.BnSide(a[0].data_ptr(), a[1].data_ptr(), a[2].data_ptr(), None, None, a[5], None)
    sb = H.BnSide(b[0].data_ptr(), b[1].data_ptr(), b[2].data_ptr(), None, None, b[5], None)
    H.check(L.hgk_bn_apply2_add(st, dt, H.ctypes.byref(sa), H.ctypes.byref(sb), out.data_ptr(), M, C,
                                part.data_ptr(), H.ctypes.byref(rows)))
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    assert rows.value == rows_ref.value
    n = rows.value * 3 * C
    assert torch.equal(part[:n], p_ref[:n])


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("M,C", [(131072, 256), (2048, 256), (520, 128)])
def test_bn_bwd_reduce2_bitwise(dtype, M, C):
    L = H.load_library()
    st = H.stream_handle()
    g = torch.Generator(device=DEV).manual_seed(7 * M + C)
    dA = (torch.randn(M, C, device=DEV, generator=g)).to(dtype)
    sides = [_side(g, M, C, dtype, r) for r in (0, 1)]
    dt = DT[dtype]
    cap = min(2048, (M + 7) // 8 + 1)
    refs = []
    for y, sc, sh, mu, iv, relu in sides:
        p = torch.full((cap * 2 * C,), float("nan"), device=DEV)
        rows = H.ctypes.c_int(0)
        H.check(L.hgk_bn_bwd_reduce(st, dt, dA.data_ptr(), y.data_ptr(), M, C, sc.data_ptr(), sh.data_ptr(),
                                    relu, mu.data_ptr(), iv.data_ptr(), p.data_ptr(), H.ctypes.byref(rows)))
        refs.append((p, rows.value))
    parts = [torch.full((cap * 2 * C,), float("nan"), device=DEV) for _ in sides]
    ss = [H.BnSide(y.data_ptr(), sc.data_ptr(), sh.data_ptr(), mu.data_ptr(), iv.data_ptr(), relu, p.data_ptr())
          for (y, sc, sh, mu, iv, relu), p in zip(sides, parts)]
    rows = H.ctypes.c_int(0)
    H.check(L.hgk_bn_bwd_reduce2(st, dt, dA.data_ptr(), M, C, H.ctypes.byref(ss[0]), H.ctypes.byref(ss[1]),
                                 H.ctypes.byref(rows)))
    torch.cuda.synchronize()
    for p, (pr, rr) in zip(parts, refs):
        assert rows.value == rr
        n = rr * 2 * C
        assert torch.equal(p[:n], pr[:n])


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_hourglass_compare_fused_block_output_bitwise(dtype):
    from progressive_process_for_human_pose_estimation_amd.presets import hourglass_compare as HC
    x = synthetic_images(2, 128, 128, seed=21).to(DEV)
    t = gaussian_targets(2, 16, 32, seed=22)[0].to(DEV)
    res = []
    for fused in (True, False):
        with E.routing(bn_add=fused):
            torch.manual_seed(0)
            m = HC.creatModel().to(DEV).set_engine_dtype(dtype).set_graph_mode(False).train()
            outs = m(x)
            loss = sum(F.mse_loss(o, t) for o in outs)
            loss.backward()
            torch.cuda.synchronize()
            res.append((torch.stack([o.detach() for o in outs]).cpu(),
                        [None if p.grad is None else p.grad.cpu() for p in m.parameters()],
                        {k: v.detach().cpu() for k, v in m.named_buffers()}))
    (h0, g0, b0), (h1, g1, b1) = res
    assert torch.equal(h0, h1)
    for a, b in zip(g0, g1):
        assert (a is None) == (b is None) and (a is None or torch.equal(a, b))
    for k in b0:
        assert torch.equal(b0[k], b1[k]), k


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("M,C,fused", [(131072, 256, False), (32768, 128, False), (2048, 256, True),
                                       (512, 256, True), (520, 128, True), (32, 256, True)])
@pytest.mark.parametrize("training", [1, 0])
def test_bn_bwd_pair_bitwise(dtype, M, C, fused, training):
    """hgk_bn_bwd_pair = two hgk_bn_bwd_finalize_apply calls (fused: partial rows in-kernel) or two
    hgk_bn_bwd_apply calls over hgk_bn_bwd_finalize's coefficients, bitwise: dy of both sides and
    (fused) the accumulated dgamma / dbeta."""
    L = H.load_library()
    st = H.stream_handle()
    g = torch.Generator(device=DEV).manual_seed(11 * M + C + training)
    dA = torch.randn(M, C, device=DEV, generator=g).to(dtype)
    sides = [_side(g, M, C, dtype, r) for r in (1, 0)]
    dt = DT[dtype]
    cap = min(2048, (M + 7) // 8 + 1)
    parts = []
    for y, sc, sh, mu, iv, relu in sides:
        p = torch.empty(cap * 2 * C, device=DEV)
        rows = H.ctypes.c_int(0)
        H.check(L.hgk_bn_bwd_reduce(st, dt, dA.data_ptr(), y.data_ptr(), M, C, sc.data_ptr(), sh.data_ptr(),
                                    relu, mu.data_ptr(), iv.data_ptr(), p.data_ptr(), H.ctypes.byref(rows)))
        parts.append((p, rows.value))
    assert (max(r for _, r in parts) <= L.hgk_bn_bwd_fused_max_rows()) == fused
    dg0 = [torch.randn(C, device=DEV, generator=g) for _ in range(4)]
    ref_dy, ref_dg, coefs = [], [], []
    for k, ((y, sc, sh, mu, iv, relu), (p, rows)) in enumerate(zip(sides, parts)):
        dy = torch.empty(M, C, device=DEV, dtype=dtype)
        dgam, dbet = dg0[2 * k].clone(), dg0[2 * k + 1].clone()
        if fused:
            H.check(L.hgk_bn_bwd_finalize_apply(st, dt, p.data_ptr(), rows, M, C, sc.data_ptr(), sh.data_ptr(),
                                                relu, mu.data_ptr(), iv.data_ptr(), training, dgam.data_ptr(),
                                                dbet.data_ptr(), dA.data_ptr(), y.data_ptr(), None,
                                                dy.data_ptr(), 0))
        else:
            coef = torch.empty(4, C, device=DEV)
            nb = L.hgk_bn_finalize_scratch(rows, C)
            scr = torch.empty(max(1, nb // 4), device=DEV)
            H.check(L.hgk_bn_bwd_finalize(st, p.data_ptr(), rows, M, C, sc.data_ptr(), mu.data_ptr(),
                                          iv.data_ptr(), training, dgam.data_ptr(), dbet.data_ptr(),
                                          coef.data_ptr(), scr.data_ptr() if nb else None))
            H.check(L.hgk_bn_bwd_apply(st, dt, dA.data_ptr(), y.data_ptr(), M, C, sc.data_ptr(), sh.data_ptr(),
                                       relu, coef.data_ptr(), None, dy.data_ptr(), 0))
            coefs.append(coef)
        ref_dy.append(dy)
        ref_dg.append((dgam, dbet))
    outs = [torch.full((M, C), float("nan"), device=DEV).to(dtype) for _ in sides]
    dgs = [(dg0[2 * k].clone(), dg0[2 * k + 1].clone()) for k in range(2)]
    ss = []
    for k, ((y, sc, sh, mu, iv, relu), (p, rows)) in enumerate(zip(sides, parts)):
        ss.append(H.BnbSide(y.data_ptr(), sc.data_ptr(), sh.data_ptr(), mu.data_ptr(), iv.data_ptr(), relu,
                            p.data_ptr() if fused else None, rows, None if fused else coefs[k].data_ptr(),
                            dgs[k][0].data_ptr() if fused else None, dgs[k][1].data_ptr() if fused else None,
                            outs[k].data_ptr()))
    H.check(L.hgk_bn_bwd_pair(st, dt, dA.data_ptr(), M, C, training, H.ctypes.byref(ss[0]),
                              H.ctypes.byref(ss[1])))
    torch.cuda.synchronize()
    for k in range(2):
        assert torch.equal(outs[k], ref_dy[k]), k
        if fused:
            assert torch.equal(dgs[k][0], ref_dg[k][0]) and torch.equal(dgs[k][1], ref_dg[k][1]), k


def test_bn_bwd_pair_rejects_mixed_modes():
    L = H.load_library()
    st = H.stream_handle()
    M, C = 64, 256
    t = torch.zeros(M, C, device=DEV, dtype=torch.bfloat16)
    v = torch.zeros(4 * C, device=DEV)
    a = H.BnbSide(t.data_ptr(), v.data_ptr(), v.data_ptr(), v.data_ptr(), v.data_ptr(), 0, v.data_ptr(), 2,
                  None, None, None, t.data_ptr())
    b = H.BnbSide(t.data_ptr(), v.data_ptr(), v.data_ptr(), v.data_ptr(), v.data_ptr(), 0, None, 2,
                  v.data_ptr(), None, None, t.data_ptr())
    assert L.hgk_bn_bwd_pair(st, H.BF16, t.data_ptr(), M, C, 1, H.ctypes.byref(a), H.ctypes.byref(b)) != 0


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_hourglass_compare_pair_backward_bitwise(dtype, monkeypatch):
    """engine route bn_pair_bwd (hgk_bn_bwd_pair after the dual reduction, the default) bitwise the
    two sides' own finalize / apply (bn_pair_bwd=0) over a whole hourglass_compare training step;
    both modes (in-kernel finalize at the small levels, coefficients at the big ones) are taken."""
    from progressive_process_for_human_pose_estimation_amd.presets import hourglass_compare as HC
    orig, taken = E.Ctx._bn_pair_bwd, []

    def spy(self, va, vb, g):
        rows = va.bwd_part[1]
        ok = orig(self, va, vb, g)
        if ok:
            taken.append(rows <= self.lib.hgk_bn_bwd_fused_max_rows())
        return ok
    monkeypatch.setattr(E.Ctx, "_bn_pair_bwd", spy)
    x = synthetic_images(4, 256, 256, seed=23).to(DEV)  # the 64x64 level: > 128 partial rows
    t = gaussian_targets(4, 16, 64, seed=24)[0].to(DEV)
    res = []
    for on in (True, False):
        with E.routing(bn_pair_bwd=on):
            torch.manual_seed(0)
            m = HC.creatModel().to(DEV).set_engine_dtype(dtype).set_graph_mode(False).train()
            outs = m(x)
            loss = sum(F.mse_loss(o, t) for o in outs)
            loss.backward()
            torch.cuda.synchronize()
            res.append([None if p.grad is None else p.grad.cpu() for p in m.parameters()])
    assert True in taken and False in taken, taken
    for a, b in zip(*res):
        assert (a is None) == (b is None) and (a is None or torch.equal(a, b))


def _shared_operand_step(order, fused, hw):
    """x -> conv_a -> relu(bn_a) = va, x -> conv_b -> bn_b = vb, s = va + vb (Ctx.bn_add when
    `fused`, else materialize + add), z = conv_c(va): va has a SECOND consumer, recorded before
    ("before": its backward runs after bn_add's) or after bn_add. Returns the engine's fp32
    gradients (x, conv / BN parameters) and a torch fp32 autograd reference of the same graph."""
    import copy
    import torch.nn as nn
    torch.manual_seed(0)
    C = 128
    mods = nn.ModuleDict({"a": nn.Conv2d(C, C, 1), "b": nn.Conv2d(C, C, 1), "c": nn.Conv2d(C, C, 1),
                          "bn_a": nn.BatchNorm2d(C), "bn_b": nn.BatchNorm2d(C)}).to(DEV)
    with torch.no_grad():
        for k in ("bn_a", "bn_b"):
            mods[k].weight.uniform_(0.5, 1.5)
            mods[k].bias.uniform_(-0.3, 0.3)
    ref = copy.deepcopy(mods)
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, C, hw, hw, generator=g).to(DEV)
    gs = torch.randn(2, C, hw, hw, generator=g).to(DEV)
    gz = torch.randn(2, C, hw, hw, generator=g).to(DEV)

    ctx = E.Ctx(torch.float32, True, torch.device(DEV), grad_enabled=True)
    xa = ctx.input(x, requires_grad=True)
    va = ctx.bn_relu(ctx.conv(xa, mods["a"]), mods["bn_a"])
    vb = ctx.bn_relu(ctx.conv(xa, mods["b"]), mods["bn_b"], relu=False)
    z = ctx.conv(va, mods["c"]) if order == "before" else None
    s = ctx.bn_add(va, vb) if fused else ctx.add(ctx.materialize(va), ctx.materialize(vb))
    if z is None:
        z = ctx.conv(va, mods["c"])
    ctx.finish_forward()
    ctx.grad_from_nchw(s, gs)
    ctx.grad_from_nchw(z, gz)
    ctx.backward()
    gx = xa.grad.view(2, hw, hw, C).permute(0, 3, 1, 2).float()
    got = {"x": gx.cpu()}
    for k, m in mods.items():
        for n, p in m.named_parameters():
            if id(p) in ctx.pgrads:
                got[f"{k}.{n}"] = ctx.pgrads[id(p)].cpu()
    torch.cuda.synchronize()

    xr = x.clone().requires_grad_(True)
    a = torch.relu(ref["bn_a"](ref["a"](xr)))
    b = ref["bn_b"](ref["b"](xr))
    ((a + b) * gs).sum().backward(retain_graph=True)
    (ref["c"](a) * gz).sum().backward()
    want = {"x": xr.grad.cpu()}
    for k, m in ref.items():
        for n, p in m.named_parameters():
            want[f"{k}.{n}"] = p.grad.cpu()
    return got, want


@pytest.mark.parametrize("order", ["before", "after"])
@pytest.mark.parametrize("hw", [16, 64])
def test_bn_add_shared_operand(order, hw):
    """Ctx.bn_add's backward precomputes both BNs' reductions over the sum's gradient only when
    that gradient is each side's whole gradient; an operand with a second consumer (either order)
    must get the BN backward of its accumulated gradient (engine fp32 vs torch fp32 autograd, and
    the fused vs unfused engine paths)."""
    res = {}
    for fused in (True, False):
        got, want = _shared_operand_step(order, fused, hw)
        res[fused] = got
        for k, w in want.items():
            if k in ("a.bias", "b.bias"):
                continue  # a conv bias feeding a train-mode BN: mathematically zero gradient
            assert k in got, k
            err = float((got[k] - w).norm() / w.norm())
            assert err < 1e-4, (fused, k, err)
    for k in res[True]:
        torch.testing.assert_close(res[True][k], res[False][k], rtol=1e-4, atol=1e-5 * float(res[False][k].abs().max()))
