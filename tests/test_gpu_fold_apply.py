"""Folded BN-backward apply (hgk_conv_fwd_bnbwd_vg, hgk_conv_seg.vg; engine PendingApply): the
input gradient of conv1 (try_with_torch.py:186) reads bn2's upstream gradient dA and the BN input y
and applies bn2's backward (hgk_bn_bwd_apply's arithmetic, bnb_apply) while staging its operand,
writing the applied gradient for the weight gradient on the side. The separate apply pass is gone;
the results must be BITWISE those of hgk_bn_bwd_apply followed by hgk_conv_fwd_bnbwd.
"""
import pytest
import torch

from progressive_process_for_human_pose_estimation_amd import hgk as H

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _operands(g, N, hw, K, Cout):
    """dgrad input channels K (= the folded BN's channels), output Cout (= the fused BN-bwd's)"""
    bf = torch.bfloat16
    d = dict(
        dA=(torch.randn(N, hw, hw, K, device=DEV, generator=g) * 0.5).to(bf),
        y=(torch.randn(N, hw, hw, K, device=DEV, generator=g) * 0.8 + 0.1).to(bf),
        vsc=torch.rand(K, device=DEV, generator=g) + 0.5,
        vsh=torch.randn(K, device=DEV, generator=g) * 0.3,
        coef=torch.randn(4, K, device=DEV, generator=g) * 0.2,
        bny=(torch.randn(N, hw, hw, Cout, device=DEV, generator=g)).to(bf),
        bsc=torch.rand(Cout, device=DEV, generator=g) + 0.5,
        bsh=torch.randn(Cout, device=DEV, generator=g) * 0.3,
        bmu=torch.randn(Cout, device=DEV, generator=g) * 0.1,
        bis=torch.rand(Cout, device=DEV, generator=g) + 0.5,
    )
    return d


def _packed_dgrad(L, g, K, Cout):
    # conv1 weight [K][Cout] (forward Cout=K from Cin=Cout); its dgrad packing: rows = Cout
    w = torch.randn(K, Cout, 1, 1, device=DEV, generator=g) * 0.05
    ld = L.hgk_conv_w_ld(K)
    wp = torch.empty(((Cout + 127) // 128) * 128, ld, device=DEV, dtype=torch.bfloat16)
    H.check(L.hgk_pack_conv_weight(H.stream_handle(), H.BF16, w.data_ptr(), wp.data_ptr(), ld, K, Cout,
                                   1, 1, 1, K, Cout))
    return wp, ld


def _reference(L, d, wp, ld, N, hw, K, Cout):
    st = H.stream_handle()
    M = N * hw * hw
    dy = torch.empty_like(d["dA"])
    H.check(L.hgk_bn_bwd_apply(st, H.BF16, d["dA"].data_ptr(), d["y"].data_ptr(), M, K,
                               d["vsc"].data_ptr(), d["vsh"].data_ptr(), 1, d["coef"].data_ptr(), None,
                               dy.data_ptr(), 0))
    out = torch.empty(N, hw, hw, Cout, device=DEV, dtype=torch.bfloat16)
    part = torch.zeros(H.load_library().hgk_max_stats_rows() * 2 * Cout, device=DEV)
    rows = H.ctypes.c_int(0)
    H.check(L.hgk_conv_fwd_bnbwd(st, H.BF16, dy.data_ptr(), wp.data_ptr(), ld, None, out.data_ptr(),
                                 N, hw, hw, K, Cout, 1, 1, 1, 0, 1, None, 0, d["bny"].data_ptr(),
                                 d["bsc"].data_ptr(), d["bsh"].data_ptr(), 1, d["bmu"].data_ptr(),
                                 d["bis"].data_ptr(), part.data_ptr(), H.ctypes.byref(rows)))
    return dy, out, part[: rows.value * 2 * Cout].clone(), rows.value


def test_vgrad_ok_query():
    L = H.load_library()
    assert L.hgk_conv_vgrad_ok(H.BF16, 32, 64, 64, 0, 0, 0, 128, 256, 1, 1, 1, 0, 1, 1) == 1
    assert L.hgk_conv_vgrad_ok(H.BF16, 32, 64, 64, 32, 32, 32, 128, 256, 1, 1, 1, 0, 1, 1) == 1
    assert L.hgk_conv_vgrad_ok(H.F32, 32, 64, 64, 0, 0, 0, 128, 256, 1, 1, 1, 0, 1, 1) == 0
    # small M: the image-tile kernel (128-channel input only)
    assert L.hgk_conv_vgrad_ok(H.BF16, 2, 8, 8, 0, 0, 0, 128, 256, 1, 1, 1, 0, 1, 1) == 1
    assert L.hgk_conv_vgrad_ok(H.BF16, 2, 8, 8, 0, 0, 0, 256, 128, 1, 1, 1, 0, 1, 1) == 0
    assert L.hgk_conv_vgrad_ok(H.BF16, 32, 8, 8, 32, 4, 4, 128, 128, 3, 3, 1, 1, 1, 1) == 1
    # the folded finalize too: image tiles only, <= 32 partial rows
    assert L.hgk_conv_vgrad_fin_ok(H.BF16, 32, 8, 8, 0, 0, 0, 128, 128, 3, 3, 1, 1, 1, 1, 32, 0, 0) == 1
    assert L.hgk_conv_vgrad_fin_ok(H.BF16, 32, 8, 8, 32, 4, 4, 128, 256, 1, 1, 1, 0, 1, 1, 32, 8, 0) == 1
    assert L.hgk_conv_vgrad_fin_ok(H.BF16, 32, 16, 16, 0, 0, 0, 128, 256, 1, 1, 1, 0, 1, 1, 128, 0, 0) == 0
    assert L.hgk_conv_vgrad_fin_ok(H.BF16, 32, 64, 64, 0, 0, 0, 128, 256, 1, 1, 1, 0, 1, 1, 32, 0, 0) == 0
    # with the skip gradient added (bn1): the 256-channel 1x1 only
    assert L.hgk_conv_vgrad_fin_ok(H.BF16, 32, 8, 8, 32, 4, 4, 256, 128, 1, 1, 1, 0, 1, 1, 32, 8, 1) == 1
    assert L.hgk_conv_vgrad_fin_ok(H.BF16, 32, 8, 8, 0, 0, 0, 256, 128, 1, 1, 1, 0, 1, 1, 32, 0, 0) == 0
    assert L.hgk_conv_vgrad_fin_ok(H.BF16, 32, 8, 8, 0, 0, 0, 128, 256, 1, 1, 1, 0, 1, 1, 32, 0, 1) == 0
    # 3x3 128 -> 128: the row-streaming kernel at 64x64 (and 64x64 + 32x32 twins), not 32x32 alone
    assert L.hgk_conv_vgrad_ok(H.BF16, 32, 64, 64, 0, 0, 0, 128, 128, 3, 3, 1, 1, 1, 1) == 1
    assert L.hgk_conv_vgrad_ok(H.BF16, 32, 64, 64, 32, 32, 32, 128, 128, 3, 3, 1, 1, 1, 1) == 1
    assert L.hgk_conv_vgrad_ok(H.BF16, 32, 32, 32, 0, 0, 0, 128, 128, 3, 3, 1, 1, 1, 1) == 0
    assert L.hgk_conv_vgrad_ok(H.BF16, 32, 64, 64, 0, 0, 0, 128, 256, 1, 1, 1, 0, 1, 0) == 0  # no bnbwd


def test_conv_bnbwd_vg_bitwise_single():
    L = H.load_library()
    g = torch.Generator(device=DEV).manual_seed(7)
    N, hw, K, Cout = 32, 64, 128, 256
    d = _operands(g, N, hw, K, Cout)
    wp, ld = _packed_dgrad(L, g, K, Cout)
    dy_ref, out_ref, part_ref, rows_ref = _reference(L, d, wp, ld, N, hw, K, Cout)
    st = H.stream_handle()
    side = torch.full_like(d["dA"], float("nan"))
    out = torch.empty_like(out_ref)
    part = torch.zeros(L.hgk_max_stats_rows() * 2 * Cout, device=DEV)
    rows = H.ctypes.c_int(0)
    vg = H.BnVgrad(d["y"].data_ptr(), d["vsc"].data_ptr(), d["vsh"].data_ptr(), d["coef"].data_ptr(),
                   1, side.data_ptr())
    H.check(L.hgk_conv_fwd_bnbwd_vg(st, H.BF16, d["dA"].data_ptr(), wp.data_ptr(), ld, None,
                                    out.data_ptr(), N, hw, hw, K, Cout, 1, 1, 1, 0, 1, None, 0,
                                    d["bny"].data_ptr(), d["bsc"].data_ptr(), d["bsh"].data_ptr(), 1,
                                    d["bmu"].data_ptr(), d["bis"].data_ptr(), part.data_ptr(),
                                    H.ctypes.byref(rows), H.ctypes.byref(vg)))
    torch.cuda.synchronize()
    assert rows.value == rows_ref
    assert torch.equal(side.view(torch.int16), dy_ref.view(torch.int16))
    assert torch.equal(out.view(torch.int16), out_ref.view(torch.int16))
    assert torch.equal(part[: rows_ref * 2 * Cout], part_ref)


def test_conv_bnbwd_vg_bitwise_twin():
    """64x64 + 32x32 segments in one ring launch: against hgk_bn_bwd_apply per segment + the same
    twin launch on the applied gradients"""
    L = H.load_library()
    g = torch.Generator(device=DEV).manual_seed(11)
    N, K, Cout = 32, 128, 256
    wp, ld = _packed_dgrad(L, g, K, Cout)
    st = H.stream_handle()
    ops = [_operands(g, N, hw, K, Cout) for hw in (64, 32)]

    def twin(vg_on):
        keep, segs, res = [], [], []
        for hw, d in zip((64, 32), ops):
            M = N * hw * hw
            side = torch.full_like(d["dA"], float("nan"))
            if vg_on:
                x = d["dA"]
                vg = H.BnVgrad(d["y"].data_ptr(), d["vsc"].data_ptr(), d["vsh"].data_ptr(),
                               d["coef"].data_ptr(), 1, side.data_ptr())
                keep.append(vg)
                vgp = H.ctypes.pointer(vg)
            else:
                H.check(L.hgk_bn_bwd_apply(st, H.BF16, d["dA"].data_ptr(), d["y"].data_ptr(), M, K,
                                           d["vsc"].data_ptr(), d["vsh"].data_ptr(), 1,
                                           d["coef"].data_ptr(), None, side.data_ptr(), 0))
                x, vgp = side, None
            out = torch.empty(N, hw, hw, Cout, device=DEV, dtype=torch.bfloat16)
            part = torch.zeros(L.hgk_max_stats_rows() * 2 * Cout, device=DEV)
            rc = H.ctypes.c_int(0)
            keep.append(rc)
            segs.append(H.ConvSeg(x.data_ptr(), None, out.data_ptr(), None, None, None, None, N, hw, hw,
                                  d["bny"].data_ptr(), d["bsc"].data_ptr(), d["bsh"].data_ptr(),
                                  d["bmu"].data_ptr(), d["bis"].data_ptr(), part.data_ptr(), 1,
                                  H.ctypes.pointer(rc), vgp))
            res.append((side, out, part, rc))
        arr = (H.ConvSeg * 2)(*segs)
        H.check(L.hgk_conv_fwd_twin(st, H.BF16, wp.data_ptr(), ld, None, 0, 0, K, Cout, 1, 1, 1, 0, 1,
                                    arr, None, 0))
        torch.cuda.synchronize()
        return [(s_, o, p[: rc.value * 2 * Cout].clone(), rc.value) for s_, o, p, rc in res]

    ref, got = twin(False), twin(True)
    for (s0, o0, p0, r0), (s1, o1, p1, r1) in zip(ref, got):
        assert r1 == r0 > 0
        assert torch.equal(s1.view(torch.int16), s0.view(torch.int16))
        assert torch.equal(o1.view(torch.int16), o0.view(torch.int16))
        assert torch.equal(p1, p0)


def _packed_dgrad3(L, g, C):
    w = torch.randn(C, C, 3, 3, device=DEV, generator=g) * (1.0 / (9 * C) ** 0.5)
    ld = L.hgk_conv_w_ld(9 * C)
    wp = torch.empty(C, ld, device=DEV, dtype=torch.bfloat16)
    H.check(L.hgk_pack_conv_weight(H.stream_handle(), H.BF16, w.data_ptr(), wp.data_ptr(), ld, C, C,
                                   3, 3, 1, C, C))
    return wp, ld


@pytest.mark.parametrize("relu", [1, 0], ids=["relu", "norelu"])
@pytest.mark.parametrize("shape", [(32, (64,)), (3, (64,)), (8, (64, 32))], ids=["n32", "n3", "twin"])
def test_conv3x3_bnbwd_vg_bitwise(shape, relu):
    """the 3x3 input gradient of conv2 (try_with_torch.py:189) with bn3's backward apply folded in
    (row-streaming kernel, mode 20): dA, the BN-backward partials of bn2 and the applied gradient
    (vout) BITWISE those of hgk_bn_bwd_apply + the unfolded launch, single and 64x64 + 32x32 twin"""
    L = H.load_library()
    g = torch.Generator(device=DEV).manual_seed(13)
    N, hws = shape
    C = 128
    wp, ld = _packed_dgrad3(L, g, C)
    st = H.stream_handle()
    ops = [_operands(g, N, hw, C, C) for hw in hws]

    def run(vg_on):
        keep, segs, res = [], [], []
        for hw, d in zip(hws, ops):
            M = N * hw * hw
            side = torch.full_like(d["dA"], float("nan"))
            if vg_on:
                x = d["dA"]
                vg = H.BnVgrad(d["y"].data_ptr(), d["vsc"].data_ptr(), d["vsh"].data_ptr(),
                               d["coef"].data_ptr(), relu, side.data_ptr())
                keep.append(vg)
                vgp = H.ctypes.pointer(vg)
            else:
                H.check(L.hgk_bn_bwd_apply(st, H.BF16, d["dA"].data_ptr(), d["y"].data_ptr(), M, C,
                                           d["vsc"].data_ptr(), d["vsh"].data_ptr(), relu,
                                           d["coef"].data_ptr(), None, side.data_ptr(), 0))
                x, vgp = side, None
            out = torch.empty(N, hw, hw, C, device=DEV, dtype=torch.bfloat16)
            part = torch.zeros(L.hgk_max_stats_rows() * 2 * C, device=DEV)
            rc = H.ctypes.c_int(0)
            keep.append(rc)
            if len(hws) == 1:
                if vg_on:
                    H.check(L.hgk_conv_fwd_bnbwd_vg(st, H.BF16, x.data_ptr(), wp.data_ptr(), ld, None,
                                                    out.data_ptr(), N, hw, hw, C, C, 3, 3, 1, 1, 1, None,
                                                    0, d["bny"].data_ptr(), d["bsc"].data_ptr(),
                                                    d["bsh"].data_ptr(), 1, d["bmu"].data_ptr(),
                                                    d["bis"].data_ptr(), part.data_ptr(),
                                                    H.ctypes.byref(rc), vgp))
                else:
                    H.check(L.hgk_conv_fwd_bnbwd(st, H.BF16, x.data_ptr(), wp.data_ptr(), ld, None,
                                                 out.data_ptr(), N, hw, hw, C, C, 3, 3, 1, 1, 1, None, 0,
                                                 d["bny"].data_ptr(), d["bsc"].data_ptr(),
                                                 d["bsh"].data_ptr(), 1, d["bmu"].data_ptr(),
                                                 d["bis"].data_ptr(), part.data_ptr(), H.ctypes.byref(rc)))
            segs.append(H.ConvSeg(x.data_ptr(), None, out.data_ptr(), None, None, None, None, N, hw, hw,
                                  d["bny"].data_ptr(), d["bsc"].data_ptr(), d["bsh"].data_ptr(),
                                  d["bmu"].data_ptr(), d["bis"].data_ptr(), part.data_ptr(), 1,
                                  H.ctypes.pointer(rc), vgp))
            res.append((side, out, part, rc))
        if len(hws) == 2:
            arr = (H.ConvSeg * 2)(*segs)
            H.check(L.hgk_conv_fwd_twin(st, H.BF16, wp.data_ptr(), ld, None, 0, 0, C, C, 3, 3, 1, 1, 1,
                                        arr, None, 0))
        torch.cuda.synchronize()
        return [(s_, o, p[: rc.value * 2 * C].clone(), rc.value) for s_, o, p, rc in res]

    ref, got = run(False), run(True)
    for (s0, o0, p0, r0), (s1, o1, p1, r1) in zip(ref, got):
        assert r1 == r0 > 0
        assert torch.equal(s1.view(torch.int16), s0.view(torch.int16))
        assert torch.equal(o1.view(torch.int16), o0.view(torch.int16))
        assert torch.equal(p1, p0)


def test_vg_refuses_unsupported_route():
    """a folded apply on a shape no kernel stages must fail loudly, launching nothing"""
    L = H.load_library()
    g = torch.Generator(device=DEV).manual_seed(5)
    N, hw, K, Cout = 2, 8, 256, 128  # small M, 256-channel input: neither ring nor image tiles
    d = _operands(g, N, hw, K, Cout)
    wp, ld = _packed_dgrad(L, g, K, Cout)
    out = torch.zeros(N, hw, hw, Cout, device=DEV, dtype=torch.bfloat16)
    part = torch.zeros(L.hgk_max_stats_rows() * 2 * Cout, device=DEV)
    side = torch.zeros_like(d["dA"])
    vg = H.BnVgrad(d["y"].data_ptr(), d["vsc"].data_ptr(), d["vsh"].data_ptr(), d["coef"].data_ptr(),
                   1, side.data_ptr())
    rc = L.hgk_conv_fwd_bnbwd_vg(H.stream_handle(), H.BF16, d["dA"].data_ptr(), wp.data_ptr(), ld, None,
                                 out.data_ptr(), N, hw, hw, K, Cout, 1, 1, 1, 0, 1, None, 0,
                                 d["bny"].data_ptr(), d["bsc"].data_ptr(), d["bsh"].data_ptr(), 1,
                                 d["bmu"].data_ptr(), d["bis"].data_ptr(), part.data_ptr(), None,
                                 H.ctypes.byref(vg))
    assert rc == -2
    torch.cuda.synchronize()
    assert int(out.view(torch.int16).abs().sum()) == 0


@pytest.mark.parametrize("use_graph", [False, True])
def test_engine_fold_apply_bitwise_whole_model(routes, use_graph):
    """2-stack hourglass, 256x256, N=32, bf16 (single and twin 64x64 blocks take the fold): a
    training step with HGK_FOLD_APPLY=1 gives bit-identical heatmaps, loss, parameter gradients
    and BN running statistics to HGK_FOLD_APPLY=0 (separate apply passes), and folds happened."""
    import progressive_process_for_human_pose_estimation_amd as P
    from progressive_process_for_human_pose_estimation_amd import engine
    from progressive_process_for_human_pose_estimation_amd.data import gaussian_targets, synthetic_images
    from progressive_process_for_human_pose_estimation_amd.trainer import Trainer

    x = synthetic_images(32, 256, 256, seed=1234).cuda()
    t = gaussian_targets(32, 17, 64, 64, seed=1)[0].cuda()

    def run(fold):
        routes(fold_apply="1" if fold else "0")
        torch.manual_seed(0)
        m = P.creatModel(nStack=2).cuda()
        before = engine.STATS["folded"]
        if use_graph:
            tr = Trainer(m, lr=1e-4, dtype=torch.bfloat16, use_graph=True)
            loss = tr.step(x, t)
            loss = tr.step(x, t)  # replay
            torch.cuda.synchronize()
            grads = tr.fp.grad.detach().clone()
            params = tr.fp.flat.detach().clone()
            out = None
        else:
            m.set_engine_dtype(torch.bfloat16)
            outs = m(x)
            loss = sum(torch.nn.functional.mse_loss(o, t) for o in outs)
            loss.backward()
            torch.cuda.synchronize()
            grads = torch.cat([p.grad.reshape(-1) for p in m.parameters() if p.grad is not None])
            params = None
            out = torch.cat([o.reshape(-1) for o in outs])
        bufs = torch.cat([b.detach().double().reshape(-1) for b in m.buffers()])
        return engine.STATS["folded"] - before, float(loss.detach()), grads, params, out, bufs

    f1, l1, g1, p1, o1, b1 = run(True)
    f0, l0, g0, p0, o0, b0 = run(False)
    assert f1 > 0 and f0 == 0, (f1, f0)
    assert l1 == l0
    assert torch.equal(g1, g0)
    assert torch.equal(b1, b0)
    if use_graph:
        assert torch.equal(p1, p0)
    else:
        assert torch.equal(o1, o0)


def _bnb_fin_operands(g, N, hw, C, rows):
    """a BN-backward's inputs for a folded finalize: partial rows [rows][2][C] (sum g, sum g xhat),
    forward stat [4][C] = mean | invstd | scale | shift"""
    return dict(part=torch.randn(rows, 2, C, device=DEV, generator=g) * 20,
                stat=torch.stack([torch.randn(C, device=DEV, generator=g) * 0.1,
                                  torch.rand(C, device=DEV, generator=g) + 0.5,
                                  torch.rand(C, device=DEV, generator=g) + 0.5,
                                  torch.randn(C, device=DEV, generator=g) * 0.3]).contiguous())


@pytest.mark.parametrize("training", [1, 0], ids=["train", "eval"])
@pytest.mark.parametrize("relu", [1, 0], ids=["relu", "norelu"])
@pytest.mark.parametrize("case", ["3x3_8", "3x3_4", "3x3_twin", "1x1_8", "1x1_twin", "1x1c256add_8",
                                  "1x1c256add_twin"])
def test_img_vg_fin_bitwise(case, relu, training):
    """the small-level input gradients with the BN-backward FINALIZE and apply folded in
    (image-tile kernel, hgk_bn_vgrad.partial; try_with_torch.py:186-192): the applied gradient,
    dA, the producer BN's partials AND dgamma / dbeta (accumulated onto non-zero values; a twin
    adds segment 0 then segment 1) BITWISE those of hgk_bn_bwd_finalize_apply / hgk_bn_bwd_twin
    followed by the unfolded launch"""
    L = H.load_library()
    g = torch.Generator(device=DEV).manual_seed(17)
    ks = 3 if case.startswith("3x3") else 1
    hws = (8, 4) if case.endswith("twin") else (4,) if case.endswith("_4") else (8,)
    add = "add" in case  # bn1: the skip gradient added (hgk_bn_vgrad.add)
    N = 32
    C = 256 if add else 128
    Cout = 128 if (ks == 3 or add) else 256
    if ks == 3:
        wp, ld = _packed_dgrad3(L, g, C)
    else:
        wp, ld = _packed_dgrad(L, g, C, Cout)
    st = H.stream_handle()
    ops = []
    for hw in hws:
        d = _operands(g, N, hw, C, Cout)
        d.update(_bnb_fin_operands(g, N, hw, C, N * hw * hw // 64))
        d["add"] = (torch.randn(N, hw, hw, C, device=DEV, generator=g) * 0.3).to(torch.bfloat16) if add else None
        ops.append(d)
    dg0 = torch.randn(C, device=DEV, generator=g)
    db0 = torch.randn(C, device=DEV, generator=g)
    pad = 1 if ks == 3 else 0
    fam = L.hgk_conv_fwd_kernel_family(H.BF16, N, hws[0], hws[0], N if len(hws) > 1 else 0,
                                       hws[-1] if len(hws) > 1 else 0, hws[-1] if len(hws) > 1 else 0,
                                       C, Cout, ks, ks, 1, pad, 1)
    assert H.KFAM[fam] == "img"

    def run(fold):
        dgamma, dbeta = dg0.clone(), db0.clone()
        keep, segs, res, bsegs = [], [], [], []
        for hw, d in zip(hws, ops):
            M = N * hw * hw
            rows = d["part"].shape[0]
            side = torch.full_like(d["dA"], float("nan"))
            mean, invstd, sc, sh = d["stat"]
            if fold:
                x = d["dA"]
                vg = H.BnVgrad(d["y"].data_ptr(), sc.data_ptr(), sh.data_ptr(), None, relu,
                               side.data_ptr(), d["part"].data_ptr(), rows, M, mean.data_ptr(),
                               invstd.data_ptr(), training, dgamma.data_ptr(), dbeta.data_ptr(),
                               None if d["add"] is None else d["add"].data_ptr())
                keep.append(vg)
                vgp = H.ctypes.pointer(vg)
            else:
                bsegs.append(H.BnbSeg(d["part"].data_ptr(), rows, M, d["stat"].data_ptr(),
                                      d["dA"].data_ptr(), d["y"].data_ptr(),
                                      None if d["add"] is None else d["add"].data_ptr(),
                                      side.data_ptr(), 0))
                x, vgp = side, None
            out = torch.empty(N, hw, hw, Cout, device=DEV, dtype=torch.bfloat16)
            part = torch.zeros(L.hgk_max_stats_rows() * 2 * Cout, device=DEV)
            rc = H.ctypes.c_int(0)
            keep.append(rc)
            segs.append((x, vgp, out, part, rc, hw, d))
            res.append((side, out, part, rc))
        if not fold:
            arr = (H.BnbSeg * len(bsegs))(*bsegs)
            H.check(L.hgk_bn_bwd_twin(st, H.BF16, arr, len(bsegs), C, relu, training,
                                      dgamma.data_ptr(), dbeta.data_ptr(), None))
        cs = [H.ConvSeg(x.data_ptr(), None, out.data_ptr(), None, None, None, None, N, hw, hw,
                        d["bny"].data_ptr(), d["bsc"].data_ptr(), d["bsh"].data_ptr(),
                        d["bmu"].data_ptr(), d["bis"].data_ptr(), part.data_ptr(), 1,
                        H.ctypes.pointer(rc), vgp) for x, vgp, out, part, rc, hw, d in segs]
        if len(hws) == 2:
            arr = (H.ConvSeg * 2)(*cs)
            H.check(L.hgk_conv_fwd_twin(st, H.BF16, wp.data_ptr(), ld, None, 0, 0, C, Cout, ks, ks, 1,
                                        pad, 1, arr, None, 0))
        else:
            x, vgp, out, part, rc, hw, d = segs[0]
            args = (st, H.BF16, x.data_ptr(), wp.data_ptr(), ld, None, out.data_ptr(), N, hw, hw, C,
                    Cout, ks, ks, 1, pad, 1, None, 0, d["bny"].data_ptr(), d["bsc"].data_ptr(),
                    d["bsh"].data_ptr(), 1, d["bmu"].data_ptr(), d["bis"].data_ptr(), part.data_ptr(),
                    H.ctypes.byref(rc))
            if fold:
                H.check(L.hgk_conv_fwd_bnbwd_vg(*args, vgp))
            else:
                H.check(L.hgk_conv_fwd_bnbwd(*args))
        torch.cuda.synchronize()
        return [(s_, o, p[: rc.value * 2 * Cout].clone(), rc.value) for s_, o, p, rc in res], dgamma, dbeta

    (ref, g0, b0), (got, g1, b1) = run(False), run(True)
    assert torch.equal(g1, g0) and torch.equal(b1, b0)
    assert not torch.equal(g1, dg0)
    for (s0, o0, p0, r0), (s1, o1, p1, r1) in zip(ref, got):
        assert r1 == r0 > 0
        assert torch.equal(s1.view(torch.int16), s0.view(torch.int16))
        assert torch.equal(o1.view(torch.int16), o0.view(torch.int16))
        assert torch.equal(p1, p0)


@pytest.mark.parametrize("add", [False, True], ids=["default", "with_bn1_add"])
@pytest.mark.parametrize("use_graph", [False, True])
def test_engine_fold_bwd_fin_bitwise_whole_model(routes, use_graph, add):
    """4-stack hourglass, 256x256, N=32, bf16: with the small-level BN-backward finalize+apply
    folded into the image-tile input gradients (fold_bwd_fin) a training step is bit-identical
    (heatmaps, loss, gradients, BN running statistics) to the separate fused finalize+apply
    launches, and folds happened"""
    import progressive_process_for_human_pose_estimation_amd as P
    from progressive_process_for_human_pose_estimation_amd import engine
    from progressive_process_for_human_pose_estimation_amd.data import gaussian_targets, synthetic_images
    from progressive_process_for_human_pose_estimation_amd.trainer import Trainer

    x = synthetic_images(32, 256, 256, seed=4321).cuda()
    t = gaussian_targets(32, 17, 64, 64, seed=2)[0].cuda()

    def run(fold):
        routes(fold_bwd_fin="1" if fold else "0", fold_bwd_add="1" if (fold and add) else "0")
        torch.manual_seed(0)
        m = P.creatModel(nStack=4).cuda()
        before = engine.STATS["fin_folded"]
        if use_graph:
            tr = Trainer(m, lr=1e-4, dtype=torch.bfloat16, use_graph=True)
            loss = tr.step(x, t)
            loss = tr.step(x, t)  # replay
            torch.cuda.synchronize()
            grads = tr.fp.grad.detach().clone()
            out = tr.fp.flat.detach().clone()
        else:
            m.set_engine_dtype(torch.bfloat16)
            outs = m(x)
            loss = sum(torch.nn.functional.mse_loss(o, t) for o in outs)
            loss.backward()
            torch.cuda.synchronize()
            grads = torch.cat([p.grad.reshape(-1) for p in m.parameters() if p.grad is not None])
            out = torch.cat([o.reshape(-1) for o in outs])
        bufs = torch.cat([b.detach().double().reshape(-1) for b in m.buffers()])
        return engine.STATS["fin_folded"] - before, float(loss.detach()), grads, out, bufs

    f1, l1, g1, o1, b1 = run(True)
    f0, l0, g0, o0, b0 = run(False)
    assert f1 > 0 and f0 == 0, (f1, f0)
    assert l1 == l0
    assert torch.equal(g1, g0)
    assert torch.equal(o1, o0)
    assert torch.equal(b1, b0)
