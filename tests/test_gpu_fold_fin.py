"""Folded BN finalize (hgk_conv_fwd_fold, hgk_conv_seg.fold; engine BNUse.pending): at the 8x8 /
4x4 levels the conv consuming relu(bn(x)) computes the BN's scale / shift from the producer's
statistics partials itself (every workgroup; the first one publishes stat and the running-stats
record) instead of a hgk_bn_finalize_deferred launch. Against finalize + conv: the statistics
agree to fp64 rounding (two-pass sum vs Chan tree), the outputs to within one bf16 rounding.
"""
import pytest
import torch

from progressive_process_for_human_pose_estimation_amd import hgk as H

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _pack(L, w, dt, tdt):
    cout, cin, k, _ = w.shape
    ld = L.hgk_conv_w_ld(k * k * cin)
    wp = torch.empty(((cout + 127) // 128) * 128, ld, device=DEV, dtype=tdt)
    H.check(L.hgk_pack_conv_weight(H.stream_handle(), dt, w.data_ptr(), wp.data_ptr(), ld, cout, cin,
                                   k, k, 0, cout, cin))
    return wp, ld


def _producer(L, g, N, hw, C):
    """a BN input with realistic channel-major statistics partials: the output of a 1x1 conv"""
    x = (torch.randn(N, hw, hw, 256, device=DEV, generator=g)).to(torch.bfloat16)
    w = torch.randn(C, 256, 1, 1, device=DEV, generator=g) * 0.06
    # (a 64-channel producer at N=8, 8x8: 8 partial rows)
    wp, ld = _pack(L, w, H.BF16, torch.bfloat16)
    b = torch.randn(C, device=DEV, generator=g) * 0.5 + 0.3
    y = torch.empty(N, hw, hw, C, device=DEV, dtype=torch.bfloat16)
    part = torch.zeros(L.hgk_max_stats_rows() * 3 * C, device=DEV)
    rows = H.ctypes.c_int(0)
    ws = torch.zeros(64 << 20, dtype=torch.uint8, device=DEV)
    H.check(L.hgk_conv_fwd(H.stream_handle(), H.BF16, x.data_ptr(), wp.data_ptr(), ld, b.data_ptr(),
                           None, y.data_ptr(), None, None, 0, 0, part.data_ptr(), H.ctypes.byref(rows),
                           N, hw, hw, 256, C, 1, 1, 1, 0, 1, ws.data_ptr(), ws.numel()))
    return y, part, rows.value


CASES = [  # N, hw, Cin (BN channels), Cout, k
    (32, 8, 128, 128, 3),   # conv2 @8x8: split-K all-ahead
    (32, 4, 128, 128, 3),   # conv2 @4x4
    (32, 8, 128, 256, 1),   # conv3 @8x8
    (32, 4, 256, 128, 1),   # conv1 @4x4 (256 BN channels)
    (8, 8, 64, 64, 3),      # 64 BN channels (the stem block at a small input): idle threads clamp
]


@pytest.mark.parametrize("case", CASES)
def test_conv_fold_matches_finalize_then_conv(case):
    N, hw, C, Cout, k = case
    L = H.load_library()
    g = torch.Generator(device=DEV).manual_seed(17)
    x, part, rows = _producer(L, g, N, hw, C)
    assert rows <= 32 and rows % 4 == 0
    M = N * hw * hw
    assert L.hgk_conv_fold_ok(H.BF16, N, hw, hw, 0, 0, 0, C, Cout, k, k, 1, k // 2, 1, rows, 0) == 1
    gamma = torch.rand(C, device=DEV, generator=g) + 0.5
    beta = torch.randn(C, device=DEV, generator=g) * 0.2
    w = torch.randn(Cout, C, k, k, device=DEV, generator=g) * 0.05
    wp, ld = _pack(L, w, H.BF16, torch.bfloat16)
    bias = torch.randn(Cout, device=DEV, generator=g) * 0.1
    ws_b = L.hgk_conv_fwd_workspace(H.BF16, N, hw, hw, C, Cout, k, k, 1, k // 2, 1)
    st = H.stream_handle()

    def run(fold):
        stat = torch.full((4, C), float("nan"), device=DEV)
        rec = torch.full((2, C), float("nan"), device=DEV, dtype=torch.float64)
        y = torch.empty(N, hw, hw, Cout, device=DEV, dtype=torch.bfloat16)
        ostat = torch.zeros(L.hgk_max_stats_rows() * 3 * Cout, device=DEV)
        orows = H.ctypes.c_int(0)
        ws = torch.zeros(max(ws_b, 1 << 20), dtype=torch.uint8, device=DEV)
        if fold:
            fd = H.BnFold(part.data_ptr(), rows, M, gamma.data_ptr(), beta.data_ptr(), 1e-5,
                          stat.data_ptr(), rec.data_ptr())
            H.check(L.hgk_conv_fwd_fold(st, H.BF16, x.data_ptr(), wp.data_ptr(), ld, bias.data_ptr(),
                                        None, y.data_ptr(), 1, 0, ostat.data_ptr(), H.ctypes.byref(orows),
                                        N, hw, hw, C, Cout, k, k, 1, k // 2, 1, ws.data_ptr(), ws.numel(),
                                        H.ctypes.byref(fd)))
        else:
            arr = (H.BnSeg * 1)(H.BnSeg(part.data_ptr(), rows, M, rec.data_ptr(), stat.data_ptr()))
            H.check(L.hgk_bn_finalize_deferred(st, arr, 1, C, gamma.data_ptr(), beta.data_ptr(), 1e-5))
            H.check(L.hgk_conv_fwd(st, H.BF16, x.data_ptr(), wp.data_ptr(), ld, bias.data_ptr(), None,
                                   y.data_ptr(), stat[2].data_ptr(), stat[3].data_ptr(), 1, 0,
                                   ostat.data_ptr(), H.ctypes.byref(orows), N, hw, hw, C, Cout, k, k, 1,
                                   k // 2, 1, ws.data_ptr(), ws.numel()))
        torch.cuda.synchronize()
        return stat, rec, y.float(), ostat[: orows.value * 3 * Cout].clone(), orows.value

    s1, r1, y1, o1, n1 = run(True)
    s0, r0, y0, o0, n0 = run(False)
    assert torch.isfinite(s1).all() and torch.isfinite(r1).all()
    assert torch.allclose(r1, r0, rtol=1e-9, atol=1e-12), (r1 - r0).abs().max()
    assert torch.allclose(s1, s0, rtol=2e-6, atol=1e-7), (s1 - s0).abs().max()
    # outputs: the same conv on (at most 1-ulp) different BN constants -> within one bf16 rounding
    err = (y1 - y0).abs()
    assert float(err.max()) <= 2 ** -7 * float(y0.abs().max()), float(err.max())
    assert float(err.mean()) <= 1e-4 * float(y0.abs().mean())
    assert n1 == n0
    assert torch.allclose(o1, o0, rtol=1e-2, atol=1e-2 * float(o0.abs().max()))


def test_conv_fold_twin_and_refusals():
    L = H.load_library()
    g = torch.Generator(device=DEV).manual_seed(23)
    N, C, Cout = 32, 128, 128
    xs = [_producer(L, g, N, hw, C) for hw in (8, 4)]
    r0, r1 = xs[0][2], xs[1][2]
    assert L.hgk_conv_fold_ok(H.BF16, N, 8, 8, N, 4, 4, C, Cout, 3, 3, 1, 1, 1, r0, r1) == 1
    # refusals: 16x16 (128 partial rows), fp32, the 64x64 ring route
    assert L.hgk_conv_fold_ok(H.BF16, N, 16, 16, 0, 0, 0, C, Cout, 3, 3, 1, 1, 1, 128, 0) == 0
    assert L.hgk_conv_fold_ok(H.F32, N, 8, 8, 0, 0, 0, C, Cout, 3, 3, 1, 1, 1, r0, 0) == 0
    assert L.hgk_conv_fold_ok(H.BF16, N, 64, 64, 0, 0, 0, 256, 128, 1, 1, 1, 0, 1, 32, 0) == 0
    gamma = torch.rand(C, device=DEV, generator=g) + 0.5
    beta = torch.randn(C, device=DEV, generator=g) * 0.2
    w = torch.randn(Cout, C, 3, 3, device=DEV, generator=g) * 0.05
    wp, ld = _pack(L, w, H.BF16, torch.bfloat16)
    ws_b = L.hgk_conv_fwd_twin_workspace(H.BF16, N, 8, 8, N, 4, 4, C, Cout, 3, 3, 1, 1, 1)
    st = H.stream_handle()

    def run(fold):
        keep, segs, outs = [], [], []
        for (x, part, rows), hw in zip(xs, (8, 4)):
            M = N * hw * hw
            stat = torch.full((4, C), float("nan"), device=DEV)
            rec = torch.full((2, C), float("nan"), device=DEV, dtype=torch.float64)
            y = torch.empty(N, hw, hw, Cout, device=DEV, dtype=torch.bfloat16)
            ost = torch.zeros(L.hgk_max_stats_rows() * 3 * Cout, device=DEV)
            rc = H.ctypes.c_int(0)
            fp = None
            if fold:
                fd = H.BnFold(part.data_ptr(), rows, M, gamma.data_ptr(), beta.data_ptr(), 1e-5,
                              stat.data_ptr(), rec.data_ptr())
                keep.append(fd)
                fp = H.ctypes.pointer(fd)
            else:
                arr = (H.BnSeg * 1)(H.BnSeg(part.data_ptr(), rows, M, rec.data_ptr(), stat.data_ptr()))
                H.check(L.hgk_bn_finalize_deferred(st, arr, 1, C, gamma.data_ptr(), beta.data_ptr(), 1e-5))
            keep += [stat, rec, y, ost, rc]
            segs.append(H.ConvSeg(x.data_ptr(), None, y.data_ptr(), None if fold else stat[2].data_ptr(),
                                  None if fold else stat[3].data_ptr(), ost.data_ptr(), H.ctypes.pointer(rc),
                                  N, hw, hw, None, None, None, None, None, None, 0, None, None, fp))
            outs.append((stat, rec, y))
        ws = torch.zeros(max(ws_b, 1 << 20), dtype=torch.uint8, device=DEV)
        arr = (H.ConvSeg * 2)(*segs)
        H.check(L.hgk_conv_fwd_twin(st, H.BF16, wp.data_ptr(), ld, None, 1, 0, C, Cout, 3, 3, 1, 1, 1,
                                    arr, ws.data_ptr(), ws.numel()))
        torch.cuda.synchronize()
        return [(s.clone(), r.clone(), y.float()) for s, r, y in outs]

    for (s1, r1, y1), (s0, r0_, y0) in zip(run(True), run(False)):
        assert torch.allclose(r1, r0_, rtol=1e-9, atol=1e-12)
        assert torch.allclose(s1, s0, rtol=2e-6, atol=1e-7)
        assert float((y1 - y0).abs().max()) <= 2 ** -7 * float(y0.abs().max())


def test_engine_fold_fin_whole_model(monkeypatch, routes):
    """2-stack hourglass, 256x256, N=32, bf16 Trainer step (hipGraph): HGK_FOLD_FIN=1 folds the
    small-level finalizes (counted) and trains like HGK_FOLD_FIN=0 — loss, BN running statistics
    and parameter gradients agree to the bf16 engine's own rounding noise."""
    import progressive_process_for_human_pose_estimation_amd as P
    from progressive_process_for_human_pose_estimation_amd import engine
    from progressive_process_for_human_pose_estimation_amd.data import gaussian_targets, synthetic_images
    from progressive_process_for_human_pose_estimation_amd.trainer import Trainer

    x = synthetic_images(32, 256, 256, seed=1234).cuda()
    t = gaussian_targets(32, 17, 64, 64, seed=1)[0].cuda()
    counted = []
    orig = engine.Ctx.finish_forward

    def spy(self):
        counted.append(self.n_fin_folded)
        return orig(self)

    monkeypatch.setattr(engine.Ctx, "finish_forward", spy)

    def run(fold):
        routes(fold_fin="1" if fold else "0")
        counted.clear()
        torch.manual_seed(0)
        m = P.creatModel(nStack=2).cuda()
        tr = Trainer(m, lr=1e-4, dtype=torch.bfloat16, use_graph=True)
        loss = float(tr.step(x, t))
        torch.cuda.synchronize()
        grads = tr.fp.grad.detach().clone()
        bufs = torch.cat([b.detach().double().reshape(-1) for b in m.buffers()])
        return max(counted), loss, grads, bufs

    f1, l1, g1, b1 = run(True)
    f0, l0, g0, b0 = run(False)
    assert f1 > 0 and f0 == 0, (f1, f0)
    assert abs(l1 - l0) <= 1e-3 * abs(l0)
    cos = float(torch.nn.functional.cosine_similarity(g1, g0, dim=0))
    assert cos > 0.999, cos
    assert torch.allclose(b1, b0, rtol=1e-3, atol=1e-3)
