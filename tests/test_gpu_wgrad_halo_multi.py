"""Multi-use 3x3 halo weight gradient (route wg_halo_multi, hgk_conv.hip
conv3x3_wgrad_halo_multi_kernel): the uses of one bf16 3x3 weight (ResidualBlock conv2,
try_with_torch.py:189, used at every hourglass level and by every stack) whose tiles the halo kernel
covers go to ONE launch whose splits run over the uses' concatenated 8x16-pixel tiles — a split
may end inside one use and continue in the next, switching its BN scale / shift — and every slab
element is read-modified-written once per launch instead of once per use. Checked against a float64
torch reference on the same bf16 operands (dW = sum over uses of conv2d_weight(relu?(BN(x)), dy),
db = sum dy), against the route-off path (one halo launch per big use + the implicit-GEMM multi
launch: another split plan, so fp32 re-association, not bitwise), bitwise against the single-use
halo kernel for one use (the same plan), with accumulation into earlier slabs, and with uses the
halo kernel does not tile (8x8) going to the implicit GEMM inside the same call."""
import pytest
import torch

from progressive_process_for_human_pose_estimation_amd import hgk as H

pytestmark = pytest.mark.gpu
DEV = "cuda"

# uses of one weight: (N, H, W, BN transform?, ReLU?) — conv2's levels in the 4-stack model
USES = [(32, 64, 64, True, True), (32, 32, 32, True, True), (32, 16, 16, True, True),
        (8, 32, 32, False, False), (32, 64, 64, True, False), (3, 16, 16, True, True)]


def _uses(g, Cin, Cout, uses):
    out = []
    for N, Hh, W, pre, relu in uses:
        x = (torch.randn(N, Hh, W, Cin, device=DEV, generator=g) * 0.7 + 0.1).to(torch.bfloat16)
        dy = (torch.randn(N, Hh, W, Cout, device=DEV, generator=g) * 0.05).to(torch.bfloat16)
        sc = (torch.rand(Cin, device=DEV, generator=g) + 0.5) if pre else None
        sh = (torch.randn(Cin, device=DEV, generator=g) * 0.2) if pre else None
        out.append(dict(x=x, dy=dy, sc=sc, sh=sh, relu=relu, N=N, H=Hh, W=W))
    return out


def _ref(uses, Cin, Cout):
    dw = torch.zeros(Cout, Cin, 3, 3, device=DEV, dtype=torch.float64)
    db = torch.zeros(Cout, device=DEV, dtype=torch.float64)
    for u in uses:
        x = u["x"].float()
        if u["sc"] is not None:
            # fmaf(x, sc, sh) as the kernels: the fp32 product is exact in fp64, one rounding
            x = (x.double() * u["sc"].double() + u["sh"].double()).float()
            if u["relu"]:
                x = torch.relu(x)
            x = x.to(torch.bfloat16).float()
        a = x.double().permute(0, 3, 1, 2)
        d = u["dy"].double().permute(0, 3, 1, 2)
        dw += torch.nn.grad.conv2d_weight(a, (Cout, Cin, 3, 3), d, padding=1)
        db += d.sum((0, 2, 3))
    return dw, db


def _run(uses, Cin, Cout, multi, slab=None, init=0, single=False):
    L = H.load_library()
    st = H.stream_handle()
    cap = L.hgk_conv_wgrad_max_splits()
    if slab is None:
        slab = torch.full((L.hgk_conv_wgrad_slab_bytes(Cin, Cout, 3, 3, cap) // 4,), float("nan"), device=DEV)
    sp = H.ctypes.c_int(0)
    with H.route(wg_halo_multi=multi):
        if single:   # one hgk_conv_wgrad_accum per use (the engine's per-use calls)
            for u in uses:
                H.check(L.hgk_conv_wgrad_accum(
                    st, H.BF16, u["x"].data_ptr(), u["dy"].data_ptr(), H.ptr(u["sc"]), H.ptr(u["sh"]),
                    1 if u["relu"] else 0, slab.data_ptr(), cap, init, 1, H.ctypes.byref(sp),
                    u["N"], u["H"], u["W"], Cin, Cout, 3, 3, 1, 1, 1))
                init = max(init, sp.value)
            sp.value = init
        else:
            srcs = [H.WgradSrc(u["x"].data_ptr(), u["dy"].data_ptr(), H.ptr(u["sc"]), H.ptr(u["sh"]),
                               1 if u["relu"] else 0, u["N"], u["H"], u["W"]) for u in uses]
            H.check(L.hgk_conv_wgrad_accum_multi(st, H.BF16, (H.WgradSrc * len(srcs))(*srcs), len(srcs),
                                                 slab.data_ptr(), cap, init, 1, H.ctypes.byref(sp), Cin,
                                                 Cout, 3, 3, 1, 1, 1))
    dw = torch.zeros(Cout, Cin, 3, 3, device=DEV)
    db = torch.zeros(Cout, device=DEV)
    H.check(L.hgk_conv_wgrad_finish(st, slab.data_ptr(), cap, sp.value, dw.data_ptr(), db.data_ptr(),
                                    Cin, Cout, 3, 3, Cin, Cout))
    torch.cuda.synchronize()
    return dw, db, sp.value, slab


def _close(a, ref, rel=2e-5):
    err = float((a.double() - ref).abs().max())
    scale = float(ref.abs().max())
    assert err <= rel * scale, (err, scale)
    return err / scale


@pytest.mark.parametrize("Cin,Cout", [(128, 128), (64, 64), (256, 128)])
def test_wgrad_halo_multi_matches_fp64_reference_and_per_use_route(Cin, Cout):
    g = torch.Generator(device=DEV).manual_seed(Cout * 3 + Cin)
    uses = _uses(g, Cin, Cout, USES)
    ref_w, ref_b = _ref(uses, Cin, Cout)
    dw, db, S, _ = _run(uses, Cin, Cout, multi=128)
    assert 0 < S <= 256
    e_w = _close(dw, ref_w)
    e_b = _close(db, ref_b)
    dw0, db0, _, _ = _run(uses, Cin, Cout, multi=0, single=True)
    _close(dw0, ref_w)
    assert float((dw - dw0).abs().max()) <= 4e-5 * float(ref_w.abs().max())
    assert float((db - db0).abs().max()) <= 4e-5 * float(ref_b.abs().max())
    dw2, db2, _, _ = _run(uses, Cin, Cout, multi=128)
    assert torch.equal(dw, dw2) and torch.equal(db, db2)
    print(f"{Cout}x{Cin}x3x3: {S} splits, rel err dW {e_w:.2e} db {e_b:.2e}")


@pytest.mark.parametrize("bn", [True, False])
def test_wgrad_halo_multi_one_use_bitwise_the_single_use_kernel(bn):
    """one 64x64 use: the multi launch has the single-use halo kernel's split plan, so the same
    partial sums in the same order"""
    Cin = Cout = 128
    g = torch.Generator(device=DEV).manual_seed(11 + bn)
    uses = _uses(g, Cin, Cout, [(32, 64, 64, bn, bn)])
    dw1, db1, S1, _ = _run(uses, Cin, Cout, multi=128)
    dw0, db0, S0, _ = _run(uses, Cin, Cout, multi=0, single=True)
    assert S1 == S0
    assert torch.equal(dw1, dw0) and torch.equal(db1, db0)


def test_wgrad_halo_multi_accumulates_into_earlier_slabs_and_mixes_untiled_uses():
    """two calls (the second with slabs_init = the first's splits), the second holding 8x8 uses the
    halo kernel does not tile (W % 16 != 0): they take the implicit-GEMM multi launch into the same
    slabs; the reduced gradient is that of every use"""
    Cin = Cout = 128
    g = torch.Generator(device=DEV).manual_seed(3)
    a = _uses(g, Cin, Cout, USES[:3])
    b = _uses(g, Cin, Cout, [(32, 8, 8, True, True), (32, 32, 32, True, True), (32, 8, 8, False, False)])
    ref_w, ref_b = _ref(a + b, Cin, Cout)
    _, _, S1, slab = _run(a, Cin, Cout, multi=128)
    dw, db, S2, _ = _run(b, Cin, Cout, multi=128, slab=slab, init=S1)
    assert S2 >= S1
    _close(dw, ref_w)
    _close(db, ref_b)


def test_wgrad_halo_multi_below_threshold_is_the_route_off_path():
    """uses holding fewer tiles than the route value leave the call to the route-off path, bitwise"""
    Cin = Cout = 128
    g = torch.Generator(device=DEV).manual_seed(4)
    uses = _uses(g, Cin, Cout, [(2, 16, 16, True, True), (3, 16, 16, True, False)])   # 10 tiles
    dw1, db1, _, _ = _run(uses, Cin, Cout, multi=128)
    dw0, db0, _, _ = _run(uses, Cin, Cout, multi=0)
    assert torch.equal(dw1, dw0) and torch.equal(db1, db0)


def test_wgrad_halo_multi_training_step_close_to_per_use_route():
    """a bf16 Trainer step of the 4-stack model at 256x256, N = 4 on the route vs off (the engine
    defers every 3x3 use to the end of backward only with the route on): the same loss and weight
    gradients within fp32 re-association"""
    import progressive_process_for_human_pose_estimation_amd as P
    from progressive_process_for_human_pose_estimation_amd.data import gaussian_targets, synthetic_images
    from progressive_process_for_human_pose_estimation_amd.trainer import Trainer
    x = synthetic_images(4, 256, 256, seed=41).to(DEV)
    t = gaussian_targets(4, 17, 64, seed=42)[0].to(DEV)
    res = []
    for multi in (128, 0):
        with H.route(wg_halo_multi=multi):
            torch.manual_seed(0)
            m = P.creatModel(nStack=4).to(DEV)
            tr = Trainer(m, lr=1e-4, dtype=torch.bfloat16, use_graph=False)
            loss = float(tr.step(x, t))
            torch.cuda.synchronize()
            res.append((loss, tr.fp.grad.clone()))
    (l1, g1), (l0, g0) = res
    assert l1 == l0
    cos = float((g1.double() @ g0.double()) / (g1.double().norm() * g0.double().norm()))
    assert cos > 0.99999, cos


def test_wgrad_halo_multi_too_few_slabs_launches_nothing():
    """a slab capacity below the launch's split count is an argument error raised before any
    launch: the slabs are untouched"""
    L = H.load_library()
    st = H.stream_handle()
    Cin = Cout = 128
    g = torch.Generator(device=DEV).manual_seed(6)
    uses = _uses(g, Cin, Cout, USES[:3])
    cap = 8   # the launch plans 64 splits
    slab = torch.full((L.hgk_conv_wgrad_slab_bytes(Cin, Cout, 3, 3, cap) // 4,), 7.0, device=DEV)
    srcs = [H.WgradSrc(u["x"].data_ptr(), u["dy"].data_ptr(), H.ptr(u["sc"]), H.ptr(u["sh"]),
                       1 if u["relu"] else 0, u["N"], u["H"], u["W"]) for u in uses]
    sp = H.ctypes.c_int(-1)
    rc = L.hgk_conv_wgrad_accum_multi(st, H.BF16, (H.WgradSrc * len(srcs))(*srcs), len(srcs),
                                      slab.data_ptr(), cap, 0, 1, H.ctypes.byref(sp), Cin, Cout,
                                      3, 3, 1, 1, 1)
    torch.cuda.synchronize()
    assert rc != 0 and b"slab capacity" in L.hgk_last_error()
    assert sp.value == -1
    assert bool((slab == 7.0).all())
