"""The LDS-DMA ring weight gradient of the big multi-use 1x1 weights (route wg_ring,
csrc/hgk_wgrad_ring.hip): dW = sum over uses of dy^T x' and db = sum dy (try_with_torch.py:186,192:
ResidualBlock conv1 256->128 / conv3 128->256; :248,295 lin / ll_ 256->256), x' = relu?(BN(x)) of
each use rounded to bf16 as the kernels store it. Against a torch fp32 reference of the same bf16
operands and against the tiled multi-use kernel (route off): another fp32 summation order and split
plan, so within fp32 re-association, not bitwise. Also: accumulation into earlier slabs
(slabs_init), uses that do not fit (a use whose pixels are not a multiple of 32, small totals)
falling back to the tiled kernel bit for bit, and a whole training step on the route."""
import pytest
import torch

from progressive_process_for_human_pose_estimation_amd import hgk as H

pytestmark = pytest.mark.gpu
DEV = "cuda"

# uses of one weight: (N, H, W, BN transform?, ReLU?) — the hourglass levels' mix
USES = [(32, 64, 64, True, True), (32, 32, 32, True, True), (32, 16, 16, False, False),
        (32, 4, 4, True, False), (8, 32, 32, True, True), (32, 32, 32, True, True)]


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
    dw = torch.zeros(Cout, Cin, device=DEV, dtype=torch.float64)
    db = torch.zeros(Cout, device=DEV, dtype=torch.float64)
    for u in uses:
        x = u["x"].float().reshape(-1, Cin)
        if u["sc"] is not None:
            # fmaf(x, sc, sh) as the kernels: the fp32 product is exact in fp64, one rounding
            x = (x.double() * u["sc"].double() + u["sh"].double()).float()
            if u["relu"]:
                x = torch.relu(x)
            x = x.to(torch.bfloat16).float()
        dy = u["dy"].float().reshape(-1, Cout)
        dw += dy.double().t() @ x.double()
        db += dy.double().sum(0)
    return dw, db


def _run(uses, Cin, Cout, ring, slab=None, init=0):
    L = H.load_library()
    st = H.stream_handle()
    cap = L.hgk_conv_wgrad_max_splits()
    if slab is None:
        slab = torch.full((L.hgk_conv_wgrad_slab_bytes(Cin, Cout, 1, 1, cap) // 4,), float("nan"), device=DEV)
    srcs = [H.WgradSrc(u["x"].data_ptr(), u["dy"].data_ptr(),
                       u["sc"].data_ptr() if u["sc"] is not None else None,
                       u["sh"].data_ptr() if u["sh"] is not None else None,
                       1 if u["relu"] else 0, u["N"], u["H"], u["W"]) for u in uses]
    sp = H.ctypes.c_int(0)
    with H.route(wg_ring=ring):
        H.check(L.hgk_conv_wgrad_accum_multi(st, H.BF16, (H.WgradSrc * len(srcs))(*srcs), len(srcs),
                                             slab.data_ptr(), cap, init, 1, H.ctypes.byref(sp), Cin,
                                             Cout, 1, 1, 1, 0, 1))
    dw = torch.zeros(Cout, Cin, 1, 1, device=DEV)
    db = torch.zeros(Cout, device=DEV)
    H.check(L.hgk_conv_wgrad_finish(st, slab.data_ptr(), cap, sp.value, dw.data_ptr(), db.data_ptr(),
                                    Cin, Cout, 1, 1, Cin, Cout))
    torch.cuda.synchronize()
    return dw.reshape(Cout, Cin), db, sp.value, slab


def _close(a, ref, rel=2e-5):
    err = float((a.double() - ref).abs().max())
    scale = float(ref.abs().max())
    assert err <= rel * scale, (err, scale)
    return err / scale


@pytest.mark.parametrize("Cout,Cin", [(128, 256), (256, 128), (256, 256)])
def test_wgrad_ring_matches_fp32_reference_and_tiled_route(Cout, Cin):
    g = torch.Generator(device=DEV).manual_seed(Cout * 3 + Cin)
    uses = _uses(g, Cin, Cout, USES)
    ref_w, ref_b = _ref(uses, Cin, Cout)
    dw, db, S, _ = _run(uses, Cin, Cout, ring=1)
    assert 0 < S <= 256
    e_w = _close(dw, ref_w)
    e_b = _close(db, ref_b)
    dw0, db0, _, _ = _run(uses, Cin, Cout, ring=0)
    _close(dw0, ref_w)
    # the two routes: both within fp32 re-association of the exact sum
    assert float((dw - dw0).abs().max()) <= 4e-5 * float(ref_w.abs().max())
    assert float((db - db0).abs().max()) <= 4e-5 * float(ref_b.abs().max())
    # deterministic: a second run is bitwise the first
    dw2, db2, _, _ = _run(uses, Cin, Cout, ring=1)
    assert torch.equal(dw, dw2) and torch.equal(db, db2)
    print(f"{Cout}x{Cin}: {S} splits, rel err dW {e_w:.2e} db {e_b:.2e}")


def test_wgrad_ring_accumulates_into_earlier_slabs():
    """two calls, the second with slabs_init = the first's splits: the reduced gradient is that of
    every use of both calls (the engine's slab protocol for > 40 uses / several flushes)"""
    Cout, Cin = 128, 256
    g = torch.Generator(device=DEV).manual_seed(3)
    a, b = _uses(g, Cin, Cout, USES[:3]), _uses(g, Cin, Cout, USES[3:])
    ref_w, ref_b = _ref(a + b, Cin, Cout)
    _, _, S1, slab = _run(a, Cin, Cout, ring=1)
    dw, db, S2, _ = _run(b, Cin, Cout, ring=1, slab=slab, init=S1)
    assert S2 >= S1
    _close(dw, ref_w)
    _close(db, ref_b)


def test_wgrad_ring_falls_back_bitwise_when_a_use_does_not_fit():
    """a use of 4x4 pixels at N = 1 (16 pixels: not whole 32-pixel blocks) sends the whole call to
    the tiled kernel: bitwise the route-off result"""
    Cout, Cin = 128, 256
    g = torch.Generator(device=DEV).manual_seed(4)
    uses = _uses(g, Cin, Cout, USES[:2] + [(1, 4, 4, True, True)])
    dw1, db1, _, _ = _run(uses, Cin, Cout, ring=1)
    dw0, db0, _, _ = _run(uses, Cin, Cout, ring=0)
    assert torch.equal(dw1, dw0) and torch.equal(db1, db0)


def test_wgrad_ring_training_step_close_to_tiled_route():
    """a bf16 Trainer step of the 4-stack model at 256x256, N = 4 on the ring route vs off: the
    same loss (the forward does not see the route) and weight gradients within bf16-step noise"""
    import progressive_process_for_human_pose_estimation_amd as P
    from progressive_process_for_human_pose_estimation_amd.data import gaussian_targets, synthetic_images
    from progressive_process_for_human_pose_estimation_amd.trainer import Trainer
    x = synthetic_images(4, 256, 256, seed=41).to(DEV)
    t = gaussian_targets(4, 17, 64, seed=42)[0].to(DEV)
    res = []
    for ring in (1, 0):
        with H.route(wg_ring=ring):
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
