"""Full-width 1x1 weight-gradient tiles (HGK_ROUTE_WG_FULL: the whole 128x256 / 256x128 weight in
one workgroup, so a use's dy and x rows are read once). The per-output-element summation order
(pixel splits, 64-pixel stages, MFMA k order) is the 128x128 tiling's, so the reduced weight
gradient must be BITWISE that of the default route (the bias: bitwise for 128 output channels,
another fixed staging order for 256); and both match a torch fp32 reference on the same bf16
operands. Multi-use launch (two sources of different sizes, BN+ReLU
applied to x on the way in) and the single-use entry point."""
import pytest
import torch

from progressive_process_for_human_pose_estimation_amd import hgk as H

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _sources(cin, cout, sizes, g):
    srcs = []
    for n, hw in sizes:
        x = (torch.randn(n, hw, hw, cin, device=DEV, generator=g) * 0.7).to(torch.bfloat16)
        dy = (torch.randn(n, hw, hw, cout, device=DEV, generator=g) * 0.1).to(torch.bfloat16)
        sc = torch.rand(cin, device=DEV, generator=g) + 0.5
        sh = torch.randn(cin, device=DEV, generator=g) * 0.3
        srcs.append((x, dy, sc, sh, n, hw))
    return srcs


def _run(L, cin, cout, srcs, multi, full):
    st = H.stream_handle()
    cap = 256
    slab = torch.zeros(L.hgk_conv_wgrad_slab_bytes(cin, cout, 1, 1, cap) // 4, device=DEV)
    dw = torch.zeros(cout, cin, 1, 1, device=DEV)
    db = torch.zeros(cout, device=DEV)
    splits = H.ctypes.c_int(0)
    prev = H.set_route("wg_full", 1 if full else 0)
    try:
        if multi:
            arr = (H.WgradSrc * len(srcs))(*[H.WgradSrc(x.data_ptr(), dy.data_ptr(), sc.data_ptr(),
                                                         sh.data_ptr(), 1, n, hw, hw)
                                             for x, dy, sc, sh, n, hw in srcs])
            H.check(L.hgk_conv_wgrad_accum_multi(st, 1, arr, len(srcs), slab.data_ptr(), cap, 0, 1,
                                                 H.ctypes.byref(splits), cin, cout, 1, 1, 1, 0, 1))
        else:
            x, dy, sc, sh, n, hw = srcs[0]
            H.check(L.hgk_conv_wgrad_accum(st, 1, x.data_ptr(), dy.data_ptr(), sc.data_ptr(),
                                           sh.data_ptr(), 1, slab.data_ptr(), cap, 0, 1,
                                           H.ctypes.byref(splits), n, hw, hw, cin, cout, 1, 1, 1, 0, 1))
    finally:
        H.set_route("wg_full", prev)
    H.check(L.hgk_conv_wgrad_finish(st, slab.data_ptr(), cap, splits.value, dw.data_ptr(),
                                    db.data_ptr(), cin, cout, 1, 1, cin, cout))
    torch.cuda.synchronize()
    return dw, db


def _reference(srcs, cin, cout):
    dw = torch.zeros(cout, cin, device=DEV, dtype=torch.float64)
    db = torch.zeros(cout, device=DEV, dtype=torch.float64)
    for x, dy, sc, sh, n, hw in srcs:
        a = torch.relu(x.float() * sc + sh).to(torch.bfloat16).double().reshape(-1, cin)
        d = dy.double().reshape(-1, cout)
        dw += d.t() @ a
        db += d.sum(0)
    return dw, db


@pytest.mark.parametrize("cin,cout", [(256, 128), (128, 256)])
@pytest.mark.parametrize("multi", [True, False])
def test_wgrad_full_tiles_bitwise_equal_default(cin, cout, multi):
    L = H.load_library()
    g = torch.Generator(device=DEV).manual_seed(11)
    # > 16384 pixels per launch: the default route's 128x128 tiles (smaller launches take 64x64
    # tiles, whose bias sums run in another order)
    sizes = [(4, 64), (5, 32)] if multi else [(5, 64)]
    srcs = _sources(cin, cout, sizes, g)
    dw0, db0 = _run(L, cin, cout, srcs, multi, False)
    dw1, db1 = _run(L, cin, cout, srcs, multi, True)
    assert torch.equal(dw0, dw1)
    if cout == 128:
        assert torch.equal(db0, db1)
    else:
        # 256-wide dy rows: the bias column sums are staged over 16 instead of 32 row slots
        # (wgrad_fast_body's RPP_D), another fixed order
        assert ((db0 - db1).abs().max() / db0.abs().max()) < 1e-6
    rw, rb = _reference(srcs, cin, cout)
    err = (dw1.double().reshape(cout, cin) - rw).abs().max() / rw.abs().max()
    # the kernel forms the BN transform with an FMA before the bf16 rounding, torch with a multiply
    # and an add: a few inputs round to the neighbouring bf16 (measured 5.8e-5 of max |dW|)
    assert err < 2e-4, float(err)
    assert (db1.double() - rb).abs().max() / rb.abs().max() < 1e-5
