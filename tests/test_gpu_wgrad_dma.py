"""3x3 halo weight gradient with LDS-DMA staging (HGK_ROUTE_WG_DMA, hgk_conv.hip
conv3x3_wgrad_dma_kernel): the dy tile and the raw input halo go global -> LDS by DMA and the
BN+ReLU transform runs in place, with the register-staged kernel's tiles, splits, MFMA order and
epilogue — so dW and the bias gradient must be BITWISE those of the register-staged route, with
and without the fused BN+ReLU input, into fresh and accumulated slabs; and both match a float64
torch reference on the same bf16 operands (try_with_torch.py:189, conv2's weight gradient)."""
import pytest
import torch

from progressive_process_for_human_pose_estimation_amd import hgk as H

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _operands(cin, cout, n, hw, g):
    x = (torch.randn(n, hw, hw, cin, device=DEV, generator=g) * 0.7).to(torch.bfloat16)
    dy = (torch.randn(n, hw, hw, cout, device=DEV, generator=g) * 0.1).to(torch.bfloat16)
    sc = torch.rand(cin, device=DEV, generator=g) + 0.5
    sh = torch.randn(cin, device=DEV, generator=g) * 0.3
    return x, dy, sc, sh


def _run(L, ops, cin, cout, n, hw, bn, dma, twice):
    x, dy, sc, sh = ops
    st = H.stream_handle()
    cap = 256
    slab = torch.full((L.hgk_conv_wgrad_slab_bytes(cin, cout, 3, 3, cap) // 4,), float("nan"), device=DEV)
    dw = torch.zeros(cout, cin, 3, 3, device=DEV)
    db = torch.zeros(cout, device=DEV)
    splits = H.ctypes.c_int(0)
    prev = H.set_route("wg_dma", 1 if dma else 0)
    try:
        init = 0
        for _ in range(2 if twice else 1):
            H.check(L.hgk_conv_wgrad_accum(st, H.BF16, x.data_ptr(), dy.data_ptr(),
                                           sc.data_ptr() if bn else None, sh.data_ptr() if bn else None,
                                           1, slab.data_ptr(), cap, init, 1, H.ctypes.byref(splits), n, hw,
                                           hw, cin, cout, 3, 3, 1, 1, 1))
            init = splits.value
    finally:
        H.set_route("wg_dma", prev)
    H.check(L.hgk_conv_wgrad_finish(st, slab.data_ptr(), cap, splits.value, dw.data_ptr(), db.data_ptr(),
                                    cin, cout, 3, 3, cin, cout))
    torch.cuda.synchronize()
    return dw, db


@pytest.mark.parametrize("cin,cout,n,hw", [(128, 128, 32, 64), (128, 128, 32, 32), (128, 128, 2, 16),
                                           (64, 64, 4, 128), (256, 128, 3, 32)])
@pytest.mark.parametrize("bn", [True, False])
@pytest.mark.parametrize("twice", [False, True])
def test_wgrad_dma_bitwise_register_staged(cin, cout, n, hw, bn, twice):
    L = H.load_library()
    g = torch.Generator(device=DEV).manual_seed(cin + 7 * hw + n + bn)
    ops = _operands(cin, cout, n, hw, g)
    dw0, db0 = _run(L, ops, cin, cout, n, hw, bn, False, twice)
    dw1, db1 = _run(L, ops, cin, cout, n, hw, bn, True, twice)
    assert torch.isfinite(dw1).all()
    assert torch.equal(dw0, dw1)
    assert torch.equal(db0, db1)


@pytest.mark.parametrize("bn", [True, False])
def test_wgrad_dma_vs_float64_reference(bn):
    L = H.load_library()
    cin = cout = 128
    n, hw = 4, 32
    g = torch.Generator(device=DEV).manual_seed(5 + bn)
    x, dy, sc, sh = ops = _operands(cin, cout, n, hw, g)
    dw, db = _run(L, ops, cin, cout, n, hw, bn, True, False)
    a = torch.relu(x.float() * sc + sh).to(torch.bfloat16) if bn else x
    a = a.double().permute(0, 3, 1, 2)
    d = dy.double().permute(0, 3, 1, 2)
    ref = torch.nn.grad.conv2d_weight(a, (cout, cin, 3, 3), d, padding=1)
    err = (dw.double() - ref).abs().max().item()
    assert err <= 1e-4 * ref.abs().max().item() + 1e-5, err
    assert torch.allclose(db.double(), d.sum((0, 2, 3)), rtol=1e-4, atol=1e-4)
