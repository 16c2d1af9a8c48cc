"""3x3 halo launches of the 16x16 level with 64-channel output tiles (library route halo_bn64:
twice the workgroups). With two k-groups (route value 2) every output element accumulates the
same k sequence as the default 128-channel tiles: outputs BITWISE (the statistics partial rows
are reduced over another thread layout: equal to fp32 rounding); with one k-group (1) the k order
differs: within bf16 rounding of the default."""
import pytest
import torch

from progressive_process_for_human_pose_estimation_amd import hgk as H

pytestmark = pytest.mark.gpu
DEV = "cuda"
C = 128


def _run(L, x, wp, ld, bias, sc, sh, route):
    N, h, w_, _ = x.shape
    y = torch.empty(N, h, w_, C, device=DEV, dtype=torch.bfloat16)
    part = torch.full(((2 * (N * h * w_ // 64) + 4) * 3 * C,), float("nan"), device=DEV)
    rows = H.ctypes.c_int(0)
    with H.route(halo_bn64=route):
        H.check(L.hgk_conv_fwd(H.stream_handle(), H.BF16, x.data_ptr(), wp.data_ptr(), ld, bias.data_ptr(),
                               None, y.data_ptr(), sc.data_ptr(), sh.data_ptr(), 1, 0, part.data_ptr(),
                               H.ctypes.byref(rows), N, h, w_, C, C, 3, 3, 1, 1, 1, None, 0))
        fam = L.hgk_conv_fwd_kernel_family(H.BF16, N, h, w_, 0, 0, 0, C, C, 3, 3, 1, 1, 1)
    torch.cuda.synchronize()
    return y, part[: rows.value * 3 * C], fam


@pytest.mark.parametrize("n", [32, 8])
def test_halo_bn64_16x16(n):
    L = H.load_library()
    g = torch.Generator(device=DEV).manual_seed(n)
    x = (torch.randn(n, 16, 16, C, device=DEV, generator=g) * 0.7).to(torch.bfloat16)
    w = torch.randn(C, C, 3, 3, device=DEV, generator=g) * (1.0 / (9 * C) ** 0.5)
    bias = torch.randn(C, device=DEV, generator=g) * 0.1
    sc = torch.rand(C, device=DEV, generator=g) + 0.5
    sh = torch.randn(C, device=DEV, generator=g) * 0.3
    ld = L.hgk_conv_w_ld(9 * C)
    wp = torch.empty(C, ld, device=DEV, dtype=torch.bfloat16)
    H.check(L.hgk_pack_conv_weight(H.stream_handle(), H.BF16, w.data_ptr(), wp.data_ptr(), ld, C, C, 3, 3, 0, C, C))
    y0, p0, fam0 = _run(L, x, wp, ld, bias, sc, sh, 0)
    y2, p2, _ = _run(L, x, wp, ld, bias, sc, sh, 2)
    y1, p1, _ = _run(L, x, wp, ld, bias, sc, sh, 1)
    assert torch.equal(y0, y2)
    torch.testing.assert_close(p2, p0, rtol=1e-5, atol=1e-5)
    assert (y1.float() - y0.float()).abs().max().item() <= 1e-2 * y0.float().abs().max().item()
    assert p1.shape == p0.shape


@pytest.mark.parametrize("n", [16, 4])
def test_halo_bn64_32x32_outputs_bitwise(n):
    """route bit 4: the 8-row-tile launches of <= 128 workgroups (32x32 at N <= 16) with
    64-channel tiles: outputs bitwise the 128-channel tiles', statistics to fp32 rounding"""
    L = H.load_library()
    g = torch.Generator(device=DEV).manual_seed(100 + n)
    x = (torch.randn(n, 32, 32, C, device=DEV, generator=g) * 0.7).to(torch.bfloat16)
    w = torch.randn(C, C, 3, 3, device=DEV, generator=g) * (1.0 / (9 * C) ** 0.5)
    bias = torch.randn(C, device=DEV, generator=g) * 0.1
    sc = torch.rand(C, device=DEV, generator=g) + 0.5
    sh = torch.randn(C, device=DEV, generator=g) * 0.3
    ld = L.hgk_conv_w_ld(9 * C)
    wp = torch.empty(C, ld, device=DEV, dtype=torch.bfloat16)
    H.check(L.hgk_pack_conv_weight(H.stream_handle(), H.BF16, w.data_ptr(), wp.data_ptr(), ld, C, C, 3, 3, 0, C, C))
    with H.route(row3=0):
        y0, p0, _ = _run(L, x, wp, ld, bias, sc, sh, 0)
        y4, p4, _ = _run(L, x, wp, ld, bias, sc, sh, 6)
    assert torch.equal(y0, y4)
    torch.testing.assert_close(p4, p0, rtol=1e-5, atol=1e-5)
