"""The row-tile stem kernel (hgk_conv_stem.hip, route `stem`): the models' 7x7 / stride-2 / pad-3
input convolution (try_with_torch.py:262) over the channel-padded NHWC image, ReLU and BN
statistics out, as the engine launches it (no ReLU: hourglass_compare's stem feeds a BN). Against a torch fp32 convolution of the same bf16
operands per element (tests/gates.py bf16_out_close), the statistics partial rows against the
kernel's own stored output (one row per 128-pixel output row, XCD-slot order), and the implicit
GEMM's SMALLC path (route stem = 0) on the same input."""
import pytest
import torch
import torch.nn.functional as F

from gates import bf16_out_close
from progressive_process_for_human_pose_estimation_amd import hgk as H

DEV = "cuda"
pytestmark = pytest.mark.gpu


def _xcd_slot(m, n):
    x, q, r = m & 7, n >> 3, n & 7
    return (x * (q + 1) if x < r else r * (q + 1) + (x - r) * q) + (m >> 3)


def _run(L, x8, wp, ld, bias, N, R, relu):
    Ho = R // 2
    M = N * Ho * Ho
    y = torch.empty(N, Ho, Ho, 64, device=DEV, dtype=torch.bfloat16)
    part = torch.full((64 * 3 * (M // 128 + 8),), float("nan"), device=DEV)
    rows = H.ctypes.c_int(0)
    ws_b = L.hgk_conv_fwd_workspace(H.BF16, N, R, R, 8, 64, 7, 7, 2, 3, 1)
    ws = torch.zeros(max(ws_b, 1), dtype=torch.uint8, device=DEV)
    H.check(L.hgk_conv_fwd(H.stream_handle(), H.BF16, x8.data_ptr(), wp.data_ptr(), ld, bias.data_ptr(), None,
                           y.data_ptr(), None, None, 0, 1 if relu else 0, part.data_ptr(), H.ctypes.byref(rows),
                           N, R, R, 8, 64, 7, 7, 2, 3, 1, ws.data_ptr(), ws.numel()))
    torch.cuda.synchronize()
    return y, part, rows.value


@pytest.mark.parametrize("N,relu", [(2, True), (5, True), (3, False)])
def test_stem_kernel(N, relu, routes):
    L = H.load_library()
    R = 256
    g = torch.Generator(device=DEV).manual_seed(40 + N)
    x = (torch.randn(N, 3, R, R, device=DEV, generator=g) * 0.8).to(torch.bfloat16)
    x8 = torch.zeros(N, R, R, 8, device=DEV, dtype=torch.bfloat16)
    x8[..., :3] = x.permute(0, 2, 3, 1)
    w = torch.randn(64, 3, 7, 7, device=DEV, generator=g) * 0.1
    bias = torch.randn(64, device=DEV, generator=g) * 0.1
    ld = L.hgk_conv_w_ld(7 * 7 * 8)
    wp = torch.empty(128, ld, device=DEV, dtype=torch.bfloat16)
    H.check(L.hgk_pack_conv_weight(H.stream_handle(), H.BF16, w.data_ptr(), wp.data_ptr(), ld, 64, 3, 7, 7, 0,
                                   64, 8))
    assert H.KFAM[L.hgk_conv_fwd_kernel_family(H.BF16, N, R, R, 0, 0, 0, 8, 64, 7, 7, 2, 3, 1)] == "stem"
    y, part, rows = _run(L, x8, wp, ld, bias, N, R, relu)
    Ho = R // 2
    M = N * Ho * Ho
    assert rows == M // 128
    # reference: the same bf16 operands in fp32, bias, ReLU (the kernel rounds acc + bias once,
    # round(relu(v)) == relu(round(v)))
    ref = F.conv2d(x.float(), w.to(torch.bfloat16).float(), bias, stride=2, padding=3)
    ref = (torch.relu(ref) if relu else ref).permute(0, 2, 3, 1)  # hourglass_compare: BN follows
    bf16_out_close(y.float(), ref, "stem output")
    # statistics partial rows [64][3][rows] of the STORED output, row r at its XCD slot
    yr = y.float().reshape(M // 128, 128, 64)
    s = yr.sum(1)
    m2 = ((yr - s[:, None, :] / 128.0) ** 2).sum(1)
    slots = torch.tensor([_xcd_slot(r, rows) for r in range(rows)], device=DEV)
    P = part[:64 * 3 * rows].reshape(64, 3, rows)
    torch.testing.assert_close(P[:, 0, slots], s.t(), rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(P[:, 1, slots], m2.t(), rtol=1e-4, atol=1e-2)
    assert torch.all(P[:, 2, :] == 128.0)
    # the implicit GEMM (route stem = 0) on the same operands: the same output up to the fp32
    # accumulation order, statistics in the same rows
    routes(stem=0)
    assert H.KFAM[L.hgk_conv_fwd_kernel_family(H.BF16, N, R, R, 0, 0, 0, 8, 64, 7, 7, 2, 3, 1)] == "smallc"
    y0, part0, rows0 = _run(L, x8, wp, ld, bias, N, R, relu)
    assert rows0 == rows
    bf16_out_close(y0.float(), ref, "implicit stem output")
    d = (y.float() - y0.float()).abs()
    assert float((d > 0).float().mean()) < 0.01  # rare one-ulp rounding flips only
    P0 = part0[:64 * 3 * rows].reshape(64, 3, rows)
    torch.testing.assert_close(P0[:, 0], P[:, 0], rtol=1e-3, atol=0.05)
    assert torch.equal(P0[:, 2], P[:, 2])


@pytest.mark.parametrize("N", [2, 3])
def test_stem_weight_gradient(N):
    """the stem's weight / bias gradient (hgk_conv_wgrad over the channel-padded input, 16-tap k
    tiles) against torch's fp32 gradient of the same bf16 operands: fp32 split-K sums, 1e-3 of
    the largest element"""
    L = H.load_library()
    R = 256
    g = torch.Generator(device=DEV).manual_seed(70 + N)
    x = (torch.randn(N, 3, R, R, device=DEV, generator=g) * 0.8).to(torch.bfloat16)
    x8 = torch.zeros(N, R, R, 8, device=DEV, dtype=torch.bfloat16)
    x8[..., :3] = x.permute(0, 2, 3, 1)
    Ho = R // 2
    dy = (torch.randn(N, Ho, Ho, 64, device=DEV, generator=g) * 0.1).to(torch.bfloat16)
    dw = torch.zeros(64, 3, 7, 7, device=DEV)
    db = torch.zeros(64, device=DEV)
    ws_b = L.hgk_conv_wgrad_workspace(H.BF16, N, R, R, 8, 64, 7, 7, 2, 3, 1)
    ws = torch.empty(ws_b, dtype=torch.uint8, device=DEV)
    H.check(L.hgk_conv_wgrad(H.stream_handle(), H.BF16, x8.data_ptr(), dy.data_ptr(), None, None, 0,
                             dw.data_ptr(), db.data_ptr(), ws.data_ptr(), ws_b, N, R, R, 8, 64, 7, 7, 2,
                             3, 1, 3, 64))
    torch.cuda.synchronize()
    xr = x.float().requires_grad_(False)
    w = torch.zeros(64, 3, 7, 7, device=DEV, requires_grad=True)
    b = torch.zeros(64, device=DEV, requires_grad=True)
    out = F.conv2d(xr, w, b, stride=2, padding=3)
    out.backward(dy.float().permute(0, 3, 1, 2))
    torch.testing.assert_close(dw, w.grad, rtol=1e-4, atol=1e-3 * float(w.grad.abs().max()))
    torch.testing.assert_close(db, b.grad, rtol=1e-4, atol=1e-3 * float(b.grad.abs().max()))
