"""Global average pool / 1x1 broadcast kernels (hgk_spatial_sum, hgk_spatial_broadcast: the live
ASPP image-pool branch, try_more_layer.py:266-268,286-287) vs torch fp32 on the same inputs."""
import pytest
import torch
import torch.nn.functional as F

from progressive_process_for_human_pose_estimation_amd import hgk as H

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("dt", [H.F32, H.BF16])
@pytest.mark.parametrize("shape", [(2, 2, 2, 256), (3, 4, 4, 256), (2, 7, 5, 40), (1, 64, 64, 8)])
def test_spatial_mean_and_broadcast(dt, shape):
    L = H.load_library()
    s = H.stream_handle()
    N, Hh, W, C = shape
    tdt = torch.float32 if dt == H.F32 else torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(7)
    x = torch.randn(N, Hh, W, C, device=DEV, generator=g).to(tdt)
    # AdaptiveAvgPool2d((1, 1)) forward
    y = torch.empty(N, C, device=DEV, dtype=tdt)
    H.check(L.hgk_spatial_sum(s, dt, x.data_ptr(), y.data_ptr(), N, Hh * W, C, 1.0 / (Hh * W), 0))
    ref = F.adaptive_avg_pool2d(x.float().permute(0, 3, 1, 2), (1, 1)).reshape(N, C)
    tol = 1e-5 if dt == H.F32 else 1e-2
    torch.testing.assert_close(y.float(), ref, rtol=tol, atol=tol)
    # bilinear align_corners=True 1x1 -> Hh x W (forward), accumulated onto an existing buffer
    base = torch.randn(N, Hh, W, C, device=DEV, generator=g).to(tdt)
    z = base.clone()
    H.check(L.hgk_spatial_broadcast(s, dt, y.data_ptr(), z.data_ptr(), N, Hh * W, C, 1.0, 1))
    up = F.interpolate(y.float().reshape(N, C, 1, 1), size=(Hh, W), mode="bilinear",
                       align_corners=True).permute(0, 2, 3, 1)
    torch.testing.assert_close(z.float(), base.float() + up, rtol=tol, atol=tol)
    # the pair as each other's backward (autograd of the torch ops)
    xr = x.float().permute(0, 3, 1, 2).requires_grad_()
    gout = torch.randn(N, C, 1, 1, device=DEV, generator=g)
    F.adaptive_avg_pool2d(xr, (1, 1)).backward(gout)
    gq = gout.reshape(N, C).to(tdt).contiguous()
    dx = torch.empty(N, Hh, W, C, device=DEV, dtype=tdt)
    H.check(L.hgk_spatial_broadcast(s, dt, gq.data_ptr(), dx.data_ptr(), N, Hh * W, C,
                                    1.0 / (Hh * W), 0))
    torch.testing.assert_close(dx.float(), xr.grad.permute(0, 2, 3, 1), rtol=tol, atol=tol)
    yr = y.float().reshape(N, C, 1, 1).requires_grad_()
    gup = torch.randn(N, C, Hh, W, device=DEV, generator=g)
    F.interpolate(yr, size=(Hh, W), mode="bilinear", align_corners=True).backward(gup)
    gin = gup.permute(0, 2, 3, 1).to(tdt).contiguous()
    dy = torch.empty(N, C, device=DEV, dtype=tdt)
    H.check(L.hgk_spatial_sum(s, dt, gin.data_ptr(), dy.data_ptr(), N, Hh * W, C, 1.0, 0))
    ref = gin.float().sum((1, 2))  # the rounded input summed in fp32
    torch.testing.assert_close(dy.float(), ref, rtol=tol, atol=tol * Hh * W ** 0.5)
    if dt == H.F32:
        torch.testing.assert_close(dy, yr.grad.reshape(N, C), rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("dt", [H.F32, H.BF16])
@pytest.mark.parametrize("args", [(2, 4, 4, 64, 2, 8, 8), (1, 3, 3, 8, 2, 5, 5), (2, 2, 3, 12, 3, 4, 7)])
def test_zero_insert(dt, args):
    """hgk_zero_insert (strided-conv input-gradient): exact scatter onto the stride grid."""
    L = H.load_library()
    s = H.stream_handle()
    N, h, w, C, st, Hz, Wz = args
    tdt = torch.float32 if dt == H.F32 else torch.bfloat16
    src = torch.randn(N, h, w, C, device=DEV).to(tdt)
    dst = torch.full((N, Hz, Wz, C), 7.0, device=DEV, dtype=tdt)
    H.check(L.hgk_zero_insert(s, dt, src.data_ptr(), dst.data_ptr(), N, h, w, C, st, Hz, Wz))
    ref = torch.zeros(N, Hz, Wz, C, device=DEV, dtype=tdt)
    hh, ww = min(h, (Hz + st - 1) // st), min(w, (Wz + st - 1) // st)
    ref[:, : hh * st : st, : ww * st : st] = src[:, :hh, :ww]
    assert torch.equal(dst, ref)
