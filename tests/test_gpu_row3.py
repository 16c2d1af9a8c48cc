"""The row-streaming 3x3 kernel (csrc/hgk_conv_row3.hip: the ResidualBlock's 128 -> 128 conv2,
try_with_torch.py:189, at the 64x64 / 32x32 levels) through the C-ABI:

* forward (BN+ReLU input transform, statistics out) against a torch fp32 conv of the same
  bf16-rounded operands, the statistics partials (one row per output row) against the stored
  outputs, and the halo kernel (HGK_ROW3=0) to bf16 rounding;
* the input gradient (flipped / transposed weights) with the fused BN-backward sums of the STORED
  dA, against torch and against sums recomputed from the output;
* twin launches (64x64 + 32x32 segments, one grid) BITWISE equal to one launch per segment;
* ragged work splits: images whose row count does not divide over the workgroups, a single image.

Tolerances as tests/test_gpu_ring.py: bf16 outputs per element 2^-8 |ref| + 1e-4 max|ref| (gates.bf16_out_close); statistics 1e-4 mean /
1e-3 variance relative."""
import pytest
import torch
import torch.nn.functional as F

from progressive_process_for_human_pose_estimation_amd import hgk as H
from gates import bf16_out_close, bn_relu_ref

pytestmark = pytest.mark.gpu
DEV = "cuda"
C = 128


def _pack(L, w, dgrad=False):
    ld = L.hgk_conv_w_ld(9 * C)
    wp = torch.empty(C, ld, device=DEV, dtype=torch.bfloat16)
    H.check(L.hgk_pack_conv_weight(H.stream_handle(), 1, w.data_ptr(), wp.data_ptr(), ld, C, C,
                                   3, 3, 1 if dgrad else 0, C, C))
    return wp, ld


def _part(M):
    return torch.full(((2 * (M // 64) + 4) * 3 * C,), float("nan"), device=DEV)


def _fwd(L, x, wp, ld, bias, scale, shift):
    N, h, w_, _ = x.shape
    y = torch.empty(N, h, w_, C, device=DEV, dtype=torch.bfloat16)
    part = _part(N * h * w_)
    rows = H.ctypes.c_int(0)
    H.check(L.hgk_conv_fwd(H.stream_handle(), 1, x.data_ptr(), wp.data_ptr(), ld, bias.data_ptr(), None,
                           y.data_ptr(), scale.data_ptr(), shift.data_ptr(), 1, 0, part.data_ptr(),
                           H.ctypes.byref(rows), N, h, w_, C, C, 3, 3, 1, 1, 1, None, 0))
    torch.cuda.synchronize()
    return y, part, rows.value


def _check_stats(y, part, nrows):
    p = part[: nrows * 3 * C].view(C, 3, nrows).permute(2, 1, 0).double()
    yd = y.double().reshape(-1, C)
    n = p[:, 2].sum(0)
    assert torch.all(n == yd.shape[0])
    mean = p[:, 0].sum(0) / n
    torch.testing.assert_close(mean, yd.mean(0), rtol=1e-4, atol=1e-4)
    m2 = (p[:, 1] + p[:, 2] * (p[:, 0] / p[:, 2].clamp_min(1) - mean) ** 2).sum(0)
    torch.testing.assert_close(m2 / n, yd.var(0, unbiased=False), rtol=1e-3, atol=1e-4)


def _inputs(N, hw, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    x = (torch.randn(N, hw, hw, C, device=DEV, generator=g) * 0.7 + 0.2).to(torch.bfloat16)
    w = torch.randn(C, C, 3, 3, device=DEV, generator=g) * (1.0 / (9 * C) ** 0.5)
    bias = torch.randn(C, device=DEV, generator=g) * 0.1
    sc = torch.rand(C, device=DEV, generator=g) + 0.5
    sh = torch.randn(C, device=DEV, generator=g) * 0.3
    return g, x, w, bias, sc, sh


@pytest.mark.parametrize("case", [(4, 64), (8, 32), (1, 64), (3, 32), (32, 64)],
                         ids=lambda c: f"n{c[0]}h{c[1]}")
def test_row3_fwd(case, routes):
    N, hw = case
    L = H.load_library()
    g, x, w, bias, sc, sh = _inputs(N, hw, 3)
    wp, ld = _pack(L, w)
    routes(row3="1")
    y, part, nrows = _fwd(L, x, wp, ld, bias, sc, sh)
    assert nrows == N * hw, nrows  # one partial row per output row
    a = bn_relu_ref(x.float(), sc, sh)
    ref = F.conv2d(a.permute(0, 3, 1, 2), w.to(torch.bfloat16).float(), bias, padding=1).permute(0, 2, 3, 1)
    bf16_out_close(y, ref)
    _check_stats(y, part, nrows)
    routes(row3="0")  # the halo kernel
    y0, part0, nrows0 = _fwd(L, x, wp, ld, bias, sc, sh)
    bf16_out_close(y0, ref)


@pytest.mark.parametrize("relu", [True, False], ids=["relu", "norelu"])
@pytest.mark.parametrize("case", [(4, 64), (6, 32)], ids=lambda c: f"n{c[0]}h{c[1]}")
def test_row3_dgrad_bn_backward(case, relu, routes):
    """input gradient (dy -> dA with the flipped, transposed weights) + BN-backward partial sums
    of the STORED dA: sum g, sum g * xhat, g = dA [y * scale + shift > 0]"""
    N, hw = case
    L = H.load_library()
    g, dy, w, _, sc, sh = _inputs(N, hw, 5)
    ybn = torch.randn(N, hw, hw, C, device=DEV, generator=g).to(torch.bfloat16)
    mean = torch.randn(C, device=DEV, generator=g) * 0.1
    invstd = torch.rand(C, device=DEV, generator=g) + 0.5
    wd, ld = _pack(L, w, dgrad=True)
    M = N * hw * hw

    def run():
        out = torch.empty(N, hw, hw, C, device=DEV, dtype=torch.bfloat16)
        part = _part(M)
        rows = H.ctypes.c_int(0)
        H.check(L.hgk_conv_fwd_bnbwd(H.stream_handle(), 1, dy.data_ptr(), wd.data_ptr(), ld, None,
                                     out.data_ptr(), N, hw, hw, C, C, 3, 3, 1, 1, 1, None, 0,
                                     ybn.data_ptr(), sc.data_ptr(), sh.data_ptr(), 1 if relu else 0,
                                     mean.data_ptr(), invstd.data_ptr(), part.data_ptr(),
                                     H.ctypes.byref(rows)))
        torch.cuda.synchronize()
        return out, part, rows.value

    routes(row3="1")
    out, part, rows = run()
    assert rows == N * hw
    ref = F.conv_transpose2d(dy.float().permute(0, 3, 1, 2), w.to(torch.bfloat16).float(),
                             padding=1).permute(0, 2, 3, 1)
    bf16_out_close(out, ref)
    dA = out.double().reshape(-1, C)
    yb = ybn.double().reshape(-1, C)
    gg = dA * ((yb * sc.double() + sh.double()) > 0) if relu else dA
    p = part[: rows * 2 * C].view(rows, 2, C).double().sum(0)
    torch.testing.assert_close(p[0], gg.sum(0), rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(p[1], (gg * (yb - mean.double()) * invstd.double()).sum(0),
                               rtol=1e-4, atol=1e-3)
    routes(row3="0")
    out0, _, rows0 = run()
    bf16_out_close(out0, ref)


@pytest.mark.parametrize("mode", ["fwd", "dgrad"])
def test_row3_twin_bitwise_equals_single(mode, routes):
    """one grid over a 64x64 and a 32x32 segment (different BN constants per segment) == one launch
    per segment, bit for bit (outputs and partial rows)"""
    routes(row3="1")
    N = 8
    L = H.load_library()
    g = torch.Generator(device=DEV).manual_seed(9)
    w = torch.randn(C, C, 3, 3, device=DEV, generator=g) * (1.0 / (9 * C) ** 0.5)
    bias = torch.randn(C, device=DEV, generator=g) * 0.1
    wp, ld = _pack(L, w, dgrad=(mode == "dgrad"))
    fwd = mode == "fwd"
    segs, singles, outs, keep = [], [], [], []
    for hw in (64, 32):
        M = N * hw * hw
        x = (torch.randn(N, hw, hw, C, device=DEV, generator=g) * 0.7).to(torch.bfloat16)
        sc = torch.rand(C, device=DEV, generator=g) + 0.5
        sh = torch.randn(C, device=DEV, generator=g) * 0.3
        ybn = torch.randn(N, hw, hw, C, device=DEV, generator=g).to(torch.bfloat16)
        mu = torch.randn(C, device=DEV, generator=g) * 0.1
        ist = torch.rand(C, device=DEV, generator=g) + 0.5
        res = []
        for twin in (False, True):
            y = torch.empty(N, hw, hw, C, device=DEV, dtype=torch.bfloat16)
            part = _part(M)
            rows = H.ctypes.c_int(0)
            res.append((y, part, rows))
            if not twin:
                if fwd:
                    H.check(L.hgk_conv_fwd(H.stream_handle(), 1, x.data_ptr(), wp.data_ptr(), ld,
                                           bias.data_ptr(), None, y.data_ptr(), sc.data_ptr(),
                                           sh.data_ptr(), 1, 0, part.data_ptr(), H.ctypes.byref(rows),
                                           N, hw, hw, C, C, 3, 3, 1, 1, 1, None, 0))
                else:
                    H.check(L.hgk_conv_fwd_bnbwd(H.stream_handle(), 1, x.data_ptr(), wp.data_ptr(), ld,
                                                 None, y.data_ptr(), N, hw, hw, C, C, 3, 3, 1, 1, 1,
                                                 None, 0, ybn.data_ptr(), sc.data_ptr(), sh.data_ptr(),
                                                 1, mu.data_ptr(), ist.data_ptr(), part.data_ptr(),
                                                 H.ctypes.byref(rows)))
        singles.append(res[0])
        outs.append(res[1])
        y, part, rows = res[1]
        if fwd:
            segs.append(H.ConvSeg(x.data_ptr(), None, y.data_ptr(), sc.data_ptr(), sh.data_ptr(),
                                  part.data_ptr(), H.ctypes.pointer(rows), N, hw, hw, None, None,
                                  None, None, None, None, 0, None))
        else:
            segs.append(H.ConvSeg(x.data_ptr(), None, y.data_ptr(), None, None, None, None, N, hw, hw,
                                  ybn.data_ptr(), sc.data_ptr(), sh.data_ptr(), mu.data_ptr(),
                                  ist.data_ptr(), part.data_ptr(), 1, H.ctypes.pointer(rows)))
        keep.append((x, ybn, sc, sh, mu, ist))
    H.check(L.hgk_conv_fwd_twin(H.stream_handle(), 1, wp.data_ptr(), ld,
                                bias.data_ptr() if fwd else None, 1 if fwd else 0, 0, C, C, 3, 3, 1,
                                1, 1, (H.ConvSeg * 2)(*segs), None, 0))
    torch.cuda.synchronize()
    for (y, part, rows), (y1, part1, rows1) in zip(outs, singles):
        assert rows.value == rows1.value > 0
        assert torch.equal(y, y1)
        n = rows1.value * (3 if fwd else 2) * C
        assert torch.equal(part[:n], part1[:n])


@pytest.mark.parametrize("case", [(8, 64), (6, 32), (32, 64), (3, 64)], ids=lambda c: f"n{c[0]}h{c[1]}")
@pytest.mark.parametrize("mode", ["fwd", "dgrad"])
def test_row3_alternating_order_bitwise(case, mode, routes):
    """route row3_alt (odd workgroups take their rows bottom-up, so neighbours share boundary rows
    in L2): outputs and partial rows bitwise those of the top-down order"""
    N, hw = case
    L = H.load_library()
    g, x, w, bias, sc, sh = _inputs(N, hw, 11)
    ybn = torch.randn(N, hw, hw, C, device=DEV, generator=g).to(torch.bfloat16)
    mu = torch.randn(C, device=DEV, generator=g) * 0.1
    ist = torch.rand(C, device=DEV, generator=g) + 0.5
    wp, ld = _pack(L, w, dgrad=(mode == "dgrad"))
    M = N * hw * hw
    res = []
    for alt in ("0", "1"):
        routes(row3="1", row3_alt=alt)
        if mode == "fwd":
            res.append(_fwd(L, x, wp, ld, bias, sc, sh))
            continue
        out = torch.empty(N, hw, hw, C, device=DEV, dtype=torch.bfloat16)
        part = _part(M)
        rows = H.ctypes.c_int(0)
        H.check(L.hgk_conv_fwd_bnbwd(H.stream_handle(), 1, x.data_ptr(), wp.data_ptr(), ld, None,
                                     out.data_ptr(), N, hw, hw, C, C, 3, 3, 1, 1, 1, None, 0,
                                     ybn.data_ptr(), sc.data_ptr(), sh.data_ptr(), 1, mu.data_ptr(),
                                     ist.data_ptr(), part.data_ptr(), H.ctypes.byref(rows)))
        torch.cuda.synchronize()
        res.append((out, part, rows.value))
    (y0, p0, r0), (y1, p1, r1) = res
    assert r0 == r1
    assert torch.equal(y0, y1)
    n = r0 * (3 if mode == "fwd" else 2) * C
    assert torch.equal(p0[:n], p1[:n])
