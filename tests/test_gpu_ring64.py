"""The ring 1x1 kernel's 64-channel instantiations (csrc/hgk_conv_ring.hip, round 5): the stem
block ResidualBlock(64, 128) at 128x128 (conv1 64 -> 64, conv3 / skip conv4 64 -> 128 and their
input gradients), residual2's 128 -> 64 / 64 -> 128 at 64x64 and the heads' 64 -> 256
(try_with_torch.py:179-209,286-297). 64-channel pixel rows are 128 B: their chunk swizzle is
c ^ ((p >> 1) & 7) and blocks grow until a part is whole DMA rounds (ring_bp).

Per launch: the output against a torch fp32 conv of the same bf16 operands (gates.bf16_out_close),
the statistics partial rows against sums of the stored output over the RING's row layout (row =
row group x pixel group: it fails if the launch took another kernel), the BN-backward partial sums
of mode 4, and the tiled route (ring off) on the same operands."""
import pytest
import torch
import torch.nn.functional as F

from gates import bf16_out_close, bn_relu_ref
from progressive_process_for_human_pose_estimation_amd import hgk as H

pytestmark = pytest.mark.gpu
DEV = "cuda"
U = 4  # kRingU


def _slot(bp, K, C, m):
    return bp * 2 * (K + (C if m & 2 else 0) + (C if m & 4 else 0) + (K if m & 16 else 0))


def _parts(bp, K, C, nw):
    return (bp * K * 2) % (nw * 1024) == 0 and (bp * C * 2) % (nw * 1024) == 0


def _bp(K, C, m, nw):  # ring_bp
    pg = max(nw // (C // 32), 1)
    if _slot(pg * 32, K, C, m) <= (32768 if nw == 8 else 16384) and _parts(pg * 32, K, C, nw):
        return pg * 32
    bp = pg * 16
    while not _parts(bp, K, C, nw):
        bp *= 2
    return bp


def _geom(K, C, m):
    """(BP, PG, PTW) of the launch (ring_nw: the 4-wave kernel where Cout <= 128 and it fits)"""
    nw = 8
    if C <= 128:
        bp = _bp(K, C, m, 4)
        pg = 4 // (C // 32)
        if (bp // 16) // pg >= 1 and (48 * 1024) // _slot(bp, K, C, m) >= 3:
            nw = 4
    bp = _bp(K, C, m, nw)
    pg = nw // (C // 32)
    return bp, pg, (bp // 16) // pg


def _ring_row_sums(t, K, C, m):
    """per ring partial row (row group x pixel group) the channel sums of t [M][C]"""
    bp, pg, ptw = _geom(K, C, m)
    M = t.shape[0]
    v = t.reshape(M // (bp * U), U, pg, ptw * 16, C)  # row group, block, pixel group, pixels
    return v.sum(dim=(1, 3)).reshape(-1, C), bp, pg, ptw


def _pack(L, w, cout, cin):
    ld = L.hgk_conv_w_ld(cin)
    wp = torch.empty(((cout + 127) // 128) * 128, ld, device=DEV, dtype=torch.bfloat16)
    H.check(L.hgk_pack_conv_weight(H.stream_handle(), 1, w.data_ptr(), wp.data_ptr(), ld, cout, cin,
                                   1, 1, 0, cout, cin))
    return wp, ld


FWD = [  # K, Cout, mode (1 BN in, 2 residual, 8 statistics), N, hw
    (64, 64, 9, 2, 128), (64, 128, 0, 2, 128), (64, 128, 11, 2, 128), (128, 64, 0, 2, 128),
    (128, 64, 9, 8, 64), (64, 256, 10, 8, 64), (64, 256, 2, 8, 64), (64, 256, 0, 8, 64),
    (64, 256, 8, 8, 64), (64, 128, 8, 2, 128), (64, 128, 9, 8, 64)]


@pytest.mark.parametrize("case", FWD, ids=lambda c: "k{}c{}m{}h{}".format(c[0], c[1], c[2], c[4]))
def test_ring64_fwd(case, routes):
    K, C, m, N, hw = case
    L = H.load_library()
    g = torch.Generator(device=DEV).manual_seed(K + C + m)
    pre, res, stats = bool(m & 1), bool(m & 2), bool(m & 8)
    x = (torch.randn(N, hw, hw, K, device=DEV, generator=g) * 0.7 + 0.2).to(torch.bfloat16)
    w = torch.randn(C, K, 1, 1, device=DEV, generator=g) * (1.0 / K ** 0.5)
    bias = torch.randn(C, device=DEV, generator=g) * 0.1
    sc = torch.rand(K, device=DEV, generator=g) + 0.5 if pre else None
    sh = torch.randn(K, device=DEV, generator=g) * 0.3 if pre else None
    r = torch.randn(N, hw, hw, C, device=DEV, generator=g).to(torch.bfloat16) if res else None
    wp, ld = _pack(L, w, C, K)
    M = N * hw * hw

    def run():
        y = torch.empty(N, hw, hw, C, device=DEV, dtype=torch.bfloat16)
        part = torch.full(((M // 16 + 4) * 3 * C,), float("nan"), device=DEV)
        rows = H.ctypes.c_int(0)
        H.check(L.hgk_conv_fwd(H.stream_handle(), 1, x.data_ptr(), wp.data_ptr(), ld, bias.data_ptr(),
                               H.ptr(r), y.data_ptr(), H.ptr(sc), H.ptr(sh), 1 if pre else 0, 0,
                               part.data_ptr() if stats else None, H.ctypes.byref(rows),
                               N, hw, hw, K, C, 1, 1, 1, 0, 1, None, 0))
        torch.cuda.synchronize()
        return y, part, rows.value

    y, part, nrows = run()
    a = bn_relu_ref(x.float(), sc, sh) if pre else x.float()
    ref = F.conv2d(a.permute(0, 3, 1, 2), w.to(torch.bfloat16).float(), bias).permute(0, 2, 3, 1)
    conv = None
    if res:
        conv = ref
        ref = ref.to(torch.bfloat16).float() + r.float()
    bf16_out_close(y, ref, "ring64 output", stored=conv)
    if stats:
        sums, bp, pg, ptw = _ring_row_sums(y.double().reshape(M, C), K, C, m)
        assert nrows == sums.shape[0], (nrows, sums.shape)
        p = part[: nrows * 3 * C].view(C, 3, nrows).double()
        torch.testing.assert_close(p[:, 0].t(), sums, rtol=1e-5, atol=1e-3)
        assert torch.all(p[:, 2] == U * 16 * ptw)
    # ring off: the tiled kernel on the same operands
    routes(ring_minm="0")
    y0, _, _ = run()
    bf16_out_close(y0, ref, "tiled output", stored=conv)


BWD = [(64, 64, 2, 128), (64, 128, 2, 128), (64, 128, 8, 64), (64, 256, 8, 64)]


@pytest.mark.parametrize("case", BWD, ids=lambda c: "k{}c{}h{}".format(c[0], c[1], c[3]))
def test_ring64_fused_bn_backward(case):
    """input-gradient launch (mode 4) with the BN-backward partial sums of the stored dA over the
    ring's rows: sum g, sum g * xhat, g = dA * [y * scale + shift > 0]"""
    K, C, N, hw = case
    L = H.load_library()
    g = torch.Generator(device=DEV).manual_seed(3 * K + C)
    dy = (torch.randn(N, hw, hw, K, device=DEV, generator=g) * 0.5).to(torch.bfloat16)
    w = torch.randn(C, K, 1, 1, device=DEV, generator=g) * (1.0 / K ** 0.5)
    ybn = torch.randn(N, hw, hw, C, device=DEV, generator=g).to(torch.bfloat16)
    scale = torch.rand(C, device=DEV, generator=g) + 0.5
    shift = torch.randn(C, device=DEV, generator=g) * 0.3
    mean = torch.randn(C, device=DEV, generator=g) * 0.1
    invstd = torch.rand(C, device=DEV, generator=g) + 0.5
    wp, ld = _pack(L, w, C, K)
    out = torch.empty(N, hw, hw, C, device=DEV, dtype=torch.bfloat16)
    M = N * hw * hw
    part = torch.full(((M // 16 + 4) * 2 * C,), float("nan"), device=DEV)
    rows = H.ctypes.c_int(0)
    H.check(L.hgk_conv_fwd_bnbwd(H.stream_handle(), 1, dy.data_ptr(), wp.data_ptr(), ld, None,
                                 out.data_ptr(), N, hw, hw, K, C, 1, 1, 1, 0, 1, None, 0,
                                 ybn.data_ptr(), scale.data_ptr(), shift.data_ptr(), 1,
                                 mean.data_ptr(), invstd.data_ptr(), part.data_ptr(),
                                 H.ctypes.byref(rows)))
    torch.cuda.synchronize()
    ref = F.conv2d(dy.float().permute(0, 3, 1, 2), w.to(torch.bfloat16).float()).permute(0, 2, 3, 1)
    bf16_out_close(out, ref, "ring64 input gradient")
    dA = out.double().reshape(-1, C)
    yb = ybn.double().reshape(-1, C)
    gg = dA * ((yb * scale.double() + shift.double()) > 0)
    s1, _, _, _ = _ring_row_sums(gg, K, C, 4)
    s2, _, _, _ = _ring_row_sums(gg * (yb - mean.double()) * invstd.double(), K, C, 4)
    assert rows.value == s1.shape[0], (rows.value, s1.shape)
    p = part[: rows.value * 2 * C].view(rows.value, 2, C).double()
    torch.testing.assert_close(p[:, 0], s1, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(p[:, 1], s2, rtol=1e-4, atol=1e-3)
