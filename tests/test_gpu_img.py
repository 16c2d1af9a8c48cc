"""Image-tile convolution kernel (csrc/hgk_conv_img.hip: the 1x1 and 3x3 convolutions of the
small hourglass levels, 16x16 .. 4x4, 64 output pixels of whole images / row strips per
workgroup) through the C-ABI:

* forward against a torch fp32 conv of the same bf16-rounded operands (BN+ReLU transform, zero
  padding after it, bias, residual) and the statistics partials against the stored outputs;
* 1x1: bitwise equal to the implicit GEMM it replaces (same k order, same epilogue code);
* fused BN-backward sums of an input-gradient launch;
* the folded BN finalize equal to the explicit finalize + transform (the all-ahead kernel's
  fold_merge), publishing the same statistics;
* twin launches (16x16 + 8x8, 8x8 + 4x4) bitwise equal to one launch per segment.
The route is asserted with hgk_conv_fwd_kernel_family before each launch."""
import pytest
import torch
import torch.nn.functional as F

from progressive_process_for_human_pose_estimation_amd import hgk as H
from gates import bf16_out_close, bn_relu_ref

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF16 = 1


def _fam(L, N, hw, cin, cout, k, N1=0, hw1=0):
    return H.KFAM[L.hgk_conv_fwd_kernel_family(BF16, N, hw, hw, N1, hw1, hw1, cin, cout, k, k, 1,
                                               k // 2, 1)]


def _pack(L, w, dgrad=False):
    cout, cin, k, _ = w.shape
    ld = L.hgk_conv_w_ld(k * k * cin)
    wp = torch.empty(((cout + 127) // 128) * 128, ld, device=DEV, dtype=torch.bfloat16)
    H.check(L.hgk_pack_conv_weight(H.stream_handle(), BF16, w.data_ptr(), wp.data_ptr(), ld, cout,
                                   cin, k, k, 1 if dgrad else 0, cout, cin))
    return wp, ld


def _inputs(N, hw, cin, cout, k, res, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    x = (torch.randn(N, hw, hw, cin, device=DEV, generator=g) * 0.7).to(torch.bfloat16)
    w = torch.randn(cout, cin, k, k, device=DEV, generator=g) * (1.0 / (cin * k * k) ** 0.5)
    bias = torch.randn(cout, device=DEV, generator=g) * 0.1
    sc = torch.rand(cin, device=DEV, generator=g) + 0.5
    sh = torch.randn(cin, device=DEV, generator=g) * 0.3
    r = torch.randn(N, hw, hw, cout, device=DEV, generator=g).to(torch.bfloat16) if res else None
    return x, w, bias, sc, sh, r


def _fwd(L, x, wp, ld, bias, r, sc, sh, cout, k):
    N, hw, _, cin = x.shape
    M = N * hw * hw
    y = torch.empty(N, hw, hw, cout, device=DEV, dtype=torch.bfloat16)
    part = torch.full(((2 * (M // 64) + 4) * 3 * cout,), float("nan"), device=DEV)
    rows = H.ctypes.c_int(0)
    ws_b = L.hgk_conv_fwd_workspace(BF16, N, hw, hw, cin, cout, k, k, 1, k // 2, 1)
    ws = torch.zeros(max(ws_b, 1), dtype=torch.uint8, device=DEV)
    H.check(L.hgk_conv_fwd(H.stream_handle(), BF16, x.data_ptr(), wp.data_ptr(), ld, bias.data_ptr(),
                           H.ptr(r), y.data_ptr(), H.ptr(sc), H.ptr(sh), 1 if sc is not None else 0,
                           0, part.data_ptr(), H.ctypes.byref(rows), N, hw, hw, cin, cout, k, k, 1,
                           k // 2, 1, ws.data_ptr(), ws_b))
    torch.cuda.synchronize()
    return y, part, rows.value


CASES = [
    # N, hw, cin, cout, k, pre, res
    (32, 4, 128, 128, 3, True, False),
    (32, 8, 128, 128, 3, True, True),
    (8, 8, 128, 128, 3, False, False),
    (4, 4, 128, 128, 3, True, True),     # one tile: four 4x4 images
    (32, 4, 256, 128, 1, True, False),
    (32, 8, 128, 256, 1, True, True),
    (32, 16, 256, 256, 1, False, False),
    (32, 4, 256, 64, 1, True, False),    # head conv2 (17 outputs, stored 64 wide)
    (16, 16, 128, 128, 3, True, False),  # 4-row strips of 16x16 (N = 16: one round)
    (16, 16, 128, 128, 3, True, True),
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "n{}h{}c{}-{}k{}{}{}".format(
    c[0], c[1], c[2], c[3], c[4], "p" if c[5] else "", "r" if c[6] else ""))
def test_img_fwd_vs_reference(case):
    N, hw, cin, cout, k, pre, res = case
    L = H.load_library()
    assert _fam(L, N, hw, cin, cout, k) == "img"
    x, w, bias, sc, sh, r = _inputs(N, hw, cin, cout, k, res, 11)
    if not pre:
        sc = sh = None
    wp, ld = _pack(L, w)
    y, part, nrows = _fwd(L, x, wp, ld, bias, r, sc, sh, cout, k)
    assert nrows == N * hw * hw // 64
    a = x.float()
    if pre:
        a = bn_relu_ref(a, sc, sh)
    ref = F.conv2d(a.permute(0, 3, 1, 2), w.to(torch.bfloat16).float(), bias, padding=k // 2)
    ref = ref.permute(0, 2, 3, 1)
    conv = None
    if res:
        conv = ref
        ref = ref.to(torch.bfloat16).float() + r.float()  # the conv output is stored, then the residual added
    bf16_out_close(y, ref, stored=conv)
    p = part[: nrows * 3 * cout].view(cout, 3, nrows).permute(2, 1, 0).double()
    yd = y.double().reshape(-1, cout)
    n = p[:, 2].sum(0)
    assert torch.all(n == yd.shape[0])
    mean = p[:, 0].sum(0) / n
    torch.testing.assert_close(mean, yd.mean(0), rtol=1e-4, atol=1e-4)
    m2 = (p[:, 1] + p[:, 2] * (p[:, 0] / p[:, 2].clamp_min(1) - mean) ** 2).sum(0)
    torch.testing.assert_close(m2 / n, yd.var(0, unbiased=False), rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize("case", [(32, 4, 256, 128, True, False), (32, 8, 128, 256, True, True),
                                  (32, 16, 256, 128, True, False)], ids=["c1@4", "c3r@8", "c1@16"])
def test_img_1x1_bitwise_equals_implicit(case, routes):
    """1x1: the same k order and epilogue code as the 64x64 implicit-GEMM tiles it replaces"""
    N, hw, cin, cout, pre, res = case
    L = H.load_library()
    x, w, bias, sc, sh, r = _inputs(N, hw, cin, cout, 1, res, 3)
    wp, ld = _pack(L, w)
    assert _fam(L, N, hw, cin, cout, 1) == "img"
    y1, p1, n1 = _fwd(L, x, wp, ld, bias, r, sc, sh, cout, 1)
    routes(img=0)
    assert _fam(L, N, hw, cin, cout, 1) == "implicit"
    y0, p0, n0 = _fwd(L, x, wp, ld, bias, r, sc, sh, cout, 1)
    assert n0 == n1
    assert torch.equal(y0, y1)
    assert torch.equal(p0[: n0 * 3 * cout], p1[: n1 * 3 * cout])


@pytest.mark.parametrize("case", [(32, 4, 256, 128, True, False), (32, 8, 128, 256, True, True),
                                  (32, 16, 256, 128, True, False), (32, 4, 256, 64, True, False)],
                         ids=["c1@4", "c3r@8", "c1@16", "head@4"])
def test_img_1x1_narrow_tiles(case, routes):
    """route img_narrow: 32-channel output tiles (twice the workgroups) give the same outputs bit
    for bit (every output keeps its k order); the statistics partials (another per-thread row
    grouping in the epilogue) match the stored output's moments"""
    N, hw, cin, cout, pre, res = case
    L = H.load_library()
    x, w, bias, sc, sh, r = _inputs(N, hw, cin, cout, 1, res, 9)
    wp, ld = _pack(L, w)
    y0, p0, n0 = _fwd(L, x, wp, ld, bias, r, sc, sh, cout, 1)
    routes(img_narrow=1 << 20)
    assert _fam(L, N, hw, cin, cout, 1) == "img"
    y1, p1, n1 = _fwd(L, x, wp, ld, bias, r, sc, sh, cout, 1)
    assert n1 == n0 == N * hw * hw // 64
    assert torch.equal(y0, y1)
    p = p1[: n1 * 3 * cout].view(cout, 3, n1).permute(2, 1, 0).double()
    yd = y1.double().reshape(-1, cout)
    n = p[:, 2].sum(0)
    assert torch.all(n == yd.shape[0])
    mean = p[:, 0].sum(0) / n
    torch.testing.assert_close(mean, yd.mean(0), rtol=1e-4, atol=1e-4)
    m2 = (p[:, 1] + p[:, 2] * (p[:, 0] / p[:, 2].clamp_min(1) - mean) ** 2).sum(0)
    torch.testing.assert_close(m2 / n, yd.var(0, unbiased=False), rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(p1[: n1 * 3 * cout], p0[: n0 * 3 * cout], rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("case", [(32, 8, 128, 128, 3), (32, 4, 128, 128, 3), (32, 4, 128, 256, 1),
                                  (32, 16, 256, 128, 1)], ids=["3x3@8", "3x3@4", "1x1@4", "1x1@16"])
def test_img_input_gradient_bn_backward_sums(case):
    """input-gradient launch with the fused BN-backward sums of the stored dA"""
    N, hw, cin, cout, k = case
    L = H.load_library()
    assert _fam(L, N, hw, cin, cout, k) == "img"
    g = torch.Generator(device=DEV).manual_seed(5)
    dy = (torch.randn(N, hw, hw, cin, device=DEV, generator=g) * 0.5).to(torch.bfloat16)
    w = torch.randn(cout, cin, k, k, device=DEV, generator=g) * (1.0 / (cin * k * k) ** 0.5)
    ybn = torch.randn(N, hw, hw, cout, device=DEV, generator=g).to(torch.bfloat16)
    scale = torch.rand(cout, device=DEV, generator=g) + 0.5
    shift = torch.randn(cout, device=DEV, generator=g) * 0.3
    mean = torch.randn(cout, device=DEV, generator=g) * 0.1
    invstd = torch.rand(cout, device=DEV, generator=g) + 0.5
    wp, ld = _pack(L, w)
    out = torch.empty(N, hw, hw, cout, device=DEV, dtype=torch.bfloat16)
    M = N * hw * hw
    part = torch.full(((2 * (M // 64) + 4) * 2 * cout,), float("nan"), device=DEV)
    rows = H.ctypes.c_int(0)
    ws_b = L.hgk_conv_fwd_workspace(BF16, N, hw, hw, cin, cout, k, k, 1, k // 2, 1)
    ws = torch.zeros(max(ws_b, 1), dtype=torch.uint8, device=DEV)
    H.check(L.hgk_conv_fwd_bnbwd(H.stream_handle(), BF16, dy.data_ptr(), wp.data_ptr(), ld, None,
                                 out.data_ptr(), N, hw, hw, cin, cout, k, k, 1, k // 2, 1,
                                 ws.data_ptr(), ws_b, ybn.data_ptr(), scale.data_ptr(),
                                 shift.data_ptr(), 1, mean.data_ptr(), invstd.data_ptr(),
                                 part.data_ptr(), H.ctypes.byref(rows)))
    torch.cuda.synchronize()
    assert rows.value == M // 64
    ref = F.conv2d(dy.float().permute(0, 3, 1, 2), w.to(torch.bfloat16).float(),
                   padding=k // 2).permute(0, 2, 3, 1)
    bf16_out_close(out, ref)
    dA = out.double().reshape(-1, cout)
    yb = ybn.double().reshape(-1, cout)
    gg = dA * ((yb * scale.double() + shift.double()) > 0)
    p = part[: rows.value * 2 * cout].view(rows.value, 2, cout).double().sum(0)
    torch.testing.assert_close(p[0], gg.sum(0), rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(p[1], (gg * (yb - mean.double()) * invstd.double()).sum(0),
                               rtol=1e-4, atol=1e-3)


def _fold_partials(cin, rows, M, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    part = torch.empty(cin, 3, rows, device=DEV)
    part[:, 0] = torch.randn(cin, rows, device=DEV, generator=g) * 20
    part[:, 1] = torch.rand(cin, rows, device=DEV, generator=g) * 40 + 1
    part[:, 2] = float(M) / rows
    return part


@pytest.mark.parametrize("case", [(32, 8, 128, 128, 3), (32, 4, 128, 128, 3), (32, 4, 256, 128, 1),
                                  (32, 8, 128, 256, 1)], ids=["3x3@8", "3x3@4", "1x1@4", "1x1@8"])
def test_img_folded_finalize_equals_explicit(case, routes):
    """hgk_conv_fwd_fold on the image-tile kernel: published statistics and outputs bitwise equal
    to the all-ahead implicit GEMM's fold (same fold_merge); outputs also equal a launch with the
    published scale / shift as an explicit transform"""
    N, hw, cin, cout, k = case
    L = H.load_library()
    M = N * hw * hw
    frows = 8 if M // 64 < 32 else 32
    x, w, bias, _, _, _ = _inputs(N, hw, cin, cout, k, False, 21)
    wp, ld = _pack(L, w)
    fpart = _fold_partials(cin, frows, M, 4)
    gamma = torch.rand(cin, device=DEV) + 0.5
    beta = torch.randn(cin, device=DEV) * 0.1
    assert L.hgk_conv_fold_ok(BF16, N, hw, hw, 0, 0, 0, cin, cout, k, k, 1, k // 2, 1, frows, 0)

    def run_fold():
        stat = torch.full((4, cin), float("nan"), device=DEV)
        rec = torch.full((2, cin), float("nan"), device=DEV, dtype=torch.float64)
        fd = H.BnFold(fpart.data_ptr(), frows, M, gamma.data_ptr(), beta.data_ptr(), 1e-5,
                      stat.data_ptr(), rec.data_ptr())
        y = torch.empty(N, hw, hw, cout, device=DEV, dtype=torch.bfloat16)
        part = torch.full(((2 * (M // 64) + 4) * 3 * cout,), float("nan"), device=DEV)
        rows = H.ctypes.c_int(0)
        ws_b = L.hgk_conv_fwd_workspace(BF16, N, hw, hw, cin, cout, k, k, 1, k // 2, 1)
        ws = torch.zeros(max(ws_b, 1 << 16), dtype=torch.uint8, device=DEV)
        H.check(L.hgk_conv_fwd_fold(H.stream_handle(), BF16, x.data_ptr(), wp.data_ptr(), ld,
                                    bias.data_ptr(), None, y.data_ptr(), 1, 0, part.data_ptr(),
                                    H.ctypes.byref(rows), N, hw, hw, cin, cout, k, k, 1, k // 2, 1,
                                    ws.data_ptr(), ws.numel(), H.ctypes.byref(fd)))
        torch.cuda.synchronize()
        return y, stat, rec, part[: rows.value * 3 * cout]

    assert _fam(L, N, hw, cin, cout, k) == "img"
    y, stat, rec, part = run_fold()
    routes(img=0)
    assert _fam(L, N, hw, cin, cout, k) == "implicit"
    y0, stat0, rec0, part0 = run_fold()
    assert torch.equal(stat, stat0) and torch.equal(rec, rec0)
    if k == 1:  # same accumulation order as the implicit GEMM (3x3: split-K there)
        assert torch.equal(y, y0) and torch.equal(part, part0)
    routes(img=8192)
    ye, _, _ = _fwd(L, x, wp, ld, bias, None, stat[2].contiguous(), stat[3].contiguous(), cout, k)
    assert torch.equal(y, ye)


@pytest.mark.parametrize("case", [(32, 8, 4, 128, 128, 3), (32, 8, 4, 128, 256, 1),
                                  (32, 16, 8, 128, 256, 1)], ids=["3x3@8+4", "1x1@8+4", "1x1@16+8"])
def test_img_twin_bitwise_equals_single(case):
    N, hw0, hw1, cin, cout, k = case
    L = H.load_library()
    assert _fam(L, N, hw0, cin, cout, k, N, hw1) == "img"
    g = torch.Generator(device=DEV).manual_seed(9)
    w = torch.randn(cout, cin, k, k, device=DEV, generator=g) * (1.0 / (cin * k * k) ** 0.5)
    bias = torch.randn(cout, device=DEV, generator=g) * 0.1
    wp, ld = _pack(L, w)
    segs, singles = [], []
    for hw in (hw0, hw1):
        x = (torch.randn(N, hw, hw, cin, device=DEV, generator=g) * 0.7).to(torch.bfloat16)
        sc = torch.rand(cin, device=DEV, generator=g) + 0.5
        sh = torch.randn(cin, device=DEV, generator=g) * 0.3
        segs.append((x, sc, sh))
        singles.append(_fwd(L, x, wp, ld, bias, None, sc, sh, cout, k))
    cs, outs = [], []
    for (x, sc, sh) in segs:
        N_, hw, _, _ = x.shape
        M = N_ * hw * hw
        y = torch.empty(N_, hw, hw, cout, device=DEV, dtype=torch.bfloat16)
        part = torch.full(((2 * (M // 64) + 4) * 3 * cout,), float("nan"), device=DEV)
        rows = H.ctypes.c_int(0)
        outs.append((y, part, rows))
        cs.append(H.ConvSeg(x.data_ptr(), None, y.data_ptr(), H.ptr(sc), H.ptr(sh),
                            part.data_ptr(), H.ctypes.pointer(rows), N_, hw, hw, None, None, None,
                            None, None, None, 0, None))
    ws_b = L.hgk_conv_fwd_twin_workspace(BF16, N, hw0, hw0, N, hw1, hw1, cin, cout, k, k, 1, k // 2, 1)
    ws = torch.zeros(max(ws_b, 1), dtype=torch.uint8, device=DEV)
    H.check(L.hgk_conv_fwd_twin(H.stream_handle(), BF16, wp.data_ptr(), ld, bias.data_ptr(), 1, 0,
                                cin, cout, k, k, 1, k // 2, 1, (H.ConvSeg * 2)(*cs), ws.data_ptr(),
                                ws_b))
    torch.cuda.synchronize()
    for (y, part, rows), (y1, part1, rows1) in zip(outs, singles):
        assert rows.value == rows1
        assert torch.equal(y, y1)
        n = rows1 * 3 * cout
        assert torch.equal(part[:n], part1[:n])
