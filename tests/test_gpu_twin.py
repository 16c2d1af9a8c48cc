"""Twin launches (an hourglass level's up-branch and down-branch blocks share ONE ResidualBlock,
try_with_torch.py:217-237, so each conv / BN launch serves both uses) against the single-use
entry points, through the C-ABI:

* hgk_conv_fwd_twin == hgk_conv_fwd / hgk_conv_fwd_bnbwd per segment. The twin launch plans its
  tiles / split-K for the combined M, so the k-summation order may differ: fp32 within 1e-5
  relative, bf16 within one output rounding (1e-2 relative).
* hgk_bn_finalize_deferred + hgk_bn_running_update == hgk_bn_finalize with immediate running
  updates, and hgk_bn_bwd_twin == hgk_bn_bwd_finalize_apply / finalize + apply per segment:
  BITWISE (the twin kernels run the single kernels' arithmetic per segment).
* whole model: the engine with twin chains (default) against HGK_TWIN=0 and the reference
  fixture (tests/test_gpu_parity.py holds the fixture gates; here the twin-vs-single agreement).
"""
import pytest
import torch

from progressive_process_for_human_pose_estimation_amd import hgk as H

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _pack(L, w, dt, tdt, dgrad=False):
    cout, cin, k, _ = w.shape
    rows, kk = (cin, cout) if dgrad else (cout, cin)
    ld = L.hgk_conv_w_ld(k * k * kk)
    wp = torch.empty(((rows + 127) // 128) * 128, ld, device=DEV, dtype=tdt)
    H.check(L.hgk_pack_conv_weight(H.stream_handle(), dt, w.data_ptr(), wp.data_ptr(), ld, cout, cin,
                                   k, k, 1 if dgrad else 0, cout, cin))
    return wp, ld


def _seg_tensors(g, N, hw, cin, cout, pre, res, tdt):
    x = (torch.randn(N, hw, hw, cin, device=DEV, generator=g) * 0.7).to(tdt)
    sc = torch.rand(cin, device=DEV, generator=g) + 0.5 if pre else None
    sh = torch.randn(cin, device=DEV, generator=g) * 0.3 if pre else None
    r = torch.randn(N, hw, hw, cout, device=DEV, generator=g).to(tdt) if res else None
    return x, sc, sh, r


TWIN_CASES = [
    # N, hw0, hw1, cin, cout, k, pre, res, dtype
    (32, 16, 8, 256, 128, 1, True, False, torch.bfloat16),   # conv1 @ 16+8
    (32, 8, 4, 128, 256, 1, True, True, torch.bfloat16),     # conv3 + residual @ 8+4
    (32, 8, 4, 128, 128, 3, True, False, torch.bfloat16),    # 3x3 @ 8+4: split-K twin
    (32, 16, 8, 128, 128, 3, True, False, torch.bfloat16),   # halo 16x16 + implicit 8x8: 2 launches
    (32, 64, 32, 128, 128, 3, True, False, torch.bfloat16),  # twin halo kernel, 8-row tiles
    (32, 32, 16, 128, 128, 3, True, True, torch.bfloat16),   # twin halo, 2 k-groups, residual
    (8, 64, 32, 256, 128, 3, False, False, torch.bfloat16),  # twin halo, 4 input chunks
    (32, 64, 32, 256, 128, 1, True, False, torch.bfloat16),  # conv1 @ 64+32
    (4, 16, 8, 256, 128, 1, True, True, torch.float32),
    (4, 8, 4, 128, 128, 3, True, False, torch.float32),
    (2, 4, 2, 128, 128, 3, False, True, torch.float32),      # ragged tiles (M 32 + 8)
]


@pytest.mark.parametrize("case", TWIN_CASES)
def test_conv_twin_matches_single_launches(case):
    N, hw0, hw1, cin, cout, k, pre, res, tdt = case
    L = H.load_library()
    dt = H.dtype_code(tdt)
    g = torch.Generator(device=DEV).manual_seed(1)
    w = torch.randn(cout, cin, k, k, device=DEV, generator=g) * (1.0 / (cin * k * k) ** 0.5)
    bias = torch.randn(cout, device=DEV, generator=g) * 0.1
    wp, ld = _pack(L, w, dt, tdt)
    pad = k // 2
    segs = [_seg_tensors(g, N, hw, cin, cout, pre, res, tdt) for hw in (hw0, hw1)]
    st = H.stream_handle()

    def single(i):
        x, sc, sh, r = segs[i]
        hw = (hw0, hw1)[i]
        y = torch.empty(N, hw, hw, cout, device=DEV, dtype=tdt)
        part = torch.zeros((2 * (N * hw * hw // 64) + 4) * 3 * cout, device=DEV)
        rows = H.ctypes.c_int(0)
        ws_b = L.hgk_conv_fwd_workspace(dt, N, hw, hw, cin, cout, k, k, 1, pad, 1)
        ws = torch.zeros(max(ws_b, 1), dtype=torch.uint8, device=DEV)
        H.check(L.hgk_conv_fwd(st, dt, x.data_ptr(), wp.data_ptr(), ld, bias.data_ptr(), H.ptr(r),
                               y.data_ptr(), H.ptr(sc), H.ptr(sh), 1 if pre else 0, 0,
                               part.data_ptr(), H.ctypes.byref(rows), N, hw, hw, cin, cout, k, k, 1,
                               pad, 1, ws.data_ptr(), ws_b))
        return y, part, rows.value

    ref = [single(0), single(1)]
    outs, parts, rows = [], [], [H.ctypes.c_int(0), H.ctypes.c_int(0)]
    cs = []
    for i, hw in enumerate((hw0, hw1)):
        x, sc, sh, r = segs[i]
        y = torch.empty(N, hw, hw, cout, device=DEV, dtype=tdt)
        part = torch.zeros((2 * (N * hw * hw // 64) + 4) * 3 * cout, device=DEV)
        outs.append(y)
        parts.append(part)
        cs.append(H.ConvSeg(x.data_ptr(), H.ptr(r), y.data_ptr(), H.ptr(sc), H.ptr(sh),
                            part.data_ptr(), H.ctypes.pointer(rows[i]), N, hw, hw, None, None, None,
                            None, None, None, 0, None))
    ws_b = L.hgk_conv_fwd_twin_workspace(dt, N, hw0, hw0, N, hw1, hw1, cin, cout, k, k, 1, pad, 1)
    ws = torch.zeros(max(ws_b, 1), dtype=torch.uint8, device=DEV)
    H.check(L.hgk_conv_fwd_twin(st, dt, wp.data_ptr(), ld, bias.data_ptr(), 1 if pre else 0, 0, cin,
                                cout, k, k, 1, pad, 1, (H.ConvSeg * 2)(*cs), ws.data_ptr(), ws_b))
    torch.cuda.synchronize()
    tol = 1e-2 if tdt == torch.bfloat16 else 1e-5
    for i in range(2):
        y_ref, p_ref, r_ref = ref[i]
        a, b = outs[i].float(), y_ref.float()
        assert (a - b).abs().max().item() <= tol * b.abs().max().item() + 1e-6, f"segment {i}"
        # channel sums of the statistics partials (channel-major [C][3][rows])
        R, Rr = rows[i].value, r_ref
        assert R > 0 and Rr > 0
        s_t = parts[i][:cout * 3 * R].view(cout, 3, R)[:, 0].double().sum(1)
        s_r = p_ref[:cout * 3 * Rr].view(cout, 3, Rr)[:, 0].double().sum(1)
        n_t = parts[i][:cout * 3 * R].view(cout, 3, R)[:, 2].double().sum(1)
        assert torch.all(n_t == N * (hw0, hw1)[i] ** 2)
        assert (s_t - s_r).abs().max().item() <= 1e-3 * s_r.abs().max().item() + 1e-3


@pytest.mark.parametrize("tdt", [torch.float32, torch.bfloat16])
def test_conv_twin_bnbwd_matches_single(tdt):
    """input gradient with the BN-backward epilogue (1x1 conv1 dgrad @ 16+8, N=32)"""
    L = H.load_library()
    dt = H.dtype_code(tdt)
    N, cin, cout = 32, 128, 256  # dgrad: dy has 128 channels, dx 256
    g = torch.Generator(device=DEV).manual_seed(2)
    w = torch.randn(cin, cout, 1, 1, device=DEV, generator=g) * 0.06  # conv 256 -> 128
    wd, ld = _pack(L, w, dt, tdt, dgrad=True)
    st = H.stream_handle()
    data = []
    for hw in (16, 8):
        dy = torch.randn(N, hw, hw, cin, device=DEV, generator=g).to(tdt)
        yb = torch.randn(N, hw, hw, cout, device=DEV, generator=g).to(tdt)
        stat = torch.stack([torch.randn(cout, device=DEV, generator=g) * 0.1,
                            torch.rand(cout, device=DEV, generator=g) + 0.5,
                            torch.rand(cout, device=DEV, generator=g) + 0.5,
                            torch.randn(cout, device=DEV, generator=g) * 0.2])
        data.append((hw, dy, yb, stat))

    def run(twin):
        res = []
        cs, rows = [], [H.ctypes.c_int(0), H.ctypes.c_int(0)]
        for i, (hw, dy, yb, stat) in enumerate(data):
            dx = torch.empty(N, hw, hw, cout, device=DEV, dtype=tdt)
            part = torch.zeros((2 * (N * hw * hw // 64) + 4) * 2 * cout, device=DEV)
            res.append((dx, part))
            if not twin:
                H.check(L.hgk_conv_fwd_bnbwd(st, dt, dy.data_ptr(), wd.data_ptr(), ld, None,
                                             dx.data_ptr(), N, hw, hw, cin, cout, 1, 1, 1, 0, 1,
                                             None, 0, yb.data_ptr(), stat[2].data_ptr(),
                                             stat[3].data_ptr(), 1, stat[0].data_ptr(),
                                             stat[1].data_ptr(), part.data_ptr(),
                                             H.ctypes.byref(rows[i])))
            else:
                cs.append(H.ConvSeg(dy.data_ptr(), None, dx.data_ptr(), None, None, None, None, N, hw,
                                    hw, yb.data_ptr(), stat[2].data_ptr(), stat[3].data_ptr(),
                                    stat[0].data_ptr(), stat[1].data_ptr(), part.data_ptr(), 1,
                                    H.ctypes.pointer(rows[i])))
        if twin:
            H.check(L.hgk_conv_fwd_twin(st, dt, wd.data_ptr(), ld, None, 0, 0, cin, cout, 1, 1, 1, 0,
                                        1, (H.ConvSeg * 2)(*cs), None, 0))
        torch.cuda.synchronize()
        return [(dx, part, r.value) for (dx, part), r in zip(res, rows)]

    a, b = run(False), run(True)
    tol = 1e-2 if tdt == torch.bfloat16 else 1e-5
    for (dx0, p0, r0), (dx1, p1, r1) in zip(a, b):
        assert (dx0.float() - dx1.float()).abs().max().item() <= tol * dx0.float().abs().max().item()
        s0 = p0[:r0 * 2 * cout].view(r0, 2, cout).double().sum(0)
        s1 = p1[:r1 * 2 * cout].view(r1, 2, cout).double().sum(0)
        assert (s0 - s1).abs().max().item() <= 1e-3 * s0.abs().max().item() + 1e-3


@pytest.mark.parametrize("hws", [(16, 8), (8, 4), (64, 32)])
def test_bn_finalize_deferred_and_running_update_bitwise(hws):
    L = H.load_library()
    st = H.stream_handle()
    N, C = 32, 128
    g = torch.Generator(device=DEV).manual_seed(3)
    gamma = torch.rand(C, device=DEV, generator=g) + 0.5
    beta = torch.randn(C, device=DEV, generator=g) * 0.1
    segs = []
    for hw in hws:
        x = (torch.randn(N * hw * hw, C, device=DEV, generator=g) * 2 + 0.5).to(torch.bfloat16)
        part = torch.empty(2048 * 3 * C, device=DEV)
        rows = H.ctypes.c_int(0)
        H.check(L.hgk_bn_stats(st, 1, x.data_ptr(), x.shape[0], C, part.data_ptr(), H.ctypes.byref(rows)))
        segs.append((part, rows.value, x.shape[0]))
    rm0 = torch.randn(C, device=DEV, generator=g)
    rv0 = torch.rand(C, device=DEV, generator=g) + 0.5
    # single finalizes, immediate updates: use 0, use 1, use 0 again (order matters)
    rm, rv = rm0.clone(), rv0.clone()
    stats_ref = []
    for part, rows, M in (segs[0], segs[1], segs[0]):
        stat = torch.empty(4, C, device=DEV)
        H.check(L.hgk_bn_finalize(st, part.data_ptr(), rows, M, C, gamma.data_ptr(), beta.data_ptr(),
                                  rm.data_ptr(), rv.data_ptr(), 0.1, 1e-5, 1, stat[0].data_ptr(),
                                  stat[1].data_ptr(), stat[2].data_ptr(), stat[3].data_ptr(), None))
        stats_ref.append(stat)
    # deferred: a twin finalize (uses 0 and 1) + a single one, then the records in order
    rm2, rv2 = rm0.clone(), rv0.clone()
    recs = [torch.empty(2, C, device=DEV, dtype=torch.float64) for _ in range(3)]
    stats = [torch.empty(4, C, device=DEV) for _ in range(3)]
    bs = [H.BnSeg(p.data_ptr(), r, M, recs[i].data_ptr(), stats[i].data_ptr())
          for i, (p, r, M) in enumerate((segs[0], segs[1]))]
    H.check(L.hgk_bn_finalize_deferred(st, (H.BnSeg * 2)(*bs), 2, C, gamma.data_ptr(),
                                       beta.data_ptr(), 1e-5))
    b3 = H.BnSeg(segs[0][0].data_ptr(), segs[0][1], segs[0][2], recs[2].data_ptr(), stats[2].data_ptr())
    H.check(L.hgk_bn_finalize_deferred(st, (H.BnSeg * 1)(b3), 1, C, gamma.data_ptr(),
                                       beta.data_ptr(), 1e-5))
    ents = [H.BnRunning(rm2.data_ptr(), rv2.data_ptr(), r.data_ptr(), C, 0.1) for r in recs]
    H.check(L.hgk_bn_running_update(st, (H.BnRunning * 3)(*ents), 3))
    torch.cuda.synchronize()
    for a, b in zip(stats, stats_ref):
        assert torch.equal(a, b)
    assert torch.equal(rm, rm2) and torch.equal(rv, rv2)


def test_bn_running_update_many_records_in_order():
    """hgk_bn_running_update over 230 records of 7 modules (interleaved, channel counts 64..512):
    more records than one launch holds (96) and than one load batch (8) per module. Bitwise equal
    to applying the records one call at a time in order, and within fp32 rounding of a float64
    host restatement of the EMA (running = (1 - m) * running + m * record, rounded to fp32 per
    record, as PyTorch's in-place update)."""
    import numpy as np
    L = H.load_library()
    st = H.stream_handle()
    g = torch.Generator(device=DEV).manual_seed(11)
    cs = [64, 128, 256, 512, 128, 256, 64]
    mods = [(torch.randn(c, device=DEV, generator=g), torch.rand(c, device=DEV, generator=g) + 0.5)
            for c in cs]
    order = torch.randint(0, len(cs), (230,), generator=torch.Generator().manual_seed(5)).tolist()
    recs = [torch.randn(2, cs[k], device=DEV, generator=g, dtype=torch.float64).abs_() for k in order]
    mom = 0.1
    batch = [(m[0].clone(), m[1].clone()) for m in mods]
    ents = [H.BnRunning(batch[k][0].data_ptr(), batch[k][1].data_ptr(), r.data_ptr(), cs[k], mom)
            for k, r in zip(order, recs)]
    H.check(L.hgk_bn_running_update(st, (H.BnRunning * len(ents))(*ents), len(ents)))
    one = [(m[0].clone(), m[1].clone()) for m in mods]
    for k, r in zip(order, recs):
        e = H.BnRunning(one[k][0].data_ptr(), one[k][1].data_ptr(), r.data_ptr(), cs[k], mom)
        H.check(L.hgk_bn_running_update(st, (H.BnRunning * 1)(e), 1))
    torch.cuda.synchronize()
    m64 = float(np.float32(mom))
    host = [(m[0].cpu().numpy().copy(), m[1].cpu().numpy().copy()) for m in mods]
    for k, r in zip(order, recs):
        rr = r.cpu().numpy()
        for j in range(2):
            host[k][j][:] = ((1.0 - m64) * host[k][j].astype(np.float64) + m64 * rr[j]).astype(np.float32)
    for k in range(len(cs)):
        for j in range(2):
            assert torch.equal(batch[k][j], one[k][j]), (k, j)
            ref = torch.from_numpy(host[k][j])
            assert torch.allclose(batch[k][j].cpu(), ref, rtol=2e-6, atol=1e-6), (k, j)


@pytest.mark.parametrize("hws,C", [((16, 8), 128), ((8, 4), 256), ((64, 32), 128)])
def test_bn_bwd_twin_bitwise(hws, C):
    """fused (<= 128 partial rows) and finalize+apply forms vs the single-use kernels"""
    L = H.load_library()
    st = H.stream_handle()
    N = 32
    g = torch.Generator(device=DEV).manual_seed(4)
    data = []
    for hw in hws:
        M = N * hw * hw
        rows = max(1, M // 64)
        part = torch.randn(rows, 2, C, device=DEV, generator=g) * 0.1
        stat = torch.stack([torch.randn(C, device=DEV, generator=g) * 0.1,
                            torch.rand(C, device=DEV, generator=g) + 0.5,
                            torch.rand(C, device=DEV, generator=g) + 0.5,
                            torch.randn(C, device=DEV, generator=g) * 0.2])
        dA = torch.randn(M, C, device=DEV, generator=g).to(torch.bfloat16)
        y = torch.randn(M, C, device=DEV, generator=g).to(torch.bfloat16)
        old = torch.randn(M, C, device=DEV, generator=g).to(torch.bfloat16)
        data.append((M, rows, part, stat, dA, y, old))
    dg0 = torch.randn(C, device=DEV, generator=g)
    db0 = torch.randn(C, device=DEV, generator=g)
    fmax = L.hgk_bn_bwd_fused_max_rows()

    # singles (accumulate into a copy of `old`)
    dg, db = dg0.clone(), db0.clone()
    outs_ref = []
    for M, rows, part, stat, dA, y, old in data:
        dy = old.clone()
        if all(d[1] <= fmax for d in data):
            H.check(L.hgk_bn_bwd_finalize_apply(st, 1, part.data_ptr(), rows, M, C, stat[2].data_ptr(),
                                                stat[3].data_ptr(), 1, stat[0].data_ptr(),
                                                stat[1].data_ptr(), 1, dg.data_ptr(), db.data_ptr(),
                                                dA.data_ptr(), y.data_ptr(), None, dy.data_ptr(), 1))
        else:
            coef = torch.empty(4, C, device=DEV)
            H.check(L.hgk_bn_bwd_finalize(st, part.data_ptr(), rows, M, C, stat[2].data_ptr(),
                                          stat[0].data_ptr(), stat[1].data_ptr(), 1, dg.data_ptr(),
                                          db.data_ptr(), coef.data_ptr(), None))
            H.check(L.hgk_bn_bwd_apply(st, 1, dA.data_ptr(), y.data_ptr(), M, C, stat[2].data_ptr(),
                                       stat[3].data_ptr(), 1, coef.data_ptr(), None, dy.data_ptr(), 1))
        outs_ref.append(dy)
    dg2, db2 = dg0.clone(), db0.clone()
    outs = [d[6].clone() for d in data]
    segs = [H.BnbSeg(part.data_ptr(), rows, M, stat.data_ptr(), dA.data_ptr(), y.data_ptr(), None,
                     o.data_ptr(), 1) for (M, rows, part, stat, dA, y, old), o in zip(data, outs)]
    coef = torch.empty(2, 6, C, device=DEV)
    H.check(L.hgk_bn_bwd_twin(st, 1, (H.BnbSeg * 2)(*segs), 2, C, 1, 1, dg2.data_ptr(),
                              db2.data_ptr(), coef.data_ptr()))
    torch.cuda.synchronize()
    for a, b in zip(outs, outs_ref):
        assert torch.equal(a, b)
    if all(d[1] <= fmax for d in data):
        assert torch.equal(dg, dg2) and torch.equal(db, db2)
    else:
        # the wave finaliser (<= 256 rows) and the workgroup one sum the rows in different orders
        assert torch.allclose(dg, dg2, rtol=1e-6, atol=1e-6) and torch.allclose(db, db2, rtol=1e-6, atol=1e-6)


def test_engine_twin_matches_single_schedule(routes):
    """1-stack hourglass, 128x128, N=8 (levels 32..2, twin chains at every level): one fp32 train
    step with twin chains (HGK_TWIN=1) and one without, each gated on the REFERENCE's own fp32
    rounding noise per parameter (tests/golden/primary_s1_n8_128.npz: ||g32 - g64|| / ||g64||
    of the reference classes, make_golden.py twin), not on the other schedule. The fp64 gradients
    come from the CPU oracle (the test checker), pinned to the fixture's fp64 grad norms."""
    import os
    import numpy as np
    from conftest import GOLDEN
    import progressive_process_for_human_pose_estimation_amd as P
    from progressive_process_for_human_pose_estimation_amd.data import gaussian_targets, synthetic_images
    from oracle.hourglass_oracle import OracleModel, stack_mse

    fx = dict(np.load(os.path.join(GOLDEN, "primary_s1_n8_128.npz")))
    x = synthetic_images(8, 128, 128, seed=1234)
    t = gaussian_targets(8, 17, 32, 32, seed=1)[0]

    def step(twin):
        routes(twin="1" if twin else "0")
        torch.manual_seed(0)
        m = P.creatModel(nStack=1).cuda()
        outs = m(x.cuda())
        loss = sum(torch.nn.functional.mse_loss(o, t.cuda()) for o in outs)
        loss.backward()
        torch.cuda.synchronize()
        grads = [None if p.grad is None else p.grad.detach().double().cpu() for p in m.parameters()]
        bufs = {k: b.detach().cpu() for k, b in m.named_buffers()}
        return outs[0].detach().double().cpu(), float(loss.detach()), grads, bufs

    torch.manual_seed(0)
    o = OracleModel(nStack=1).double()
    ref = o(x.double())
    rloss = stack_mse(ref, t.double())
    rloss.backward()
    rg = [p.grad for p in o.parameters()]
    n64 = fx["grad_norm64"]
    on = np.array([-1.0 if g is None else float(g.norm()) for g in rg])
    assert np.allclose(on, n64, rtol=1e-9, atol=1e-12), "oracle fp64 grads off the reference's"
    assert abs(float(rloss.detach()) - float(fx["loss64"])) <= 1e-12
    noise = fx["grad_noise32"]
    live = n64 > 1e-5 * n64.max()
    med_noise = float(np.median(noise[live]))
    r = ref[0].detach()
    b = 1e-3 + 2 * np.abs(fx["train32_sample"] - fx["train64_sample"]).max()
    st = int(fx["sample_stride"])
    for twin in (True, False):
        out, loss, grads, bufs = step(twin)
        assert (out - r).abs().max().item() <= b, twin
        assert np.abs(out.numpy().reshape(-1)[::st] - fx["train64_sample"]).max() <= b
        assert abs(loss - float(fx["loss64"])) <= 1e-4 + 2 * abs(float(fx["loss32"]) - float(fx["loss64"]))
        errs = []
        for i, (gg, g64) in enumerate(zip(grads, rg)):
            assert (gg is None) == (g64 is None), i
            if gg is None or not live[i]:
                continue
            e = float((gg - g64).norm() / g64.norm())
            errs.append(e / max(noise[i], med_noise))
            assert e <= 4 * max(noise[i], med_noise) + 1e-5, (twin, fx["param_names"][i], e, noise[i])
        print(f"twin={twin}: grad error / reference fp32 noise: median {np.median(errs):.3f}, "
              f"max {np.max(errs):.3f}")
        assert np.median(errs) <= 2.0
        nbt = [int(v) for k, v in bufs.items() if k.endswith("num_batches_tracked")]
        assert nbt == list(fx["bn_num_batches_tracked"])
        for kind in ("running_mean", "running_var"):
            got = torch.cat([v.reshape(-1) for k, v in bufs.items() if k.endswith(kind)]).numpy()
            r32, r64 = fx["bn_" + kind + "32"], fx["bn_" + kind + "64"]
            assert np.all(np.abs(got - r64) <= 1e-4 + 1e-4 * np.abs(r64) + 4 * np.abs(r32 - r64).max()), kind


def test_wgrad_finish_multi_bitwise_equals_single_calls():
    """hgk_conv_wgrad_finish_multi (every weight of a flush point in one launch) against the
    per-weight hgk_conv_wgrad_finish: bitwise, for >= 64 and < 64 slabs, ragged K, bias, logical
    channel counts below the stored ones."""
    L = H.load_library()
    st = H.stream_handle()
    g = torch.Generator(device=DEV).manual_seed(6)
    shapes = [  # Cin, Cout, KH, KW, nslabs, Cin_log, Cout_log, bias
        (256, 128, 1, 1, 200, 256, 128, True), (128, 128, 3, 3, 40, 128, 128, True),
        (64, 64, 7, 7, 3, 3, 64, False), (256, 64, 1, 1, 64, 256, 17, True),
        (128, 256, 1, 1, 1, 128, 256, False),
        # < 64 slabs: four column chunks per workgroup (a partial last workgroup, bias chunks
        # beyond the logical channels)
        (256, 256, 1, 1, 39, 256, 256, True), (128, 128, 3, 3, 26, 128, 100, True),
        (64, 256, 1, 1, 63, 64, 250, True), (256, 64, 1, 1, 5, 200, 64, True)]
    ents, outs_ref, outs = [], [], []
    for Cin, Cout, KH, KW, S, Cil, Col, bias in shapes:
        cap = max(S, 4)
        K = KH * KW * Cin
        nb = L.hgk_conv_wgrad_slab_bytes(Cin, Cout, KH, KW, cap)
        slab = torch.randn(nb // 4, device=DEV, generator=g)
        dw0 = torch.randn(Col, Cil, KH, KW, device=DEV, generator=g)
        db0 = torch.randn(Col, device=DEV, generator=g) if bias else None
        a_dw, a_db = dw0.clone(), None if db0 is None else db0.clone()
        H.check(L.hgk_conv_wgrad_finish(st, slab.data_ptr(), cap, S, a_dw.data_ptr(), H.ptr(a_db),
                                        Cin, Cout, KH, KW, Cil, Col))
        outs_ref.append((a_dw, a_db))
        b_dw, b_db = dw0.clone(), None if db0 is None else db0.clone()
        outs.append((b_dw, b_db, slab))
        ents.append(H.WgradFin(slab.data_ptr(), cap, S, b_dw.data_ptr(), H.ptr(b_db), Cin, Cout, KH, KW,
                               Cil, Col))
    H.check(L.hgk_conv_wgrad_finish_multi(st, (H.WgradFin * len(ents))(*ents), len(ents)))
    torch.cuda.synchronize()
    for (a_dw, a_db), (b_dw, b_db, _) in zip(outs_ref, outs):
        assert torch.equal(a_dw, b_dw)
        assert (a_db is None) == (b_db is None) and (a_db is None or torch.equal(a_db, b_db))
