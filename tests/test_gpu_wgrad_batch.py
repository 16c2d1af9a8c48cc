"""Weight gradients of DIFFERENT weights batched into shared launches (hgk_conv_wgrad_accum_batch:
the unshared blocks of hourglass_compare / train.py, one use per weight): every job's slabs and
split count must be BITWISE those of its own hgk_conv_wgrad_accum_multi(nsrc = 1) call — mixed
shapes (1x1, 3x3, 64- and 128-wide tiles), bias, accumulation into earlier slabs, more jobs than
one launch holds — and the engine's batched flush (route wg_batch, the default) bitwise the
per-weight one over a whole hourglass_compare training step. Both with the library routes
wg_batch_target = 0 (each job planned alone) and wg_batch_slab_x10 = 20 (the per-weight slab cap); with the batch planned as a whole (fewer pixel
splits per weight, the default) the reduced weight gradients equal the single calls' up to fp32
re-association."""
import pytest
import torch
import torch.nn.functional as F

from progressive_process_for_human_pose_estimation_amd import engine as E
from progressive_process_for_human_pose_estimation_amd import hgk as H
from progressive_process_for_human_pose_estimation_amd.data import gaussian_targets, synthetic_images

pytestmark = pytest.mark.gpu
DEV = "cuda"

# (N, H, W, Cin, Cout, K, bias, slabs_init)
JOBS = [(32, 16, 16, 256, 128, 1, True, 0), (32, 8, 8, 128, 128, 3, True, 0),
        (32, 4, 4, 128, 256, 1, False, 0), (32, 32, 32, 256, 128, 1, True, 3),
        (8, 8, 8, 256, 256, 1, True, 0), (32, 16, 16, 128, 128, 3, False, 0),
        # halo-tileable 3x3 jobs (route wg_halo_multi): their own halo launch inside the batch
        (32, 32, 32, 128, 128, 3, True, 0), (4, 64, 64, 64, 64, 3, True, 2)] * 3


def _job(L, g, N, Hh, W, Cin, Cout, K, bias, init, dtype):
    x = (torch.randn(N, Hh, W, Cin, device=DEV, generator=g) * 0.5).to(dtype)
    dy = (torch.randn(N, Hh, W, Cout, device=DEV, generator=g) * 0.1).to(dtype)
    sc = torch.rand(Cin, device=DEV, generator=g) + 0.5
    sh = torch.randn(Cin, device=DEV, generator=g) * 0.2
    cap = L.hgk_conv_wgrad_max_splits()
    slab = torch.randn(L.hgk_conv_wgrad_slab_bytes(Cin, Cout, K, K, cap) // 4, device=DEV, generator=g)
    src = H.WgradSrc(x.data_ptr(), dy.data_ptr(), sc.data_ptr(), sh.data_ptr(), 1, N, Hh, W)
    return dict(keep=(x, dy, sc, sh), slab=slab, src=src, cap=cap, init=init, bias=bias, Cin=Cin,
                Cout=Cout, K=K)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_wgrad_batch_bitwise_equals_single_calls(dtype):
    L = H.load_library()
    st = H.stream_handle()
    dt = H.BF16 if dtype == torch.bfloat16 else H.F32
    g = torch.Generator(device=DEV).manual_seed(5)
    jobs = [_job(L, g, *j, dtype) for j in JOBS]
    ref_slabs, ref_splits = [], []
    for j in jobs:
        s = j["slab"].clone()
        sp = H.ctypes.c_int(0)
        arr = (H.WgradSrc * 1)(j["src"])
        H.check(L.hgk_conv_wgrad_accum_multi(st, dt, arr, 1, s.data_ptr(), j["cap"], j["init"],
                                             1 if j["bias"] else 0, H.ctypes.byref(sp), j["Cin"],
                                             j["Cout"], j["K"], j["K"], 1, j["K"] // 2, 1))
        ref_slabs.append(s)
        ref_splits.append(sp.value)
    descs = [H.WgradJob(j["src"], j["slab"].data_ptr(), j["cap"], j["init"], 1 if j["bias"] else 0,
                        j["Cin"], j["Cout"], j["K"], j["K"], 1, j["K"] // 2, 1) for j in jobs]
    splits = (H.ctypes.c_int * len(jobs))()
    with H.route(wg_batch_target=0, wg_batch_slab_x10=20):
        H.check(L.hgk_conv_wgrad_accum_batch(st, dt, (H.WgradJob * len(jobs))(*descs), len(jobs), splits))
    torch.cuda.synchronize()
    for i, j in enumerate(jobs):
        assert splits[i] == ref_splits[i], i
        assert torch.equal(j["slab"], ref_slabs[i]), i


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_hourglass_compare_batched_wgrads_bitwise(dtype):
    from progressive_process_for_human_pose_estimation_amd.presets import hourglass_compare as HC
    x = synthetic_images(2, 128, 128, seed=31).to(DEV)
    t = gaussian_targets(2, 16, 32, seed=32)[0].to(DEV)
    res = []
    for batched in (True, False):
        with E.routing(wg_batch=batched), H.route(wg_batch_target=0, wg_batch_slab_x10=20):
            torch.manual_seed(0)
            m = HC.creatModel().to(DEV).set_engine_dtype(dtype).set_graph_mode(False).train()
            outs = m(x)
            sum(F.mse_loss(o, t) for o in outs).backward()
            torch.cuda.synchronize()
            res.append([None if p.grad is None else p.grad.cpu() for p in m.parameters()])
    for a, b in zip(*res):
        assert (a is None) == (b is None) and (a is None or torch.equal(a, b))


def _reduce(L, st, j, slab, nslabs):
    dw = torch.zeros(j["Cout"], j["Cin"], j["K"], j["K"], device=DEV)
    db = torch.zeros(j["Cout"], device=DEV)
    H.check(L.hgk_conv_wgrad_finish(st, slab.data_ptr(), j["cap"], nslabs, dw.data_ptr(),
                                    db.data_ptr() if j["bias"] else None, j["Cin"], j["Cout"], j["K"],
                                    j["K"], j["Cin"], j["Cout"]))
    return dw, db


@pytest.mark.parametrize("target", [1024, 256])
def test_wgrad_batch_planned_as_a_whole(target):
    """route wg_batch_target: fewer splits per job (never more than alone), reduced dW / db equal
    the single calls' within fp32 re-association (1e-5 of the largest element)."""
    L = H.load_library()
    st = H.stream_handle()
    g = torch.Generator(device=DEV).manual_seed(9)
    jobs = [_job(L, g, *j, torch.bfloat16) for j in JOBS]
    refs = []
    for j in jobs:
        s = j["slab"].clone()
        sp = H.ctypes.c_int(0)
        arr = (H.WgradSrc * 1)(j["src"])
        H.check(L.hgk_conv_wgrad_accum_multi(st, H.BF16, arr, 1, s.data_ptr(), j["cap"], j["init"],
                                             1 if j["bias"] else 0, H.ctypes.byref(sp), j["Cin"],
                                             j["Cout"], j["K"], j["K"], 1, j["K"] // 2, 1))
        refs.append((_reduce(L, st, j, s, sp.value), sp.value))
    descs = [H.WgradJob(j["src"], j["slab"].data_ptr(), j["cap"], j["init"], 1 if j["bias"] else 0,
                        j["Cin"], j["Cout"], j["K"], j["K"], 1, j["K"] // 2, 1) for j in jobs]
    splits = (H.ctypes.c_int * len(jobs))()
    with H.route(wg_batch_target=target, wg_batch_slab_x10=20):
        H.check(L.hgk_conv_wgrad_accum_batch(st, H.BF16, (H.WgradJob * len(jobs))(*descs), len(jobs),
                                             splits))
    fewer = 0
    for i, j in enumerate(jobs):
        (dw0, db0), sp0 = refs[i]
        assert j["init"] <= splits[i] <= max(sp0, j["init"]), (i, splits[i], sp0)
        fewer += splits[i] < sp0
        dw, db = _reduce(L, st, j, j["slab"], splits[i])
        torch.cuda.synchronize()
        tol = 1e-5 * dw0.abs().max().item()
        assert (dw - dw0).abs().max().item() <= tol, i
        if j["bias"]:
            assert (db - db0).abs().max().item() <= 1e-5 * db0.abs().max().item() + 1e-6, i
    assert fewer > 0


@pytest.mark.parametrize("cap", [5, 10])
def test_wgrad_batch_slab_cap(cap):
    """route wg_batch_slab_x10 (default 5): fewer pixel splits for a batched job (its slabs capped
    at cap / 10 x its operand bytes), reduced dW / db equal the single calls' to fp32
    re-association"""
    L = H.load_library()
    st = H.stream_handle()
    g = torch.Generator(device=DEV).manual_seed(19)
    jobs = [_job(L, g, *j, torch.bfloat16) for j in JOBS[:6]]
    refs = []
    for j in jobs:
        s = j["slab"].clone()
        sp = H.ctypes.c_int(0)
        arr = (H.WgradSrc * 1)(j["src"])
        H.check(L.hgk_conv_wgrad_accum_multi(st, H.BF16, arr, 1, s.data_ptr(), j["cap"], j["init"],
                                             1 if j["bias"] else 0, H.ctypes.byref(sp), j["Cin"],
                                             j["Cout"], j["K"], j["K"], 1, j["K"] // 2, 1))
        refs.append((_reduce(L, st, j, s, sp.value), sp.value))
    descs = [H.WgradJob(j["src"], j["slab"].data_ptr(), j["cap"], j["init"], 1 if j["bias"] else 0,
                        j["Cin"], j["Cout"], j["K"], j["K"], 1, j["K"] // 2, 1) for j in jobs]
    splits = (H.ctypes.c_int * len(jobs))()
    with H.route(wg_batch_slab_x10=cap):
        H.check(L.hgk_conv_wgrad_accum_batch(st, H.BF16, (H.WgradJob * len(jobs))(*descs), len(jobs),
                                             splits))
    for i, j in enumerate(jobs):
        (dw0, db0), sp0 = refs[i]
        assert splits[i] <= max(sp0, j["init"])
        dw, db = _reduce(L, st, j, j["slab"], splits[i])
        torch.cuda.synchronize()
        assert (dw - dw0).abs().max().item() <= 1e-5 * dw0.abs().max().item(), i
        if j["bias"]:
            assert (db - db0).abs().max().item() <= 1e-5 * db0.abs().max().item() + 1e-6, i


def test_wgrad_batch_invalid_job_launches_nothing():
    """Every job is validated before the first launch: a batch whose LAST job is
    invalid returns an error with the earlier jobs' slabs untouched and splits_out unwritten —
    including a full-width (route wg_full) job, which takes a launch of its own."""
    L = H.load_library()
    st = H.stream_handle()
    g = torch.Generator(device=DEV).manual_seed(23)
    jobs = [_job(L, g, *j, torch.bfloat16) for j in [(32, 16, 16, 256, 128, 1, True, 0),
                                                       (32, 8, 8, 128, 128, 3, True, 0)]]
    before = [j["slab"].clone() for j in jobs]
    descs = [H.WgradJob(j["src"], j["slab"].data_ptr(), j["cap"], j["init"], 1 if j["bias"] else 0,
                        j["Cin"], j["Cout"], j["K"], j["K"], 1, j["K"] // 2, 1) for j in jobs]
    bad = H.WgradJob(jobs[0]["src"], None, jobs[0]["cap"], 0, 1, 256, 128, 1, 1, 1, 0, 1)  # no slabs
    splits = (H.ctypes.c_int * 3)(-7, -7, -7)
    with H.route(wg_full=1):  # job 0 (1x1 256->128, 8192 px) takes the full-width launch
        rc = L.hgk_conv_wgrad_accum_batch(st, H.BF16, (H.WgradJob * 3)(*descs, bad), 3, splits)
    torch.cuda.synchronize()
    assert rc != 0 and "bad slabs" in L.hgk_last_error().decode()
    assert list(splits) == [-7, -7, -7]
    for j, b in zip(jobs, before):
        assert torch.equal(j["slab"], b)
