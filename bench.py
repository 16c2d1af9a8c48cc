"""Benchmark: images/sec of the fused training step (fwd + 4x MSE + bwd [+ RCCL all-reduce] + Adam)
of the 4-stack hourglass (try_with_torch.creatModel) at 256x256, bs=32 per GPU, bf16 storage /
fp32 accumulate (BASELINE.json configs[1] at N=1, configs[2] for N>1).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

With --gpus N > 1 and no WORLD_SIZE in the environment, bench.py starts the N ranks itself (a
`torch.distributed.run` child process, one rank per GPU, before anything touches a GPU) and exits
with the child's status. Rank 0 prints ONE JSON line. `value` = images processed by all ranks /
max-over-ranks wall time of the K timed steps (inputs resident in HBM before the timed region).

`roofline` = the kernel family with the largest share of the step (rocprofv3 table
profiles/r06_step_kernel_stats_v8.csv: the 1x1 convs of the 128x128 .. 32x32 levels on the LDS-DMA ring
kernel, `conv1x1_ring_kernel<K,Cout,mode,NW>`, 24.7 % over its instantiations), here the residual block's
conv1 (<256,128,9>: BN+ReLU fused into the slot transform, BN-statistics epilogue) timed live with
HIP events on its stream, each launch after a read-only 512 MB cache flush (its operands come from
HBM, as in the step: 32.3 us vs 32.3 us in the step table); algorithmic bytes per launch = x + y + w.
`roofline_second` = the second family (14.3 %: the small-level image-tile convs, `conv_img_kernel`),
its largest instantiation's
launch shape (1x1 256->128 at 16x16); `roofline_mfma` = the 3x3 bottleneck conv (the MFMA-heaviest
kernel). `cpu_baseline` times the CPU restatement (oracle/hourglass_oracle.py) per
BASELINE.md §3 on rank 0 at N=1; `dropin` times the reference's own loop (model(x), 4x
nn.MSELoss, backward, torch.optim.Adam) on the drop-in HIP modules: graph-captured module calls
(the default) and, as `dropin.eager`, with graph_calls off.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "images/sec fwd+bwd, 4-stack hourglass 256×256 bs=32/GPU at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s HBM3E (spec)
BF16_MFMA_PEAK_TFS = 2500.0    # dense bf16 MFMA (spec, no sparsity)
FP32_MFMA_PEAK_TFS = 157.3     # dense fp32 matrix (spec)
# (stacks, res, dtype) -> (algorithmic bytes / image, FLOPs / image, step bound) per SURVEY.md §8(d)
ALG_PER_CONFIG = {("primary", 4, 256, "bf16"): (2.478e9, 151.26e9, "hbm"),
                  ("primary", 4, 256, "fp32"): (4.956e9, 151.26e9, "mfma"),
                  ("try_with_aspp", 3, 256, "bf16"): (1.899e9, 115.61e9, "hbm"),
                  ("hourglass_compare", 4, 256, "bf16"): (2.058e9, 107.62e9, "hbm"),
                  ("try_more_layer", 4, 256, "bf16"): (2.445e9, 149.49e9, "hbm"),
                  ("primary", 8, 384, "fp32"): (21.156e9, 653.54e9, "mfma")}
ROOFLINE_PMC = os.path.join(ROOT, "profiles", "r06_roofline_pmc_v8.json")
# the dominant kernel family's share of the headline step (rocprofv3 step table), per
# instantiation <K, Cout, mode> (mode bits: 1 BN transform in, 2 residual / accumulate source,
# 4 fused BN-backward sums, 8 BN statistics out, 16 folded BN-backward apply; twin launches included)
STEP_SHARE = {"table": "profiles/r06_step_kernel_stats_v8.csv",
              "<128,256,20> conv1 input grad (bn2 apply folded in; 64x64, 64+32, 32x32)": {"launches_per_step": 32, "us_per_step": 1183.3, "share": 0.0586},
              "<128,256,11> conv3 fwd (64x64, 64+32, 32x32)": {"launches_per_step": 33, "us_per_step": 983.1, "share": 0.0487},
              "<256,128,4,4> conv3 input grad (64x64, 64+32, 32x32, 16+8)": {"launches_per_step": 41, "us_per_step": 921.1, "share": 0.0456},
              "<256,128,9,4> conv1 fwd (timed; 64x64, 64+32, 32x32, 16+8)": {"launches_per_step": 40, "us_per_step": 874.2, "share": 0.0433},
              "<256,256,*> lin / ll_, the 64-channel stem-block / head launches and the rest": {"launches_per_step": 32, "us_per_step": 1026.7, "share": 0.0508},
              "combined_share": 0.247}
# step share per kernel family (same table; share of the kernels' busy time)
FAMILY_SHARE = {"table": "profiles/r06_step_kernel_stats_v8.csv",
                "conv1x1_ring_kernel": 0.247, "conv_img_kernel": 0.1431, "conv3x3_row_kernel": 0.0965,
                "bn_bwd_apply(_twin)_kernel": 0.0928, "conv3x3_halo_kernel": 0.0773,
                "conv1x1_wgrad_ring_kernel": 0.061, "conv3x3_wgrad_halo_multi_kernel": 0.0537,
                "sample_stats_kernel": 0.0255, "bn_finalize_multi_kernel": 0.0218}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (32; 16 for try_with_aspp)")
    ap.add_argument("--res", type=int, default=256)
    ap.add_argument("--stacks", type=int, default=None, help="4 (primary) / 3 (try_with_aspp)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--preset", default="primary",
                    choices=["primary", "try_with_aspp", "hourglass_compare", "try_more_layer",
                             "train"],
                    help="primary = try_with_torch.creatModel (4xMSE); try_with_aspp = BASELINE "
                         "configs[3] (3 progressive stacks, CE/CE/MSE heads, Adam lr 1e-4); "
                         "hourglass_compare = its 4 unshared stages, nearest up-sampling, 16 "
                         "heatmaps, 4xMSE, Adam lr 1e-4 eps 1e-4 (hourglass_compare.py:885); "
                         "try_more_layer = the live-ASPP progressive model (4 stacks, CE/CE/MSE on "
                         "outputs 0-2, Adam lr 1e-4; try_more_layer.py:387,398-401); train = "
                         "train.py's stride-2 model (3 stages, bootstrapped top-k CE + CE on "
                         "outputs 1-2, Adam lr 1e-4 eps 1e-4; train.py:834,886-890) through the "
                         "drop-in modules (graph-captured calls) and the HIP loss kernels")
    ap.add_argument("--no-fp32-leg", action="store_true",
                    help="skip the fp32 leg of the headline config (the reference's precision)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-overlap", action="store_true",
                    help="all-reduce after the whole backward (no side-stream overlap)")
    ap.add_argument("--branches", action="store_true",
                    help="hourglass up-branches on side streams (Trainer(branches=True))")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-bs32-steps", type=int, default=3)
    ap.add_argument("--dropin-steps", type=int, default=10)
    ap.add_argument("--route", default="",
                    help="A/B only: 'name=value,...' engine routes (twin, fold_apply, fold_fin) and "
                         "library routes (ring_nw, ring_minm, ring_small, row3, splitk_fixup); the "
                         "defaults are compiled in, nothing is read from the environment")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: launcher + gloo grad all-reduce of the real flat layout only")
    a = ap.parse_args()
    if a.batch is None:
        a.batch = 16 if a.preset in ("try_with_aspp", "try_more_layer", "train") else 32
    if a.stacks is None:
        a.stacks = {"try_with_aspp": 3, "train": 3}.get(a.preset, 4)
    if a.preset == "hourglass_compare" and a.stacks != 4:
        ap.error("hourglass_compare has 4 hard-wired stages")
    if a.preset == "train" and a.stacks != 3:
        ap.error("train.py's model has 3 hard-wired stages")
    if a.preset == "train" and a.gpus > 1:
        ap.error("the train preset's line is a single-GPU drop-in loop (no DP all-reduce)")
    return a


# ------------------------------------------------------------------------------ launcher
def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv):
    """Run this script as n ranks under torch.distributed.run (one process per GPU) and return
    its exit status. Called before any GPU call, so the parent never initialises the device."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}",
           os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    return subprocess.call(cmd, env=env)


# ------------------------------------------------------------------------------ roofline kernels
def _conv_launcher(dtype, N, hw, Cin, Cout, k, pre, stats):
    """A bound hgk_conv_fwd launch of one residual-block conv at N x hw x hw (bf16 inputs,
    BN+ReLU fused into staging when `pre`, BN-statistics epilogue when `stats`)."""
    from progressive_process_for_human_pose_estimation_amd import hgk as H
    L = H.lib()
    dev = torch.device("cuda")
    M = N * hw * hw
    x = torch.randn(N, hw, hw, Cin, device=dev).to(dtype)
    ld = L.hgk_conv_w_ld(k * k * Cin)
    w = torch.randn(Cout, Cin, k, k, device=dev) * 0.05
    wp = torch.empty((Cout + 127) // 128 * 128, ld, device=dev, dtype=dtype)
    stream = H.stream_handle()
    dt = H.dtype_code(dtype)
    H.check(L.hgk_pack_conv_weight(stream, dt, w.data_ptr(), wp.data_ptr(), ld, Cout, Cin, k, k, 0,
                                   Cout, Cin))
    bias = torch.zeros(Cout, device=dev)
    scale = torch.rand(Cin, device=dev) + 0.5
    shift = torch.randn(Cin, device=dev) * 0.1
    y = torch.empty(N, hw, hw, Cout, device=dev, dtype=dtype)
    part = torch.empty((2 * (M // 64) + 4) * 3 * Cout, device=dev)
    rows = H.ctypes.c_int(0)
    pad = k // 2
    ws_b = L.hgk_conv_fwd_workspace(dt, N, hw, hw, Cin, Cout, k, k, 1, pad, 1)
    ws = torch.zeros(max(ws_b, 1), dtype=torch.uint8, device=dev)
    keep = (x, wp, bias, scale, shift, y, part, ws)

    def launch():
        H.check(L.hgk_conv_fwd(stream, dt, x.data_ptr(), wp.data_ptr(), ld, bias.data_ptr(), None,
                               y.data_ptr(), scale.data_ptr() if pre else None,
                               shift.data_ptr() if pre else None, 1 if pre else 0, 0,
                               part.data_ptr() if stats else None, H.ctypes.byref(rows),
                               N, hw, hw, Cin, Cout, k, k, 1, pad, 1,
                               ws.data_ptr() if ws_b else None, ws_b))
    launch.keep = keep
    return launch


FLUSH_BYTES = 512 << 20   # > the 256 MB Infinity Cache (MALL) + 8 x 4 MB L2 (MI355X_MICROARCH.md)
_FLUSH = []


def _flush_caches(st):
    """READ a 512 MB buffer on stream `st` (a sum): evicts the launch's operands from L2 and the
    MALL with CLEAN lines, so the next launch reads them from HBM as it does inside the training
    step. (A write flush leaves up to 256 MB of dirty lines whose write-back then lands in the timed
    launch: 45 vs 32 us in-step for the ring conv1, round-6 evidence run r06a.)"""
    if not _FLUSH:
        _FLUSH.append(torch.ones(FLUSH_BYTES // 4, dtype=torch.float32, device="cuda"))
        _FLUSH.append(torch.zeros((), dtype=torch.float32, device="cuda"))
    with torch.cuda.stream(st):
        torch.sum(_FLUSH[0], dim=0, out=_FLUSH[1])


def _time_launch(launch, reps=20):
    """(cold, warm) average duration of `launch` by HIP events recorded on the stream it launches
    on. cold: every rep bracketed by its own event pair after a 512 MB cache flush (outside the
    bracket) — the launch as the step sees it (round-5 verdict: the warm loop re-reads a 67 MB
    input from the Infinity Cache); warm: `reps` launches back to back between one pair."""
    from progressive_process_for_human_pose_estimation_amd import hgk as H  # noqa: F401
    for _ in range(3):
        launch()
    st = torch.cuda.current_stream()   # hgk launches go to H.stream_handle() == this stream
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        launch()
    e1.record(st)
    torch.cuda.synchronize()
    warm = e0.elapsed_time(e1) / 1e3 / reps
    pairs = []
    for _ in range(reps):
        _flush_caches(st)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        launch()
        b.record(st)
        pairs.append((a, b))
    torch.cuda.synchronize()
    cold = sum(a.elapsed_time(b) for a, b in pairs) / 1e3 / reps
    return cold, warm


def _pmc_traffic(key):
    if os.path.exists(ROOFLINE_PMC):
        pmc = json.load(open(ROOFLINE_PMC)).get(key)
        if pmc:
            return pmc["hbm_bytes_per_launch"]
    return None


def roofline_dominant(dtype, batch, res):
    """Residual-block conv1 (1x1 256->128 at the 64x64 level, BN+ReLU fused, BN-stats epilogue):
    the launch shape of the kernel with the largest step share. HBM-bound: algorithmic bytes =
    x (M x 256) + y (M x 128) + w (128 x 256) in the storage dtype."""
    hw = res // 4
    esz = 2 if dtype == torch.bfloat16 else 4
    M = batch * hw * hw
    avg, warm = _time_launch(_conv_launcher(dtype, batch, hw, 256, 128, 1, True, True))
    alg = (M * 256 + M * 128 + 128 * 256) * esz
    gbs = alg / avg / 1e9
    tn = "bf16_t" if dtype == torch.bfloat16 else "float"
    profiled = (batch, res, dtype) == (32, 256, torch.bfloat16)
    kname = ("conv1x1_ring_kernel<256,128,9> 1x1 256->128 @%dx%d N=%d (BN+ReLU fused in, BN stats "
             "out; LDS-DMA ring, two 4-wave workgroups per CU)" % (hw, hw, batch)
             if dtype == torch.bfloat16 and M >= 65536 else
             "conv_fwd_kernel<%s,...> 1x1 256->128 @%dx%d N=%d (BN+ReLU fused in, BN stats out)"
             % (tn, hw, hw, batch))
    return {"kernel": kname,
            "step_share": STEP_SHARE if profiled else None,
            "family_shares": FAMILY_SHARE if profiled else None,
            "bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(gbs / HBM_PEAK_GBS, 4),
            "traffic": _pmc_traffic("conv1x1") if profiled else None,
            "traffic_unit": "bytes/launch (2*FETCH_SIZE+WRITE_SIZE, %s)" % os.path.relpath(ROOFLINE_PMC, ROOT),
            "avg_us": round(avg * 1e6, 2), "alg_bytes_per_launch": alg,
            "timing": "cold: each launch after a 512 MB read-only cache flush (as inside the step); warm: "
                      "back-to-back launches re-reading their operands from the Infinity Cache",
            "warm_us": round(warm * 1e6, 2), "warm_frac": round(alg / warm / 1e9 / HBM_PEAK_GBS, 4)}


def roofline_second(dtype, batch, res):
    """The second family by step share: the small-level image-tile convs (conv_img_kernel), at its
    largest instantiation's shape — 1x1 256->128 at 16x16 (res / 16), BN+ReLU fused in, BN
    statistics out. Latency-bound (a chain of dependent memory round trips per launch, ~9 us for
    0.5 GFLOP / 6.3 MB): both fractions reported, `bound` = the larger."""
    hw = res // 16
    esz = 2 if dtype == torch.bfloat16 else 4
    M = batch * hw * hw
    avg, warm = _time_launch(_conv_launcher(dtype, batch, hw, 256, 128, 1, True, True))
    alg = (M * 256 + M * 128 + 128 * 256) * esz
    flops = 2.0 * M * 256 * 128
    gbs, tfs = alg / avg / 1e9, flops / avg / 1e12
    peak_tf = BF16_MFMA_PEAK_TFS if dtype == torch.bfloat16 else FP32_MFMA_PEAK_TFS
    fh, fm = gbs / HBM_PEAK_GBS, tfs / peak_tf
    from progressive_process_for_human_pose_estimation_amd import hgk as H
    fam = H.KFAM.get(H.lib().hgk_conv_fwd_kernel_family(H.dtype_code(dtype), batch, hw, hw, 0, 0, 0,
                                                         256, 128, 1, 1, 1, 0, 1))
    return {"kernel": "1x1 256->128 @%dx%d N=%d (BN+ReLU fused in, BN stats out) on the %s kernel "
                      "family" % (hw, hw, batch, fam),
            "family_share": FAMILY_SHARE.get("conv_img_kernel") if fam == "img" else None,
            "bound": "hbm" if fh >= fm else "mfma", "latency_bound": True,
            "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(fh, 4),
            "achieved_tflops": round(tfs, 2), "frac_mfma": round(fm, 4),
            "avg_us": round(avg * 1e6, 2), "warm_us": round(warm * 1e6, 2),
            "alg_bytes_per_launch": alg, "flops_per_launch": flops}


def roofline_mfma(dtype, batch, res):
    """3x3 bottleneck conv (128->128 at 64x64, BN+ReLU fused): algorithmic FLOPs = 2*M*9*C*C."""
    hw = res // 4
    M = batch * hw * hw
    avg, warm = _time_launch(_conv_launcher(dtype, batch, hw, 128, 128, 3, True, True))
    flops = 2.0 * M * 9 * 128 * 128
    tfs = flops / avg / 1e12
    peak = BF16_MFMA_PEAK_TFS if dtype == torch.bfloat16 else FP32_MFMA_PEAK_TFS
    profiled = (batch, res, dtype) == (32, 256, torch.bfloat16)
    return {"kernel": "3x3 128->128 @%dx%d N=%d %s (BN+ReLU fused; bf16: conv3x3_row_kernel<9,64,64>, "
                      "weights resident in registers, input rows streamed)"
                      % (hw, hw, batch, "bf16" if dtype == torch.bfloat16 else "fp32"),
            "bound": "mfma", "achieved": round(tfs, 2), "peak": peak, "unit": "TFLOP/s",
            "frac": round(tfs / peak, 4), "traffic": _pmc_traffic("conv3x3") if profiled else None,
            "traffic_unit": "bytes/launch", "avg_us": round(avg * 1e6, 2),
            "warm_us": round(warm * 1e6, 2), "flops_per_launch": flops}


def roofline_wgrad(dtype, batch, res):
    """The multi-use 1x1 weight gradient (round 6: conv1x1_wgrad_ring_kernel, 5.7 % of the step) of
    the outermost hourglass level's conv1 (256->128, try_with_torch.py:186): its 24 uses per step —
    2 per stack at 64x64 (up-branch) and 4 per stack at 32x32 (down-branch, innermost levels'
    inputs) — in one launch, each use's x BN+ReLU-transformed on the fly; HBM-bound: algorithmic
    bytes = every use's x (M x 256) + dy (M x 128) once, bf16. Cold launches as `roofline`."""
    from progressive_process_for_human_pose_estimation_amd import hgk as H
    if dtype != torch.bfloat16:
        return None
    L = H.lib()
    st = H.stream_handle()
    cap = L.hgk_conv_wgrad_max_splits()
    hw = res // 4
    uses = [(batch, hw, hw)] * 8 + [(batch, hw // 2, hw // 2)] * 16
    keep, srcs = [], []
    for n, hh, ww in uses:
        x = torch.randn(n, hh, ww, 256, device="cuda").to(dtype)
        dy = (torch.randn(n, hh, ww, 128, device="cuda") * 0.05).to(dtype)
        sc = torch.rand(256, device="cuda") + 0.5
        sh = torch.randn(256, device="cuda") * 0.1
        keep += [x, dy, sc, sh]
        srcs.append(H.WgradSrc(x.data_ptr(), dy.data_ptr(), sc.data_ptr(), sh.data_ptr(), 1, n, hh, ww))
    arr = (H.WgradSrc * len(srcs))(*srcs)
    slab = torch.zeros(L.hgk_conv_wgrad_slab_bytes(256, 128, 1, 1, cap) // 4, device="cuda")
    sp = H.ctypes.c_int(0)

    def launch():
        H.check(L.hgk_conv_wgrad_accum_multi(st, H.BF16, arr, len(srcs), slab.data_ptr(), cap, 0, 1,
                                             H.ctypes.byref(sp), 256, 128, 1, 1, 1, 0, 1))
    avg, warm = _time_launch(launch, reps=10)
    alg = sum(n * hh * ww for n, hh, ww in uses) * (256 + 128) * 2
    gbs = alg / avg / 1e9
    out = {"kernel": "conv1x1_wgrad_ring_kernel<128,256>: dW of a 1x1 256->128 over its 24 uses "
                     "(8 x %dx%d + 16 x %dx%d, N=%d), BN+ReLU of x in place, fp32 split slabs"
                     % (hw, hw, hw // 2, hw // 2, batch),
           "family_share": FAMILY_SHARE.get("conv1x1_wgrad_ring_kernel"),
           "bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(gbs / HBM_PEAK_GBS, 4), "avg_us": round(avg * 1e6, 2),
           "warm_us": round(warm * 1e6, 2), "alg_bytes_per_launch": alg, "splits": sp.value}
    del keep, slab
    torch.cuda.empty_cache()
    return out


def roofline_wgrad3x3(dtype, batch, res):
    """The multi-use 3x3 halo weight gradient (round 6: conv3x3_wgrad_halo_multi_kernel, 5.4 % of
    the step) of the outermost hourglass level's conv2 (128->128, try_with_torch.py:189): its 24
    uses per step (8 at 64x64, 16 at 32x32, as roofline_wgrad) in ONE launch over the uses'
    concatenated 8x16-pixel tiles, each use's x BN+ReLU-transformed on the fly; MFMA-bound:
    algorithmic FLOPs = 2 x 9 x 128 x 128 per pixel of every use. Cold launches as `roofline`."""
    from progressive_process_for_human_pose_estimation_amd import hgk as H
    if dtype != torch.bfloat16:
        return None
    L = H.lib()
    st = H.stream_handle()
    cap = L.hgk_conv_wgrad_max_splits()
    hw = res // 4
    uses = [(batch, hw, hw)] * 8 + [(batch, hw // 2, hw // 2)] * 16
    keep, srcs = [], []
    for n, hh, ww in uses:
        x = torch.randn(n, hh, ww, 128, device="cuda").to(dtype)
        dy = (torch.randn(n, hh, ww, 128, device="cuda") * 0.05).to(dtype)
        sc = torch.rand(128, device="cuda") + 0.5
        sh = torch.randn(128, device="cuda") * 0.1
        keep += [x, dy, sc, sh]
        srcs.append(H.WgradSrc(x.data_ptr(), dy.data_ptr(), sc.data_ptr(), sh.data_ptr(), 1, n, hh, ww))
    arr = (H.WgradSrc * len(srcs))(*srcs)
    slab = torch.zeros(L.hgk_conv_wgrad_slab_bytes(128, 128, 3, 3, cap) // 4, device="cuda")
    sp = H.ctypes.c_int(0)

    def launch():
        H.check(L.hgk_conv_wgrad_accum_multi(st, H.BF16, arr, len(srcs), slab.data_ptr(), cap, 0, 1,
                                             H.ctypes.byref(sp), 128, 128, 3, 3, 1, 1, 1))
    avg, warm = _time_launch(launch, reps=10)
    pix = sum(n * hh * ww for n, hh, ww in uses)
    flops = float(pix) * 2 * 9 * 128 * 128
    tfs = flops / avg / 1e12
    out = {"kernel": "conv3x3_wgrad_halo_multi_kernel<8>: dW of a 3x3 128->128 over its 24 uses "
                     "(8 x %dx%d + 16 x %dx%d, N=%d) in one launch, BN+ReLU of x in place, fp32 split slabs"
                     % (hw, hw, hw // 2, hw // 2, batch),
           "family_share": FAMILY_SHARE.get("conv3x3_wgrad_halo_multi_kernel"),
           "bound": "mfma", "achieved": round(tfs, 1), "peak": BF16_MFMA_PEAK_TFS, "unit": "TFLOP/s",
           "frac": round(tfs / BF16_MFMA_PEAK_TFS, 4), "avg_us": round(avg * 1e6, 2),
           "warm_us": round(warm * 1e6, 2), "flops_per_launch": flops,
           "alg_bytes_per_launch": pix * (128 + 128) * 2, "splits": sp.value}
    del keep, slab
    torch.cuda.empty_cache()
    return out


# ------------------------------------------------------------------------------ baselines
def cpu_model():
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(bs32_steps):
    """the CPU restatement of try_with_torch.py:179-343 (oracle, fp32, same aten
    ops), fwd + 4xMSE + bwd + Adam on synthetic 256x256 crops + Gaussian targets, at bs 2 (min of
    3 steps after 1 warm-up) and bs 32 (bs32_steps timed after 1 warm-up: the bounded sample).
    Threads: every CPU this process may use (OMP_NUM_THREADS caps it where the host sets it:
    16 per GPU on the pool's boxes, whose os.cpu_count() shows the whole machine)."""
    from oracle.hourglass_oracle import OracleModel, stack_mse
    from progressive_process_for_human_pose_estimation_amd.data import gaussian_targets, synthetic_images
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    cap = int(os.environ.get("OMP_NUM_THREADS") or 0)
    threads = min(avail, cap) if cap > 0 else avail
    torch.set_num_threads(threads)
    res = {}
    for n, steps in ((2, 3), (32, bs32_steps)):
        if steps <= 0:
            continue
        torch.manual_seed(0)
        m = OracleModel()
        opt = torch.optim.Adam(m.parameters(), lr=1e-5)
        x = synthetic_images(n, 256, 256, seed=0)
        t = gaussian_targets(n, 17, 64, seed=1)[0]

        def one():
            opt.zero_grad()
            stack_mse(m(x), t).backward()
            opt.step()
        one()
        times = []
        for _ in range(steps):
            t0 = time.perf_counter()
            one()
            times.append(time.perf_counter() - t0)
        res[n] = (n / min(times), min(times), steps)
        del m, opt
    main_bs = 32 if 32 in res else 2
    v = res[main_bs]
    out = {"value": round(v[0], 3), "unit": "images/sec", "cores": threads, "kind": "port",
           "cores_note": (f"{threads} threads = OMP_NUM_THREADS, the host CPU share the pool gives "
                          f"one GPU's job; os.cpu_count() ({os.cpu_count()}) counts the whole "
                          f"machine, shared with the other GPUs' jobs" if cap > 0 and cap < avail
                          else "every CPU this process may use"),
           "cpu_model": cpu_model(), "os_cpu_count": os.cpu_count(), "affinity_cpus": avail,
           "sample": f"oracle creatModel 4-stack 256x256 fp32, bs={main_bs}, fwd+4xMSE+bwd+Adam, "
                     f"min of {v[2]} step(s) after 1 warm-up, {threads} threads"}
    for n, (ips, s, k) in res.items():
        out[f"bs{n}"] = {"images_per_sec": round(ips, 3), "s_per_step": round(s, 3), "steps": k}
    return out


def dropin(dtype, batch, res, stacks, steps, graph=True):
    """The reference loop (try_with_torch.py:330-344) unchanged on the drop-in HIP modules:
    outs = model(x); loss = sum of nn.MSELoss per stack; opt.zero_grad(); loss.backward();
    opt.step() with torch.optim.Adam(lr=1e-5). graph: the module call and its backward replay
    captured hipGraphs (the default, modules.py); else every engine launch is a ctypes call from
    Python. Two untimed warm-up steps (eager warm-up, capture)."""
    import torch.nn as nn
    import progressive_process_for_human_pose_estimation_amd as P
    from progressive_process_for_human_pose_estimation_amd.data import gaussian_targets, synthetic_images
    torch.manual_seed(0)
    model = P.creatModel(nStack=stacks).cuda().set_engine_dtype(dtype).set_graph_mode(graph)
    opt = torch.optim.Adam(model.parameters(), lr=1e-5)
    crit = nn.MSELoss()
    x = synthetic_images(batch, res, res, seed=1234).cuda()
    t = gaussian_targets(batch, 17, res // 4, seed=1)[0].cuda()

    def one():
        outs = model(x)
        loss = sum(crit(o, t) for o in outs)
        opt.zero_grad()
        loss.backward()
        opt.step()
        return loss
    one()
    one()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = one()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    out = {"value": round(batch * steps / el, 2), "unit": "images/sec",
           "ms_per_step": round(el / steps * 1e3, 2), "steps": steps,
           "loss_last_step": float(loss.detach()),
           "path": "model(x) -> 4x nn.MSELoss -> backward -> torch.optim.Adam, one autograd node "
                   "per model call, " + ("its forward and backward replayed as hipGraphs"
                                         if graph else "eager (graph_calls off)")}
    del model, opt
    torch.cuda.empty_cache()
    return out


def inference(dtype, batch, res, stacks, steps=20):
    """The reference's evaluation path (hourglass_compare.py:1263-1273 times `model.eval()`
    forwards): eval-mode forward of the drop-in model under no_grad, graph-captured module calls
    (modules.py), batch `batch`; heatmaps copied out (NCHW fp32) every call."""
    import progressive_process_for_human_pose_estimation_amd as P
    from progressive_process_for_human_pose_estimation_amd.data import synthetic_images
    torch.manual_seed(0)
    model = P.creatModel(nStack=stacks).cuda().set_engine_dtype(dtype).eval()
    x = synthetic_images(batch, res, res, seed=7).cuda()
    with torch.no_grad():
        for _ in range(3):
            model(x)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            outs = model(x)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
    out = {"value": round(batch * steps / el, 1), "unit": "images/sec",
           "ms_per_batch": round(el / steps * 1e3, 3), "batch": batch, "steps": steps,
           "heatmap_checksum": float(sum(o.double().sum() for o in outs)),
           "path": "model.eval(); with no_grad: model(x) -> nStack heatmaps, graph-captured call"}
    del model
    torch.cuda.empty_cache()
    return out


# ------------------------------------------------------------------------------ dry run (CPU)
def dry_run(args, world, rank):
    """Plumbing check without a GPU: gloo process group, the engine model's real flat layout
    (FlatParams: [trunk | stem | never-grad tail]), each rank's gradient pre-scaled by 1/world as
    the MSE kernel does, segment-wise GradSync in grad-ready order; verifies the mean and prints
    the rank-0 line with n_gpus = world."""
    import progressive_process_for_human_pose_estimation_amd as P
    from progressive_process_for_human_pose_estimation_amd import dp
    from progressive_process_for_human_pose_estimation_amd.trainer import FlatParams
    if world > 1:
        dist.init_process_group("gloo")
    torch.manual_seed(0)
    fp = FlatParams(P.creatModel(nStack=args.stacks))
    sync = dp.GradSync(fp.grad, fp.segments)
    idx = torch.arange(fp.numel, dtype=torch.float32)
    sync.timing = True
    t0 = time.perf_counter()
    for _ in range(args.steps):
        fp.grad.zero_()
        fp.grad[:fp.active] = (rank + 1) * torch.sin(idx[:fp.active]) / world
        for i in range(len(fp.segments)):
            sync.launch(i)
        sync.wait()
    el = time.perf_counter() - t0
    st = sync.comm_stats()
    per_rank = [el]
    if world > 1:
        tt = torch.zeros(world, dtype=torch.float64)
        tt[rank] = el
        dist.all_reduce(tt)
        per_rank = tt.tolist()
    comm = {"bytes_reduced_per_step": sync.reduced_bytes(), "buckets_per_step": sync.buckets(),
            "bucket_bytes": sync.bucket_bytes, "segments": len(sync.segments),
            "per_rank_ms_per_step": [round(s / args.steps * 1e3, 3) for s in per_rank],
            "allreduce_ms_per_step_max": round(gather_max(st["allreduce_ms"], "cpu"), 4),
            "exposed_allreduce_ms_per_step_max": round(gather_max(st["exposed_ms"], "cpu"), 4),
            "probe_steps": st["steps"], "note": "gloo on the CPU: synchronous, fully exposed"}
    expect = (world + 1) / 2.0 * torch.sin(idx[:fp.active])
    ok = bool(torch.allclose(fp.grad[:fp.active], expect, rtol=1e-5, atol=1e-6)) and \
        bool((fp.grad[fp.active:] == 0).all())
    if rank == 0:
        print(json.dumps({
            "metric": METRIC, "value": 0.0, "unit": "images/sec", "n_gpus": world,
            "steps": args.steps, "warmup": 0, "ms_per_step": round(el / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "dry run: synthetic gradients, no model step", "dry_run": True,
            "config": {"workload": "flat-gradient all-reduce only (gloo)",
                       "global_batch": args.batch * world, "parallelism": f"dp{world}",
                       "segments": fp.segments, "active_params": fp.active,
                       "never_grad_params": fp.numel - fp.active},
            "comm": comm, "allreduce_ok": ok}), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0 if ok else 1


# ------------------------------------------------------------------------------ main
def build_step(preset, stacks, dtype, N, R, rank, use_graph=True, branches=False, overlap=None):
    """(trainer, x, targets, workload text) of one configuration, inputs resident in HBM.
    rank r's shard of the global batch is samples [N r, N r + N) (its own seeds)."""
    import progressive_process_for_human_pose_estimation_amd as P
    from progressive_process_for_human_pose_estimation_amd.data import (class_maps, gaussian_targets,
                                                                       synthetic_images)
    from progressive_process_for_human_pose_estimation_amd.trainer import Trainer
    torch.manual_seed(0)
    x = synthetic_images(N, R, R, seed=1234 + rank).cuda()
    kp = gaussian_targets(N, 17, R // 4, seed=1 + rank)[0].cuda()
    if preset == "try_with_aspp":
        from progressive_process_for_human_pose_estimation_amd.presets import try_with_aspp as AS
        model = AS.creatModel(nStack=stacks).cuda()
        trainer = Trainer(model, lr=1e-4, dtype=dtype, use_graph=use_graph, branches=branches,
                          overlap=overlap, heads=("ce", "ce", "mse")[:stacks])
        bg = class_maps(N, 2, R // 4, seed=2 + rank).cuda()
        sk = class_maps(N, 20, R // 4, seed=3 + rank).cuda()
        target = (bg, sk, kp)[:stacks]
        work = (f"try_with_aspp.creatModel ({stacks} progressive stacks) {R}x{R}, bs={N}/GPU, "
                f"fwd + CE(bg) + CE(skeleton) + MSE(keypoints) + bwd + Adam")
    elif preset == "try_more_layer":
        from progressive_process_for_human_pose_estimation_amd.presets import try_more_layer as TM
        model = TM.creatModel(nStack=stacks).cuda()
        trainer = Trainer(model, lr=1e-4, dtype=dtype, use_graph=use_graph, branches=branches,
                          overlap=overlap, heads=("ce", "ce", "mse", "none")[:stacks])
        bg = class_maps(N, 2, R // 4, seed=2 + rank).cuda()
        sk = class_maps(N, 20, R // 4, seed=3 + rank).cuda()
        target = (bg, sk, kp, None)[:stacks]
        work = (f"try_more_layer.creatModel ({stacks} progressive stacks, live ASPP) {R}x{R}, "
                f"bs={N}/GPU, fwd + CE(bg) + CE(skeleton) + MSE(keypoints) on outputs 0-2 + bwd + Adam")
    elif preset == "train":
        from progressive_process_for_human_pose_estimation_amd.presets import train as TP
        model = TP.creatModel().cuda()
        sk = class_maps(N, 16, R // 4, seed=3 + rank).cuda()
        kc = class_maps(N, 17, R // 4, seed=4 + rank).cuda()
        trainer = DropinStep(model, dtype, lr=1e-4, eps=1e-4)
        target = (sk, kc)
        work = (f"train.creatModel (3 stages, stride-2 residual blocks, live ASPP_Block) {R}x{R}, "
                f"bs={N}/GPU, fwd + bootstrapped top-k CE + CE on outputs 1-2 + bwd + Adam "
                f"(drop-in modules, graph-captured calls, HIP loss kernels)")
    elif preset == "hourglass_compare":
        from progressive_process_for_human_pose_estimation_amd.presets import hourglass_compare as HC
        model = HC.creatModel().cuda()
        trainer = Trainer(model, lr=1e-4, eps=1e-4, dtype=dtype, use_graph=use_graph,
                          branches=branches, overlap=overlap)
        target = gaussian_targets(N, 16, R // 4, seed=1 + rank)[0].cuda()
        work = (f"hourglass_compare.creatModel (4 unshared stages, nearest up-sampling) {R}x{R}, "
                f"bs={N}/GPU, fwd+4xMSE(16 heatmaps)+bwd+Adam")
    else:
        model = P.creatModel(nStack=stacks).cuda()
        trainer = Trainer(model, lr=1e-5, dtype=dtype, use_graph=use_graph, branches=branches,
                          overlap=overlap)
        target = kp
        work = (f"{stacks}-stack hourglass (try_with_torch.creatModel) {R}x{R}, bs={N}/GPU, "
                f"fwd+{stacks}xMSE+bwd+Adam")
    return trainer, x, target, work


class DropinStep:
    """train.py's loop on the drop-in modules (train.py:834,886-890): outs = model(x); loss =
    boot(out1, skeleton, 0.5) + CE(out1, skeleton) + boot(out2, keypoints, 0.5) + CE(out2,
    keypoints) on the HIP loss kernels (losses.py); backward; torch.optim.Adam. Module calls and
    their backward replay captured hipGraphs from the second step (modules.py)."""

    overlap = False
    fp = None

    def __init__(self, model, dtype, lr, eps, fraction=0.5):
        from progressive_process_for_human_pose_estimation_amd import losses as Lo
        self.model = model.set_engine_dtype(dtype)
        self.model.train()
        self.opt = torch.optim.Adam(model.parameters(), lr=lr, eps=eps)
        self.boot = Lo.Costomer_CrossEntropyLoss()
        self.ce = Lo.cross_entropy
        self.fraction = fraction

    def step(self, x, target):
        sk, kc = target
        outs = self.model(x)
        loss = (self.boot(outs[1], sk, self.fraction) + self.ce(outs[1], sk)
                + self.boot(outs[2], kc, self.fraction) + self.ce(outs[2], kc))
        self.opt.zero_grad()
        loss.backward()
        self.opt.step()
        return loss.detach()


def timed_steps(trainer, x, target, warmup, steps, world):
    """W untimed steps, then K steps between barriers + device syncs; max over ranks.
    Returns (max-over-ranks seconds, last loss, every rank's seconds)."""
    for _ in range(warmup):
        trainer.step(x, target)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = trainer.step(x, target)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    per_rank = [elapsed]
    if world > 1:
        tt = torch.zeros(world, device="cuda")
        tt[dist.get_rank()] = elapsed
        dist.all_reduce(tt, op=dist.ReduceOp.SUM)
        per_rank = tt.tolist()
        elapsed = max(per_rank)
    return elapsed, float(loss.detach()), per_rank


def gather_max(v, device):
    """max over ranks of a float (identity at world 1)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return v
    t = torch.tensor([v], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t)


def comm_object(sync, per_rank_s, steps, probe, device):
    """The DP step's communication, for reading a SCALE line: bytes and buckets the SUM
    all-reduce moves per step, each rank's ms per timed step, and — from `probe` extra steps run
    AFTER the timed region with events around the collectives (GradSync.timing) — the collective
    time per step and how much of it the backward overlap did not hide (max over ranks)."""
    sync.timing = True
    probe()
    st = sync.comm_stats()
    sync.timing = False
    return {"bytes_reduced_per_step": sync.reduced_bytes(), "buckets_per_step": sync.buckets(),
            "bucket_bytes": sync.bucket_bytes, "segments": len(sync.segments),
            "per_rank_ms_per_step": [round(s / steps * 1e3, 3) for s in per_rank_s],
            "allreduce_ms_per_step_max": round(gather_max(st["allreduce_ms"], device), 4),
            "exposed_allreduce_ms_per_step_max": round(gather_max(st["exposed_ms"], device), 4),
            "probe_steps": st["steps"],
            "note": "allreduce/exposed from untimed probe steps after the timed region (events on "
                    "the side stream; exposed = last collective end - main stream ready for Adam)"}


def step_roofline(key, N, ms, dtype):
    alg = ALG_PER_CONFIG.get(key)
    if alg is None:
        return None
    gbs = alg[0] * N / (ms / 1e3) / 1e9
    tfs = alg[1] * N / (ms / 1e3) / 1e12
    peak_tf = BF16_MFMA_PEAK_TFS if dtype == torch.bfloat16 else FP32_MFMA_PEAK_TFS
    return {"bound": alg[2], "alg_bytes_per_img": alg[0], "alg_flops_per_img": alg[1],
            "achieved_GBps": round(gbs, 1), "peak_GBps": HBM_PEAK_GBS,
            "alg_tflops": round(tfs, 1), "peak_tflops": peak_tf,
            "frac": round(gbs / HBM_PEAK_GBS if alg[2] == "hbm" else tfs / peak_tf, 4)}


def fp32_leg(args):
    """The headline configuration at the reference's own precision (fp32 storage and MFMA
    inputs; try_with_torch.py trains in fp32): a few timed steps on one GPU."""
    tr, x, t, work = build_step("primary", 4, torch.float32, 32, 256, 0)
    steps = 6
    el, loss, _ = timed_steps(tr, x, t, 2, steps, 1)
    ms = el / steps * 1e3
    out = {"value": round(32 * steps / el, 2), "unit": "images/sec", "ms_per_step": round(ms, 3),
           "steps": steps, "warmup": 2, "dtype": "f32", "workload": work,
           "step_roofline": step_roofline(("primary", 4, 256, "fp32"), 32, ms, torch.float32),
           "loss_last_step": loss}
    del tr
    torch.cuda.empty_cache()
    return out


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args.gpus, sys.argv[1:])
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        return dry_run(args, world, rank)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    N, R = args.batch, args.res
    if args.route:
        from progressive_process_for_human_pose_estimation_amd import engine as E
        E.apply_route_spec(args.route)
    trainer, x, t, work = build_step(args.preset, args.stacks, dtype, N, R, rank,
                                     use_graph=not args.no_graph, branches=args.branches,
                                     overlap=False if args.no_overlap else None)
    elapsed, final_loss, per_rank = timed_steps(trainer, x, t, args.warmup, args.steps, world)
    comm = None
    if world > 1 and getattr(trainer, "sync", None) is not None:
        comm = comm_object(trainer.sync, per_rank, args.steps,
                           lambda: [trainer.step(x, t) for _ in range(5)], "cuda")
    ms = elapsed / args.steps * 1e3
    value = N * world * args.steps / elapsed
    headline = (args.preset, args.stacks, R, N, args.dtype) == ("primary", 4, 256, 32, "bf16")

    if rank == 0:
        roof = roofline_dominant(dtype, N, R)
        roof_2 = roofline_second(dtype, N, R)
        roof_m = roofline_mfma(dtype, N, R)
        roof_w = roofline_wgrad(dtype, N, R) if args.preset == "primary" else None
        roof_w3 = roofline_wgrad3x3(dtype, N, R) if args.preset == "primary" else None
        step_roof = step_roofline((args.preset, args.stacks, R, args.dtype), N, ms, dtype)
        f32 = None
        if world == 1 and headline and not args.no_fp32_leg:
            f32 = fp32_leg(args)
        drop = None
        if world == 1 and args.dropin_steps > 0 and args.preset == "primary":
            drop = dropin(dtype, N, R, args.stacks, args.dropin_steps)
            drop["frac_of_trainer"] = round(drop["value"] / value, 4)
            drop["eager"] = dropin(dtype, N, R, args.stacks, 3, graph=False)
        infer = None
        if world == 1 and args.preset == "primary":
            infer = inference(dtype, N, R, args.stacks)
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(args.cpu_bs32_steps)
        rec = {
            "metric": METRIC, "value": round(value, 2), "unit": "images/sec", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "bf16" if dtype == torch.bfloat16 else "f32",
            "data": "synthetic (rand*2-1 images, sigma=1 Gaussian heatmap targets"
                    + (", uniform class maps" if args.preset in ("try_with_aspp", "try_more_layer",
                                                                 "train") else "")
                    + "); random init",
            "config": {"workload": work + (" + RCCL grad all-reduce (trunk overlapped with stem "
                                           "bwd)" if world > 1 else ""),
                       "model": {"try_with_aspp": f"try_with_aspp.creatModel nStack={args.stacks}",
                                 "try_more_layer": f"try_more_layer.creatModel nStack={args.stacks}",
                                 "train": "train.creatModel (3 stages)",
                                 "hourglass_compare": "hourglass_compare.creatModel nFeats=256 nOut=16"
                                 }.get(args.preset, f"creatModel nStack={args.stacks} nFeats=256 nOut=17"),
                       "global_batch": N * world, "seq_len": None, "parallelism": f"dp{world}",
                       "hipgraph": not args.no_graph, "overlap": trainer.overlap,
                       "never_grad_params": (None if trainer.fp is None
                                             else trainer.fp.numel - trainer.fp.active),
                       "route": args.route or "default"},
            "roofline": roof,
            "roofline_second": roof_2,
            "roofline_mfma": roof_m,
            "roofline_wgrad": roof_w,
            "roofline_wgrad3x3": roof_w3,
            "step_roofline": step_roof,
            "fp32_leg": f32,
            "cpu_baseline": cpu,
            "dropin": drop,
            "inference": infer,
            "comm": comm,
            "loss_last_step": final_loss,
        }
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
