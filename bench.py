"""Benchmark: images/sec of the fused training step (fwd + 4x MSE + bwd [+ RCCL all-reduce] + Adam)
of the 4-stack hourglass (try_with_torch.creatModel) at 256x256, bs=32 per GPU, bf16 storage /
fp32 accumulate (BASELINE.json configs[1] at N=1, configs[2] for N>1).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Rank 0 prints ONE JSON line. `value` = images processed by all ranks / max-over-ranks wall time of
the K timed steps (inputs resident in HBM before the timed region). `roofline` reports the dominant
kernel (the 3x3 bottleneck conv at 64x64, bf16 MFMA) timed live with HIP events on its stream;
`cpu_baseline` times the CPU oracle (oracle/hourglass_oracle.py, PyTorch-CPU restatement of the
reference) on a bounded sample on rank 0.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "images/sec fwd+bwd, 4-stack hourglass 256×256 bs=32/GPU at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s HBM3E (spec)
BF16_MFMA_PEAK_TFS = 2500.0    # dense bf16 MFMA (spec, no sparsity)
ALG_BYTES_PER_IMG = 2.478e9    # algorithmic bytes / image (bf16, N=32)
ALG_FLOPS_PER_IMG = 151.26e9
# (stacks, res, dtype) -> (algorithmic bytes / image, FLOPs / image, step bound) per SURVEY.md §8(d)
ALG_PER_CONFIG = {(4, 256, "bf16"): (2.478e9, 151.26e9, "hbm"),
                  (8, 384, "fp32"): (21.156e9, 653.54e9, "mfma")}
FP32_MFMA_PEAK_TFS = 157.3     # dense fp32 matrix (spec)
ROOFLINE_KERNEL_SYMBOL = "conv3x3_halo_kernel"   # what the 3x3 @64x64 bf16 launch runs
ROOFLINE_PMC = os.path.join(ROOT, "profiles", "r01_roofline_pmc.json")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--res", type=int, default=256)
    ap.add_argument("--stacks", type=int, default=4)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--branches", action="store_true",
                    help="hourglass up-branches on side streams (Trainer(branches=True))")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=3)
    return ap.parse_args()


def dominant_kernel_roofline(dtype, batch, res, lib_mod):
    """Time the 3x3 bottleneck conv (mid=128, at the 64x64 level, BN+ReLU fused into its input
    staging) with HIP events on the stream it launches on; algorithmic FLOPs = 2*M*K*N."""
    from progressive_process_for_human_pose_estimation_amd import hgk as H
    L = H.lib()
    dev = torch.device("cuda")
    hw = res // 4
    N, C = batch, 128
    M = N * hw * hw
    x = torch.randn(N, hw, hw, C, device=dev).to(dtype)
    ld = L.hgk_conv_w_ld(9 * C)
    w = torch.randn(C, C, 3, 3, device=dev) * 0.05
    wp = torch.empty(128, ld, device=dev, dtype=dtype)
    stream = H.stream_handle()
    dt = H.dtype_code(dtype)
    H.check(L.hgk_pack_conv_weight(stream, dt, w.data_ptr(), wp.data_ptr(), ld, C, C, 3, 3, 0, C, C))
    bias = torch.zeros(C, device=dev)
    scale = torch.ones(C, device=dev)
    shift = torch.zeros(C, device=dev)
    y = torch.empty_like(x)
    part = torch.empty((2 * (M // 64) + 4) * 3 * C, device=dev)
    rows = H.ctypes.c_int(0)

    def launch():
        H.check(L.hgk_conv_fwd(stream, dt, x.data_ptr(), wp.data_ptr(), ld, bias.data_ptr(), None,
                               y.data_ptr(), scale.data_ptr(), shift.data_ptr(), 1, 0,
                               part.data_ptr(), H.ctypes.byref(rows), N, hw, hw, C, C, 3, 3, 1, 1, 1, None, 0))
    for _ in range(3):
        launch()
    reps = 20
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        launch()
    e1.record(st)
    torch.cuda.synchronize()
    avg_s = e0.elapsed_time(e1) / 1e3 / reps
    flops = 2.0 * M * (9 * C) * C
    achieved = flops / avg_s / 1e12
    peak = BF16_MFMA_PEAK_TFS if dtype == torch.bfloat16 else FP32_MFMA_PEAK_TFS
    traffic = None  # HBM bytes per launch from rocprofv3 PMC passes (scripts/roofline_pmc.py)
    if dtype == torch.bfloat16 and os.path.exists(ROOFLINE_PMC):
        pmc = json.load(open(ROOFLINE_PMC))
        if pmc.get("kernel_symbol") == ROOFLINE_KERNEL_SYMBOL:
            traffic = pmc["hbm_bytes_per_launch"]
    sym = ROOFLINE_KERNEL_SYMBOL if dtype == torch.bfloat16 else "conv_fwd_kernel<float> (implicit GEMM)"
    return {"kernel": "%s 3x3 128->128 @%dx%d N=%d (BN+ReLU fused)" % (sym, hw, hw, N),
            "bound": "mfma", "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
            "frac": round(achieved / peak, 4), "traffic": traffic, "traffic_unit": "bytes/launch",
            "avg_us": round(avg_s * 1e6, 2), "flops_per_launch": flops}


def cpu_baseline(steps):
    """Oracle (PyTorch-CPU restatement of try_with_torch.py:179-343) fp32, bounded sample."""
    from oracle.hourglass_oracle import OracleModel, stack_mse
    from progressive_process_for_human_pose_estimation_amd.data import gaussian_targets, synthetic_images
    cores = min(16, os.cpu_count() or 1)
    torch.set_num_threads(cores)
    n = 2
    torch.manual_seed(0)
    m = OracleModel()
    opt = torch.optim.Adam(m.parameters(), lr=1e-5)
    x = synthetic_images(n, 256, 256)
    t = gaussian_targets(n, 17, 64)[0]

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
    best = min(times)
    return {"value": round(n / best, 3), "unit": "images/sec", "cores": cores, "kind": "port",
            "sample": f"oracle creatModel 4-stack 256x256 fp32, bs={n}, fwd+4xMSE+bwd+Adam, "
                      f"min of {steps} steps after 1 warm-up"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    import progressive_process_for_human_pose_estimation_amd as P
    from progressive_process_for_human_pose_estimation_amd.data import gaussian_targets, synthetic_images
    from progressive_process_for_human_pose_estimation_amd.trainer import Trainer

    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    torch.manual_seed(0)
    model = P.creatModel(nStack=args.stacks).cuda()
    trainer = Trainer(model, lr=1e-5, dtype=dtype, use_graph=not args.no_graph,
                      branches=args.branches)
    N, R = args.batch, args.res
    x = synthetic_images(N, R, R, seed=1234 + rank).cuda()
    t = gaussian_targets(N, 17, R // 4, seed=1 + rank)[0].cuda()

    for _ in range(args.warmup):
        trainer.step(x, t)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = trainer.step(x, t)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt)
    ms = elapsed / args.steps * 1e3
    value = N * world * args.steps / elapsed
    final_loss = float(loss)

    if rank == 0:
        roof = dominant_kernel_roofline(dtype, N, R, P)
        alg = ALG_PER_CONFIG.get((args.stacks, R, args.dtype))
        step_roof = None
        if alg is not None:
            gbs = alg[0] * N / (ms / 1e3) / 1e9
            tfs = alg[1] * N / (ms / 1e3) / 1e12
            peak_tf = BF16_MFMA_PEAK_TFS if dtype == torch.bfloat16 else FP32_MFMA_PEAK_TFS
            step_roof = {"bound": alg[2], "alg_bytes_per_img": alg[0], "alg_flops_per_img": alg[1],
                         "achieved_GBps": round(gbs, 1), "peak_GBps": HBM_PEAK_GBS,
                         "alg_tflops": round(tfs, 1), "peak_tflops": peak_tf,
                         "frac": round(gbs / HBM_PEAK_GBS if alg[2] == "hbm" else tfs / peak_tf, 4)}
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(args.cpu_steps)
        rec = {
            "metric": METRIC, "value": round(value, 2), "unit": "images/sec", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "bf16" if dtype == torch.bfloat16 else "f32",
            "data": "synthetic (rand*2-1 images, sigma=1 Gaussian heatmap targets); random init",
            "config": {"workload": f"{args.stacks}-stack hourglass (try_with_torch.creatModel) "
                                   f"{R}x{R}, bs={N}/GPU, fwd+{args.stacks}xMSE+bwd+Adam"
                                   + (" + RCCL grad all-reduce" if world > 1 else ""),
                       "model": f"creatModel nStack={args.stacks} nFeats=256 nOut=17",
                       "global_batch": N * world, "seq_len": None, "parallelism": f"dp{world}",
                       "hipgraph": not args.no_graph},
            "roofline": roof,
            "step_roofline": step_roof,
            "cpu_baseline": cpu,
            "loss_last_step": final_loss,
        }
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
