"""Micro-benchmark of the libhgk convolution kernels on the hot path's shapes (N=32, 256x256 model).

  python scripts/conv_bench.py [--dtype bf16] [--reps 20]

Prints per shape: average µs per launch (HIP events on the launch stream) and TFLOP/s
(algorithmic 2*M*K*N). Shapes: the bottleneck convs of a ResidualBlock at every hourglass level,
forward / input-grad (as forward conv of dy with the flipped weight) / weight-grad.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from progressive_process_for_human_pose_estimation_amd import hgk as H  # noqa: E402


GRAPH = False


def timeit(fn, reps):
    """us per call; with --graph the reps are captured into one hipGraph and replayed (what the
    training step sees: no host launch cost between dependent kernels)."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if GRAPH:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                for _ in range(reps):
                    fn()
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        e0.record()
        g.replay()
        e1.record()
    else:
        st = torch.cuda.current_stream()
        e0.record(st)
        for _ in range(reps):
            fn()
        e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps  # us


NOSTATS = False


def bench_conv(L, dt, dtype, N, hw, cin, cout, k, pre, res, reps, mode):
    dev = "cuda"
    stream = H.stream_handle()
    pad = k // 2
    x = (torch.randn(N, hw, hw, cin, device=dev) * 0.5).to(dtype)
    w = torch.randn(cout, cin, k, k, device=dev) * 0.05
    M = N * hw * hw
    flops = 2.0 * M * cin * k * k * cout
    scale = torch.rand(max(cin, cout), device=dev) + 0.5
    shift = torch.randn(max(cin, cout), device=dev) * 0.1
    rows = H.ctypes.c_int(0)
    if mode in ("fwd", "dgrad"):
        ci, co = (cin, cout) if mode == "fwd" else (cout, cin)
        xin = x if mode == "fwd" else (torch.randn(N, hw, hw, ci, device=dev) * 0.5).to(dtype)
        ld = L.hgk_conv_w_ld(k * k * ci)
        wp = torch.empty(((co + 127) // 128) * 128, ld, device=dev, dtype=dtype)
        H.check(L.hgk_pack_conv_weight(stream, dt, w.data_ptr(), wp.data_ptr(), ld, cout, cin, k, k,
                                       0 if mode == "fwd" else 1, cout, cin))
        y = torch.empty(N, hw, hw, co, device=dev, dtype=dtype)
        bias = torch.zeros(co, device=dev)
        part = torch.empty((2 * (M // 64) + 4) * 3 * co, device=dev)
        r = y if res else None
        use_pre = pre and mode == "fwd"
        ws_b = L.hgk_conv_fwd_workspace(dt, N, hw, hw, ci, co, k, k, 1, pad, 1)
        ws = torch.zeros(ws_b, dtype=torch.uint8, device=dev) if ws_b else None

        def fn():
            H.check(L.hgk_conv_fwd(H.stream_handle(), dt, xin.data_ptr(), wp.data_ptr(), ld,
                                   bias.data_ptr() if mode == "fwd" else None,
                                   None if r is None else r.data_ptr(), y.data_ptr(),
                                   scale.data_ptr() if use_pre else None,
                                   shift.data_ptr() if use_pre else None, 1 if use_pre else 0, 0,
                                   part.data_ptr() if (mode == "fwd" and not NOSTATS) else None,
                                   H.ctypes.byref(rows),
                                   N, hw, hw, ci, co, k, k, 1, pad, 1,
                                   None if ws is None else ws.data_ptr(),
                                   0 if ws is None else ws.numel()))
    else:
        dy = (torch.randn(N, hw, hw, cout, device=dev) * 0.5).to(dtype)
        dw = torch.zeros(cout, cin, k, k, device=dev)
        db = torch.zeros(cout, device=dev)
        ws_b = L.hgk_conv_wgrad_workspace(dt, N, hw, hw, cin, cout, k, k, 1, pad, 1)
        ws = torch.empty(ws_b, dtype=torch.uint8, device=dev)

        def fn():
            H.check(L.hgk_conv_wgrad(H.stream_handle(), dt, x.data_ptr(), dy.data_ptr(),
                                     scale.data_ptr() if pre else None,
                                     shift.data_ptr() if pre else None, 1 if pre else 0,
                                     dw.data_ptr(), db.data_ptr(), ws.data_ptr(), ws_b,
                                     N, hw, hw, cin, cout, k, k, 1, pad, 1, cin, cout))
    us = timeit(fn, reps)
    es = 2 if dtype == torch.bfloat16 else 4
    nbytes = M * (cin + cout + (cout if (res and mode == "fwd") else 0)) * es
    return us, flops / us / 1e6, nbytes / us / 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--N", type=int, default=32)
    ap.add_argument("--only", default="")
    ap.add_argument("--modes", default="fwd,dgrad,wgrad")
    ap.add_argument("--nopre", action="store_true", help="drop the fused BN+ReLU input transform")
    ap.add_argument("--nostats", action="store_true", help="no BN statistics in the fwd epilogue")
    ap.add_argument("--graph", action="store_true", help="time hipGraph replays of the reps")
    args = ap.parse_args()
    global GRAPH
    GRAPH = args.graph
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    L = H.load_library()
    dt = H.dtype_code(dtype)
    shapes = [  # name, hw, cin, cout, k, pre, res
        ("conv1 1x1 256->128", 64, 256, 128, 1, True, False),
        ("conv2 3x3 128->128", 64, 128, 128, 3, True, False),
        ("conv3 1x1 128->256", 64, 128, 256, 1, True, True),
        ("lin 1x1 256->256", 64, 256, 256, 1, False, False),
        ("conv1 1x1 256->128 @32", 32, 256, 128, 1, True, False),
        ("conv3 1x1 128->256 @32", 32, 128, 256, 1, True, True),
        ("conv1 1x1 256->128 @16", 16, 256, 128, 1, True, False),
        ("conv1 1x1 256->128 @8", 8, 256, 128, 1, True, False),
        ("conv1 1x1 256->128 @4", 4, 256, 128, 1, True, False),
        ("conv2 3x3 @32", 32, 128, 128, 3, True, False),
        ("conv2 3x3 @16", 16, 128, 128, 3, True, False),
        ("conv2 3x3 @8", 8, 128, 128, 3, True, False),
        ("conv2 3x3 @4", 4, 128, 128, 3, True, False),
        ("stem RB conv2 3x3 64->64 @128", 128, 64, 64, 3, True, False),
    ]
    global NOSTATS
    NOSTATS = args.nostats
    tot = {}
    for mode in args.modes.split(","):
        for name, hw, cin, cout, k, pre, res in shapes:
            if args.only and args.only not in name:
                continue
            us, tf, gbs = bench_conv(L, dt, dtype, args.N, hw, cin, cout, k, pre and not args.nopre, res,
                                args.reps, mode)
            tot[mode] = tot.get(mode, 0) + us
            print(f"{mode:6s} {name:32s} {us:9.1f} us {tf:8.1f} TF/s {gbs:8.1f} GB/s", flush=True)
    print({k: round(v, 1) for k, v in tot.items()})


if __name__ == "__main__":
    main()
