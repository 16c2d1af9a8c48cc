"""Micro-benchmark of the stem convolution (try_with_torch.py:262: nn.Conv2d(3, 64, 7, 2, 3) on the
channel-padded NHWC input, 256x256 -> 128x128) through hgk_conv_fwd (ReLU + statistics out, as the
engine launches it) and its weight gradient: us per launch, hipGraph replays.
  python scripts/stem_bench.py [--N 32] [--reps 20]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from progressive_process_for_human_pose_estimation_amd import hgk as H  # noqa: E402


def timeit(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
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
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=32)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    L = H.load_library()
    dt = H.BF16
    N, R, Cs, Co = a.N, 256, 8, 64
    Ho = R // 2
    x = torch.zeros(N, R, R, Cs, device="cuda", dtype=torch.bfloat16)
    x[..., :3] = torch.randn(N, R, R, 3, device="cuda").to(torch.bfloat16)
    w = torch.randn(Co, 3, 7, 7, device="cuda") * 0.05
    ld = L.hgk_conv_w_ld(7 * 7 * Cs)
    wp = torch.empty(128, ld, device="cuda", dtype=torch.bfloat16)
    st = H.stream_handle()
    H.check(L.hgk_pack_conv_weight(st, dt, w.data_ptr(), wp.data_ptr(), ld, Co, 3, 7, 7, 0, Co, Cs))
    y = torch.empty(N, Ho, Ho, Co, device="cuda", dtype=torch.bfloat16)
    bias = torch.randn(Co, device="cuda") * 0.1
    M = N * Ho * Ho
    part = torch.empty((2 * (M // 64) + 4) * 3 * Co, device="cuda")
    rows = H.ctypes.c_int(0)
    ws_b = L.hgk_conv_fwd_workspace(dt, N, R, R, Cs, Co, 7, 7, 2, 3, 1)
    ws = torch.zeros(max(ws_b, 1), dtype=torch.uint8, device="cuda")

    def fwd():
        H.check(L.hgk_conv_fwd(H.stream_handle(), dt, x.data_ptr(), wp.data_ptr(), ld, bias.data_ptr(), None,
                               y.data_ptr(), None, None, 0, 1, part.data_ptr(), H.ctypes.byref(rows),
                               N, R, R, Cs, Co, 7, 7, 2, 3, 1, ws.data_ptr(), ws.numel()))

    dy = (torch.randn(N, Ho, Ho, Co, device="cuda") * 0.1).to(torch.bfloat16)
    dw = torch.zeros(Co, 3, 7, 7, device="cuda")
    db = torch.zeros(Co, device="cuda")
    wws_b = L.hgk_conv_wgrad_workspace(dt, N, R, R, Cs, Co, 7, 7, 2, 3, 1)
    wws = torch.empty(wws_b, dtype=torch.uint8, device="cuda")

    def wgrad():
        H.check(L.hgk_conv_wgrad(H.stream_handle(), dt, x.data_ptr(), dy.data_ptr(), None, None, 0,
                                 dw.data_ptr(), db.data_ptr(), wws.data_ptr(), wws_b,
                                 N, R, R, Cs, Co, 7, 7, 2, 3, 1, 3, Co))

    flops = 2.0 * M * 3 * 49 * Co
    for stem in (1, 0):
        with H.route(stem=stem):
            for name, fn in (("fwd", fwd), ("wgrad", wgrad)):
                us = timeit(fn, a.reps)
                print(f"stem {name:6s} N={N} route stem={stem}: {us:8.1f} us  {flops / us / 1e6:7.1f} TF/s "
                      f"(algorithmic, Cin=3)", flush=True)


if __name__ == "__main__":
    main()
