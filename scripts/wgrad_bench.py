"""Micro-benchmark: weight-grad of a shared 3x3 / 1x1 weight over many small uses, one launch per
use (hgk_conv_wgrad_accum) vs one multi-use launch (hgk_conv_wgrad_accum_multi). hipGraph timing.

  python scripts/wgrad_bench.py [--prod | --halo]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from progressive_process_for_human_pose_estimation_amd import hgk as H  # noqa: E402


def graph_time(fn, reps=10):
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
    L = H.load_library()
    dt = H.BF16
    dev = "cuda"
    cap = L.hgk_conv_wgrad_max_splits()
    shapes = [(128, 128, 3, [(32, 16)] * 8), (128, 128, 3, [(32, 8)] * 8 + [(32, 4)] * 16),
              (256, 128, 1, [(32, 16)] * 8), (128, 128, 3, [(32, 64)])]
    if "--prod" in sys.argv:
        # the 64x64 level's shared 1x1 weights: 4 stacks x (2 up-branch uses at 64^2 + 4 at 32^2)
        # and residual4's (8 uses at 64^2)
        shapes = [(256, 128, 1, [(32, 64)] * 8 + [(32, 32)] * 16), (128, 256, 1, [(32, 64)] * 8 + [(32, 32)] * 16),
                  (256, 128, 1, [(32, 64)] * 8), (128, 256, 1, [(32, 64)] * 8), (256, 128, 1, [(32, 64)])]
    if "--halo" in sys.argv:
        # the 3x3 halo weight-grad kernel, one use per launch: 64x64 and 32x32 levels, stem block
        shapes = [(128, 128, 3, [(32, 64)]), (128, 128, 3, [(32, 32)]), (64, 64, 3, [(32, 128)])]
    for (cin, cout, k, uses) in shapes:
        pad = k // 2
        srcs = []
        for (n, hw) in uses:
            x = torch.randn(n, hw, hw, cin, device=dev).to(torch.bfloat16)
            dy = torch.randn(n, hw, hw, cout, device=dev).to(torch.bfloat16)
            sc = torch.rand(cin, device=dev) + 0.5
            sh = torch.randn(cin, device=dev) * 0.1
            srcs.append((x, dy, sc, sh, n, hw))
        nbytes = L.hgk_conv_wgrad_slab_bytes(cin, cout, k, k, cap)
        slabs = torch.zeros(nbytes // 4, device=dev)
        rows = H.ctypes.c_int(0)
        flops = sum(2.0 * n * hw * hw * cin * k * k * cout for (_, _, _, _, n, hw) in srcs)

        def per_use():
            init = 0
            for (x, dy, sc, sh, n, hw) in srcs:
                H.check(L.hgk_conv_wgrad_accum(H.stream_handle(), dt, x.data_ptr(), dy.data_ptr(),
                                               sc.data_ptr(), sh.data_ptr(), 1, slabs.data_ptr(),
                                               cap, init, 1, H.ctypes.byref(rows), n, hw, hw, cin,
                                               cout, k, k, 1, pad, 1))
                init = max(init, rows.value)

        arr = (H.WgradSrc * len(srcs))(*[H.WgradSrc(x.data_ptr(), dy.data_ptr(), sc.data_ptr(),
                                                      sh.data_ptr(), 1, n, hw, hw)
                                         for (x, dy, sc, sh, n, hw) in srcs])

        def multi():
            H.check(L.hgk_conv_wgrad_accum_multi(H.stream_handle(), dt, arr, len(srcs),
                                                 slabs.data_ptr(), cap, 0, 1, H.ctypes.byref(rows),
                                                 cin, cout, k, k, 1, pad, 1))
        t1 = graph_time(per_use)
        t2 = graph_time(multi)
        gb = sum(n * hw * hw * (cin + cout) * (2 if dt == H.BF16 else 4) for (_, _, _, _, n, hw) in srcs) / 1e9
        print(f"  algorithmic x+dy {gb:.3f} GB: multi {gb / t2 * 1e3:.2f} TB/s")
        print(f"{cin}->{cout} k{k} uses={[u[1] for u in uses]}: per-use {t1:8.1f} us "
              f"({flops / t1 / 1e6:6.1f} TF/s)  multi {t2:8.1f} us ({flops / t2 / 1e6:6.1f} TF/s) "
              f"splits={rows.value}", flush=True)


if __name__ == "__main__":
    main()
