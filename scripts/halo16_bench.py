"""Per-launch time of the 16x16-level 3x3 (N=32, 128->128, BN+ReLU in, statistics out) for library
route halo_bn64 = 0 (128-channel tiles, 128 workgroups), 1, 2 (64-channel tiles: 256 workgroups,
one / two k-groups); hipGraph replay, alternating rounds.

  python scripts/halo16_bench.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from progressive_process_for_human_pose_estimation_amd import hgk as H  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from wgrad_bench import graph_time  # noqa: E402


def main():
    L = H.load_library()
    g = torch.Generator(device="cuda").manual_seed(0)
    N, hw, C = 32, 16, 128
    x = (torch.randn(N, hw, hw, C, device="cuda", generator=g) * 0.7).to(torch.bfloat16)
    w = torch.randn(C, C, 3, 3, device="cuda", generator=g) * (1.0 / (9 * C) ** 0.5)
    bias = torch.randn(C, device="cuda", generator=g) * 0.1
    sc = torch.rand(C, device="cuda", generator=g) + 0.5
    sh = torch.randn(C, device="cuda", generator=g) * 0.3
    ld = L.hgk_conv_w_ld(9 * C)
    wp = torch.empty(C, ld, device="cuda", dtype=torch.bfloat16)
    H.check(L.hgk_pack_conv_weight(H.stream_handle(), H.BF16, w.data_ptr(), wp.data_ptr(), ld, C, C, 3, 3, 0, C, C))
    y = torch.empty(N, hw, hw, C, device="cuda", dtype=torch.bfloat16)
    part = torch.empty((2 * (N * hw * hw // 64) + 4) * 3 * C, device="cuda")
    rows = H.ctypes.c_int(0)
    print("route,us_per_launch")
    for rnd in range(3):
        for r in (0, 1, 2):
            prev = H.set_route("halo_bn64", r)

            def fn():
                H.check(L.hgk_conv_fwd(H.stream_handle(), H.BF16, x.data_ptr(), wp.data_ptr(), ld,
                                       bias.data_ptr(), None, y.data_ptr(), sc.data_ptr(), sh.data_ptr(),
                                       1, 0, part.data_ptr(), H.ctypes.byref(rows), N, hw, hw, C, C, 3,
                                       3, 1, 1, 1, None, 0))
            us = graph_time(fn, reps=20)
            H.set_route("halo_bn64", prev)
            print(f"{r},{us:.2f}", flush=True)


if __name__ == "__main__":
    main()
