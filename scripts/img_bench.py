"""Image-tile kernel vs the routes it replaces, per small-level conv shape of the headline step
(N = 32, bf16): us per launch as hipGraph replays of 20 launches (HIP events), route img on / off.

  python scripts/img_bench.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from progressive_process_for_human_pose_estimation_amd import hgk as H  # noqa: E402
from fwd_trace import graph_us, make  # noqa: E402

CASES = [
    # name, N, hw, cin, cout, k, pre, stats, res, fold
    ("3x3 128->128 @4", 32, 4, 128, 128, 3, True, True, False, False),
    ("3x3 128->128 @4 folded", 32, 4, 128, 128, 3, True, True, False, True),
    ("3x3 128->128 @8", 32, 8, 128, 128, 3, True, True, False, False),
    ("3x3 128->128 @8 folded", 32, 8, 128, 128, 3, True, True, False, True),
    ("3x3 128->128 @16", 32, 16, 128, 128, 3, True, True, False, False),
    ("1x1 256->128 @4", 32, 4, 256, 128, 1, True, True, False, False),
    ("1x1 256->128 @4 folded", 32, 4, 256, 128, 1, True, True, False, True),
    ("1x1 128->256 @4 +res", 32, 4, 128, 256, 1, True, True, True, False),
    ("1x1 256->128 @8", 32, 8, 256, 128, 1, True, True, False, False),
    ("1x1 128->256 @8 +res", 32, 8, 128, 256, 1, True, True, True, False),
    ("1x1 256->128 @16", 32, 16, 256, 128, 1, True, True, False, False),
    ("1x1 128->256 @16 +res", 32, 16, 128, 256, 1, True, True, True, False),
    ("1x1 256->256 @16 (lin)", 32, 16, 256, 256, 1, False, True, False, False),
]


def main():
    L = H.load_library()
    for name, N, hw, cin, cout, k, pre, stats, res, fold in CASES:
        out = []
        for img in (0, 8192):
            with H.route(img=img):
                fam = H.KFAM[L.hgk_conv_fwd_kernel_family(1, N, hw, hw, 0, 0, 0, cin, cout, k, k, 1,
                                                          k // 2, 1)]
                fn = make(L, N, hw, cin, cout, k, pre, stats, res, fold)
                out.append((fam, graph_us(fn)))
        print(f"{name:28s} {out[0][0]:8s} {out[0][1]:6.2f} us | {out[1][0]:8s} {out[1][1]:6.2f} us "
              f"x{out[0][1] / out[1][1]:.2f}", flush=True)


if __name__ == "__main__":
    main()
