"""Per-launch time of the 3x3 halo weight gradient, register-staged (wg_dma=0) vs LDS-DMA staged
(wg_dma=1), hipGraph replay, alternating rounds (same box).

  python scripts/wgrad_dma_bench.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from progressive_process_for_human_pose_estimation_amd import hgk as H  # noqa: E402
from wgrad_bench import graph_time  # noqa: E402


def main():
    L = H.load_library()
    g = torch.Generator(device="cuda").manual_seed(0)
    cases = [(128, 128, 32, 64, True), (128, 128, 32, 64, False), (128, 128, 32, 32, True),
             (128, 128, 32, 16, True)]
    cap = 256
    print("case,route,us_per_launch,TF/s")
    for rnd in range(3):
        for cin, cout, n, hw, bn in cases:
            x = (torch.randn(n, hw, hw, cin, device="cuda", generator=g) * 0.7).to(torch.bfloat16)
            dy = (torch.randn(n, hw, hw, cout, device="cuda", generator=g) * 0.1).to(torch.bfloat16)
            sc = torch.rand(cin, device="cuda", generator=g) + 0.5
            sh = torch.randn(cin, device="cuda", generator=g) * 0.3
            slab = torch.zeros(L.hgk_conv_wgrad_slab_bytes(cin, cout, 3, 3, cap) // 4, device="cuda")
            splits = H.ctypes.c_int(0)
            for dma in (0, 1):
                prev = H.set_route("wg_dma", dma)

                def fn():
                    H.check(L.hgk_conv_wgrad_accum(H.stream_handle(), H.BF16, x.data_ptr(), dy.data_ptr(),
                                                   sc.data_ptr() if bn else None,
                                                   sh.data_ptr() if bn else None, 1, slab.data_ptr(), cap,
                                                   0, 1, H.ctypes.byref(splits), n, hw, hw, cin, cout, 3, 3,
                                                   1, 1, 1))
                us = graph_time(fn, reps=20)
                H.set_route("wg_dma", prev)
                fl = 2.0 * n * hw * hw * cin * cout * 9
                print(f"{cin}->{cout} @{hw} N={n} bn={int(bn)},{dma},{us:.2f},{fl / us / 1e6:.1f}", flush=True)


if __name__ == "__main__":
    main()
