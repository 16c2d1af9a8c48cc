"""Per-launch time of the multi-use 1x1 weight gradient, ring kernel (route wg_ring) vs the tiled
multi kernel, at the headline step's use mixes (4-stack 256x256, N = 32): the outermost hourglass
level's conv1 / conv3 (8 uses at 64x64 + 16 at 32x32), residual4's (8 at 64x64), lin / ll_ 256x256
(4 at 64x64), the second level's (8 at 32x32 + 16 at 16x16). Algorithmic bytes = every use's x + dy
(bf16) once. usage (GPU box): python scripts/wgrad_ring_bench.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from progressive_process_for_human_pose_estimation_amd import hgk as H  # noqa: E402

MIXES = {"level4": [(32, 64, 64)] * 8 + [(32, 32, 32)] * 16,
         "residual4": [(32, 64, 64)] * 8,
         "lin": [(32, 64, 64)] * 4,
         "level3": [(32, 32, 32)] * 8 + [(32, 16, 16)] * 16}
SHAPES = {"level4": [(128, 256), (256, 128)], "residual4": [(128, 256), (256, 128)],
          "lin": [(256, 256)], "level3": [(128, 256), (256, 128)]}


def main():
    L = H.load_library()
    st = H.stream_handle()
    cap = L.hgk_conv_wgrad_max_splits()
    print("mix,Cout,Cin,uses,alg_MB,route,us,TBps,frac_8TBps")
    for mix, uses in MIXES.items():
        for Cout, Cin in SHAPES[mix]:
            keep, srcs = [], []
            for N, Hh, W in uses:
                x = torch.randn(N, Hh, W, Cin, device="cuda").to(torch.bfloat16)
                dy = torch.randn(N, Hh, W, Cout, device="cuda").to(torch.bfloat16)
                sc = torch.rand(Cin, device="cuda") + 0.5
                sh = torch.randn(Cin, device="cuda") * 0.1
                keep += [x, dy, sc, sh]
                srcs.append(H.WgradSrc(x.data_ptr(), dy.data_ptr(), sc.data_ptr(), sh.data_ptr(), 1, N, Hh, W))
            arr = (H.WgradSrc * len(srcs))(*srcs)
            slab = torch.zeros(L.hgk_conv_wgrad_slab_bytes(Cin, Cout, 1, 1, cap) // 4, device="cuda")
            alg = sum(N * Hh * W for N, Hh, W in uses) * (Cin + Cout) * 2
            sp = H.ctypes.c_int(0)
            for ring in (0, 1, 0, 1):
                with H.route(wg_ring=ring):
                    def one():
                        H.check(L.hgk_conv_wgrad_accum_multi(st, H.BF16, arr, len(srcs), slab.data_ptr(), cap,
                                                             0, 1, H.ctypes.byref(sp), Cin, Cout, 1, 1, 1, 0, 1))
                    for _ in range(2):
                        one()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(10):
                        one()
                    e1.record()
                    torch.cuda.synchronize()
                    us = e0.elapsed_time(e1) * 1e3 / 10
                tb = alg / us / 1e6
                print(f"{mix},{Cout},{Cin},{len(uses)},{alg / 1e6:.1f},{'ring' if ring else 'tiled'},{us:.1f},"
                      f"{tb:.2f},{tb / 8:.3f}", flush=True)
            del keep, slab
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
