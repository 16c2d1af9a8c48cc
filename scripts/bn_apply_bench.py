"""BN-backward apply (hgk_bn_bwd_apply) on the production shapes, hipGraph replays of `reps`
launches timed with HIP events; HBM bytes = read dA + y (+ add) + write dy.

  HGK_LIB=<ablation build> python scripts/bn_apply_bench.py [--reps 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from progressive_process_for_human_pose_estimation_amd import hgk as H  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from ring_bench import graph_time  # noqa: E402

DEV = "cuda"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    L = H.load_library()
    g = torch.Generator(device=DEV).manual_seed(0)
    for M, C, add in ((131072, 256, False), (131072, 128, False), (131072, 256, True),
                      (32768, 128, False), (32768, 256, False)):
        dA = torch.randn(M, C, device=DEV, generator=g).to(torch.bfloat16)
        y = torch.randn(M, C, device=DEV, generator=g).to(torch.bfloat16)
        a = torch.randn(M, C, device=DEV, generator=g).to(torch.bfloat16) if add else None
        out = torch.empty(M, C, device=DEV, dtype=torch.bfloat16)
        sc = torch.rand(C, device=DEV, generator=g) + 0.5
        sh = torch.randn(C, device=DEV, generator=g) * 0.1
        coef = torch.randn(4, C, device=DEV, generator=g)

        def fn():
            H.check(L.hgk_bn_bwd_apply(H.stream_handle(), 1, dA.data_ptr(), y.data_ptr(), M, C,
                                       sc.data_ptr(), sh.data_ptr(), 1, coef.data_ptr(),
                                       H.ptr(a), out.data_ptr(), 0))
        us = graph_time(fn, args.reps)
        nb = M * C * 2 * (3 + (1 if add else 0))
        print(f"apply M {M:6d} C {C} add {int(add)}: {us:6.1f} us {nb / us / 1e3:6.0f} GB/s "
              f"({nb / us / 1e3 / 8000:.3f} of 8 TB/s)", flush=True)


if __name__ == "__main__":
    main()
