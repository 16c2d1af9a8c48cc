"""Per-launch time / bandwidth of the BN elementwise kernels at the 64x64 level (M = 131072,
C = 256, bf16): hgk_bn_apply2_add (3 streams), hgk_bn_bwd_reduce2 (3), hgk_bn_bwd_pair (coef
mode: 5), hgk_bn_bwd_apply (3; + add: 4), hgk_bn_bwd_reduce (2). hipGraph replay.

  python scripts/bn_pair_bench.py
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
    st = H.stream_handle
    dt = H.BF16
    M, C = 131072, 256
    g = torch.Generator(device="cuda").manual_seed(0)
    t = lambda: (torch.randn(M, C, device="cuda", generator=g)).to(torch.bfloat16)  # noqa: E731
    v = lambda: torch.rand(C, device="cuda", generator=g) + 0.5  # noqa: E731
    dA, ya, yb, out, out2, add = t(), t(), t(), t(), t(), t()
    sca, sha, mua, iva, scb, shb, mub, ivb = (v() for _ in range(8))
    part = torch.empty(2048 * 3 * C, device="cuda")
    pa, pb = torch.empty(2048 * 2 * C, device="cuda"), torch.empty(2048 * 2 * C, device="cuda")
    coef_a, coef_b = torch.rand(4, C, device="cuda"), torch.rand(4, C, device="cuda")
    rows = H.ctypes.c_int(0)
    sa = H.BnSide(ya.data_ptr(), sca.data_ptr(), sha.data_ptr(), mua.data_ptr(), iva.data_ptr(), 0, pa.data_ptr())
    sb = H.BnSide(yb.data_ptr(), scb.data_ptr(), shb.data_ptr(), mub.data_ptr(), ivb.data_ptr(), 0, pb.data_ptr())
    fa = H.BnbSide(ya.data_ptr(), sca.data_ptr(), sha.data_ptr(), mua.data_ptr(), iva.data_ptr(), 0, None, 2048,
                   coef_a.data_ptr(), None, None, out.data_ptr())
    fb = H.BnbSide(yb.data_ptr(), scb.data_ptr(), shb.data_ptr(), mub.data_ptr(), ivb.data_ptr(), 0, None, 2048,
                   coef_b.data_ptr(), None, None, out2.data_ptr())
    E = M * C * 2
    cases = [
        ("apply2_add", 3, lambda: H.check(L.hgk_bn_apply2_add(st(), dt, H.ctypes.byref(sa), H.ctypes.byref(sb),
                                                              out.data_ptr(), M, C, part.data_ptr(), H.ctypes.byref(rows)))),
        ("bwd_reduce2", 3, lambda: H.check(L.hgk_bn_bwd_reduce2(st(), dt, dA.data_ptr(), M, C, H.ctypes.byref(sa),
                                                                H.ctypes.byref(sb), H.ctypes.byref(rows)))),
        ("bwd_pair(coef)", 5, lambda: H.check(L.hgk_bn_bwd_pair(st(), dt, dA.data_ptr(), M, C, 1, H.ctypes.byref(fa),
                                                                H.ctypes.byref(fb)))),
        ("bwd_apply", 3, lambda: H.check(L.hgk_bn_bwd_apply(st(), dt, dA.data_ptr(), ya.data_ptr(), M, C, sca.data_ptr(),
                                                            sha.data_ptr(), 1, coef_a.data_ptr(), None, out.data_ptr(), 0))),
        ("bwd_apply+add", 4, lambda: H.check(L.hgk_bn_bwd_apply(st(), dt, dA.data_ptr(), ya.data_ptr(), M, C, sca.data_ptr(),
                                                                sha.data_ptr(), 1, coef_a.data_ptr(), add.data_ptr(),
                                                                out.data_ptr(), 0))),
        ("bwd_reduce", 2, lambda: H.check(L.hgk_bn_bwd_reduce(st(), dt, dA.data_ptr(), ya.data_ptr(), M, C, sca.data_ptr(),
                                                              sha.data_ptr(), 1, mua.data_ptr(), iva.data_ptr(),
                                                              pa.data_ptr(), H.ctypes.byref(rows)))),
        ("bn_stats", 1, lambda: H.check(L.hgk_bn_stats(st(), dt, ya.data_ptr(), M, C, part.data_ptr(), H.ctypes.byref(rows)))),
    ]
    print("kernel,streams,us,TB/s")
    for rnd in range(2):
        for name, ns, fn in cases:
            us = graph_time(fn, reps=20)
            print(f"{name},{ns},{us:.2f},{ns * E / us / 1e6:.2f}", flush=True)


if __name__ == "__main__":
    main()
