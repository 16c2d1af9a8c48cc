"""Ring 1x1 kernel vs the tiled implicit-GEMM kernel on the production shapes (N=32, bf16, 64x64
level; twin = 64x64 + 32x32 in one launch). Each launch timed as hipGraph replays of `reps`
launches (HIP events on the replay stream); the ring_minm route (hgk.set_route) toggles the route
per call.

  python scripts/ring_bench.py [--reps 20] [--N 32] [--route ring_nw=8]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from progressive_process_for_human_pose_estimation_amd import hgk as H  # noqa: E402

DEV = "cuda"


def graph_time(fn, reps):
    for _ in range(2):
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
    best = 1e30
    for _ in range(3):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / reps)
    return best


def make_case(L, N, hws, cin, cout, pre, res, bbm, stats):
    """one (twin when len(hws) == 2) 1x1 launch; returns (fn, algorithmic bytes)"""
    g = torch.Generator(device=DEV).manual_seed(0)
    w = torch.randn(cout, cin, 1, 1, device=DEV, generator=g) * (1.0 / cin ** 0.5)
    ld = L.hgk_conv_w_ld(cin)
    wp = torch.empty(((cout + 127) // 128) * 128, ld, device=DEV, dtype=torch.bfloat16)
    H.check(L.hgk_pack_conv_weight(H.stream_handle(), 1, w.data_ptr(), wp.data_ptr(), ld, cout, cin,
                                   1, 1, 0, cout, cin))
    bias = torch.zeros(cout, device=DEV)
    segs, keep, nbytes = [], [], 0
    for hw in hws:
        M = N * hw * hw
        x = (torch.randn(N, hw, hw, cin, device=DEV, generator=g) * 0.5).to(torch.bfloat16)
        y = torch.empty(N, hw, hw, cout, device=DEV, dtype=torch.bfloat16)
        r = torch.randn(N, hw, hw, cout, device=DEV, generator=g).to(torch.bfloat16) if res else None
        sc = torch.rand(cin, device=DEV, generator=g) + 0.5 if pre else None
        sh = torch.randn(cin, device=DEV, generator=g) * 0.1 if pre else None
        part = torch.empty((2 * (M // 64) + 4) * 3 * cout, device=DEV) if (stats or bbm) else None
        yb = torch.randn(N, hw, hw, cout, device=DEV, generator=g).to(torch.bfloat16) if bbm else None
        cst = torch.rand(cout, device=DEV, generator=g) + 0.5 if bbm else None
        rows = H.ctypes.c_int(0)
        keep += [x, y, r, sc, sh, part, yb, cst, rows]
        segs.append(H.ConvSeg(x.data_ptr(), H.ptr(r), y.data_ptr(), H.ptr(sc), H.ptr(sh),
                              H.ptr(part) if stats else None, H.ctypes.pointer(rows), N, hw, hw,
                              H.ptr(yb), H.ptr(cst), H.ptr(cst), H.ptr(cst), H.ptr(cst),
                              H.ptr(part) if bbm else None, 1, H.ctypes.pointer(rows)))
        nbytes += M * 2 * (cin + cout + (cout if res else 0) + (cout if bbm else 0))
    nbytes += cout * cin * 2
    arr = (H.ConvSeg * 2)(*(segs * (2 if len(segs) == 1 else 1)))

    def fn():
        if len(hws) == 2:
            H.check(L.hgk_conv_fwd_twin(H.stream_handle(), 1, wp.data_ptr(), ld, bias.data_ptr(),
                                        1 if pre else 0, 0, cin, cout, 1, 1, 1, 0, 1, arr, None, 0))
        else:
            s = segs[0]
            if bbm:
                H.check(L.hgk_conv_fwd_bnbwd(H.stream_handle(), 1, s.x, wp.data_ptr(), ld, s.res, s.y,
                                             N, hws[0], hws[0], cin, cout, 1, 1, 1, 0, 1, None, 0,
                                             s.bb_y, s.bb_scale, s.bb_shift, 1, s.bb_mean,
                                             s.bb_invstd, s.bb_partial, s.bb_rows))
            else:
                H.check(L.hgk_conv_fwd(H.stream_handle(), 1, s.x, wp.data_ptr(), ld, bias.data_ptr(),
                                       s.res, s.y, s.pre_scale, s.pre_shift, 1 if pre else 0, 0,
                                       s.stats, s.rows_out, N, hws[0], hws[0], cin, cout, 1, 1, 1,
                                       0, 1, None, 0))
    fn.keep = (keep, arr, wp, bias)
    return fn, nbytes


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--N", type=int, default=32)
    ap.add_argument("--only", default="")
    ap.add_argument("--route", default="", help="library routes, e.g. ring_nw=8")
    args = ap.parse_args()
    if args.route:
        from progressive_process_for_human_pose_estimation_amd import engine as E
        E.apply_route_spec(args.route)
    L = H.load_library()
    cases = [  # name, hws, cin, cout, pre, res, bbm, stats
        ("conv1 fwd 256->128 @64", (64,), 256, 128, True, False, False, True),
        ("conv3 fwd 128->256 +res @64", (64,), 128, 256, True, True, False, True),
        ("dgrad conv1 128->256 acc+bnb @64", (64,), 128, 256, False, True, True, False),
        ("dgrad conv3 256->128 bnb @64", (64,), 256, 128, False, False, True, False),
        ("lin fwd 256->256 @64", (64,), 256, 256, False, False, False, True),
        ("conv1 fwd twin @64+32", (64, 32), 256, 128, True, False, False, True),
        ("conv3 fwd twin @64+32", (64, 32), 128, 256, True, True, False, True),
        ("dgrad conv1 twin @64+32", (64, 32), 128, 256, False, True, True, False),
        ("dgrad conv3 twin @64+32", (64, 32), 256, 128, False, False, True, False),
        ("conv1 fwd 256->128 @32", (32,), 256, 128, True, False, False, True),
        ("conv3 fwd 128->256 +res @32", (32,), 128, 256, True, True, False, True),
        ("dgrad conv1 128->256 acc+bnb @32", (32,), 128, 256, False, True, True, False),
        ("dgrad conv3 256->128 bnb @32", (32,), 256, 128, False, False, True, False),
        ("conv1 fwd twin @32+16", (32, 16), 256, 128, True, False, False, True),
        ("conv3 fwd twin @32+16", (32, 16), 128, 256, True, True, False, True),
        ("dgrad conv1 twin @32+16", (32, 16), 128, 256, False, True, True, False),
        ("dgrad conv3 twin @32+16", (32, 16), 256, 128, False, False, True, False),
        ("conv1 fwd 256->128 @16", (16,), 256, 128, True, False, False, True),
        ("dgrad conv3 256->128 bnb @16", (16,), 256, 128, False, False, True, False),
        ("conv1 fwd twin @16+8", (16, 8), 256, 128, True, False, False, True),
        ("dgrad conv3 twin @16+8", (16, 8), 256, 128, False, False, True, False),
    ]
    for name, hws, cin, cout, pre, res, bbm, stats in cases:
        if args.only and args.only not in name:
            continue
        fn, nbytes = make_case(L, args.N, hws, cin, cout, pre, res, bbm, stats)
        out = []
        for minm in ("0", "1024"):
            with H.route(ring_minm=int(minm)):
                us = graph_time(fn, args.reps)
            out.append((us, nbytes / us / 1e3))
        print(f"{name:36s} tiled {out[0][0]:7.1f} us {out[0][1]:6.0f} GB/s | ring {out[1][0]:7.1f} us "
              f"{out[1][1]:6.0f} GB/s ({out[1][1] / 8000:.3f} of 8 TB/s)  x{out[0][0] / out[1][0]:.2f}",
              flush=True)


if __name__ == "__main__":
    main()
