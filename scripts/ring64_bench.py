"""Per-shape timing of the ring 1x1 kernel's 64-channel launches against the tiled route (ring off,
route ring_minm = 0) at the primary's sizes (N = 32): us per launch from hipGraph replays.
  python scripts/ring64_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from progressive_process_for_human_pose_estimation_amd import hgk as H  # noqa: E402

DEV = "cuda"
CASES = [  # K, Cout, mode, hw (N = 32); mode 4 = input gradient with BN-backward sums
    (64, 64, 9, 128), (64, 64, 4, 128), (64, 128, 0, 128), (64, 128, 11, 128), (64, 128, 4, 128),
    (128, 64, 0, 128), (128, 64, 4, 128), (128, 64, 9, 64), (128, 64, 4, 64), (64, 128, 11, 64),
    (64, 128, 4, 64), (256, 64, 1, 64), (256, 64, 2, 64), (64, 256, 10, 64), (64, 256, 2, 64),
    (64, 256, 4, 64), (64, 256, 0, 64), (64, 256, 8, 64), (64, 128, 8, 128), (64, 128, 9, 64)]


def timeit(fn, reps=20):
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
    L = H.load_library()
    N = 32
    for K, C, m, hw in CASES:
        M = N * hw * hw
        x = (torch.randn(N, hw, hw, K, device=DEV) * 0.5).to(torch.bfloat16)
        w = torch.randn(C, K, 1, 1, device=DEV) * 0.05
        ld = L.hgk_conv_w_ld(K)
        wp = torch.empty(((C + 127) // 128) * 128, ld, device=DEV, dtype=torch.bfloat16)
        H.check(L.hgk_pack_conv_weight(H.stream_handle(), 1, w.data_ptr(), wp.data_ptr(), ld, C, K, 1, 1, 0, C, K))
        bias = torch.zeros(C, device=DEV)
        sc = torch.rand(K, device=DEV) + 0.5
        sh = torch.randn(K, device=DEV) * 0.1
        r = torch.randn(N, hw, hw, C, device=DEV).to(torch.bfloat16)
        y = torch.empty(N, hw, hw, C, device=DEV, dtype=torch.bfloat16)
        part = torch.empty((M // 16 + 4) * 3 * C, device=DEV)
        ybn = torch.randn(N, hw, hw, C, device=DEV).to(torch.bfloat16)
        cs = torch.rand(C, device=DEV) + 0.5
        rows = H.ctypes.c_int(0)
        pre, res, stats = m & 1, m & 2, m & 8

        def fn():
            if m == 4:
                H.check(L.hgk_conv_fwd_bnbwd(H.stream_handle(), 1, x.data_ptr(), wp.data_ptr(), ld, None,
                                             y.data_ptr(), N, hw, hw, K, C, 1, 1, 1, 0, 1, None, 0,
                                             ybn.data_ptr(), cs.data_ptr(), cs.data_ptr(), 1, cs.data_ptr(),
                                             cs.data_ptr(), part.data_ptr(), H.ctypes.byref(rows)))
            else:
                H.check(L.hgk_conv_fwd(H.stream_handle(), 1, x.data_ptr(), wp.data_ptr(), ld, bias.data_ptr(),
                                       r.data_ptr() if res else None, y.data_ptr(),
                                       sc.data_ptr() if pre else None, sh.data_ptr() if pre else None,
                                       1 if pre else 0, 0, part.data_ptr() if stats else None,
                                       H.ctypes.byref(rows), N, hw, hw, K, C, 1, 1, 1, 0, 1, None, 0))

        t_ring = timeit(fn)
        with H.route(ring_minm=0):
            t_tiled = timeit(fn)
        nbytes = M * (K + C + (C if (res or m == 4) else 0)) * 2
        print(f"K {K:3d} Cout {C:3d} mode {m:2d} @{hw:3d}: ring {t_ring:7.1f} us ({nbytes / t_ring / 1e6:5.2f} TB/s)"
              f"  tiled {t_tiled:7.1f} us  ratio {t_tiled / t_ring:5.2f}", flush=True)


if __name__ == "__main__":
    main()
