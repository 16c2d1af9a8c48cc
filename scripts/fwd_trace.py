"""Per-phase timing of the all-ahead implicit-GEMM conv (conv_fwd_kernel, PF = 6) on the small
hourglass levels (timing build: HGK_EXTRA_FLAGS=-DHGK_FWD_TRACE HGK_OUT=ablib/fwdtrace.so
python -m progressive_process_for_human_pose_estimation_amd.build_ext; then
HGK_LIB=ablib/fwdtrace.so python scripts/fwd_trace.py [--img]; --img: the image-tile kernel's stamps,
for the shapes it takes).

Stamps (thread 0 of each workgroup, s_memrealtime = 100 MHz, i.e. 10 ns): 0 kernel entry, 1 body
(after the twin argument pick / tile remap), 2 row geometry done, 3 every k-tile's loads issued,
4 folded finalize / BN constants landed, 5 first barrier, 6 first k-tile landed, transformed and
staged, 7-10 after each further k-tile's MFMAs + barrier, 11 MFMAs done, 12 split-K: arrival
counter returned / else epilogue tile staged, 13 second half staged, 15 exit. Per launch: the host-side duration (hipGraph of 20 launches, HIP
events), the in-kernel span (first entry -> last exit over workgroups) and the dispatch skew, and
the median phase durations over workgroups.
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from progressive_process_for_human_pose_estimation_amd import hgk as H  # noqa: E402

DEV = "cuda"


def make(L, N, hw, cin, cout, k, pre=True, stats=True, res=False, fold=False):
    dt = H.BF16
    M = N * hw * hw
    x = (torch.randn(N, hw, hw, cin, device=DEV) * 0.5).to(torch.bfloat16)
    w = torch.randn(cout, cin, k, k, device=DEV) * 0.05
    ld = L.hgk_conv_w_ld(k * k * cin)
    wp = torch.empty((cout + 127) // 128 * 128, ld, device=DEV, dtype=torch.bfloat16)
    H.check(L.hgk_pack_conv_weight(H.stream_handle(), dt, w.data_ptr(), wp.data_ptr(), ld, cout, cin,
                                   k, k, 0, cout, cin))
    bias = torch.randn(cout, device=DEV) * 0.1
    sc = torch.rand(cin, device=DEV) + 0.5
    sh = torch.randn(cin, device=DEV) * 0.1
    y = torch.empty(N, hw, hw, cout, device=DEV, dtype=torch.bfloat16)
    r = (torch.randn(N, hw, hw, cout, device=DEV) * 0.5).to(torch.bfloat16) if res else None
    part = torch.empty((2 * (M // 64) + 4) * 3 * cout, device=DEV)
    rows = ctypes.c_int(0)
    pad = k // 2
    ws_b = L.hgk_conv_fwd_workspace(dt, N, hw, hw, cin, cout, k, k, 1, pad, 1)
    ws = torch.zeros(max(ws_b, 1 << 16), dtype=torch.uint8, device=DEV)
    keep = [x, wp, bias, sc, sh, y, r, part, ws]
    if fold:
        frows = 16
        fpart = torch.empty(cin, 3, frows, device=DEV)
        fpart[:, 0] = torch.randn(cin, frows, device=DEV) * 10
        fpart[:, 1] = torch.rand(cin, frows, device=DEV) * 50 + 1
        fpart[:, 2] = float(M) / frows
        gamma = torch.rand(cin, device=DEV) + 0.5
        beta = torch.randn(cin, device=DEV) * 0.1
        stat = torch.empty(4, cin, device=DEV)
        rec = torch.empty(2, cin, device=DEV, dtype=torch.float64)
        fd = H.BnFold(fpart.data_ptr(), frows, M, gamma.data_ptr(), beta.data_ptr(), 1e-5,
                      stat.data_ptr(), rec.data_ptr())
        keep += [fpart, gamma, beta, stat, rec, fd]
        assert L.hgk_conv_fold_ok(dt, N, hw, hw, 0, 0, 0, cin, cout, k, k, 1, pad, 1, frows, 0)

        def launch():
            H.check(L.hgk_conv_fwd_fold(H.stream_handle(), dt, x.data_ptr(), wp.data_ptr(), ld, bias.data_ptr(),
                                        None if r is None else r.data_ptr(), y.data_ptr(), 1, 0,
                                        part.data_ptr() if stats else None, ctypes.byref(rows),
                                        N, hw, hw, cin, cout, k, k, 1, pad, 1, ws.data_ptr(),
                                        ws.numel(), ctypes.byref(fd)))
    else:
        def launch():
            H.check(L.hgk_conv_fwd(H.stream_handle(), dt, x.data_ptr(), wp.data_ptr(), ld, bias.data_ptr(),
                                   None if r is None else r.data_ptr(), y.data_ptr(),
                                   sc.data_ptr() if pre else None, sh.data_ptr() if pre else None,
                                   1 if pre else 0, 0, part.data_ptr() if stats else None,
                                   ctypes.byref(rows), N, hw, hw, cin, cout, k, k, 1, pad, 1,
                                   ws.data_ptr(), ws.numel()))
    launch.keep = keep
    return launch


def graph_us(fn, reps=20):
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
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    g.replay()
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (5 * reps)


CASES = [
    # name, N, hw, cin, cout, k, pre, stats, res, fold
    ("1x1 256->128 @4 BN-in stats (conv1)", 32, 4, 256, 128, 1, True, True, False, False),
    ("1x1 256->128 @4 folded finalize", 32, 4, 256, 128, 1, True, True, False, True),
    ("1x1 128->256 @4 +res stats (conv3)", 32, 4, 128, 256, 1, True, True, True, False),
    ("1x1 256->128 @16 BN-in stats", 32, 16, 256, 128, 1, True, True, False, False),
    ("3x3 128->128 @4 split-K", 32, 4, 128, 128, 3, True, True, False, False),
    ("3x3 128->128 @8 split-K", 32, 8, 128, 128, 3, True, True, False, False),
    ("3x3 128->128 @8 split-K folded", 32, 8, 128, 128, 3, True, True, False, True),
    ("1x1 256->128 @4 no BN no stats", 32, 4, 256, 128, 1, False, False, False, False),
]


NAMES_FWD = {1: "args", 2: "geom", 3: "issue", 4: "consts", 5: "bar", 6: "tile0", 7: "k1", 8: "k2",
             9: "k3", 10: "k4", 11: "mfma", 12: "arrive/stage", 13: "half2", 15: "exit"}
# image-tile kernel (hgk_conv_img.hip)
NAMES_IMG = {1: "geom", 2: "issue", 3: "consts", 4: "bar", 5: "halo", 6: "dma-wait", 7: "bar",
             8: "mfma", 9: "stage", 15: "exit"}


def main():
    L = H.load_library()
    img = "--img" in sys.argv
    dbg = L.hgk_debug_img_trace if img else L.hgk_debug_fwd_trace
    dbg.argtypes = [ctypes.c_void_p, ctypes.c_int]
    names = NAMES_IMG if img else NAMES_FWD
    for name, N, hw, cin, cout, k, pre, stats, res, fold in CASES:
        fn = make(L, N, hw, cin, cout, k, pre, stats, res, fold)
        us = graph_us(fn)
        torch.cuda.synchronize()
        assert dbg(None, 1) == 0
        fn()
        torch.cuda.synchronize()
        buf = np.zeros(512 * 16, dtype=np.uint64)
        assert dbg(buf.ctypes.data_as(ctypes.c_void_p), 0) == 0
        t = buf.reshape(512, 16).astype(np.int64)
        live = t[:, 0] > 0
        t = t[live]
        nwg = len(t)
        t0 = t[:, 0].min()
        span = (t[:, 15].max() - t0) / 100.0
        skew = (t[:, 0].max() - t0) / 100.0
        print(f"== {name}: {us:6.2f} us/launch (graph), {nwg} WGs traced, in-kernel span {span:5.2f} us, "
              f"entry skew {skew:4.2f} us")
        rel = (t - t0) / 100.0
        # per phase: median duration over workgroups (stamps missing on a path are skipped)
        prev = rel[:, 0]
        parts = []
        for j in range(1, 16):
            col = np.where(t[:, j] > 0, rel[:, j], np.nan)
            d = col - prev
            if np.isfinite(d).any():
                parts.append(f"{names[j]} {np.nanmedian(d):4.2f}")
                prev = np.where(np.isfinite(col), col, prev)
        print("   median per WG: " + " | ".join(parts))
        print("   exit time: median %.2f  max %.2f us after first entry" %
              (np.median(rel[:, 15][t[:, 15] > 0]) if (t[:, 15] > 0).any() else -1, span))


if __name__ == "__main__":
    main()
