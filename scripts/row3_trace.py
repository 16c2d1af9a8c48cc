"""Per-iteration phase timing of the row-streaming 3x3 kernel (timing build: HGK_EXTRA_FLAGS=
-DHGK_R3_TRACE HGK_OUT=ablib/trace.so; HGK_LIB=ablib/trace.so python scripts/row3_trace.py).
Phases (wave 0 of workgroups 0-3, clock64 cycles): wait = top vmcnt wait, bar = top barrier,
mma = DMA issue + transform + fragment/MFMA stream, xch = exchange (+ BN input wait) barrier,
epi = epilogue."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from progressive_process_for_human_pose_estimation_amd import hgk as H  # noqa: E402

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import test_gpu_row3 as T  # noqa: E402


def main():
    L = H.load_library()
    for mode in ("fwd", "dgrad", "dgrad_vg"):
        for hw in ((64,) if mode == "dgrad_vg" else (64, 32)):
            N = 32
            g, x, w, bias, sc, sh = T._inputs(N, hw, 3)
            wp, ld = T._pack(L, w, dgrad=(mode != "fwd"))
            for _ in range(3):
                if mode == "fwd":
                    T._fwd(L, x, wp, ld, bias, sc, sh)
                elif mode == "dgrad_vg":
                    out = torch.empty_like(x)
                    side = torch.empty_like(x)
                    part = T._part(N * hw * hw)
                    rows = H.ctypes.c_int(0)
                    coef = torch.randn(4, 128, device="cuda") * 0.1
                    vg = H.BnVgrad(x.data_ptr(), sc.data_ptr(), sh.data_ptr(), coef.data_ptr(), 1,
                                   side.data_ptr())
                    H.check(L.hgk_conv_fwd_bnbwd_vg(H.stream_handle(), 1, x.data_ptr(), wp.data_ptr(), ld,
                                                    None, out.data_ptr(), N, hw, hw, 128, 128, 3, 3, 1, 1,
                                                    1, None, 0, x.data_ptr(), sc.data_ptr(), sh.data_ptr(),
                                                    1, sc.data_ptr(), sc.data_ptr(), part.data_ptr(),
                                                    H.ctypes.byref(rows), H.ctypes.byref(vg)))
                    torch.cuda.synchronize()
                else:
                    out = torch.empty_like(x)
                    part = T._part(N * hw * hw)
                    rows = H.ctypes.c_int(0)
                    H.check(L.hgk_conv_fwd_bnbwd(H.stream_handle(), 1, x.data_ptr(), wp.data_ptr(), ld, None,
                                                 out.data_ptr(), N, hw, hw, 128, 128, 3, 3, 1, 1, 1, None, 0,
                                                 x.data_ptr(), sc.data_ptr(), sh.data_ptr(), 1, sc.data_ptr(),
                                                 sc.data_ptr(), part.data_ptr(), H.ctypes.byref(rows)))
                    torch.cuda.synchronize()
            buf = np.zeros(4 * 16 * 6, dtype=np.uint64)
            assert L.hgk_debug_row3_trace(buf.ctypes.data_as(ctypes.c_void_p)) == 0
            t = buf.reshape(4, 16, 6).astype(np.int64)
            print(f"== {mode} @{hw}")
            for wg in range(2):
                for i in range(16):
                    r = t[wg, i]
                    if r[0] == 0 or r[5] == 0:
                        continue
                    d = np.diff(r)
                    nxt = t[wg, i + 1, 0] - r[5] if i + 1 < 16 and t[wg, i + 1, 0] else 0
                    print(f"  wg{wg} row{i:2d}: wait {d[0]:6d} bar {d[1]:6d} mma {d[2]:6d} xch {d[3]:6d} "
                          f"epi {d[4]:6d} (loop {nxt:5d})")


if __name__ == "__main__":
    main()
