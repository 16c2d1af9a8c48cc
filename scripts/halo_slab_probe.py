"""How much of the per-use 3x3 halo weight gradient is the slab read-modify-write: the outermost
level's 3x3 (128->128) over its 24 uses per step (8 at 64x64, 16 at 32x32), one launch per use as
the engine issues them, hipGraph timing. Run with the default library and with the
HGK_ABL_WG_NOSLAB ablation build (HGK_LIB=...: the kernels skip the slab read-modify-write; wrong
results, timing only). usage (GPU box): [HGK_LIB=abx/noslab.so] python scripts/halo_slab_probe.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
from progressive_process_for_human_pose_estimation_amd import hgk as H  # noqa: E402
from wgrad_bench import graph_time  # noqa: E402

L = H.load_library()
cap = L.hgk_conv_wgrad_max_splits()
for label, uses in (("64x64 x8", [(32, 64)] * 8), ("32x32 x16", [(32, 32)] * 16)):
    srcs = []
    for n, hw in uses:
        x = torch.randn(n, hw, hw, 128, device="cuda").to(torch.bfloat16)
        dy = torch.randn(n, hw, hw, 128, device="cuda").to(torch.bfloat16)
        sc = torch.rand(128, device="cuda") + 0.5
        sh = torch.randn(128, device="cuda") * 0.1
        srcs.append((x, dy, sc, sh, n, hw))
    slabs = torch.zeros(L.hgk_conv_wgrad_slab_bytes(128, 128, 3, 3, cap) // 4, device="cuda")
    rows = H.ctypes.c_int(0)

    def per_use():
        init = 0
        for (x, dy, sc, sh, n, hw) in srcs:
            H.check(L.hgk_conv_wgrad_accum(H.stream_handle(), H.BF16, x.data_ptr(), dy.data_ptr(),
                                           sc.data_ptr(), sh.data_ptr(), 1, slabs.data_ptr(), cap, init,
                                           1, H.ctypes.byref(rows), n, hw, hw, 128, 128, 3, 3, 1, 1, 1))
            init = max(init, rows.value)
    t = graph_time(per_use)
    print(f"{os.environ.get('HGK_LIB', 'default')}: {label}: {t:8.1f} us for {len(uses)} launches "
          f"({t / len(uses):6.2f} us each), splits {rows.value}", flush=True)
