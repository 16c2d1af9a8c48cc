"""Census of one eager bf16 training step's library calls (the headline config by default): per
entry point and geometry, how many calls and which forward kernel family the conv launches take
(hgk_conv_fwd_kernel_family). usage (GPU box): python scripts/launch_census.py [--preset P]"""
import argparse
import collections
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from progressive_process_for_human_pose_estimation_amd import engine as E  # noqa: E402
from progressive_process_for_human_pose_estimation_amd import hgk as H  # noqa: E402
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--preset", default="primary")
ap.add_argument("--batch", type=int, default=32)
ap.add_argument("--stacks", type=int, default=4)
args = ap.parse_args()
L = H.load_library()
census = collections.Counter()
GEO = {"hgk_conv_fwd": 14, "hgk_conv_fwd_fold": 12, "hgk_conv_fwd_bnbwd": 7, "hgk_conv_fwd_bnbwd_vg": 7}


class Proxy:
    def __getattr__(self, name):
        fn = getattr(L, name)

        def call(*a):
            key = name
            if name in GEO:
                i = GEO[name]
                N, Hh, W, Cin, Cout, KH, KW, st, pad, dil = [int(v) for v in a[i:i + 10]]
                fam = L.hgk_conv_fwd_kernel_family(1, N, Hh, W, 0, 0, 0, Cin, Cout, KH, KW, st, pad, dil)
                if name == "hgk_conv_fwd":
                    mode = (1 if a[8] else 0) | (2 if a[6] else 0) | (8 if a[12] else 0)
                elif name == "hgk_conv_fwd_fold":
                    mode = 1 | (2 if a[6] else 0) | (8 if a[10] else 0)
                else:
                    mode = 4 | (2 if a[5] else 0) | (16 if name.endswith("_vg") else 0)
                key = (f"{name} M={N * Hh * W} {Hh}x{W} {Cin}->{Cout} k{KH} s{st} mode{mode} "
                       f"fam={H.KFAM.get(fam, fam)}")
            census[key] += 1
            return fn(*a)
        return call


orig_lib = H.lib
H.lib = lambda: Proxy()
E.H.lib = H.lib
tr, x, t, _ = bench.build_step(args.preset, args.stacks, torch.bfloat16, args.batch, 256, 0,
                               use_graph=False)
tr.lib = Proxy()
tr.step(x, t)
torch.cuda.synchronize()
census.clear()
tr.step(x, t)
torch.cuda.synchronize()
for k, v in sorted(census.items(), key=lambda kv: str(kv[0])):
    print(f"{v:4d}  {k}")
