"""Determinism probe of the training step: the same Trainer step (fresh Trainer, same seed, same
batch) repeated R times in ONE process must give bitwise-identical flat gradients. Prints, per
repeat, the max |diff| against the first run for the trunk and stem segments.

  python scripts/twin_determinism.py [--graph] [--reps 4] [--n 2] [--res 128] [--stacks 2]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import progressive_process_for_human_pose_estimation_amd as P  # noqa: E402
from progressive_process_for_human_pose_estimation_amd.data import gaussian_targets, synthetic_images  # noqa: E402
from progressive_process_for_human_pose_estimation_amd.trainer import Trainer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graph", action="store_true")
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--n", type=int, default=2)
    ap.add_argument("--res", type=int, default=128)
    ap.add_argument("--stacks", type=int, default=2)
    ap.add_argument("--dtype", default="fp32")
    a = ap.parse_args()
    dt = torch.float32 if a.dtype == "fp32" else torch.bfloat16
    x = synthetic_images(a.n, a.res, a.res, seed=100).cuda()
    t = gaussian_targets(a.n, 17, a.res // 4, seed=200)[0].cuda()
    first = None
    for r in range(a.reps):
        torch.manual_seed(0)
        m = P.creatModel(nStack=a.stacks).cuda()
        tr = Trainer(m, lr=1e-4, dtype=dt, use_graph=a.graph)
        tr.step(x, t)
        if a.graph:
            tr.step(x, t)  # second replay: grads of the same weights? no: Adam moved them
        torch.cuda.synchronize()
        g = tr.fp.grad.clone()
        segs = tr.fp.segments
        if first is None:
            first = g
            print("run 0: trunk norm %.6e stem norm %.6e" % (g[segs[0][0]:segs[0][1]].norm(),
                                                              g[segs[1][0]:segs[1][1]].norm()))
            continue
        d = (g - first).abs()
        print("run %d: trunk max diff %.3e, stem max diff %.3e, n diff %d" % (
            r, d[segs[0][0]:segs[0][1]].max(), d[segs[1][0]:segs[1][1]].max(), int((d > 0).sum())),
            flush=True)


if __name__ == "__main__":
    main()
