"""Short-training probe on the GPU: the headline Trainer (4-stack 256x256, N=32, hipGraph, default
routes) on a fixed keypoint batch (data.keypoint_task), loss per step and the PCKh curve
(train.py:759-791 on the HIP kernel) every `--every` steps, bf16 and fp32. Used to pick the
convergence fixture's step count / lr (tests/golden/make_golden.py converge).
usage (GPU box): python scripts/converge_probe.py [--steps 150] [--lr 1e-3] [--n 32]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import progressive_process_for_human_pose_estimation_amd as P  # noqa: E402
from progressive_process_for_human_pose_estimation_amd import engine as E  # noqa: E402
from progressive_process_for_human_pose_estimation_amd.data import keypoint_task  # noqa: E402
from progressive_process_for_human_pose_estimation_amd.targets import PCKh  # noqa: E402
from progressive_process_for_human_pose_estimation_amd.trainer import Trainer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=150)
    ap.add_argument("--every", type=int, default=10)
    ap.add_argument("--lrs", default="1e-3")
    ap.add_argument("--ns", default="32")
    ap.add_argument("--res", type=int, default=256)
    ap.add_argument("--stacks", type=int, default=4)
    ap.add_argument("--task", default="keypoint", choices=["keypoint", "noise"])
    ap.add_argument("--dtypes", default="bf16,fp32")
    ap.add_argument("--route", default="")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "converge_probe.json"))
    a = ap.parse_args()
    if a.route:
        E.apply_route_spec(a.route)
    res = {}
    for n, dn, lr in [(int(n), d, float(l)) for n in a.ns.split(",") for l in a.lrs.split(",")
                      for d in a.dtypes.split(",")]:
        x, t, lab = keypoint_task(n, 17, a.res // 4, seed=5, background=1.0 if a.task == "noise" else 0.25)
        x, t = x.cuda(), t.cuda()
        rects = {s: np.tile(np.array([0.0, 0.0, s, s]), (n, 1)) for s in (4.0, 8.0)}
        dt = torch.bfloat16 if dn == "bf16" else torch.float32
        torch.manual_seed(0)
        m = P.creatModel(nStack=a.stacks).cuda()
        tr = Trainer(m, lr=lr, dtype=dt, use_graph=True)
        losses, curves = [], {}
        t0 = time.time()
        for s in range(1, a.steps + 1):
            losses.append(float(tr.step(x, t)))
            if s % a.every == 0:
                with torch.no_grad():
                    hm = m.train()(x)[-1]
                c = {str(int(r)): np.nanmean(PCKh()(hm, lab, rects[r])[0], axis=0).round(4).tolist()
                     for r in rects}
                curves[s] = c
                print(f"n {n} {dn} lr {lr:g} step {s} loss {losses[-1]:.5f} PCKh@0.5 box4 {c['4'][10]:.3f} "
                      f"box8 {c['8'][10]:.3f}", flush=True)
        torch.cuda.synchronize()
        res[f"n{n}_{dn}_lr{lr:g}"] = {"loss": losses, "pckh": curves, "seconds": time.time() - t0}
        del tr, m
        torch.cuda.empty_cache()
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump({"args": vars(a), "runs": res}, open(a.out, "w"))


if __name__ == "__main__":
    main()
