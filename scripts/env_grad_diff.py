"""Per-parameter gradient difference of ONE Trainer step between two route settings
(engine.apply_route_spec, e.g. a kernel-route switch): each setting runs in its own child process,
grads are saved under gpurun_out/, then compared parameter by parameter.

  python scripts/env_grad_diff.py "ring_minm=0" "ring_minm=65536" [--n 4] [--res 128] [--dtype fp32]
"""
import argparse
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child(a, out):
    import progressive_process_for_human_pose_estimation_amd as P
    from progressive_process_for_human_pose_estimation_amd.data import gaussian_targets, synthetic_images
    from progressive_process_for_human_pose_estimation_amd.trainer import Trainer
    from progressive_process_for_human_pose_estimation_amd import engine as E
    E.apply_route_spec(a.route)
    dt = torch.float32 if a.dtype == "fp32" else torch.bfloat16
    x = synthetic_images(a.n, a.res, a.res, seed=100).cuda()
    t = gaussian_targets(a.n, 17, a.res // 4, seed=200)[0].cuda()
    torch.manual_seed(0)
    m = P.creatModel(nStack=a.stacks).cuda()
    tr = Trainer(m, lr=1e-4, dtype=dt, use_graph=False)
    tr.step(x, t)
    torch.cuda.synchronize()
    g = tr.fp.grad.detach().float().cpu()
    base = tr.fp.flat.data_ptr()
    grads = {}
    for n, p in m.named_parameters():
        o = (p.data_ptr() - base) // 4
        grads[n] = g[o:o + p.numel()].clone()
    torch.save(grads, out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("envs", nargs=2)
    ap.add_argument("--n", type=int, default=4)
    ap.add_argument("--res", type=int, default=128)
    ap.add_argument("--stacks", type=int, default=2)
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--child", default=None)
    ap.add_argument("--route", default="")
    a = ap.parse_args()
    if a.child:
        child(a, a.child)
        return
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    outs = []
    for i, e in enumerate(a.envs):
        out = os.path.join(ROOT, "gpurun_out", f"grads_{i}.pt")
        cmd = [sys.executable, os.path.abspath(__file__), *a.envs, "--n", str(a.n), "--res", str(a.res),
               "--stacks", str(a.stacks), "--dtype", a.dtype, "--child", out, "--route", e]
        subprocess.run(cmd, check=True, timeout=240)
        outs.append(torch.load(out, weights_only=True))
    g0, g1 = outs
    rows = []
    for k in g0:
        d = (g0[k] - g1[k]).norm().item()
        n = g0[k].norm().item()
        rows.append((d / max(n, 1e-30), d, n, k))
    rows.sort(reverse=True)
    for r in rows[:15]:
        print("rel %.3e  abs %.3e  norm %.3e  %s" % r)


if __name__ == "__main__":
    main()
