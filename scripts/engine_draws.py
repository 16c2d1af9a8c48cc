"""Engine fp32 'draws' of the configs[4] step (8-stack 384x384, N=16 or 8) under equally valid
routings, saved for a per-parameter comparison with the reference's fp32 draws
(scripts/draw_compare.py). A spec is 'name=value,...' over engine / library routes ('' = the
defaults); `--perturb K` adds K more draws per spec whose input differs from the fixture's in the
last bit of a few hundred seeded elements (the same size of perturbation as one fp32 rounding), so
the spread of ONE routing under the step's chaotic train-mode BN is measured next to the spread
between routings.
usage (GPU box): python scripts/engine_draws.py [--n 16] [--specs ';twin=0'] [--perturb 0]
  -> gpurun_out/engine_draws_s8_n<N>.npz"""
import argparse
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import progressive_process_for_human_pose_estimation_amd as P  # noqa: E402
from progressive_process_for_human_pose_estimation_amd import engine as E  # noqa: E402
from progressive_process_for_human_pose_estimation_amd.data import gaussian_targets, synthetic_images  # noqa: E402


def perturbed(x, seed, count=256):
    """x with `count` seeded elements moved by one ulp (fp32 nextafter, alternating direction)."""
    g = torch.Generator().manual_seed(seed)
    idx = torch.randperm(x.numel(), generator=g)[:count]
    flat = x.clone().reshape(-1)
    up = torch.full((count,), float("inf"))
    up[1::2] = -float("inf")
    flat[idx] = torch.nextafter(flat[idx], up)
    return flat.view_as(x)


def tag_of(spec, k):
    base = spec.replace("=", "").replace(",", "_") or "default"
    return base if k == 0 else f"{base}_p{k}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16)
    ap.add_argument("--specs", default=";twin=0")
    ap.add_argument("--perturb", type=int, default=0)
    a = ap.parse_args()
    n = a.n
    x0 = synthetic_images(n, 384, 384, seed=1234)
    t = gaussian_targets(n, 17, 96, 96, seed=1)[0].cuda()
    out = {}
    for spec in a.specs.split(";"):
        for k in range(a.perturb + 1):
            tag = tag_of(spec, k)
            x = (x0 if k == 0 else perturbed(x0, 100 + k)).cuda()
            cms = E.apply_route_spec(spec) if spec else ()
            torch.manual_seed(0)
            m = P.creatModel(nStack=8).cuda().set_graph_mode(False)
            outs = m(x)
            loss = sum(F.mse_loss(o, t) for o in outs)
            loss.backward()
            torch.cuda.synchronize()
            out[f"{tag}_loss"] = np.array(float(loss.detach()))
            out[f"{tag}_grad_norm"] = np.array([-1.0 if p.grad is None else float(p.grad.double().norm())
                                                for p in m.parameters()])
            out[f"{tag}_grad_sample"] = np.concatenate(
                [p.grad.detach().double().reshape(-1)[::97].cpu().numpy()
                 for p in m.parameters() if p.grad is not None])
            for cm in reversed(cms):
                cm.__exit__(None, None, None)
            print(tag, "loss", float(loss.detach()), flush=True)
            del m, outs, loss
            torch.cuda.empty_cache()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez(os.path.join(ROOT, "gpurun_out", f"engine_draws_s8_n{n}.npz"), **out)


if __name__ == "__main__":
    main()
