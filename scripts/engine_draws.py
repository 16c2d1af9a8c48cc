"""Engine fp32 'draws' of the configs[4] step (8-stack 384x384, N=16 or 8) under equally valid
routings, saved for a per-parameter comparison with the reference's fp32 draws
(scripts/draw_compare.py). usage (GPU box): python scripts/engine_draws.py [N] -> gpurun_out/"""
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

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
x = synthetic_images(n, 384, 384, seed=1234).cuda()
t = gaussian_targets(n, 17, 96, 96, seed=1)[0].cuda()
out = {}
for tag, spec in (("default", ""), ("twin0", "twin=0")):
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
    out[f"{tag}_grad_sample"] = np.concatenate([p.grad.detach().double().reshape(-1)[::97].cpu().numpy()
                                                for p in m.parameters() if p.grad is not None])
    for cm in reversed(cms):
        cm.__exit__(None, None, None)
    print(tag, "loss", float(loss.detach()), flush=True)
    del m, outs, loss
    torch.cuda.empty_cache()
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", f"engine_draws_s8_n{n}.npz"), **out)
