"""Engine weight gradients (fp32 and bf16 paths) at N=32 (4-stack, 256x256, first step from the
seeded init) against the reference's fp64 gradients (strided samples in
tests/golden/primary_s4_n32_256.npz): per-parameter cosine similarity and norm ratio, worst
first. Diagnostic for the bf16 gate of test_gpu_parity.py."""
import os
import sys

import numpy as np
import torch
import torch.nn as nn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import progressive_process_for_human_pose_estimation_amd as P  # noqa: E402
from progressive_process_for_human_pose_estimation_amd.data import gaussian_targets, synthetic_images  # noqa: E402

g = np.load(os.path.join(ROOT, "tests", "golden", "primary_s4_n32_256.npz"))
x = synthetic_images(32, 256, 256, seed=1234).cuda()
t = gaussian_targets(32, 17, 64, 64, seed=1)[0].cuda()
for dt in (torch.float32, torch.bfloat16):
    torch.manual_seed(0)
    m = P.creatModel().cuda().set_engine_dtype(dt)
    m.train()
    outs = m(x)
    loss = sum(nn.functional.mse_loss(o, t) for o in outs)
    loss.backward()
    rows, off = [], 0
    for k, p in m.named_parameters():
        if p.grad is None:
            continue
        s = p.grad.detach().double().reshape(-1)[::97].cpu().numpy()
        r = g["grad_sample64"][off:off + len(s)]
        off += len(s)
        cos = float((s * r).sum() / (np.linalg.norm(s) * np.linalg.norm(r) + 1e-300))
        rows.append((cos, float(np.linalg.norm(s) / (np.linalg.norm(r) + 1e-300)), k, float(np.linalg.norm(r))))
    assert off == len(g["grad_sample64"])
    rows.sort()
    big = [r for r in rows if r[3] > 1e-6]
    print(dt, "loss", float(loss.detach()), "median cos (non-zero grads)", np.median([r[0] for r in big]))
    for r in big[:12]:
        print("  cos %.5f ratio %.4f %s ref-norm %.4g" % r)
