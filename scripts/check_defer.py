"""Gradient of one training step with the deferred (multi-use) weight-grads vs per-use launches
(bench configuration). The two differ only in fp32 summation order.

  python scripts/check_defer.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import progressive_process_for_human_pose_estimation_amd as P  # noqa: E402
from progressive_process_for_human_pose_estimation_amd.data import gaussian_targets, synthetic_images  # noqa: E402
from progressive_process_for_human_pose_estimation_amd.trainer import Trainer  # noqa: E402


def grads(tr, x, t, defer):
    os.environ["HGK_WGRAD_DEFER_M"] = "8192" if defer else "0"
    os.environ["HGK_WGRAD_DEFER_M_1X1"] = str(1 << 30) if defer else "0"
    tr._fwd_bwd(x, t)
    torch.cuda.synchronize()
    return tr.fp.grad.clone()


def main():
    torch.manual_seed(0)
    model = P.creatModel(nStack=int(os.environ.get("CD_STACKS", "4"))).cuda()
    tr = Trainer(model, dtype=torch.bfloat16, use_graph=False)
    n, r = 32, 256
    x = synthetic_images(n, r, r, seed=1234).cuda()
    t = gaussian_targets(n, 17, r // 4, seed=1)[0].cuda()
    g0 = grads(tr, x, t, False)
    g1 = grads(tr, x, t, True)
    g2 = grads(tr, x, t, False)
    off = 0
    worst = []
    for name, p in model.named_parameters():
        k = p.numel()
        a, b, c = g0[off:off + k], g1[off:off + k], g2[off:off + k]
        den = float(a.norm()) + 1e-30
        worst.append((float((a - b).norm()) / den, float((a - c).norm()) / den, name))
        off += k
    worst.sort(reverse=True)
    for w in worst[:8]:
        print(f"defer-vs-not {w[0]:.3e}   rerun {w[1]:.3e}   {w[2]}")


if __name__ == "__main__":
    main()
