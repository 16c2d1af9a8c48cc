"""bf16 gradient sensitivity to kernel routing: the batch-32 production step (the parity test's
inputs) under several route configurations (engine.apply_route_spec) in ONE process; per-parameter relative gradient
difference and cosine between configurations, next to the fp64 fixture's norms.

  python scripts/grad_noise.py "ring_nw=8" "ring_nw=4,ring_small=0" "ring_nw=4"
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_gpu_parity as T  # noqa: E402


def run(cfg):
    from progressive_process_for_human_pose_estimation_amd import engine as E
    cms = E.apply_route_spec(cfg)
    g, st, x, t = T._batch32()
    m = T.build(4, 17).to(T.DEV).set_engine_dtype(torch.bfloat16)
    out, loss = T.train_step(m, x, t)
    grads = [p.grad.detach().double().cpu().reshape(-1) for p in m.parameters() if p.grad is not None]
    names = [n for n, p in m.named_parameters() if p.grad is not None]
    for cm in reversed(cms):
        cm.__exit__(None, None, None)
    return names, grads, out, loss, g


def main():
    cfgs = sys.argv[1:]
    res = [run(c) for c in cfgs]
    names, g = res[0][0], res[0][4]
    n64 = g["grad_norm64"]
    n64 = n64[n64 >= 0]
    nbf = g["grad_normbf16"]
    ok = g["grad_norm64"] >= 0
    n64a, nbfa = g["grad_norm64"][ok], nbf[ok]
    for c, r in zip(cfgs, res):
        # the parity test's per-parameter gate (tests/test_gpu_parity.py)
        norms = np.array([float(x.norm()) for x in r[1]])
        err, err_ref = np.abs(norms - n64a), np.abs(nbfa - n64a)
        lim = 0.1 * n64a + 4 * err_ref + 1e-4 * n64a.max()
        bad = np.nonzero(err > lim)[0]
        ratio = np.median(err / np.maximum(err_ref, 1e-12))
        print(f"[{c}] gate: {len(bad)} of {len(err)} params over; median ratio {ratio:.3f}; over: "
              + ", ".join(f"{r[0][k]} err {err[k]:.3g} lim {lim[k]:.3g} n64 {n64a[k]:.3g}" for k in bad[:6]))
    for i in range(len(cfgs)):
        for j in range(i + 1, len(cfgs)):
            ga, gb = res[i][1], res[j][1]
            rel = np.array([float((a - b).norm() / max(a.norm(), 1e-30)) for a, b in zip(ga, gb)])
            cos = np.array([float((a * b).sum() / max(a.norm() * b.norm(), 1e-30)) for a, b in zip(ga, gb)])
            nerr = np.array([abs(float(a.norm()) - float(b.norm())) for a, b in zip(ga, gb)])
            print(f"[{cfgs[i]}] vs [{cfgs[j]}]: loss {res[i][3]:.6f} / {res[j][3]:.6f}; out max diff "
                  f"{np.abs(res[i][2] - res[j][2]).max():.4f}; grad rel diff median {np.median(rel):.3f} "
                  f"max {rel.max():.3f}; cosine median {np.median(cos):.3f} min {cos.min():.3f}; "
                  f"norm diff / fp64 norm max {np.max(nerr / np.maximum(n64, 1e-12)):.3f}")
            worst = np.argsort(-rel)[:5]
            print("   worst:", ", ".join(f"{names[k]} rel {rel[k]:.2f} cos {cos[k]:.2f}" for k in worst))


if __name__ == "__main__":
    main()
