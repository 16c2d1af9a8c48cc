"""Convergence of the BENCHED configuration (round-5 verdict, next-round item 1; BASELINE.json
north_star "PCKh@0.5 within 0.2 of the CPU reference").

The reference's own training loop (try_with_torch.py:330-344: model(x) -> sum of per-stack
nn.MSELoss -> zero_grad -> backward -> Adam.step) was run on the CPU with the reference classes
(tests/golden/make_golden.py converge <draw>) for 1200 Adam steps (lr 4e-4) from the seeded init on a
fixed learnable synthetic pose batch (data.keypoint_task: 2 crops, 16 scored joints drawn as
coloured cells), in fp32 under several CPU reduction orders ("draws": the train-mode step is
chaotic, tests/gates.py), recording the loss of every step and, every 100 steps, the PCKh curve of
the reference's own PCKh class (train.py:759-791) on the train-mode forward's last stack.

Here the bench's Trainer (bench.build_step: 4-stack creatModel, bf16, hipGraph, default routes,
N = 32) trains on 16 copies of the same 2 crops: BN batch statistics and the mean MSE are unchanged
by duplicating a batch, so this is the same training run at the benched batch and kernel routing
(the duplicates' heatmaps are checked bitwise equal). Rule, fixed before the engine was compared
with the draws:
* PCKh@0.5 after the last step (head boxes of 4 and 8 heatmap pixels), the HIP PCKh kernel
  (targets.PCKh, bit-exact with the reference's class): within 0.2 of the mean over the reference
  draws (north_star), whose own value must be >= 0.5 (the fixture learned the task: 0.85 / 0.96
  over the four draws orig / avx2 / sse41 / nomkl — the 1-pixel box 4 differs between draws by up
  to 0.41, so the originally written 0.8 applied to the fixture, not the engine, was relaxed to 0.5
  after the first GPU run showed the two-draw mean at 0.72; the engine's own criterion is unchanged);
* loss trajectory: the mean loss of every 100-step window within [lo - w, hi + w], lo / hi the
  draws' minimum / maximum of that window, w = max(hi - lo, 0.1 x their mean).
The engine's fp32 path runs the same gates (control)."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
DEV = "cuda"
FIXTURE = os.path.join(GOLDEN, "converge_s4_n2_256.npz")
DRAWS = ("orig", "avx2", "sse41", "nomkl")


def _fixture():
    if not os.path.exists(FIXTURE):
        pytest.skip("no convergence fixture (make_golden.py converge <draw>)")
    g = dict(np.load(FIXTURE))
    runs = [(d, g[f"{d}_loss"], g[f"{d}_pckh"]) for d in DRAWS if f"{d}_loss" in g]
    assert len(runs) >= 2, "the band needs at least two reference draws"
    return g, runs


def _train(dtype, g, rep=16):
    import progressive_process_for_human_pose_estimation_amd as P
    from progressive_process_for_human_pose_estimation_amd.data import keypoint_task
    from progressive_process_for_human_pose_estimation_amd.targets import PCKh
    from progressive_process_for_human_pose_estimation_amd.trainer import Trainer
    n, steps, every, lr = int(g["n"]), int(g["steps"]), int(g["every"]), float(g["lr"])
    x, t, lab = keypoint_task(n, 17, 64, seed=5)
    assert np.array_equal(lab.numpy(), g["labels"])
    xb = x.repeat(rep, 1, 1, 1).to(DEV)
    tb = t.repeat(rep, 1, 1, 1).to(DEV)
    torch.manual_seed(0)
    m = P.creatModel(nStack=4).to(DEV)
    tr = Trainer(m, lr=lr, dtype=dtype, use_graph=True)   # as bench.build_step, at the fixture's lr
    rects = {b: np.tile(np.array([0.0, 0.0, b, b]), (n, 1)) for b in g["boxes"]}
    losses, curves = [], []
    for s in range(1, steps + 1):
        losses.append(tr.step(xb, tb).clone())
        if s % every == 0:
            with torch.no_grad():
                hm = m.train()(xb)[-1]
            # the copies of one crop produce the same heatmaps bit for bit
            assert torch.equal(hm[:n].repeat(rep, 1, 1, 1), hm)
            curves.append(np.stack([np.nanmean(PCKh()(hm[:n], lab, rects[b])[0], axis=0)
                                    for b in g["boxes"]]))
    return torch.cat(losses).cpu().numpy().astype(np.float64), np.stack(curves)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32], ids=["bf16", "fp32"])
def test_benched_trainer_converges_like_the_reference(dtype):
    g, runs = _fixture()
    every = int(g["every"])
    loss, pckh = _train(dtype, g)
    ref_final = np.mean([p[-1] for _, _, p in runs], axis=0)   # [boxes, 11]
    assert np.all(ref_final[:, 10] >= 0.5), ref_final[:, 10]
    for bi, b in enumerate(g["boxes"]):
        print(f"PCKh@0.5 box {b:g}: engine {pckh[-1, bi, 10]:.3f}, reference draws "
              + " ".join(f"{d} {p[-1, bi, 10]:.3f}" for d, _, p in runs))
        assert abs(pckh[-1, bi, 10] - ref_final[bi, 10]) <= 0.2, (b, pckh[-1, bi, 10], ref_final[bi, 10])
    win = lambda v: v.reshape(-1, every).mean(1)  # noqa: E731
    ref_w = np.stack([win(lv) for _, lv, _ in runs])
    eng_w = win(loss)
    lo, hi = ref_w.min(0), ref_w.max(0)
    w = np.maximum(hi - lo, 0.1 * ref_w.mean(0))
    for k in range(len(eng_w)):
        print(f"steps {k * every + 1:5d}-{(k + 1) * every:5d}: engine {eng_w[k]:.6f}  draws "
              f"[{lo[k]:.6f}, {hi[k]:.6f}]  band [{lo[k] - w[k]:.6f}, {hi[k] + w[k]:.6f}]")
    bad = [k for k in range(len(eng_w)) if not (lo[k] - w[k] <= eng_w[k] <= hi[k] + w[k])]
    assert not bad, [(k, eng_w[k], lo[k] - w[k], hi[k] + w[k]) for k in bad]
