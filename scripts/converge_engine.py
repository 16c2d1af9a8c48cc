"""The engine side of tests/test_gpu_converge.py without the fixture: trains the bench's Trainer
(N = 32 = 16 copies of data.keypoint_task's 2 crops) for the fixture's schedule and saves the loss
of every step and the PCKh curves to gpurun_out/converge_engine_<dtype>.npz (for the tables in
DESIGN.md; the test gates the same numbers). usage (GPU box): python scripts/converge_engine.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_gpu_converge as T  # noqa: E402

g = {"n": 2, "steps": 1200, "every": 100, "lr": 4e-4, "boxes": np.array([4.0, 8.0]), "labels": None}
from progressive_process_for_human_pose_estimation_amd.data import keypoint_task  # noqa: E402
g["labels"] = keypoint_task(2, 17, 64, seed=5)[2].numpy()
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
for dt, tag in ((torch.bfloat16, "bf16"), (torch.float32, "fp32")):
    loss, pckh = T._train(dt, g)
    np.savez(os.path.join(ROOT, "gpurun_out", f"converge_engine_{tag}.npz"), loss=loss, pckh=pckh)
    print(tag, "final PCKh@0.5 box4 %.3f box8 %.3f" % (pckh[-1, 0, 10], pckh[-1, 1, 10]),
          "window losses", np.round(loss.reshape(-1, 100).mean(1), 6).tolist(), flush=True)
