"""Per-step wall time of a bench.py configuration (each step synchronised), to see how many steps
a line needs before it is steady state (round-5 verdict: the `train` preset measured 768.7 img/s
over 10 steps vs ~950 over 30). usage (GPU box):
  python scripts/step_times.py --preset train --steps 60 [--warmup 0]"""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="train")
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--batch", type=int, default=None)
    a = ap.parse_args()
    N = a.batch or (16 if a.preset in ("try_with_aspp", "try_more_layer", "train") else 32)
    stacks = {"try_with_aspp": 3, "train": 3}.get(a.preset, 4)
    tr, x, t, work = bench.build_step(a.preset, stacks, torch.bfloat16, N, 256, 0)
    print(work, flush=True)
    times = []
    for s in range(a.steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tr.step(x, t)
        torch.cuda.synchronize()
        times.append((time.perf_counter() - t0) * 1e3)
        print(f"step {s:3d} {times[-1]:8.2f} ms  {N / times[-1] * 1e3:8.1f} img/s", flush=True)
    for lo in (5, 10, 20, 30):
        if lo < len(times):
            w = times[lo:]
            print(f"mean over steps {lo}..{len(times) - 1}: {sum(w) / len(w):.2f} ms "
                  f"= {N * len(w) / sum(w) * 1e3:.1f} img/s")


if __name__ == "__main__":
    main()
