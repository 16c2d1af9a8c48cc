"""Is a preset's graph-replayed step bound by the host? Times K trainer.step() calls on the host
(no device sync: the graph launches are asynchronous) against the device time of the same K steps.
A host time per step close to the device time means the CPU-side graph submission paces the GPU.
  python scripts/host_launch_probe.py [preset ...]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    for p in sys.argv[1:] or ["primary", "try_with_aspp"]:
        N, S = (16, 3) if p == "try_with_aspp" else (32, 4)
        trainer, x, t, _ = bench.build_step(p, S, torch.bfloat16, N, 256, 0)
        for _ in range(5):
            trainer.step(x, t)
        torch.cuda.synchronize()
        K = 20
        g = trainer.graph
        # the graph alone: K replays, host time of the launches vs device time
        t0 = time.perf_counter()
        for _ in range(K):
            g.replay()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        # whole steps
        t3 = time.perf_counter()
        for _ in range(K):
            trainer.step(x, t)
        t4 = time.perf_counter()
        torch.cuda.synchronize()
        t5 = time.perf_counter()
        print(f"{p}: graph replay host {1e3 * (t1 - t0) / K:.2f} ms/replay, device {1e3 * (t2 - t0) / K:.2f} ms/replay; "
              f"step host {1e3 * (t4 - t3) / K:.2f} ms, wall {1e3 * (t5 - t3) / K:.2f} ms", flush=True)
        del trainer


if __name__ == "__main__":
    main()
