"""Per-launch cost of dependent back-to-back kernels, eager and in a hipGraph, and whether two
independent chains captured on two streams overlap inside one graph.

  python scripts/launch_floor.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from progressive_process_for_human_pose_estimation_amd import hgk as H  # noqa: E402


def timed(fn, reps=5):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    L = H.load_library()
    n = 2000
    elems = int(os.environ.get("LF_ELEMS", "64"))
    xa = torch.zeros(elems, device="cuda", dtype=torch.bfloat16)
    xb = torch.zeros(elems, device="cuda", dtype=torch.bfloat16)

    def chain(x, count):
        st = H.stream_handle()
        for _ in range(count):
            H.check(L.hgk_add(st, H.BF16, x.data_ptr(), None, x.data_ptr(), elems, 1))

    chain(xa, 10)
    print(f"eager: {timed(lambda: chain(xa, n), 1) / n:.2f} us per launch")
    cap = torch.cuda.Stream()
    side = torch.cuda.Stream()
    cap.wait_stream(torch.cuda.current_stream())
    g1 = torch.cuda.CUDAGraph()
    with torch.cuda.stream(cap):
        with torch.cuda.graph(g1, stream=cap):
            chain(xa, 2 * n)
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.stream(cap):
        with torch.cuda.graph(g2, stream=cap):
            side.wait_stream(cap)
            chain(xa, n)
            with torch.cuda.stream(side):
                chain(xb, n)
            cap.wait_stream(side)
    torch.cuda.synchronize()
    g1.replay()
    g2.replay()
    t1 = timed(g1.replay)
    t2 = timed(g2.replay)
    print(f"graph, one chain of {2 * n}: {t1:.0f} us ({t1 / (2 * n):.2f} us per launch)")
    print(f"graph, two chains of {n} on two streams: {t2:.0f} us ({t2 / n:.2f} us per launch-pair)")


if __name__ == "__main__":
    main()
