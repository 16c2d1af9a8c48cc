"""Can throughput work hide under the latency-bound small-level chain? (hipGraph, MI355X)

chain = the 8x8 level's conv1 (1x1 256->128, N=32, BN in, stats out) launched `--chain` times back
to back on the main stream (each ~7 us, few workgroups); side = the 64x64 3x3 halo weight grad
(hgk_conv_wgrad_accum, ~42 us, full GPU) `--side` times on a second stream. Times: each alone and
both in one graph (fork/join by events). If chain+side ~= max(chain, side), weight grads can be
moved off the backward's critical path onto a side stream.

  python scripts/overlap_probe.py [--chain 400] [--side 40]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from progressive_process_for_human_pose_estimation_amd import hgk as H  # noqa: E402

DEV = "cuda"


def conv_small(L):
    N, hw, cin, cout = 32, 8, 256, 128
    M = N * hw * hw
    x = (torch.randn(N, hw, hw, cin, device=DEV) * 0.5).to(torch.bfloat16)
    w = torch.randn(cout, cin, 1, 1, device=DEV) * 0.05
    ld = L.hgk_conv_w_ld(cin)
    wp = torch.empty(128, ld, device=DEV, dtype=torch.bfloat16)
    H.check(L.hgk_pack_conv_weight(H.stream_handle(), 1, w.data_ptr(), wp.data_ptr(), ld, cout, cin,
                                   1, 1, 0, cout, cin))
    sc = torch.rand(cin, device=DEV) + 0.5
    sh = torch.randn(cin, device=DEV) * 0.1
    y = torch.empty(N, hw, hw, cout, device=DEV, dtype=torch.bfloat16)
    part = torch.empty((2 * (M // 64) + 4) * 3 * cout, device=DEV)
    rows = H.ctypes.c_int(0)
    ws_b = L.hgk_conv_fwd_workspace(1, N, hw, hw, cin, cout, 1, 1, 1, 0, 1)
    ws = torch.zeros(max(ws_b, 1), dtype=torch.uint8, device=DEV)

    def fn():
        H.check(L.hgk_conv_fwd(H.stream_handle(), 1, x.data_ptr(), wp.data_ptr(), ld, None, None,
                               y.data_ptr(), sc.data_ptr(), sh.data_ptr(), 1, 0, part.data_ptr(),
                               H.ctypes.byref(rows), N, hw, hw, cin, cout, 1, 1, 1, 0, 1,
                               ws.data_ptr(), ws_b))
    fn.keep = (x, wp, sc, sh, y, part, ws)
    return fn


def wgrad_big(L):
    N, hw, cin, cout = 32, 64, 128, 128
    x = (torch.randn(N, hw, hw, cin, device=DEV) * 0.5).to(torch.bfloat16)
    dy = (torch.randn(N, hw, hw, cout, device=DEV) * 0.5).to(torch.bfloat16)
    sc = torch.rand(cin, device=DEV) + 0.5
    sh = torch.randn(cin, device=DEV) * 0.1
    cap = L.hgk_conv_wgrad_max_splits()
    slabs = torch.zeros(L.hgk_conv_wgrad_slab_bytes(cin, cout, 3, 3, cap), dtype=torch.uint8,
                        device=DEV)
    splits = H.ctypes.c_int(0)

    def fn():
        H.check(L.hgk_conv_wgrad_accum(H.stream_handle(), 1, x.data_ptr(), dy.data_ptr(),
                                       sc.data_ptr(), sh.data_ptr(), 1, slabs.data_ptr(), cap, cap,
                                       1, H.ctypes.byref(splits), N, hw, hw, cin, cout, 3, 3, 1, 1, 1))
    fn.keep = (x, dy, sc, sh, slabs)
    return fn


EAGER = False


def graph_us(body):
    if EAGER:
        body()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        body()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3
    s0 = torch.cuda.Stream()
    s0.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s0):
        body()  # warm
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s0):
            body()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e30
    for _ in range(3):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3)
    return best


def _capture(body, stream):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(stream):
        body()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=stream):
            body()
    torch.cuda.synchronize()
    return g


def two_graphs_us(chain, sidework, side_eager=False):
    """chain graph replayed on stream A while the side graph replays (or the side work is
    launched eagerly) on stream B"""
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    ga = _capture(chain, sa)
    gb = None if side_eager else _capture(sidework, sb)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e30
    for _ in range(3):
        torch.cuda.synchronize()
        e0.record(sa)
        sb.wait_event(e0)
        with torch.cuda.stream(sb):
            if gb is None:
                sidework()
            else:
                gb.replay()
        with torch.cuda.stream(sa):
            ga.replay()
        sa.wait_stream(sb)
        e1.record(sa)
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chain", type=int, default=400)
    ap.add_argument("--side", type=int, default=40)
    ap.add_argument("--eager", action="store_true", help="no graph: host-launched streams")
    ap.add_argument("--graph-eager", action="store_true",
                    help="chain graph on stream A, side work launched eagerly on stream B")
    ap.add_argument("--two-graphs", action="store_true",
                    help="chain and side work as two graphs replayed on two streams")
    args = ap.parse_args()
    global EAGER
    EAGER = args.eager
    L = H.load_library()
    small, big = conv_small(L), wgrad_big(L)
    side = torch.cuda.Stream()

    def chain():
        for _ in range(args.chain):
            small()

    def sidework():
        for _ in range(args.side):
            big()

    def both():
        cur = torch.cuda.current_stream()
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            sidework()
        chain()
        cur.wait_stream(side)

    tc = graph_us(chain)
    ts = graph_us(sidework)
    if args.two_graphs:
        tb = two_graphs_us(chain, sidework)
    elif args.graph_eager:
        tb = two_graphs_us(chain, sidework, side_eager=True)
    else:
        tb = graph_us(both)
    print(f"chain alone {tc:9.1f} us ({tc / args.chain:.2f} us/launch) | side alone {ts:9.1f} us "
          f"({ts / args.side:.1f} us/launch) | both {tb:9.1f} us | sum {tc + ts:9.1f} max "
          f"{max(tc, ts):9.1f} -> hidden {(tc + ts - tb) / ts:.2f} of the side work", flush=True)


if __name__ == "__main__":
    main()
