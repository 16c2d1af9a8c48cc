"""Per-step kernel statistics from a rocprofv3 sqlite database (rocprofv3 --kernel-trace -o run).

usage: python scripts/db_stats.py gpurun_out/prof/run_results.db [--csv out.csv] [--steps K]

Steps are delimited by the Adam kernel (the last launch of a training step). Prints, per step
averaged over the last K steps: wall time, summed kernel time, idle gap time, the launch count,
and a per-kernel table (calls/step, us/step, avg us, share).
"""
import argparse
import collections
import sqlite3


def short(name):
    n = name.split("(")[0]
    return n.replace("void ", "").replace("hgk::", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--by-grid", help="also write a per (kernel, grid_x, workgroup_x) table here")
    ap.add_argument("--gaps", type=int, default=0,
                    help="print the N largest idle gaps of the last step (kernels either side)")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end, grid_x, workgroup_x from kernels order by start").fetchall()
    ends = [i for i, r in enumerate(rows) if r[0].startswith("hgk::adam_kernel")]
    if len(ends) < a.steps + 1:
        raise SystemExit(f"only {len(ends)} steps in trace")
    sel = ends[-(a.steps + 1):]
    agg = collections.defaultdict(lambda: [0, 0.0])
    aggg = collections.defaultdict(lambda: [0, 0.0])
    wall = busy = 0.0
    nl = 0
    for s0, s1 in zip(sel[:-1], sel[1:]):
        seg = rows[s0 + 1:s1 + 1]
        wall += (seg[-1][2] - rows[s0][2]) / 1e3
        for name, st, en, gx, wx in seg:
            d = (en - st) / 1e3
            busy += d
            nl += 1
            key = short(name)
            agg[key][0] += 1
            agg[key][1] += d
            aggg[(key, gx, wx)][0] += 1
            aggg[(key, gx, wx)][1] += d
    if a.gaps:
        seg = rows[sel[-2]:sel[-1] + 1]
        gl, last_end = [], seg[0][2]
        for i in range(1, len(seg)):
            g = (seg[i][1] - last_end) / 1e3
            if g > 0:
                gl.append((g, short(seg[i - 1][0])[:50], short(seg[i][0])[:50], i))
            last_end = max(last_end, seg[i][2])
        gl.sort(reverse=True)
        print(f"largest gaps of the last step (total {sum(x[0] for x in gl):.1f} us over {len(gl)}):")
        for g, p0, p1, i in gl[:a.gaps]:
            print(f"  {g:8.1f} us  before launch {i}: {p0} -> {p1}")
    k = a.steps
    print(f"per step: wall {wall / k:.1f} us, kernel busy {busy / k:.1f} us, "
          f"idle {(wall - busy) / k:.1f} us, launches {nl / k:.0f}")
    items = sorted(agg.items(), key=lambda kv: -kv[1][1])
    lines = ["kernel,calls_per_step,us_per_step,avg_us,share"]
    for key, (n, t) in items:
        lines.append(f"\"{key}\",{n / k:.0f},{t / k:.1f},{t / n:.2f},{t / busy:.4f}")
    for ln in lines[:a.top + 1]:
        print(ln)
    if a.by_grid:
        with open(a.by_grid, "w") as f:
            f.write("kernel,grid_x,workgroup_x,calls_per_step,us_per_step,avg_us,share\n")
            for (key, gx, wx), (n, t) in sorted(aggg.items(), key=lambda kv: -kv[1][1]):
                f.write(f"\"{key}\",{gx},{wx},{n / k:.0f},{t / k:.1f},{t / n:.2f},{t / busy:.4f}\n")
    if a.csv:
        with open(a.csv, "w") as f:
            f.write(f"# per step over the last {k} steps: wall {wall / k:.1f} us, busy {busy / k:.1f} us, "
                    f"launches {nl / k:.0f}\n")
            f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
