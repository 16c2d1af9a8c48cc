"""Per-step kernel breakdown from a rocprofv3 kernel trace of `bench.py`.

  python scripts/trace_breakdown.py gpurun_out/prof/run_kernel_trace.csv [--top 40]

Takes the last complete training step (delimited by the Adam kernel), groups launches by
(kernel, grid, block) and prints time per step, launch counts and the idle gaps between
consecutive kernels (dispatch overhead inside the hipGraph).
"""
import argparse
import csv
import re
from collections import defaultdict


def short(name):
    name = re.sub(r"\(.*$", "", name) if not name.startswith("void ") else name
    name = name.replace("void ", "").replace("hgk::", "").replace("bf16_t", "bf16")
    return re.sub(r"\((hgk::)?Conv\w+Args\)|\(.*\)$", "", name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    adam = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
    lo, hi = adam[-2] + 1, adam[-1] + 1
    step = rows[lo:hi]
    t0, t1 = int(step[0]["Start_Timestamp"]), int(step[-1]["End_Timestamp"])
    busy = 0
    gaps = []
    agg = defaultdict(lambda: [0, 0.0])
    prev_end = None
    for r in step:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        busy += e - s
        if prev_end is not None:
            gaps.append(s - prev_end)
        prev_end = e
        key = (short(r["Kernel_Name"]),
               f'{int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])}x'
               f'{r["Grid_Size_Y"]}x{r["Grid_Size_Z"]}/{r["Workgroup_Size_X"]}')
        agg[key][0] += 1
        agg[key][1] += (e - s) / 1e3
    span = (t1 - t0) / 1e3
    print(f"step span {span:.1f} us, kernel busy {busy / 1e3:.1f} us, launches {len(step)}, "
          f"sum gaps {sum(gaps) / 1e3:.1f} us (median gap {sorted(gaps)[len(gaps) // 2] / 1e3:.2f} us)")
    byk = defaultdict(lambda: [0, 0.0])
    for (k, g), (n, t) in agg.items():
        byk[k][0] += n
        byk[k][1] += t
    print("\n-- by kernel --")
    for k, (n, t) in sorted(byk.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{t:9.1f} us {100 * t / span:5.1f}%  n={n:4d}  avg={t / n:7.1f}  {k}")
    print("\n-- by kernel x grid --")
    for (k, g), (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{t:9.1f} us {100 * t / span:5.1f}%  n={n:4d}  avg={t / n:7.1f}  {g:>18s}  {k}")


if __name__ == "__main__":
    main()
