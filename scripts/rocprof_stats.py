"""From a rocprofv3 kernel-trace database of a bench.py run: (1) every dispatch per (kernel, grid)
-> csv (calls, avg / min / max / total us); (2) the back-to-back runs of one (kernel, grid) of at
least --run dispatches (bench.py's warm roofline timing loops) with their average, and (3) the
"cold" dispatches of a kernel — each right after the read-only cache flush (torch's sum kernel,
bench._flush_caches), bench.py's cold loops since round 6 — to set beside the bench line's live
HIP-event averages.
  python scripts/rocprof_stats.py run_results.db --csv out.csv [--run 20]"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv")
    ap.add_argument("--run", type=int, default=20)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end, grid_x, workgroup_x from kernels order by start").fetchall()
    agg = {}
    for name, st, en, gx, wx in rows:
        n = name.split("(")[0].replace("void ", "").replace("hgk::", "")
        d = (en - st) / 1e3
        e = agg.setdefault((n, gx, wx), [0, 0.0, 1e30, 0.0])
        e[0] += 1
        e[1] += d
        e[2] = min(e[2], d)
        e[3] = max(e[3], d)
    if a.csv:
        with open(a.csv, "w") as f:
            f.write("kernel,grid_x,workgroup_x,calls,avg_us,min_us,max_us,total_us\n")
            for (n, gx, wx), (k, t, lo, hi) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
                f.write(f'"{n}",{gx},{wx},{k},{t / k:.2f},{lo:.2f},{hi:.2f},{t:.1f}\n')
    # cold dispatches: the kernel right after a flush (a torch reduce kernel), grouped by grid
    cold = {}
    for k in range(1, len(rows)):
        if "reduce_kernel" in rows[k - 1][0] and "hgk::" in rows[k][0]:
            n = rows[k][0].split("(")[0].replace("void ", "").replace("hgk::", "")
            cold.setdefault((n, rows[k][3]), []).append((rows[k][2] - rows[k][1]) / 1e3)
    for (n, gx), ds in sorted(cold.items()):
        if len(ds) >= a.run // 2:
            print(f"cold: {len(ds)} dispatches after a flush  avg {sum(ds) / len(ds):8.2f} us  grid {gx}  {n}")
    # back-to-back runs
    i = 0
    while i < len(rows):
        j = i
        key = (rows[i][0], rows[i][3])
        while j + 1 < len(rows) and (rows[j + 1][0], rows[j + 1][3]) == key:
            j += 1
        if j - i + 1 >= a.run:
            ds = [(rows[k][2] - rows[k][1]) / 1e3 for k in range(i, j + 1)]
            n = key[0].split("(")[0].replace("void ", "").replace("hgk::", "")
            print(f"run of {len(ds)} dispatches  avg {sum(ds) / len(ds):8.2f} us  grid {key[1]}  {n}")
        i = j + 1


if __name__ == "__main__":
    main()
