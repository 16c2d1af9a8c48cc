"""Ordered kernel list of ONE training step from a rocprofv3 sqlite database (kernel trace):
start offset, duration, gap to the previous kernel, grid (workgroups) and block size, kernel name.
The step is the last complete one (delimited by the Adam kernel).

usage: python scripts/step_dump.py gpurun_out/prof/run_results.db > step.txt
"""
import sqlite3
import sys


def main():
    c = sqlite3.connect(sys.argv[1])
    rows = c.execute("select name, start, end, grid_x, grid_y, grid_z, workgroup_x from kernels "
                     "order by start").fetchall()
    ends = [i for i, r in enumerate(rows) if r[0].startswith("hgk::adam_kernel")]
    s0, s1 = ends[-2], ends[-1]
    seg = rows[s0 + 1:s1 + 1]
    t0 = rows[s0][2]
    prev = t0
    for name, st, en, gx, gy, gz, wx in seg:
        n = name.split("(")[0].replace("void ", "").replace("hgk::", "")
        print(f"{(st - t0) / 1e3:9.2f} {(en - st) / 1e3:7.2f} {(st - prev) / 1e3:6.2f} "
              f"{gx // max(wx, 1)}x{gy}x{gz}/{wx} {n}")
        prev = en


if __name__ == "__main__":
    main()
