"""Average rocprofv3 PMC counters per dispatch of the kernels whose name contains a substring.

  rocprofv3 --pmc C1 C2 ... --output-format csv -d D -o run -- python3 scripts/conv_bench.py ...
  python3 scripts/pmc_kernel.py D <kernel-substring>
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    d, sub = sys.argv[1], sys.argv[2]
    per = defaultdict(lambda: defaultdict(float))
    names = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if sub in r["Kernel_Name"]:
                per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
                names[r["Dispatch_Id"]] = r["Kernel_Name"].split("(")[0]
    if not per:
        raise SystemExit("no dispatch of " + sub)
    keys = sorted({k for v in per.values() for k in v})
    n = len(per)
    print(f"{n} dispatches of {sorted(set(names.values()))}")
    for k in keys:
        print(f"  {k:32s} {sum(v.get(k, 0.0) for v in per.values()) / n:16.1f}")


if __name__ == "__main__":
    main()
