"""HBM traffic of bench.py's roofline kernels from rocprofv3 PMC counters.

Run each counter in its OWN pass (FETCH_SIZE and WRITE_SIZE cannot share one on gfx950):

  rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- \
      python3 scripts/roofline_pmc.py run
  rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- \
      python3 scripts/roofline_pmc.py run
  python3 scripts/roofline_pmc.py parse gpurun_out/pmc_fetch gpurun_out/pmc_write > profiles/r02_roofline_pmc.json

`run` launches exactly bench.py's two roofline launches (roofline_dominant: the 1x1 conv1 at
64x64; roofline_mfma: the 3x3 conv). `parse` averages the per-dispatch counters of each kernel:
bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (KiB units; FETCH_SIZE counts half of a
16-B-per-lane streaming read on gfx950: MI355X_MICROARCH.md §HBM). bench.py reports the result as
roofline.traffic / roofline_mfma.traffic.
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# bench key -> kernel-name substring of its launch
KERNELS = {"conv1x1": "conv1x1_ring_kernel", "conv3x3": "conv3x3_row_kernel"}


def run():
    import torch
    import bench
    torch.cuda.set_device(0)
    r1 = bench.roofline_dominant(torch.bfloat16, 32, 256)
    r2 = bench.roofline_mfma(torch.bfloat16, 32, 256)
    print(json.dumps([r1, r2]))


def counter_avg(d, name, kernel_sub):
    vals, names = {}, set()
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if kernel_sub in row["Kernel_Name"] and row["Counter_Name"] == name:
                vals[row["Dispatch_Id"]] = vals.get(row["Dispatch_Id"], 0.0) + float(row["Counter_Value"])
                names.add(row["Kernel_Name"].split("(")[0])
    return sum(vals.values()) / max(1, len(vals)), len(vals), sorted(names)


def parse(dfetch, dwrite):
    out = {"note": "FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM (gfx950 counts half of a "
                   "16-B/lane streaming read); separate --pmc passes; averages over every "
                   "dispatch of the kernel in bench.py's roofline timing loops"}
    for key, sub in KERNELS.items():
        f, nf, names = counter_avg(dfetch, "FETCH_SIZE", sub)
        w, nw, _ = counter_avg(dwrite, "WRITE_SIZE", sub)
        out[key] = {"kernel": names, "dispatches": [nf, nw], "fetch_size_kib": f,
                    "write_size_kib": w, "hbm_bytes_per_launch": (2.0 * f + w) * 1024.0}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        parse(sys.argv[2], sys.argv[3])
