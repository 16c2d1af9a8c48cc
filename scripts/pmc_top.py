"""Per-kernel HBM traffic and MFMA / wave-state counters of one training step (rocprofv3 PMC).

Three PMC passes, each its own rocprofv3 run (gfx950 slot limits: FETCH_SIZE takes 3 of the 4 TCC
slots, WRITE_SIZE 2, so they cannot share a pass; <= 8 SQ and <= 2 GRBM counters per pass):

  rocprofv3 --pmc FETCH_SIZE -d D/fetch -o run --output-format csv -- python3 scripts/pmc_top.py run
  rocprofv3 --pmc WRITE_SIZE -d D/write -o run --output-format csv -- python3 scripts/pmc_top.py run
  rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY \
      SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_MOPS SQ_LDS_BANK_CONFLICT \
      GRBM_GUI_ACTIVE -d D/sq -o run --output-format csv -- python3 scripts/pmc_top.py run
  python3 scripts/pmc_top.py parse D/fetch D/write D/sq STEP_STATS.csv > profiles/<round>_pmc_top5.json

`run` executes STEPS eager (un-graphed, so every dispatch is attributed) training steps of bench.py's
workload (4-stack, 256x256, N=32, bf16). `parse` sums every counter per (kernel, grid) and per
kernel over the run, divides by STEPS, and joins the per-step time of each kernel from the
graph-replayed kernel trace (`STEP_STATS.csv`, scripts/db_stats.py --csv). Units and corrections
(MI355X_MICROARCH.md §HBM, §rocprofv3): HBM bytes = 2 * FETCH_SIZE + WRITE_SIZE (KiB); MFMA busy
= SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 1024 SIMDs) (GRBM_GUI_ACTIVE is summed
over the 8 XCDs; 256 CUs x 4 SIMDs); SQ_WAVE_CYCLES / SQ_WAIT_* count quad-cycles.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
STEPS = 2


def run():
    import torch
    import progressive_process_for_human_pose_estimation_amd as P
    from progressive_process_for_human_pose_estimation_amd.data import gaussian_targets, synthetic_images
    from progressive_process_for_human_pose_estimation_amd.trainer import Trainer
    torch.cuda.set_device(0)
    torch.manual_seed(0)
    model = P.creatModel(nStack=4).cuda()
    tr = Trainer(model, lr=1e-5, dtype=torch.bfloat16, use_graph=False)
    x = synthetic_images(32, 256, 256, seed=1234).cuda()
    t = gaussian_targets(32, 17, 64, seed=1)[0].cuda()
    for _ in range(STEPS):
        tr.step(x, t)
    torch.cuda.synchronize()
    print("pmc_top run: %d eager steps done" % STEPS)


def short(name):
    """same key as scripts/db_stats.py"""
    return name.replace("void ", "").split("(")[0].replace("hgk::", "")


def load(d):
    """{(kernel, grid): {counter: (sum over dispatches, dispatches)}}"""
    out = defaultdict(lambda: defaultdict(lambda: [0.0, set()]))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if not k.startswith(("conv", "bn_", "wgrad", "sample_stats", "maxpool", "upsample",
                                 "add_", "mse", "adam", "nchw", "nhwc", "pack", "channel")):
                continue
            key = (k, r["Grid_Size"])
            ent = out[key][r["Counter_Name"]]
            ent[0] += float(r["Counter_Value"])
            ent[1].add(r["Dispatch_Id"])
    return out


def parse(dfetch, dwrite, dsq, step_stats):
    merged = defaultdict(dict)
    for d in (dfetch, dwrite, dsq):
        for key, cs in load(d).items():
            for c, (v, disp) in cs.items():
                merged[key][c] = v / STEPS
                merged[key]["calls"] = len(disp) / STEPS
    times = {}
    for r in csv.DictReader(ln for ln in open(step_stats) if not ln.startswith("#")):
        times[r["kernel"]] = (float(r["us_per_step"]), float(r["calls_per_step"]))
    byk = defaultdict(lambda: defaultdict(float))
    for (k, g), cs in merged.items():
        for c, v in cs.items():
            byk[k][c] += v
    rows = []
    for k, (us, calls) in sorted(times.items(), key=lambda kv: -kv[1][0]):
        cs = byk.get(k)
        if not cs:
            continue
        hbm = (2.0 * cs.get("FETCH_SIZE", 0.0) + cs.get("WRITE_SIZE", 0.0)) * 1024.0
        grbm = cs.get("GRBM_GUI_ACTIVE", 0.0)
        mfma = cs.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        wave = cs.get("SQ_WAVE_CYCLES", 0.0)
        rows.append({
            "kernel": k, "calls_per_step": calls, "us_per_step": us,
            "fabric_bytes_per_step": hbm, "fabric_GBps": hbm / (us * 1e-6) / 1e9 if us else None,
            "fabric_frac_of_8TBps": hbm / (us * 1e-6) / 8e12 if us else None,
            "mfma_busy_frac": mfma / (grbm / 8.0 * 1024.0) if grbm else None,
            "wave_wait_any_frac": cs.get("SQ_WAIT_ANY", 0.0) / wave if wave else None,
            "wave_wait_inst_any_frac": cs.get("SQ_WAIT_INST_ANY", 0.0) / wave if wave else None,
            "wave_active_inst_frac": cs.get("SQ_ACTIVE_INST_ANY", 0.0) / wave if wave else None,
            "raw_per_step": {c: v for c, v in cs.items() if c != "calls"},
        })
    print(json.dumps({"steps_profiled": STEPS, "workload": "4-stack 256x256 N=32 bf16 eager step",
                      "fabric_bytes": "2*FETCH_SIZE+WRITE_SIZE (KiB->B), FETCH doubled per "
                                      "MI355X_MICROARCH.md gfx950 correction; L2 <-> fabric traffic, "
                                      "Infinity-Cache (MALL) hits included, so an upper bound on HBM "
                                      "bytes (a consumer of a just-written tensor can exceed 8 TB/s)",
                      "mfma_busy": "SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 * 1024 SIMDs)",
                      "kernels": rows}, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        parse(*sys.argv[2:6])
