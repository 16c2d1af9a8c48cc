"""Per-operation GPU time of one training step, attributed to the libhgk call that launched it.

  rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ops -o run -- \
      python3 scripts/op_profile.py --log gpurun_out/ops/calls.txt
  python scripts/op_profile.py --parse gpurun_out/ops/run_kernel_trace.csv --log gpurun_out/ops/calls.txt

Run mode: eager Trainer steps (no hipGraph); on the last step every launching libhgk call is
followed by a complex64 fill kernel (FillFunctor<c10::complex<float>>: no engine op fills that
type) as a separator and logged with its
integer arguments. Parse mode: kernels between separators belong to the logged call; prints the
time per call site signature (function + shape arguments), summed over the step.
"""
import argparse
import csv
import ctypes
import os
import sys
from collections import defaultdict

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NON_LAUNCH = {"hgk_abi_version", "hgk_last_error", "hgk_max_stats_rows", "hgk_conv_fwd_workspace",
              "hgk_conv_w_ld", "hgk_conv_wgrad_workspace", "hgk_conv_wgrad_max_splits",
              "hgk_conv_wgrad_slab_bytes", "hgk_bn_finalize_scratch"}


class LoggingLib:
    def __init__(self, lib, log, sep, begin):
        self._lib, self._log, self._sep, self._begin = lib, log, sep, begin
        self.on = False

    def __getattr__(self, name):
        fn = getattr(self._lib, name)
        if name in NON_LAUNCH or not name.startswith("hgk_"):
            return fn

        def call(*args):
            rc = fn(*args)
            if self.on:
                ints = [a for a in args[1:] if isinstance(a, int) and not isinstance(a, bool)
                        and a < 2 ** 31]
                self._log.append(f"{name} {' '.join(str(i) for i in ints)}")
                # drained on both sides: the separator can neither overtake nor overlap the
                # call's own kernels in the trace's start-time order
                torch.cuda.synchronize()
                self._sep.fill_(1)
                torch.cuda.synchronize()
            return rc
        return call


def run(args):
    import torch
    import progressive_process_for_human_pose_estimation_amd as P
    from progressive_process_for_human_pose_estimation_amd import hgk as H
    from progressive_process_for_human_pose_estimation_amd.data import gaussian_targets, synthetic_images
    from progressive_process_for_human_pose_estimation_amd.trainer import Trainer
    from progressive_process_for_human_pose_estimation_amd import engine, trainer as T

    real = H.load_library()
    log = []
    sep = torch.zeros(1, dtype=torch.complex64, device="cuda")
    begin = torch.zeros(1, dtype=torch.int16, device="cuda")
    proxy = LoggingLib(real, log, sep, begin)
    H._lib = proxy
    engine.H._lib = proxy
    torch.manual_seed(0)
    model = P.creatModel(nStack=args.stacks).cuda()
    dtype = torch.bfloat16
    tr = Trainer(model, lr=1e-5, dtype=dtype, use_graph=False)
    x = synthetic_images(args.batch, args.res, args.res, seed=1234).cuda()
    t = gaussian_targets(args.batch, 17, args.res // 4, seed=1)[0].cuda()
    for _ in range(2):
        tr.step(x, t)
    torch.cuda.synchronize()
    begin.fill_(1)
    proxy.on = True
    tr.step(x, t)
    proxy.on = False
    torch.cuda.synchronize()
    with open(args.log, "w") as f:
        f.write("\n".join(log) + "\n")
    print(f"logged {len(log)} launching calls")


def parse(args):
    rows = list(csv.DictReader(open(args.parse)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    calls = []
    for line in open(args.log):
        if line.strip():
            f = line.split()
            calls.append(" ".join([f[0]] + [v for v in f[1:] if int(v) < 2 ** 31]))
    start = max(i for i, r in enumerate(rows) if "FillFunctor<short>" in r["Kernel_Name"])
    groups, cur = [], []
    for r in rows[start + 1:]:
        if "FillFunctor<c10::complex<float>" in r["Kernel_Name"]:
            groups.append(cur)
            cur = []
        else:
            cur.append(r)
    if len(groups) == len(calls) + 1:
        groups = groups[:-1]  # the separator written behind the last logged call
    assert len(groups) == len(calls), (len(groups), len(calls))
    agg = defaultdict(lambda: [0, 0.0, defaultdict(float)])
    total = 0.0
    for call, ks in zip(calls, groups):
        t = sum(int(k["End_Timestamp"]) - int(k["Start_Timestamp"]) for k in ks) / 1e3
        total += t
        a = agg[call]
        a[0] += 1
        a[1] += t
        for k in ks:
            nm = k["Kernel_Name"].replace("void ", "").replace("hgk::", "").split("(")[0]
            a[2][nm] += (int(k["End_Timestamp"]) - int(k["Start_Timestamp"])) / 1e3
    print(f"total kernel time (excl. separators) {total:.1f} us over {len(calls)} calls")
    bykind = defaultdict(float)
    for call, (n, t, _) in agg.items():
        bykind[call.split()[0]] += t
    for k, t in sorted(bykind.items(), key=lambda kv: -kv[1]):
        print(f"{t:9.1f} us {100 * t / total:5.1f}%  {k}")
    print()
    for call, (n, t, ks) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:args.top]:
        kd = ", ".join(f"{k[:38]}={v / n:.1f}" for k, v in sorted(ks.items(), key=lambda kv: -kv[1]))
        print(f"{t:8.1f} us n={n:3d} avg={t / n:7.1f}  {call}\n{'':30s}{kd}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log", required=True)
    ap.add_argument("--parse")
    ap.add_argument("--top", type=int, default=60)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--res", type=int, default=256)
    ap.add_argument("--stacks", type=int, default=4)
    a = ap.parse_args()
    if a.parse:
        parse(a)
    else:
        run(a)


if __name__ == "__main__":
    main()
