"""Reference cycles left by one eager Trainer step: run a step with the cyclic GC off, then
collect with DEBUG_SAVEALL and print what the collector found (type histogram and, for a few
objects of engine types, which other garbage objects refer to them)."""
import collections
import gc
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import progressive_process_for_human_pose_estimation_amd as P  # noqa: E402
from progressive_process_for_human_pose_estimation_amd.data import gaussian_targets, synthetic_images  # noqa: E402
from progressive_process_for_human_pose_estimation_amd.trainer import Trainer  # noqa: E402

x = synthetic_images(2, 128, 128).cuda()
t = gaussian_targets(2, 17, 32)[0].cuda()
tr = Trainer(P.creatModel(nStack=2).cuda(), dtype=torch.bfloat16, use_graph=False)
tr.step(x, t)
torch.cuda.synchronize()
gc.collect()
gc.disable()
base = torch.cuda.memory_allocated()
tr.step(x, t)
torch.cuda.synchronize()
print("allocated after step without gc:", torch.cuda.memory_allocated() - base)
gc.set_debug(gc.DEBUG_SAVEALL)
n = gc.collect()
print("collected", n, "allocated after gc:", torch.cuda.memory_allocated() - base)
hist = collections.Counter(type(o).__name__ for o in gc.garbage)
print(hist.most_common(25))
ids = {id(o) for o in gc.garbage}
shown = collections.Counter()
for o in gc.garbage:
    tn = type(o).__name__
    if tn in ("Act", "Ctx", "BNUse", "PendingApply", "function", "cell") and shown[tn] < 3:
        shown[tn] += 1
        refs = [r for r in gc.get_referrers(o) if id(r) in ids]
        desc = []
        for r in refs[:6]:
            d = type(r).__name__
            if isinstance(r, dict):
                d += "{" + ",".join(str(k) for k in list(r)[:6]) + "}"
            if isinstance(r, (tuple, list)):
                d += "[" + ",".join(type(q).__name__ for q in r[:6]) + "]"
            if type(r).__name__ == "function":
                d += ":" + r.__qualname__
            desc.append(d)
        extra = o.__qualname__ if tn == "function" else ""
        print(f"{tn} {extra} <- {desc}")
