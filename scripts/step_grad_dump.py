"""One eager bf16 training step of the benched configuration (bench.build_step, graph off) on the
library HGK_LIB names; saves the flat fp32 gradient and the loss to argv[1] — two runs on two
library builds compare bit for bit (scripts: a kernel change claimed bitwise)."""
import os
import sys

import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402

tr, x, t, _ = bench.build_step("primary", 4, torch.bfloat16, int(os.environ.get("N", "8")), 256, 0,
                               use_graph=False)
loss = tr.step(x, t)
torch.cuda.synchronize()
torch.save({"grad": tr.fp.grad.cpu(), "loss": loss.cpu()}, sys.argv[1])
print("saved", sys.argv[1], float(loss))
