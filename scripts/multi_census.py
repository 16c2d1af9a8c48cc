import os, sys
sys.path.insert(0, "/root/repo")
os.chdir(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch, bench
from progressive_process_for_human_pose_estimation_amd import engine as E
orig = E.Ctx.finish_wgrads
def fin(self):
    singles = [k for k, u in self.wdefer.items() if len(u) == 1] if self.wg_batch else []
    print(f"-- flush {len(self.barriers_passed)}: {len(self.wdefer)} weights, {len(singles)} single-use")
    for key, uses in self.wdefer.items():
        ent = self.wslabs[key]
        cin_st, cout_st, KH, KW = ent[4][:4]
        Ms = [u[0][5] * u[0][6] * u[0][7] for u in uses]
        kind = "single" if key in singles else "multi "
        print(f"{kind} weight {cin_st}->{cout_st} k{KH}: {len(uses)} sources, M total {sum(Ms)}, "
              f"Ms {sorted(set(Ms))}, HW {sorted(set((u[0][6], u[0][7]) for u in uses))}")
    orig(self)
E.Ctx.finish_wgrads = fin
tr, x, t, _ = bench.build_step("primary", 4, torch.bfloat16, 32, 256, 0, use_graph=False)
tr.step(x, t)
torch.cuda.synchronize()
