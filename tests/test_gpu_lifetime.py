"""The engine's deterministic buffer-lifetime guard (engine.LifetimeGuard, HGK_DEBUG_LIFETIME=1).

The bug class it exists for (found in round 2 only through contention probes, fixed in f11e87b):
a kernel argument taken from a tensor (data_ptr() int, also inside a twin-segment descriptor)
whose last Python owner is gone before the launch — the caching allocator may already have
handed that memory to the next allocation. The guard keeps every Ctx buffer alive for the step
(no address reuse) and, at every launch, requires each pointer argument's buffer to still have an
owner other than the guard.

* the guard raises on a launch that reads a released buffer, and not on a live one;
* full training steps of the twin schedule (eager and hipGraph capture) and of the grad-barrier
  split-graph schedule (Trainer overlap: the DP path's graph cut) run clean, with thousands of
  pointer arguments resolved;
* the pre-f11e87b twin BN backward (a segment's partials released before the launch) is caught."""
import pytest
import torch

import progressive_process_for_human_pose_estimation_amd as P
from progressive_process_for_human_pose_estimation_amd import engine as E
from progressive_process_for_human_pose_estimation_amd import hgk as H
from progressive_process_for_human_pose_estimation_amd.data import gaussian_targets, synthetic_images
from progressive_process_for_human_pose_estimation_amd.trainer import Trainer

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture
def guards(monkeypatch):
    """every LifetimeGuard the engine creates during the test"""
    made = []
    init = E.LifetimeGuard.__init__

    def rec(self, lib):
        init(self, lib)
        made.append(self)
    monkeypatch.setattr(E.LifetimeGuard, "__init__", rec)
    monkeypatch.setenv("HGK_DEBUG_LIFETIME", "1")
    return made


def test_guard_flags_released_buffer():
    ctx = E.Ctx(torch.bfloat16, True, torch.device(DEV), debug_lifetime=True)
    a = ctx._empty(4096)
    b = ctx._empty(4096)
    out = ctx._empty(4096)
    a.fill_(1.0)
    b.fill_(2.0)
    # live operands: fine
    H.check(ctx.lib.hgk_add(ctx.stream, ctx.dt, a.data_ptr(), b.data_ptr(), out.data_ptr(), 4096, 0))
    torch.cuda.synchronize()
    assert float(out.float().max()) == 3.0
    assert ctx.guard.checked == 3
    # the pointer outlives its tensor: the launch must be refused before it runs
    pa = a.data_ptr()
    del a
    with pytest.raises(RuntimeError, match="lifetime: hgk_add arg 2"):
        ctx.lib.hgk_add(ctx.stream, ctx.dt, pa, b.data_ptr(), out.data_ptr(), 4096, 0)
    # a view keeps the storage owned
    v = b[1024:]
    pb = b.data_ptr()
    del b
    H.check(ctx.lib.hgk_add(ctx.stream, ctx.dt, pb, v.data_ptr(), out.data_ptr(), 1024, 0))
    torch.cuda.synchronize()


@pytest.mark.parametrize("use_graph", [False, True], ids=["eager", "graph"])
def test_twin_schedule_steps_clean(guards, use_graph):
    """2-stack, 128x128, N=4: every level runs twin chains (conv, BN finalize, BN backward twins)"""
    x = synthetic_images(4, 128, 128, seed=3)
    t = gaussian_targets(4, 17, 32, 32, seed=4)[0]
    torch.manual_seed(0)
    m = P.creatModel(nStack=2).to(DEV)
    tr = Trainer(m, lr=1e-4, dtype=torch.bfloat16, use_graph=use_graph)
    for _ in range(2):
        tr.step(x.to(DEV), t.to(DEV))
    torch.cuda.synchronize()
    assert guards and all(g.launches > 0 for g in guards)
    assert sum(g.checked for g in guards) > 2000


def test_split_graph_schedule_steps_clean(guards):
    """the DP schedule's grad barrier: backward split at the stem, trunk grads final first
    (overlap=True without a process group: the same capture cut, no collective)"""
    x = synthetic_images(4, 128, 128, seed=5)
    t = gaussian_targets(4, 17, 32, 32, seed=6)[0]
    torch.manual_seed(0)
    m = P.creatModel(nStack=2).to(DEV)
    tr = Trainer(m, lr=1e-4, dtype=torch.bfloat16, use_graph=True, overlap=True)
    tr.step(x.to(DEV), t.to(DEV))
    torch.cuda.synchronize()
    assert tr.graphs is not None and len(tr.graphs) == 2
    assert sum(g.checked for g in guards) > 1000


def _twin_bn_bwd_pre_fix(self, vs):
    """Ctx._bn_relu_bwd_twin as it was before f11e87b: the loop variable is a segment's partials'
    only owner, so the first segment's buffer is released before the launch that reads it."""
    if not all(v.grad is not None and v.bwd_part is not None and v.src.requires_grad for v in vs):
        for v in vs:
            self._bn_relu_bwd(v)
        return
    use0 = vs[0].bn
    bn, C = use0.mod, vs[0].src.C
    segs = []
    for v in vs:
        x = v.src
        part, rows = v.bwd_part
        v.bwd_part = None
        dst, acc, src = self.grad_slot(x)
        segs.append(H.BnbSeg(part.data_ptr(), rows, x.M, v.bn.stat.data_ptr(), v.grad.data_ptr(),
                             x.t.data_ptr(), None if src is dst else src.data_ptr(),
                             dst.data_ptr(), acc if src is dst else 0))
    coef = self._f32(len(vs), 6, C)
    arr = (H.BnbSeg * len(segs))(*segs)
    H.check(self.lib.hgk_bn_bwd_twin(self.stream, self.dt, arr, len(segs), C,
                                     1 if use0.relu else 0, 1 if use0.training else 0,
                                     self.pgrad(bn.weight).data_ptr(),
                                     self.pgrad(bn.bias).data_ptr(), coef.data_ptr()))
    for v in vs:
        v.grad = None


def test_guard_catches_reintroduced_twin_release(guards, monkeypatch):
    monkeypatch.setattr(E.Ctx, "_bn_relu_bwd_twin", _twin_bn_bwd_pre_fix)
    x = synthetic_images(4, 128, 128, seed=3)
    t = gaussian_targets(4, 17, 32, 32, seed=4)[0]
    torch.manual_seed(0)
    m = P.creatModel(nStack=1).to(DEV)
    tr = Trainer(m, lr=1e-4, dtype=torch.bfloat16, use_graph=False)
    with pytest.raises(RuntimeError, match=r"lifetime: hgk_bn_bwd_twin arg 2\[0\]\.partial"):
        tr.step(x.to(DEV), t.to(DEV))
    torch.cuda.synchronize()
