"""Fused training step: forward + per-stack MSE + backward + (RCCL all-reduce) + Adam.

Reference loop (try_with_torch.py:330-344): result = model(bx_); losses = sum_k MSELoss(result[k],
y); opt.zero_grad(); losses.backward(); opt.step() with Adam(lr=1e-5). Here the same step runs
entirely on libhgk kernels:

* parameters live in ONE flat fp32 buffer (the nn.Parameters become views of it, so state_dict /
  load_state_dict / torch.save keep working), grads in one flat fp32 buffer, Adam moments in two
  more -> the optimizer is a single fused kernel and the data-parallel all-reduce is ONE RCCL call;
* the per-stack MSE is the fused hgk_mse_fwd_bwd kernel; with world_size W its gradient is scaled
  by 1/W at the source, so a SUM all-reduce yields the mean gradient with no extra pass;
* forward+loss+backward is captured once into a hipGraph (torch.cuda.CUDAGraph over the current
  stream) and replayed: ~3k kernel launches per step cost no host time. BN batch statistics stay
  local to each rank (the reference has no SyncBN), exactly like running the reference per shard.
* checkpoints use the reference's layout {'epoch', 'state_dict', 'optimizer', 'loss'}
  (try_with_torch.py:321-328,361-367) with a genuine torch.optim.Adam state_dict, so reference
  scripts and this trainer load each other's files; `load_matching` is train.py:856-867's
  fine-tune load (keep the keys whose shapes match).
"""
import torch
import torch.distributed as dist

from . import dp
from . import hgk as H
from .engine import Ctx


class FlatParams:
    """Re-home every parameter of `model` into one contiguous fp32 buffer (views)."""

    def __init__(self, model):
        params = [p for p in model.parameters()]
        total = sum(p.numel() for p in params)
        dev = params[0].device
        self.flat = torch.empty(total, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(total, dtype=torch.float32, device=dev)
        self.params = params
        self.grad_views = {}
        off = 0
        for p in params:
            n = p.numel()
            self.flat[off:off + n].copy_(p.detach().reshape(-1))
            p.data = self.flat[off:off + n].view_as(p)
            self.grad_views[id(p)] = self.grad[off:off + n].view_as(p)
            off += n
        self.numel = total


class Trainer:
    def __init__(self, model, lr=1e-5, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 dtype=torch.bfloat16, use_graph=True, process_group=None, branches=False):
        self.model = model
        # hourglass up-branches on side streams (engine.Ctx.fork): exact, but measured slower on
        # MI355X (profiles/r01_branch_streams_ab.txt), so off by default
        self.branches = branches
        self.dtype = dtype
        model.set_engine_dtype(dtype)
        self.fp = FlatParams(model)
        dev = self.fp.flat.device
        self.device = dev
        self.exp_avg = torch.zeros_like(self.fp.flat)
        self.exp_avg_sq = torch.zeros_like(self.fp.flat)
        self.adam_state = torch.zeros(4, dtype=torch.float32, device=dev)
        self.lr, self.betas, self.eps, self.wd = lr, betas, eps, weight_decay
        self.use_graph = use_graph
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_available() and \
            dist.is_initialized() else 1
        self.loss = torch.zeros(1, dtype=torch.float32, device=dev)
        self.graph = None
        self.static_x = None
        self.static_t = None
        self.lib = H.lib()
        self._convs = {id(m): m for m in model.modules() if isinstance(m, torch.nn.Conv2d)}
        self._pack_plan = None
        # every BN's num_batches_tracked re-homed into one int64 buffer (0-d views, so the
        # state_dict is unchanged); the per-step increments are learned from the first pass
        bns = [m for m in model.modules()
               if isinstance(m, torch.nn.BatchNorm2d) and m.num_batches_tracked is not None]
        self._nbt_flat = torch.zeros(len(bns), dtype=torch.long, device=dev)
        for i, m in enumerate(bns):
            self._nbt_flat[i].copy_(m.num_batches_tracked)
            m.num_batches_tracked = self._nbt_flat[i]
        self._nbt_index = {id(m): i for i, m in enumerate(bns)}
        self._nbt_counts = None
        dp.broadcast_flat(self.fp.flat, src=0, group=process_group)

    # ------------------------------------------------------------------ one fwd+loss+bwd
    def _fwd_bwd(self, x, target):
        model = self.model
        model.train()
        ctx = Ctx(self.dtype, True, self.device, grad_enabled=True).enable_branches(self.branches)
        ctx.pgrads = dict(self.fp.grad_views)
        self.fp.grad.zero_()
        if self._pack_plan is not None:
            # every weight layout of the step in one launch (learned from the first pass)
            ctx.prepack(self._pack_plan, self._convs)
        if self._nbt_counts is not None:
            ctx.nbt_batch = (self._nbt_flat, self._nbt_counts)
        xin = ctx.input(x, requires_grad=False)
        heatmaps = model.hg_forward(ctx, xin)
        ctx.finish_forward()
        numel = target.numel()
        rows = H.ctypes.c_int(0)
        part = torch.empty(1024, dtype=torch.float32, device=self.device)
        for s, hm in enumerate(heatmaps):
            out = ctx.output_nchw(hm)
            grad = torch.empty_like(out)
            H.check(self.lib.hgk_mse_fwd_bwd(ctx.stream, out.data_ptr(), target.data_ptr(), numel,
                                             part.data_ptr(), H.ctypes.byref(rows), grad.data_ptr(),
                                             1.0 / self.world))
            H.check(self.lib.hgk_mse_finalize(ctx.stream, part.data_ptr(), rows.value, numel,
                                              self.loss.data_ptr(), 1 if s > 0 else 0))
            ctx.grad_from_nchw(hm, grad)
        ctx.backward()
        if self._pack_plan is None:
            self._pack_plan = ctx.pack_plan()
        if self._nbt_counts is None:
            counts = torch.zeros_like(self._nbt_flat)
            for bn, count in ctx.bn_uses.values():
                if id(bn) in self._nbt_index:
                    counts[self._nbt_index[id(bn)]] = count
            self._nbt_counts = counts

    def _adam(self):
        b1, b2 = self.betas
        H.check(self.lib.hgk_adam_step(H.stream_handle(), self.fp.flat.data_ptr(),
                                       self.fp.grad.data_ptr(), self.exp_avg.data_ptr(),
                                       self.exp_avg_sq.data_ptr(), self.fp.numel, self.lr, b1, b2,
                                       self.eps, self.wd, self.adam_state.data_ptr()))

    def _allreduce(self):
        if self.world > 1:
            dp.allreduce_flat(self.fp.grad, group=self.pg)

    def step(self, x, target):
        """One training step on this rank's shard; returns the (device) loss tensor of this rank
        (sum over stacks of the per-stack MSE, unscaled)."""
        if not self.use_graph:
            self._fwd_bwd(x, target)
        else:
            if self.graph is None:
                self._capture(x, target)
            self.static_x.copy_(x)
            self.static_t.copy_(target)
            self.graph.replay()
        self._allreduce()
        self._adam()
        return self.loss

    def _capture(self, x, target):
        self.static_x = x.clone()
        self.static_t = target.clone()
        # warm the caching allocator / library on a side stream, as torch.cuda.graphs advises
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        saved = [p.detach().clone() for p in self.fp.params]
        bn_state = {k: v.clone() for k, v in self.model.state_dict().items() if "running" in k or
                    "num_batches" in k}
        with torch.cuda.stream(s):
            self._fwd_bwd(self.static_x, self.static_t)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._fwd_bwd(self.static_x, self.static_t)
        self.graph = g
        # capture ran the step twice (warm-up + capture): restore BN running stats so the first
        # replay is the first real step (weights were not touched: Adam runs outside the graph)
        sd = self.model.state_dict()
        for k, v in bn_state.items():
            sd[k].copy_(v)
        for p, v in zip(self.fp.params, saved):
            p.data.copy_(v)

    # ------------------------------------------------------------------ checkpoints
    def _torch_adam(self):
        b1, b2 = self.betas
        return torch.optim.Adam(self.fp.params, lr=self.lr, betas=(b1, b2), eps=self.eps,
                                weight_decay=self.wd)

    def optimizer_state_dict(self):
        """torch.optim.Adam(model.parameters()).state_dict() of the fused optimizer's state."""
        opt = self._torch_adam()
        step = float(self.adam_state[0])
        if step > 0:
            off = 0
            for p in self.fp.params:
                n = p.numel()
                opt.state[p] = {"step": torch.tensor(step),
                                "exp_avg": self.exp_avg[off:off + n].view_as(p).clone(),
                                "exp_avg_sq": self.exp_avg_sq[off:off + n].view_as(p).clone()}
                off += n
        return opt.state_dict()

    def load_optimizer_state_dict(self, sd):
        """Load a torch.optim.Adam state_dict (e.g. a reference checkpoint's 'optimizer')."""
        opt = self._torch_adam()
        opt.load_state_dict(sd)  # validates the layout against this model's parameters
        g = opt.param_groups[0]
        self.lr, self.betas, self.eps, self.wd = g["lr"], tuple(g["betas"]), g["eps"], g["weight_decay"]
        steps = set()
        off = 0
        for p in self.fp.params:
            n = p.numel()
            st = opt.state.get(p)
            if st:
                self.exp_avg[off:off + n].copy_(st["exp_avg"].reshape(-1))
                self.exp_avg_sq[off:off + n].copy_(st["exp_avg_sq"].reshape(-1))
                steps.add(float(st["step"]))
            else:
                self.exp_avg[off:off + n].zero_()
                self.exp_avg_sq[off:off + n].zero_()
            off += n
        if len(steps) > 1:
            raise ValueError(f"per-parameter Adam step counts differ: {sorted(steps)}")
        self.adam_state.zero_()
        self.adam_state[0] = steps.pop() if steps else 0.0

    def checkpoint(self, epoch, loss):
        """{'epoch', 'state_dict', 'optimizer', 'loss'} as try_with_torch.py:361-367 saves it."""
        return {"epoch": epoch, "state_dict": self.model.state_dict(),
                "optimizer": self.optimizer_state_dict(), "loss": loss}

    def load_checkpoint(self, state):
        """try_with_torch.py:323-327: model weights, optimizer state; returns (epoch, loss)."""
        self.model.load_state_dict(state["state_dict"])  # copies into the flat-buffer views
        self.load_optimizer_state_dict(state["optimizer"])
        return state["epoch"], state["loss"]


def load_matching(model, pretrained_state_dict):
    """train.py:856-867 fine-tune load: take every pretrained tensor whose key exists with the same
    shape, keep the model's own values elsewhere. Returns the list of keys taken."""
    own = model.state_dict()
    take = {k: v for k, v in pretrained_state_dict.items() if k in own and v.size() == own[k].size()}
    own.update(take)
    model.load_state_dict(own)
    return sorted(take)
