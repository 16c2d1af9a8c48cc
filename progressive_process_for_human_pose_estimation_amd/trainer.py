"""Fused training step: forward + per-stack MSE + backward + (RCCL all-reduce) + Adam.

Reference loop (try_with_torch.py:330-344): result = model(bx_); losses = sum_k MSELoss(result[k],
y); opt.zero_grad(); losses.backward(); opt.step() with Adam(lr=1e-5). Here the same step runs
entirely on libhgk kernels:

* parameters live in ONE flat fp32 buffer (the nn.Parameters become views of it, so state_dict /
  load_state_dict / torch.save keep working), grads in one flat fp32 buffer, Adam moments in two
  more, all in grad-ready order [trunk | stem | never-grad tail] -> the optimizer is a single
  fused kernel over the active prefix and the data-parallel all-reduce is one RCCL call per
  segment, the trunk's overlapped with the stem's backward (dp.GradSync);
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
from .engine import ROUTE, Ctx


def param_layout(model):
    """(grad-ready groups of parameter names, never-grad names) of an engine model; a plain
    nn.Module (e.g. the CPU oracle) gets one group holding every parameter."""
    names = [k for k, _ in model.named_parameters()]
    if hasattr(model, "grad_ready_groups"):
        groups = [list(g) for g in model.grad_ready_groups()]
        frozen = list(model.never_grad_parameters())
    else:
        groups, frozen = [names], []
    seen = [k for g in groups for k in g] + frozen
    if sorted(seen) != sorted(names):
        raise ValueError("grad-ready groups + never-grad parameters must cover every parameter once")
    return groups, frozen


class FlatParams:
    """Re-home every parameter of `model` into one contiguous fp32 buffer (views), laid out in
    grad-ready order: [group 0 | group 1 | ... | never-grad tail]. `segments[i]` is group i's
    [lo, hi) range; [0, active) is what the all-reduce and Adam touch. `layout` defaults to
    param_layout(model) (pass another model's layout to give the oracle the engine's layout)."""

    def __init__(self, model, layout=None):
        groups, frozen = param_layout(model) if layout is None else layout
        named = dict(model.named_parameters())
        self.params = [p for _, p in model.named_parameters()]  # model order (optimizer state)
        dev = self.params[0].device
        total = sum(p.numel() for p in self.params)
        self.flat = torch.empty(total, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(total, dtype=torch.float32, device=dev)
        self.grad_views = {}
        self.offsets = {}      # id(param) -> (offset, numel)
        self.segments = []
        self.active_ids = set()
        self.group_ids = [{id(named[k]) for k in g} for g in groups]  # per grad-ready group
        off = 0
        for gi, names in enumerate(list(groups) + [frozen]):
            lo = off
            for k in names:
                p = named[k]
                n = p.numel()
                self.flat[off:off + n].copy_(p.detach().reshape(-1))
                p.data = self.flat[off:off + n].view_as(p)
                self.grad_views[id(p)] = self.grad[off:off + n].view_as(p)
                self.offsets[id(p)] = (off, n)
                if gi < len(groups):
                    self.active_ids.add(id(p))
                off += n
            if gi < len(groups):
                self.segments.append((lo, off))
        self.active = self.segments[-1][1] if self.segments else 0
        self.numel = total


HEAD_LOSSES = ("mse", "ce", "none")


class Trainer:
    """`heads`: the loss of each model output, "mse" (nn.MSELoss, try_with_torch.py:305-341),
    "ce" (nn.CrossEntropyLoss over the class axis, try_with_aspp.py:356-358) or "none" (computed
    but not trained: try_more_layer.py's 4th output, :398-401; its target is ignored, pass None);
    None = every output MSE against ONE target tensor. With `heads` given, step() takes one target
    per output (float heatmaps for "mse", int64 class maps [N, H, W] for "ce"); the step's loss is
    the sum."""

    def __init__(self, model, lr=1e-5, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 dtype=torch.bfloat16, use_graph=True, process_group=None, branches=False,
                 overlap=None, heads=None):
        self.model = model
        if heads is not None:
            heads = tuple(heads)
            bad = [h for h in heads if h not in HEAD_LOSSES]
            if bad:
                raise ValueError(f"unknown head loss(es) {bad}: expected one of {HEAD_LOSSES}")
        self.heads = heads
        # every MSE head in one launch on the NHWC heads (hgk_mse_heads_nhwc, round 6; engine route
        # mse_heads); False = the per-head NCHW path (A/B, tests)
        self.fused_mse = bool(ROUTE["mse_heads"])
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
        # grad all-reduce per grad-ready segment; with overlap the trunk segment's collective
        # runs on a side stream during the stem's backward (graph split at the barrier)
        self.sync = dp.GradSync(self.fp.grad, self.fp.segments, group=process_group)
        self.overlap = (self.world > 1) if overlap is None else bool(overlap)
        self.loss = torch.zeros(1, dtype=torch.float32, device=dev)
        # per-output losses (the reference prints loss_1..loss_3, try_with_aspp.py:404-411) and
        # the device flag of the CE heads' target check (read by check_targets())
        self.head_losses = torch.zeros(len(heads) if heads else 1, dtype=torch.float32, device=dev)
        self._bad_target = torch.zeros(1, dtype=torch.int32, device=dev)
        # step() reads the flag back without a sync: a pinned copy + event per step, inspected at
        # the next step (so a bad target raises at most one step late)
        self._bad_host = torch.zeros(1, dtype=torch.int32, pin_memory=True) if heads else None
        self._bad_event = None
        self.graph = None
        self.graphs = None
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
        self._probed = False
        self.dead_params = []   # active by structure, never reached by the dataflow (see _probe)
        dp.broadcast_flat(self.fp.flat, src=0, group=process_group)

    # ------------------------------------------------------------------ one fwd+loss+bwd
    def _fwd_bwd(self, x, target, on_ready=None):
        """forward + per-stack MSE + backward on the current stream; on_ready(i) runs when the
        grads of segment i (< last) are final (engine.Ctx.grad_barrier)."""
        model = self.model
        model.train()
        ctx = Ctx(self.dtype, True, self.device, grad_enabled=True).enable_branches(self.branches)
        ctx.pgrads = dict(self.fp.grad_views)
        ctx.seal_groups = self.fp.group_ids[:-1]
        seg = [0]

        def ready(tag):
            if on_ready is not None:
                on_ready(seg[0])
            seg[0] += 1
        ctx.on_grads_ready = ready
        self.fp.grad.zero_()
        if self._pack_plan is not None:
            # every weight layout of the step in one launch (learned from the first pass)
            ctx.prepack(self._pack_plan, self._convs)
        if self._nbt_counts is not None:
            ctx.nbt_batch = (self._nbt_flat, self._nbt_counts)
        xin = ctx.input(x, requires_grad=False)
        heatmaps = model.hg_forward(ctx, xin)
        ctx.finish_forward()
        self._heads_fwd_bwd(ctx, heatmaps, target)
        ctx.backward()
        if seg[0] != len(self.fp.segments) - 1:
            raise RuntimeError(f"model passed {seg[0]} grad barriers for "
                               f"{len(self.fp.segments)} grad-ready groups")
        stray = ctx.touched - self.fp.active_ids
        if stray:
            raise RuntimeError(f"{len(stray)} parameters declared never-grad received gradients")
        if self._probed and ctx.touched != self.fp.active_ids:
            raise RuntimeError("the step's dataflow changed after the first pass: "
                               f"{len(self.fp.active_ids - ctx.touched)} active parameters got no "
                               "gradient")
        if self._pack_plan is None:
            self._pack_plan = ctx.pack_plan()
        if self._nbt_counts is None:
            counts = torch.zeros_like(self._nbt_flat)
            for bn, count in ctx.bn_uses.values():
                if id(bn) in self._nbt_index:
                    counts[self._nbt_index[id(bn)]] = count
            self._nbt_counts = counts
        return ctx.touched

    def _heads_fwd_bwd(self, ctx, heatmaps, target):
        """Per-output loss + its gradient (pre-scaled by 1/world: the SUM all-reduce gives the
        mean), the total into self.loss; each head's gradient enters the engine tape."""
        if self.heads is None and self.fused_mse and self._mse_heads(ctx, heatmaps, target):
            return
        rows = H.ctypes.c_int(0)
        part = torch.empty(1024, dtype=torch.float32, device=self.device)
        if self.heads is None:
            kinds, targets = ["mse"] * len(heatmaps), [target] * len(heatmaps)
        else:
            kinds, targets = list(self.heads), list(target)
            if len(kinds) != len(heatmaps) or len(targets) != len(heatmaps):
                raise ValueError(f"{len(heatmaps)} model outputs, {len(kinds)} head losses, "
                                 f"{len(targets)} targets")
        hl = self.head_losses
        for s, (hm, kind, tgt) in enumerate(zip(heatmaps, kinds, targets)):
            if kind == "none":
                continue  # head_losses[s] stays 0; no gradient enters the tape from this output
            out = ctx.output_nchw(hm)
            grad = torch.empty_like(out)
            if kind == "mse":
                if tgt.shape != out.shape or tgt.dtype != torch.float32 or not tgt.is_contiguous():
                    raise ValueError(f"head {s}: MSE target must be contiguous fp32 {tuple(out.shape)}")
                numel = tgt.numel()
                H.check(self.lib.hgk_mse_fwd_bwd(ctx.stream, out.data_ptr(), tgt.data_ptr(), numel,
                                                 part.data_ptr(), H.ctypes.byref(rows),
                                                 grad.data_ptr(), 1.0 / self.world))
            else:
                N, K, Hh, W = out.shape
                if tuple(tgt.shape) != (N, Hh, W) or tgt.dtype != torch.int64 or not tgt.is_contiguous():
                    raise ValueError(f"head {s}: CE target must be contiguous int64 {(N, Hh, W)}")
                numel = N * Hh * W
                H.check(self.lib.hgk_ce_fwd_bwd(ctx.stream, out.data_ptr(), tgt.data_ptr(), N, K,
                                                Hh * W, part.data_ptr(), H.ctypes.byref(rows),
                                                grad.data_ptr(), 1.0 / self.world,
                                                self._bad_target.data_ptr()))
            if self.heads is None:
                H.check(self.lib.hgk_mse_finalize(ctx.stream, part.data_ptr(), rows.value, numel,
                                                  self.loss.data_ptr(), 1 if s > 0 else 0))
            else:
                H.check(self.lib.hgk_mse_finalize(ctx.stream, part.data_ptr(), rows.value, numel,
                                                  hl[s:].data_ptr(), 0))
            ctx.grad_from_nchw(hm, grad)
        if self.heads is not None:
            H.check(self.lib.hgk_mse_finalize(ctx.stream, hl.data_ptr(), len(kinds), 1,
                                              self.loss.data_ptr(), 0))

    def _mse_heads(self, ctx, heatmaps, target):
        """Every head's MSE (one target) in one hgk_mse_heads_nhwc launch + one finalize, on the
        engine's NHWC heads (no NCHW copies): the gradients hgk_nhwc_to_nchw + hgk_mse_fwd_bwd +
        hgk_nchw_to_nhwc give, bit for bit. False (nothing launched) where it does not apply."""
        hs = list(heatmaps)
        h0 = hs[0]
        if (len(hs) > 8 or any(h.bn is not None or (h.N, h.H, h.W, h.C, h.C_log) !=
                               (h0.N, h0.H, h0.W, h0.C, h0.C_log) for h in hs)
                or h0.C % 8 != 0 or h0.C_log > 64 or tuple(target.shape) != (h0.N, h0.C_log, h0.H, h0.W)
                or target.dtype != torch.float32 or not target.is_contiguous()):
            return False
        grads = [ctx._empty(h0.N, h0.H, h0.W, h0.C) for _ in hs]
        part = torch.empty(self.lib.hgk_mse_heads_partial_rows(), dtype=torch.float32,
                           device=self.device)
        H.check(self.lib.hgk_mse_heads_nhwc(
            ctx.stream, ctx.dt, (H.ctypes.c_void_p * len(hs))(*[h.t.data_ptr() for h in hs]),
            (H.ctypes.c_void_p * len(hs))(*[g.data_ptr() for g in grads]), len(hs),
            target.data_ptr(), h0.N, h0.C_log, h0.H, h0.W, h0.C, 1.0 / self.world, part.data_ptr(),
            self.loss.data_ptr()))
        for h, g in zip(hs, grads):
            ctx.add_grad(h, g)
        return True

    def check_targets(self):
        """Raise if a CE head saw a class index outside [0, K) since the last call (the fused
        kernels flag it on the device instead of synchronising every step). ignore_index (-100)
        counts as out of range: the fused head does not support ignored pixels."""
        self._bad_event = None
        if int(self._bad_target.item()):
            self._bad_target.zero_()
            raise ValueError("cross entropy: target class out of range (ignore_index -100 is not "
                             "supported by the fused CE head)")

    def _poll_targets(self):
        """step()'s non-blocking target check: the previous step's flag, if its copy landed."""
        ev = self._bad_event
        if ev is not None and ev.query():
            self._bad_event = None
            if int(self._bad_host[0]):
                self.check_targets()

    def _adam(self):
        # the active prefix only: never-grad parameters keep their values and get no state,
        # like torch.optim.Adam's skip of parameters whose grad is None
        b1, b2 = self.betas
        H.check(self.lib.hgk_adam_step(H.stream_handle(), self.fp.flat.data_ptr(),
                                       self.fp.grad.data_ptr(), self.exp_avg.data_ptr(),
                                       self.exp_avg_sq.data_ptr(), self.fp.active, self.lr, b1, b2,
                                       self.eps, self.wd, self.adam_state.data_ptr()))

    def step(self, x, target):
        """One training step on this rank's shard; returns the (device) loss tensor of this rank
        (sum over the outputs of their losses, unscaled). With CE heads, a target class outside
        [0, K) seen by an earlier step raises here (the device flag is read back without a sync)."""
        if self._bad_host is not None:
            self._poll_targets()
        if not self._probed:
            self._probe(x, target)
        nseg = len(self.fp.segments)
        if not self.use_graph:
            # eager: segment i's all-reduce is launched the moment its grads are final
            self._fwd_bwd(x, target, on_ready=self.sync.launch if self.overlap else None)
            for i in range(len(self.sync.launched) if self.overlap else 0, nseg):
                self.sync.launch(i)
        else:
            if self.graph is None and self.graphs is None:
                self._capture(x, target)
            self.static_x.copy_(x)
            if self.heads is None:
                self.static_t.copy_(target)
            else:
                for st, tg in zip(self.static_t, target):
                    if st is not None:
                        st.copy_(tg)
            if self.graphs is not None:
                # graph i = the step up to barrier i: replaying graph i+1 overlaps segment i's
                # all-reduce on the side stream
                for i, g in enumerate(self.graphs):
                    g.replay()
                    self.sync.launch(i)
            else:
                self.graph.replay()
                for i in range(nseg):
                    self.sync.launch(i)
        self.sync.wait()
        self._adam()
        if self._bad_host is not None:
            if self._bad_event is None:
                self._bad_host.copy_(self._bad_target, non_blocking=True)
                self._bad_event = torch.cuda.Event()
                self._bad_event.record()
        return self.loss

    def _bn_state(self):
        return {k: v.clone() for k, v in self.model.state_dict().items()
                if "running" in k or "num_batches" in k}

    def _restore_bn(self, bn_state):
        sd = self.model.state_dict()
        for k, v in bn_state.items():
            sd[k].copy_(v)

    def _probe(self, x, target):
        """One untimed forward+backward before the first step (BN state restored afterwards,
        weights untouched: no Adam). It learns the step's weight-pack plan and BN use counts and
        which active parameters the dataflow never reaches (e.g. the registered-but-dead ASPP
        branch of try_with_aspp.py:213-232, creatModel's conv3 / conv4 at nStack=1): those move
        to the never-grad tail — no all-reduce, no Adam update or state, as torch.optim.Adam skips
        parameters whose grad stays None."""
        bn_state = self._bn_state()
        touched = self._fwd_bwd(x, target)
        torch.cuda.current_stream().synchronize()
        self._restore_bn(bn_state)
        self._probed = True
        dead = self.fp.active_ids - touched
        if dead:
            self._relayout(dead)

    def _relayout(self, dead):
        """Move the parameters `dead` (ids) from the grad-ready groups to the never-grad tail."""
        named = list(self.model.named_parameters())
        ids = {k: id(p) for k, p in named}
        groups, frozen = param_layout(self.model)
        groups = [[k for k in g if ids[k] not in dead] for g in groups]
        frozen = frozen + [k for k, p in named if id(p) in dead]
        old, ea, eas = self.fp, self.exp_avg, self.exp_avg_sq
        new = FlatParams(self.model, layout=(groups, frozen))
        self.exp_avg = torch.zeros_like(new.flat)
        self.exp_avg_sq = torch.zeros_like(new.flat)
        for p in new.params:
            if id(p) in new.active_ids:
                o, n = old.offsets[id(p)]
                o2, _ = new.offsets[id(p)]
                self.exp_avg[o2:o2 + n].copy_(ea[o:o + n])
                self.exp_avg_sq[o2:o2 + n].copy_(eas[o:o + n])
        self.fp = new
        self.sync = dp.GradSync(new.grad, new.segments, group=self.pg)
        self.dead_params = [k for k, p in named if id(p) in dead]

    def _capture(self, x, target):
        self.static_x = x.clone()
        self.static_t = (target.clone() if self.heads is None else
                         [None if t is None else t.clone() for t in target])
        # warm the caching allocator / library on a side stream, as torch.cuda.graphs advises
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        saved = [p.detach().clone() for p in self.fp.params]
        bn_state = self._bn_state()
        with torch.cuda.stream(s):
            self._fwd_bwd(self.static_x, self.static_t)
        torch.cuda.current_stream().wait_stream(s)
        if self.overlap and len(self.fp.segments) > 1:
            # one graph per grad-ready segment, cut at each grad barrier; later graphs share the
            # first one's memory pool (they replay in capture order on one stream)
            graphs = [torch.cuda.CUDAGraph()]
            torch.cuda.synchronize()
            cap = torch.cuda.Stream()
            cap.wait_stream(torch.cuda.current_stream())

            def cut(_i):
                graphs[-1].capture_end()
                graphs.append(torch.cuda.CUDAGraph())
                graphs[-1].capture_begin(pool=graphs[0].pool())
            with torch.cuda.stream(cap):
                graphs[0].capture_begin()
                self._fwd_bwd(self.static_x, self.static_t, on_ready=cut)
                graphs[-1].capture_end()
            torch.cuda.current_stream().wait_stream(cap)
            self.graphs = graphs
        else:
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
            for p in self.fp.params:
                if id(p) not in self.fp.active_ids:
                    continue  # never had a grad: torch.optim.Adam keeps no state for it either
                off, n = self.fp.offsets[id(p)]
                opt.state[p] = {"step": torch.tensor(step),
                                "exp_avg": self.exp_avg[off:off + n].view_as(p).clone(),
                                "exp_avg_sq": self.exp_avg_sq[off:off + n].view_as(p).clone()}
        return opt.state_dict()

    def load_optimizer_state_dict(self, sd):
        """Load a torch.optim.Adam state_dict (e.g. a reference checkpoint's 'optimizer')."""
        opt = self._torch_adam()
        opt.load_state_dict(sd)  # validates the layout against this model's parameters
        g = opt.param_groups[0]
        self.lr, self.betas, self.eps, self.wd = g["lr"], tuple(g["betas"]), g["eps"], g["weight_decay"]
        steps = set()
        for p in self.fp.params:
            off, n = self.fp.offsets[id(p)]
            st = opt.state.get(p)
            if st and id(p) in self.fp.active_ids:
                self.exp_avg[off:off + n].copy_(st["exp_avg"].reshape(-1))
                self.exp_avg_sq[off:off + n].copy_(st["exp_avg_sq"].reshape(-1))
                steps.add(float(st["step"]))
            else:
                self.exp_avg[off:off + n].zero_()
                self.exp_avg_sq[off:off + n].zero_()
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
