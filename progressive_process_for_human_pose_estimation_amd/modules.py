"""Drop-in nn.Module surface of the reference (try_with_torch.py:179-298), executed on libhgk.

Same class names, constructor signatures, sub-module names and registration order as the
reference, so `torch.manual_seed(s); creatModel()` gives bit-identical initial weights and a
key-/shape-identical state_dict (199 keys for the primary model, incl. the never-used `conv4` of
square ResidualBlocks and BN running stats). The reference's module globals
(nStack / nFeats / nOutChannels / nModules, try_with_torch.py:23-28) become keyword arguments with
the reference's values as defaults.

`forward` of every public module runs the whole sub-graph through the HIP engine (engine.Ctx) and
autograd sees ONE node per call: backward replays the engine tape. Activations stay NHWC on the
GPU inside the call; inputs/outputs are NCHW fp32 like the reference's.

Graph-captured calls: the reference's own loop (try_with_torch.py:330-344: model(x) -> 4x
nn.MSELoss -> backward -> torch.optim.Adam) issues ~1,500 engine launches per step from Python.
From the second call with the same signature (input shape / dtype / grad mode, train/eval, engine
dtype, parameter and buffer addresses) a module call replays a hipGraph of its forward, and its
backward replays a hipGraph of the engine tape (captured at the first backward through a graphed
forward, in the forward graph's memory pool). The graphs read the parameters, BN buffers and
running statistics in place, so in-place optimizer updates / load_state_dict need no re-capture;
outputs, dx and parameter gradients are handed to autograd as fresh tensors. A graphed call whose
backward has not run yet keeps its saved activations: another call with the same signature
meanwhile runs eagerly. Results are bitwise those of the eager path (same launches, same order).
"""
import weakref
from collections import OrderedDict

import torch
import torch.nn as nn

from . import hgk as H
from .engine import Ctx

UPSAMPLE_MODES = {"bilinear": H.UP_BILINEAR_AC, "nearest": H.UP_NEAREST}

# module -> OrderedDict(signature -> _GraphEntry); weak, so graphs die with their module
_GRAPHS = weakref.WeakKeyDictionary()
_MAX_GRAPHS = 8  # signatures remembered per module (LRU; an uncaptured entry is a call counter)
# captured signatures kept per module by default: each holds a private graph memory pool with one
# step's activations, so a new capture evicts the least recently used captured entry beyond this
# many (train + eval of a loop fit; a smaller last batch of an epoch evicts nothing: it is captured
# only at its second call). set_graph_mode(max_graphs=k) changes it per model.
MAX_CAPTURED = 2


class _Token:
    """alive while a graphed forward's autograd node may still run its backward"""


class _GraphEntry:
    __slots__ = ("calls", "fwd", "bwd", "static_x", "outs_nchw", "ectx", "acts", "xin", "single",
                 "gouts", "gflat", "gviews", "touched", "dx", "busy")

    def __init__(self):
        self.calls = 0
        self.fwd = self.bwd = None
        self.busy = None

    def is_busy(self):
        return self.busy is not None and self.busy() is not None


def _engine_forward(module, want_grad, x, x_requires_grad):
    """(ectx, output acts, xin, single, NCHW outputs) of one engine forward on the current stream"""
    ectx = Ctx(module.engine_dtype(), module.training, x.device, grad_enabled=want_grad)
    xin = ectx.input(x, requires_grad=want_grad and x_requires_grad)
    outs = module.hg_forward(ectx, xin)
    single = not isinstance(outs, (list, tuple))
    outs = [outs] if single else list(outs)
    outs = [ectx.materialize(o) for o in outs]
    ectx.finish_forward()
    return ectx, outs, xin, single, tuple(ectx.output_nchw(o) for o in outs)


_BNS = weakref.WeakKeyDictionary()  # module -> its BatchNorm2d sub-modules


def _signature(module, want_grad, x, params):
    """Everything a captured call froze: input shape / dtype / grad mode, train / eval, engine
    dtype, parameter and buffer addresses, the engine and library routes in force, and the host
    scalars the BN launches carry (momentum, eps)."""
    from .engine import ROUTE
    bns = _BNS.get(module)
    if bns is None:
        bns = _BNS[module] = [m for m in module.modules() if isinstance(m, nn.BatchNorm2d)]
    return (tuple(x.shape), x.dtype, x.device, bool(x.requires_grad), bool(want_grad),
            bool(module.training), module.engine_dtype(),
            tuple((p.data_ptr(), bool(p.requires_grad)) for p in params),
            tuple(b.data_ptr() for b in module.buffers()),
            tuple(sorted(ROUTE.items())), H.route_key(),
            tuple((m.momentum, m.eps) for m in bns))


def _evict_captured(cache, keep, limit):
    """Drop least recently used captured entries (not `keep`, not busy) beyond `limit`."""
    captured = [k for k, e in cache.items() if e.fwd is not None and e is not keep]
    excess = len(captured) + 1 - limit
    for k in captured:
        if excess <= 0:
            break
        if not cache[k].is_busy():
            del cache[k]
            excess -= 1


def _graph_entry(module, want_grad, x, params):
    """the cache entry of this call, or None when the call must run eagerly"""
    if (not getattr(module, "graph_calls", False) or torch.cuda.is_current_stream_capturing()
            or Ctx.debug_lifetime_default()):
        return None
    cache = _GRAPHS.get(module)
    if cache is None:
        cache = _GRAPHS[module] = OrderedDict()
    key = _signature(module, want_grad, x, params)
    ent = cache.get(key)
    if ent is None:
        ent = cache[key] = _GraphEntry()
        while len(cache) > _MAX_GRAPHS:
            cache.popitem(last=False)
    cache.move_to_end(key)
    ent.calls += 1
    if ent.calls == 1 or ent.is_busy():
        return None  # first call: eager warm-up (lazy code-object loads, allocator) / in use
    return ent


def _capture_forward(ent, module, want_grad, x):
    ent.static_x = x.detach().clone()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        ent.ectx, ent.acts, ent.xin, ent.single, ent.outs_nchw = _engine_forward(
            module, want_grad, ent.static_x, x.requires_grad)
    ent.fwd = g
    if not want_grad:
        ent.ectx = ent.acts = ent.xin = None  # nothing to replay backward from


def _capture_backward(ent, params):
    ectx = ent.ectx
    total = sum(p.numel() for p in params)
    ent.gflat = torch.empty(max(total, 1), dtype=torch.float32, device=ent.static_x.device)
    ent.gviews, off = [], 0
    for p in params:
        v = ent.gflat[off:off + p.numel()].view(p.shape)
        ent.gviews.append((off, p.numel()))
        ectx.pgrads[id(p)] = v
        off += p.numel()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, pool=ent.fwd.pool()):
        ent.gflat.zero_()
        ectx.stream = H.stream_handle()
        for a, go in zip(ent.acts, ent.gouts):
            ectx.grad_from_nchw(a, go)
        ectx.backward()
        xin = ent.xin
        ent.dx = None
        if xin.requires_grad and xin.grad is not None:
            ent.dx = ectx.output_nchw(type(xin)(xin.grad, xin.N, xin.H, xin.W, xin.C, C_log=xin.C_log))
    ent.touched = [id(p) in ectx.touched for p in params]
    ent.bwd = g
    # the tape is consumed and every buffer the two graphs use lives in their private pool
    ent.ectx = ent.acts = ent.xin = None


class _EngineFunction(torch.autograd.Function):
    """forward: NCHW input -> engine dataflow -> NCHW outputs; backward: engine tape (eagerly, or
    as the replay of a captured hipGraph, see the module docstring)."""

    @staticmethod
    def forward(fctx, module, want_grad, x, *params):
        if not x.is_cuda:
            raise H.HgkError("the HIP engine runs on the GPU: move the model and input to cuda")
        fctx.params = params
        fctx.entry = ent = _graph_entry(module, want_grad, x, params)
        if ent is None:
            ectx, outs, xin, single, res = _engine_forward(module, want_grad, x, x.requires_grad)
            fctx.ectx, fctx.outs, fctx.xin, fctx.single = ectx, outs, xin, single
            return res
        if ent.fwd is None:
            _evict_captured(_GRAPHS[module], ent, getattr(module, "graph_max_captured", MAX_CAPTURED))
            _capture_forward(ent, module, want_grad, x)
        ent.static_x.copy_(x)
        ent.fwd.replay()
        if want_grad:
            fctx.token = _Token()
            ent.busy = weakref.ref(fctx.token)
        fctx.ectx, fctx.single = None, ent.single
        return tuple(o.clone() for o in ent.outs_nchw)

    @staticmethod
    def backward(fctx, *gouts):
        ent = fctx.entry
        if ent is not None:
            if getattr(fctx, "token", None) is None:
                raise RuntimeError("backward through the same engine call twice is not supported")
            if ent.bwd is None:
                ent.gouts = [torch.empty_like(o) for o in ent.outs_nchw]
            for st, g in zip(ent.gouts, gouts):
                st.copy_(g)
            if ent.bwd is None:
                _capture_backward(ent, fctx.params)
            ent.bwd.replay()
            fctx.token = None
            ent.busy = None
            gflat = ent.gflat.clone()
            grads = tuple(gflat[o:o + n].view(p.shape).to(p.dtype) if t else None
                          for p, (o, n), t in zip(fctx.params, ent.gviews, ent.touched))
            dx = None if ent.dx is None else ent.dx.clone()
            return (None, None, dx) + grads
        ectx = fctx.ectx
        if ectx is None:
            raise RuntimeError("backward through the same engine call twice is not supported")
        ectx.stream = H.stream_handle()
        for a, g in zip(fctx.outs, gouts):
            if g is not None:
                ectx.grad_from_nchw(a, g)
        ectx.backward()
        xin = fctx.xin
        dx = None
        if xin.requires_grad and xin.grad is not None:
            dx = ectx.output_nchw(type(xin)(xin.grad, xin.N, xin.H, xin.W, xin.C, C_log=xin.C_log))
        grads = []
        for p in fctx.params:
            g = ectx.pgrads.get(id(p))
            grads.append(None if g is None else g.to(p.dtype))
        fctx.ectx = None
        return (None, None, dx) + tuple(grads)


class _EngineModule(nn.Module):
    """Mixin: engine dtype selection + the autograd entry point."""

    _hgk_dtype = torch.float32
    _returns_list = False  # the stacked models return one heatmap per stack
    graph_calls = True     # replay captured hipGraphs from the second call of a signature on
    graph_max_captured = MAX_CAPTURED

    def set_graph_mode(self, on=True, max_graphs=None):
        """Graph-captured module calls (module docstring) on / off (off: every call eager). Each
        captured signature keeps a private memory pool holding one call's activations; at most
        `max_graphs` (default MAX_CAPTURED = 2) captured signatures are kept per module, a new
        capture evicting the least recently used one. Clears the module's graph cache."""
        if max_graphs is not None and int(max_graphs) < 1:
            raise ValueError("max_graphs must be >= 1 (set_graph_mode(False) turns graphs off)")
        for m in self.modules():
            if isinstance(m, _EngineModule):
                m.graph_calls = bool(on)
                if max_graphs is not None:
                    m.graph_max_captured = int(max_graphs)
                _GRAPHS.pop(m, None)
        return self

    def graph_cache_info(self):
        """{'signatures': remembered call signatures, 'captured': those holding hipGraphs (and a
        memory pool each), 'max_captured': the cap} of this module's graph cache."""
        cache = _GRAPHS.get(self) or {}
        return {"signatures": len(cache),
                "captured": sum(1 for e in cache.values() if e.fwd is not None),
                "max_captured": getattr(self, "graph_max_captured", MAX_CAPTURED)}

    def engine_dtype(self):
        return self._hgk_dtype

    def set_engine_dtype(self, dtype):
        """fp32 (parity path, default) or bf16 activations/weights in the kernels."""
        H.dtype_code(dtype)
        for m in self.modules():
            if isinstance(m, _EngineModule):
                m._hgk_dtype = dtype
        return self

    def never_grad_parameters(self):
        """Names of the parameters no forward reads: the `conv4` of every square ResidualBlock
        (registered unconditionally, used only when numIn != numOut, try_with_torch.py:193,205-208).
        PyTorch leaves their .grad None and torch.optim.Adam skips them; the Trainer keeps them at
        the tail of its flat buffers, outside the all-reduce and the Adam update."""
        out = []
        for name, m in self.named_modules():
            if isinstance(m, ResidualBlock) and m.numIn == m.numOut:
                out += [f"{name}.conv4.{k}" if name else f"conv4.{k}" for k, _ in m.conv4.named_parameters()]
        return out

    def grad_ready_groups(self):
        """Parameter names grouped in the order backward finalises their gradients (each group's
        grads are complete once the reverse tape passes the matching Ctx.grad_barrier). One group
        unless the model places barriers (creatModel: trunk, then stem)."""
        never = set(self.never_grad_parameters())
        return [[k for k, _ in self.named_parameters() if k not in never]]

    def forward(self, x):
        params = tuple(self.parameters())
        want_grad = torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in params))
        outs = _EngineFunction.apply(self, want_grad, x, *params)
        return list(outs) if self._returns_list else outs[0]


class ResidualBlock(_EngineModule):
    """Pre-activation bottleneck (try_with_torch.py:179-209).

    BN->ReLU->1x1(C->C/2)->BN->ReLU->3x3->BN->ReLU->1x1(C/2->C) (+ conv4 1x1 skip iff numIn !=
    numOut). Each BN+ReLU is fused into the next conv's input staging; the bias, the residual add
    and the next BN's statistics into the conv epilogue."""

    def __init__(self, numIn, numOut):
        super().__init__()
        self.numIn = numIn
        self.numOut = numOut
        mid = int(numOut / 2)
        self.bn1 = nn.BatchNorm2d(numIn)
        self.relu = nn.ReLU(True)
        self.conv1 = nn.Conv2d(numIn, mid, 1, 1)
        self.bn2 = nn.BatchNorm2d(mid)
        self.conv2 = nn.Conv2d(mid, mid, 3, 1, 1)
        self.bn3 = nn.BatchNorm2d(mid)
        self.conv3 = nn.Conv2d(mid, numOut, 1, 1)
        self.conv4 = nn.Conv2d(numIn, numOut, 1, 1)

    def hg_forward(self, ctx, x):
        h = ctx.conv(ctx.bn_relu(x, self.bn1), self.conv1)
        h = ctx.conv(ctx.bn_relu(h, self.bn2), self.conv2)
        a3 = ctx.bn_relu(h, self.bn3)
        if self.numIn != self.numOut:
            skip = ctx.conv(x, self.conv4, stats=False)
            return ctx.conv(a3, self.conv3, res=skip, inplace_res=True)
        return ctx.conv(a3, self.conv3, res=x)

    def hg_forward_twin(self, ctx, xs):
        """hg_forward on two independent inputs at once (square blocks): every conv / BN launch
        serves both (Ctx.conv_twin / bn_relu_twin); results equal two hg_forward calls."""
        assert self.numIn == self.numOut
        h = ctx.conv_twin(ctx.bn_relu_twin(xs, self.bn1), self.conv1)
        h = ctx.conv_twin(ctx.bn_relu_twin(h, self.bn2), self.conv2)
        return ctx.conv_twin(ctx.bn_relu_twin(h, self.bn3), self.conv3, res=xs)


class hourglass(_EngineModule):  # noqa: N801 (reference name)
    """Recursive hourglass with ONE shared ResidualBlock per level (try_with_torch.py:212-240).
    At the innermost level the primary applies one more residual chain (low2, :231-233);
    variants without it (try_with_aspp.py:245-246) set `_inner_chain = False`."""

    _inner_chain = True

    def __init__(self, n, f, nModules=2, upsample="bilinear"):
        super().__init__()
        self.n = n
        self.f = f
        self.nModules = nModules
        self.upsample = upsample
        self.residual_block = ResidualBlock(f, f)
        if n > 1:
            # type(self): a preset subclass recurses into itself (its extra sub-modules are
            # registered after this constructor, per level, like the reference's)
            self.hourglass1 = type(self)(n - 1, f, nModules, upsample)
        self.maxpool = nn.MaxPool2d(2)

    def _chain(self, ctx, a):
        for _ in range(self.nModules):
            a = self.residual_block.hg_forward(ctx, a)
        return a

    def _inner(self, ctx, low):
        """the innermost level's low2 (try_with_torch.py:231-233); presets override it"""
        return self._chain(ctx, low) if self._inner_chain else low

    def _twin_chain(self, ctx, x):
        """up1 = chain(x) and low1 = chain(maxpool(x)) side by side: both chains apply the SAME
        residual_block, so each of their conv / BN launches covers both (one launch instead of
        two for the latency-bound small levels). maxpool has no state, so issuing it before the
        up-branch changes nothing; the BN running statistics keep the reference's order
        (Ctx.twin_begin)."""
        pair = (x, ctx.maxpool2(x))
        ctx.twin_begin()
        for _ in range(self.nModules):
            pair = self.residual_block.hg_forward_twin(ctx, pair)
        ctx.twin_end()
        return pair

    def hg_forward(self, ctx, x):
        if ctx.twin and self.residual_block.numIn == self.residual_block.numOut:
            up1, low = self._twin_chain(ctx, x)
            low = self.hourglass1.hg_forward(ctx, low) if self.n > 1 else self._inner(ctx, low)
            low = self._chain(ctx, low)
            return ctx.upsample2_add(low, up1, UPSAMPLE_MODES[self.upsample])
        # the up branch is independent of the down branch until the final add: with
        # ctx.enable_branches() it runs on a side stream, overlapping the latency-bound small
        # levels of the down branch (forward and backward)
        br = ctx.fork() if ctx.branch_level(self.n) else None
        up1 = self._chain(ctx, x)
        ctx.back(br)
        low = self._chain(ctx, ctx.maxpool2(x))
        low = self.hourglass1.hg_forward(ctx, low) if self.n > 1 else self._inner(ctx, low)
        low = self._chain(ctx, low)
        ctx.join(br)
        return ctx.upsample2_add(low, up1, UPSAMPLE_MODES[self.upsample])


class lin(_EngineModule):  # noqa: N801
    """1x1 conv -> BN -> ReLU (try_with_torch.py:243-256); the BN+ReLU stays virtual (fused into
    the consumers' input staging)."""

    def __init__(self, numIn, numOut):
        super().__init__()
        self.numIn = numIn
        self.numOut = numOut
        self.conv = nn.Conv2d(numIn, numOut, 1, 1, 0)
        self.bn = nn.BatchNorm2d(numOut)
        self.relu = nn.ReLU()

    def hg_forward(self, ctx, x):
        return ctx.bn_relu(ctx.conv(x, self.conv), self.bn)


class creatModel(_EngineModule):  # noqa: N801
    """Stacked hourglass (try_with_torch.py:259-298): stem 7x7/2 conv + ReLU, RB(64,128), maxpool,
    RB(128,128), RB(128,nFeats); nStack passes through the SAME hourglass / residual4 / lin /
    heads; returns the list of nStack heatmaps [N, nOutChannels, H/4, W/4]."""

    _returns_list = True
    _hourglass_cls = hourglass

    def __init__(self, nStack=4, nFeats=256, nOutChannels=17, nModules=2, depth=4,
                 upsample="bilinear"):
        super().__init__()
        self._init_trunk(nStack, nFeats, nModules, depth, upsample)
        self.conv2 = nn.Conv2d(nFeats, nOutChannels, 1, 1, 0)
        self.conv3 = nn.Conv2d(nFeats, nFeats, 1, 1, 0)
        self.conv4 = nn.Conv2d(nOutChannels, nFeats, 1, 1, 0)

    def _init_trunk(self, nStack, nFeats, nModules, depth, upsample):
        """stem + shared hourglass / residual4 / lin, registered in the reference's order
        (try_with_torch.py:262-270; try_with_aspp.py:301-309)"""
        self.nStack = nStack
        self.nModules = nModules
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3)
        self.relu = nn.ReLU()
        self.residual1 = ResidualBlock(64, 128)
        self.max_pool1 = nn.MaxPool2d(2)
        self.residual2 = ResidualBlock(128, 128)
        self.residual3 = ResidualBlock(128, nFeats)
        self.hourglass1 = self._hourglass_cls(depth, nFeats, nModules, upsample)
        self.residual4 = ResidualBlock(nFeats, nFeats)
        self.lin = lin(nFeats, nFeats)

    _STEM = ("conv1.", "residual1.", "residual2.", "residual3.")

    def _stem(self, ctx, x):
        h = ctx.conv(x, self.conv1, post_relu=True)
        h = self.residual1.hg_forward(ctx, h)
        h = ctx.maxpool2(h)
        h = self.residual2.hg_forward(ctx, h)
        h = self.residual3.hg_forward(ctx, h)
        # everything after this point (hourglass, residual4, lin, heads: shared by all stacks,
        # try_with_torch.py:268,286-297) is used for the last time by stack 0, so its gradients
        # are final once backward gets back here — before the stem's own backward (:276-281)
        ctx.grad_barrier("trunk")
        return h

    def grad_ready_groups(self):
        """[trunk, stem]: the trunk's grads are final when the stem's backward starts, so their
        all-reduce overlaps it (Trainer / dp.GradSync)."""
        (active,) = super().grad_ready_groups()
        stem = [k for k in active if k.startswith(self._STEM)]
        return [[k for k in active if not k.startswith(self._STEM)], stem]

    def _stack_body(self, ctx, inter):
        """hourglass -> nModules x residual4 -> lin (virtual BN+ReLU output)"""
        ll = self.hourglass1.hg_forward(ctx, inter)
        for _ in range(self.nModules):
            ll = self.residual4.hg_forward(ctx, ll)
        return self.lin.hg_forward(ctx, ll)

    def hg_forward(self, ctx, x):
        inter = self._stem(ctx, x)
        heatmaps = []
        for s in range(self.nStack):
            a = self._stack_body(ctx, inter)
            hm = ctx.conv(a, self.conv2, stats=False)
            heatmaps.append(hm)
            # the reference also forms `inter` after the last stack (:294-297); it feeds nothing,
            # so skipping it changes no output, gradient or running statistic.
            if s + 1 < self.nStack:
                t = ctx.conv(a, self.conv3, stats=False)
                inter = ctx.conv(hm, self.conv4, res=t, inplace_res=True)
        return heatmaps
