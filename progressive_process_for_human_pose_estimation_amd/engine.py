"""Dataflow engine: runs a stacked-hourglass forward on libhgk and replays it backwards.

Modules describe their dataflow with the primitives of `Ctx` (conv, bn_relu, maxpool2,
upsample2_add); each primitive launches its HIP kernel(s) immediately on the current stream and
appends its backward to a tape. There is no tracing compiler: the tape IS the backward schedule,
and a caller may capture a whole forward+backward into a hipGraph (trainer.py).

Data layout in HBM: every activation is NHWC in the engine dtype (fp32 for parity, bf16 for
speed); BatchNorm is never materialised — `bn_relu` returns a *virtual* activation (the producer
tensor + per-channel scale/shift) that the consuming convolution applies while staging its input
tile (BN->ReLU->Conv). Batch statistics come from the producing kernel's
epilogue when it has them (conv), otherwise from one bn_stats pass.

Reference semantics followed (try_with_torch.py): shared modules -> every use launches its own
kernels with the same weights, grads accumulate into one fp32 buffer per parameter and BN running
stats are updated once per use in call order (:217,224-237,268,286); num_batches_tracked += uses.
"""
import bisect
import ctypes
import os
import traceback

import torch

from . import hgk as H


class LifetimeGuard:
    """Deterministic buffer-lifetime check (HGK_DEBUG_LIFETIME=1, or Ctx(debug_lifetime=True)).

    Kernels read device pointers that the engine took from tensors earlier (data_ptr() ints, also
    inside segment descriptors). If the last Python owner of such a tensor goes away before the
    launch that reads it, the caching allocator may hand the memory to the next allocation and
    the kernel reads someone else's data (the f11e87b bug: a twin segment's partials re-used as
    the other segment's gradient) — visible only under allocator contention.

    The guard holds every buffer the Ctx allocates until the step ends (so no address is reused
    inside the step) and wraps the library: at every launch each pointer argument (plain or a
    c_void_p field of a ctypes descriptor array) that falls inside a tracked buffer must still
    have an owner besides the guard (storage use count). A buffer whose only owner is the guard
    would have been free at that launch: the launch raises, naming the entry point, the argument
    and the allocation site."""

    def __init__(self, lib):
        self._lib = lib
        self._starts = []     # sorted buffer start addresses
        self._bufs = {}       # start -> (end, tensor, allocation site)
        self.launches = 0
        self.checked = 0      # pointer arguments resolved to a tracked buffer

    def track(self, t):
        if t.numel() == 0:
            return t
        a = t.data_ptr()
        if a not in self._bufs:
            bisect.insort(self._starts, a)
        site = "".join(traceback.format_stack(limit=4)[:-2]).strip()
        # an alias of its own (a second TensorImpl on the storage): the engine's tensors are
        # counted apart from it
        self._bufs[a] = (a + t.numel() * t.element_size(), t.detach(), site)
        return t

    def _owner(self, p):
        i = bisect.bisect_right(self._starts, p) - 1
        if i < 0:
            return None
        end, t, site = self._bufs[self._starts[i]]
        return (t, site) if p < end else None

    def _pointers(self, args):
        for k, a in enumerate(args):
            if isinstance(a, int) and a > 4096:
                yield f"arg {k}", a
            elif isinstance(a, ctypes.Array) and len(a) and isinstance(a[0], ctypes.Structure):
                for j, st in enumerate(a):
                    for fname, ftype in st._fields_:
                        if ftype is ctypes.c_void_p:
                            v = getattr(st, fname)
                            if v:
                                yield f"arg {k}[{j}].{fname}", v

    def __getattr__(self, name):
        fn = getattr(self._lib, name)
        if not name.startswith("hgk_") or not callable(fn):
            return fn

        def launch(*args):
            self.launches += 1
            for where, p in self._pointers(args):
                hit = self._owner(p)
                if hit is None:
                    continue
                t, site = hit
                self.checked += 1
                # owners of the storage besides the guard's alias and the temporary storage object
                if torch._C._storage_Use_Count(t.untyped_storage()._cdata) <= 2:
                    raise RuntimeError(f"lifetime: {name} {where} reads a buffer with no owner left "
                                       f"(it would be free and re-usable at this launch); "
                                       f"allocated at:\n{site}")
            return fn(*args)
        return launch

    def release(self):
        self._starts.clear()
        self._bufs.clear()


_SIDE_STREAMS = {}


def _side_stream(device, i):
    """Side HIP streams of the branch-parallel schedule, created once per device and reused (a
    captured hipGraph keeps only the dependency edges, not the streams)."""
    lst = _SIDE_STREAMS.setdefault(str(device), [])
    while len(lst) <= i:
        lst.append(torch.cuda.Stream(device=device))
    return lst[i]


def _oshape(a):
    return (a.N, a.H, a.W, a.C)


class Act:
    """An NHWC activation [N, H, W, C] (real), or relu?(bn(src)) (virtual: `bn` is a BNUse).
    C is the STORED channel count; C_log <= C the logical one (channel-padded heatmaps)."""
    __slots__ = ("t", "N", "H", "W", "C", "C_log", "stats", "bn", "src", "requires_grad", "_grad",
                 "uses", "bwd_part", "gshared", "pending", "producer")

    def __init__(self, t, N, Hh, W, C, stats=None, requires_grad=True, C_log=None):
        self.t, self.N, self.H, self.W, self.C = t, N, Hh, W, C
        self.C_log = C if C_log is None else C_log
        self.stats = stats
        self.bn = None
        self.src = None
        self.requires_grad = requires_grad
        self._grad = None
        # PendingApply: this act's grad is a BN-backward apply not launched yet (Ctx._bn_relu_bwd);
        # reading .grad launches it, a folding input-gradient conv takes it over (Ctx._conv_bwd)
        self.pending = None
        # (core, index): core = (inputs, conv, post_relu, output shapes) of the Ctx.conv /
        # conv_twin call that made this act (shared by a twin pair), index = which output this is:
        # whether that conv's input gradient can fold a pending apply (Ctx._can_defer_apply). Only
        # shapes are kept, never the outputs themselves (an act referring to itself would put
        # every conv output in a reference cycle that only the cyclic GC frees)
        self.producer = None
        self.uses = 0          # consumers of a virtual activation (forward)
        self.bwd_part = None   # (partials, rows): BN-backward sums fused into its producer
        self.gshared = False   # grad aliases a buffer a deferred weight-grad still reads

    @property
    def grad(self):
        p = self.pending
        if p is not None:
            self.pending = None
            p.materialize()
        return self._grad

    @grad.setter
    def grad(self, g):
        if self.pending is not None:
            raise RuntimeError("engine: overwriting an activation gradient whose BN-backward apply "
                               "was never launched")
        self._grad = g

    @property
    def M(self):
        return self.N * self.H * self.W

    @property
    def real(self):
        return self.src if self.bn is not None else self


# Engine-level routing: compiled-in defaults, changed only explicitly (tests, A/B scripts via
# `routing(...)` or bench.py --route), never by the environment. twin: one launch per conv / BN for
# an hourglass level's two chains; fold_apply / fold_fin: the deferred BN-backward apply / forward
# finalize folded into the consuming conv launch; fold_bwd_fin: at the small levels the BN-backward
# finalize+apply folded into the image-tile input gradient (needs fold_apply); fold_bwd_add: bn1's
# too, with the skip gradient added in the kernel (off: -0.2 % img/s same-box, the 256-channel
# input gradient's third operand costs more than the launch it saves, profiles/r04_bn1_fold_ab.txt)
# (Ctx docs).
# bn_add: a BN pair whose outputs are summed (hourglass_compare's block output) in one fused pass
# forward (Ctx.bn_add) and one dual reduction backward; off = materialize x2 + add (bitwise equal).
# bn_pair_bwd: after bn_add's dual reduction, both BNs' finalize + apply in one launch reading the
# common gradient once (hgk_bn_bwd_pair) when neither apply folds into its producer's input
# gradient; off = each side's own finalize / apply in _bn_relu_bwd (bitwise equal).
# pair_apply: with many partial rows, both applies of bn_pair_bwd in the one pair kernel too
# (off: two apply launches, dA read twice; on: +0.9 % on hourglass_compare,
# profiles/r05_pair_apply_ab.txt).
# fin_batch: a train-mode BN finalize the consuming conv cannot fold waits until a statistic is
# read, then goes out with every other such finalize pending (hgk_bn_finalize_multi; the pair
# backward's two coefficient finalizes likewise, hgk_bn_bwd_finalize_multi); off = one launch per
# BN at its bn_relu call (bitwise equal).
# pair_blocks: a preset's independent blocks run interleaved op by op (their lazy finalizes go
# out together); off = sequential (bitwise equal).
# wg_batch: the deferred weight gradients of single-use weights batched across weights into shared
# launches at the end of backward (Ctx.finish_wgrads); off = one launch per weight. Bitwise equal
# only with the library routes wg_batch_slab_x10 = 20 and wg_batch_target = 0 (the single call's
# split plan; tests/test_gpu_wgrad_batch.py pins those): the compiled default slab cap (5 = 0.5x)
# picks fewer pixel splits than the single call (2x), so the fp32 summation order differs and the
# default cap is gated with a tolerance (test_gpu_wgrad_batch.py::test_wgrad_batch_slab_cap[5]).
# mse_heads: the Trainer's per-stack MSE heads (one target) in ONE hgk_mse_heads_nhwc launch on the
# NHWC heads; off = per head nhwc_to_nchw + hgk_mse_fwd_bwd + finalize + nchw_to_nhwc (gradients
# bitwise equal, the loss to fp32 summation order).
ROUTE = {"twin": True, "fold_apply": True, "fold_fin": True, "fold_bwd_fin": True, "fold_bwd_add": False,
         "bn_add": True, "bn_pair_bwd": True, "pair_apply": True, "fin_batch": True, "pair_blocks": True,
         "wg_batch": True, "mse_heads": True}


class routing:
    """`with engine.routing(twin=False): ...`: Ctx objects created inside use these routes."""

    def __init__(self, **kw):
        bad = set(kw) - set(ROUTE)
        if bad:
            raise ValueError(f"unknown engine route(s) {sorted(bad)}: expected {sorted(ROUTE)}")
        self.kw, self.prev = kw, {}

    def __enter__(self):
        self.prev = {k: ROUTE[k] for k in self.kw}
        ROUTE.update({k: bool(v) for k, v in self.kw.items()})
        return self

    def __exit__(self, *exc):
        ROUTE.update(self.prev)
        return False


def apply_route_spec(spec):
    """'name=value,...' over engine routes (ROUTE) and library routes (hgk.ROUTES), for scripts
    and bench.py --route; returns the (engine, library) routing context managers, entered."""
    eng, libr = {}, {}
    for item in filter(None, (spec or "").split(",")):
        k, v = item.split("=")
        k = k.strip()
        if k in ROUTE:
            eng[k] = int(v) != 0
        elif k in H.ROUTES:
            libr[k] = int(v)
        else:
            raise ValueError(f"unknown route {k!r}: engine {sorted(ROUTE)}, library {sorted(H.ROUTES)}")
    cms = (routing(**eng), H.route(**libr))
    for cm in cms:
        cm.__enter__()
    return cms


# process-wide count of BN-backward applies folded into input-gradient launches (tests / evidence)
STATS = {"folded": 0, "fin_folded": 0}


class PendingApply:
    """A train-mode BN(+ReLU) backward apply dy = hgk_bn_bwd_apply(dA, y, coef) into `dst`, not
    launched yet (its finalize already ran: coef, dgamma and dbeta are final). The BN's input is a
    conv output whose only reader in backward is that conv's input gradient: when its kernel can
    stage the apply itself (hgk_conv_fwd_bnbwd_vg / hgk_conv_seg.vg, hgk_conv_vgrad_ok) the apply
    pass disappears (one read of dA and y instead of read dA, y + write dy + read dy); any other
    reader of the act's .grad launches the apply first (materialize).
    `fin` = (partials, rows): the finalize is deferred too (small levels, few partial rows: the
    image-tile input gradient computes the coefficients and accumulates dgamma / dbeta itself,
    hgk_bn_vgrad.partial; materialize launches hgk_bn_bwd_finalize_apply); coef is None then.
    `add` (with fin): the gradient already accumulated for the BN input (bn1's skip gradient),
    dst = apply + add (hgk_bn_vgrad.add); it is only read."""
    __slots__ = ("ctx", "dA", "x", "use", "coef", "dst", "fin", "add")

    def __init__(self, ctx, dA, x, use, coef, dst, fin=None, add=None):
        self.ctx, self.dA, self.x, self.use, self.coef, self.dst = ctx, dA, x, use, coef, dst
        self.fin, self.add = fin, add

    def vgrad(self):
        u = self.use
        if self.fin is None:
            return H.BnVgrad(self.x.t.data_ptr(), u.scale.data_ptr(), u.shift.data_ptr(),
                             self.coef.data_ptr(), 1 if u.relu else 0, self.dst.data_ptr())
        part, rows = self.fin
        bn = u.mod
        c = self.ctx
        return H.BnVgrad(self.x.t.data_ptr(), u.scale.data_ptr(), u.shift.data_ptr(), None,
                         1 if u.relu else 0, self.dst.data_ptr(), part.data_ptr(), rows, self.x.M,
                         u.mean.data_ptr(), u.invstd.data_ptr(), 1 if u.training else 0,
                         c.pgrad(bn.weight).data_ptr(), c.pgrad(bn.bias).data_ptr(),
                         None if self.add is None else self.add.data_ptr())

    def materialize(self):
        c, u, x = self.ctx, self.use, self.x
        if self.fin is not None:
            part, rows = self.fin
            bn = u.mod
            H.check(c.lib.hgk_bn_bwd_finalize_apply(
                c.stream, c.dt, part.data_ptr(), rows, x.M, x.C, u.scale.data_ptr(),
                u.shift.data_ptr(), 1 if u.relu else 0, u.mean.data_ptr(), u.invstd.data_ptr(),
                1 if u.training else 0, c.pgrad(bn.weight).data_ptr(), c.pgrad(bn.bias).data_ptr(),
                self.dA.data_ptr(), x.t.data_ptr(), None if self.add is None else self.add.data_ptr(),
                self.dst.data_ptr(), 0))
        else:
            H.check(c.lib.hgk_bn_bwd_apply(c.stream, c.dt, self.dA.data_ptr(), x.t.data_ptr(), x.M,
                                           x.C, u.scale.data_ptr(), u.shift.data_ptr(),
                                           1 if u.relu else 0, self.coef.data_ptr(), None,
                                           self.dst.data_ptr(), 0))
        c._pub(("g", id(x)))


class BNUse:
    """One train/eval-mode use of a BatchNorm module: stat [4][C] = mean | invstd | scale | shift.
    `pending` (training, small levels): the finalize is not launched yet — the consuming conv
    folds it into its own launch (hgk_conv_fwd_fold) and writes stat and the running-statistics
    record; reading any statistic before that launches the finalize (resolve)."""
    __slots__ = ("mod", "x", "stat", "relu", "training", "pending", "ctx", "batch")

    def __init__(self, mod, x, stat, relu, training):
        self.mod, self.x, self.stat, self.relu, self.training = mod, x, stat, relu, training
        self.pending = None  # (partials, rows, record [2][C] fp64)
        self.ctx = None
        # the pending finalize is not foldable: it runs, together with every other such finalize
        # pending at that moment, when a statistic is first read (Ctx._resolve_fin, fin_batch)
        self.batch = False

    def resolve(self):
        if self.pending is not None:
            self.ctx._resolve_fin(self)

    def fold_desc(self):
        """hgk_bn_fold of the pending finalize (the caller launches it, then clears pending)"""
        part, rows, rec = self.pending
        bn = self.mod
        return H.BnFold(part.data_ptr(), rows, self.x.M, H.ptr(bn.weight), H.ptr(bn.bias),
                        float(bn.eps), self.stat.data_ptr(), rec.data_ptr())

    @property
    def mean(self):
        self.resolve()
        return self.stat[0]

    @property
    def invstd(self):
        self.resolve()
        return self.stat[1]

    @property
    def scale(self):
        self.resolve()
        return self.stat[2]

    @property
    def shift(self):
        self.resolve()
        return self.stat[3]


class Ctx:
    def __init__(self, dtype, training, device, grad_enabled=True, debug_lifetime=None):
        self.dtype = dtype
        self.dt = H.dtype_code(dtype)
        self.training = training
        self.device = device
        self.grad_enabled = grad_enabled
        if debug_lifetime is None:
            debug_lifetime = Ctx.debug_lifetime_default()
        self.guard = LifetimeGuard(H.lib()) if debug_lifetime else None
        self.lib = self.guard if debug_lifetime else H.lib()
        self.stream = H.stream_handle()
        self.tape = []
        self.packed = {}       # id(conv) -> (w_fwd, ld)
        self.packed_dgrad = {}  # id(conv) -> (w_dgrad, ld)
        self.bn_uses = {}      # id(bn module) -> (module, count)
        self.pgrads = {}       # id(param) -> fp32 grad buffer
        self._rows = H.ctypes.c_int(0)
        self._ws = {}          # stream index -> split-K workspace
        self._keep = []        # scratch buffers referenced by enqueued kernels
        self.wslabs = {}       # id(conv) -> [slab buffer, slabs holding data, cap, conv, dims]
        # weight-grads of small-level uses, run at the end of backward as ONE multi-use launch per
        # weight (hgk_conv_wgrad_accum_multi): id(conv) -> [(hgk_wgrad_src fields, refs)]
        self.wdefer = {}
        # pixels per use up to which a weight-grad is deferred: 3x3 only below the 32x32 level
        # (there the halo weight-grad kernel beats the implicit GEMM), 1x1 always
        self.wdefer_max_m = 8192
        self.wdefer_max_m_1x1 = 1 << 30
        self.nbt_batch = None  # (flat int64 counters, per-step increments): see Trainer
        # grad_barrier callback: on_grads_ready(tag) runs when backward passes the barrier (the
        # Trainer launches that group's all-reduce there / splits its graph capture)
        self.on_grads_ready = None
        self.barriers_passed = []
        # seal_groups[i]: id(param) of the grad-ready group whose grads are final at barrier i
        # (set by the Trainer). Passing barrier i seals that group: a later gradient write into
        # it would race with the group's all-reduce already in flight, so pgrad() raises
        self.seal_groups = None
        self.sealed = set()
        self.touched = set()   # id(param) of every parameter whose grad a kernel wrote
        # maxpool / upsample outputs carry their BN statistics (fused *_fwd_stats kernels)
        self.stats_ops = True
        # BN backward with few partial rows: finalize folded into the apply launch
        self.fused_bwd_fin = True
        # BN backward with many partial rows (the 64x64 / 32x32 levels): the apply is folded into
        # the consuming input-gradient conv where its kernel stages it (PendingApply);
        # ROUTE["fold_apply"] = False: always a separate apply pass (ablation / A-B)
        self.fold_apply = bool(ROUTE["fold_apply"])
        self.n_folded = 0  # applies taken over by an input-gradient launch (tests / evidence)
        # ... and at the small levels their finalizes too (hgk_bn_vgrad.partial, image tiles);
        # _fin_pending: those not taken yet (flushed at a grad barrier / the end of backward)
        self.fold_bwd_fin = bool(ROUTE["fold_bwd_fin"])
        self.fold_bwd_add = bool(ROUTE["fold_bwd_add"])
        self._fin_pending = []
        self.n_fin_folded = 0  # forward finalizes taken over by the consuming conv
        # BN forward finalize with few partial rows (the 8x8 / 4x4 levels): folded into the
        # consuming conv's launch (BNUse.pending, hgk_conv_fwd_fold); ROUTE["fold_fin"]: ablation
        self.fold_fin = bool(ROUTE["fold_fin"])
        self._pending_fin = []
        # twin execution (hourglass.hg_forward): an hourglass level's up-branch and down-branch
        # blocks share one ResidualBlock, so each conv / BN launch serves both uses
        # (hgk_conv_fwd_twin, hgk_bn_finalize_deferred, hgk_bn_bwd_twin). BN running statistics
        # are then recorded per use and applied in the reference's call order at finish_forward
        # (hgk_bn_running_update): the momentum EMA is order dependent
        self.twin = bool(ROUTE["twin"])
        self.bn_pair = bool(ROUTE["bn_add"])
        self.bn_pair_bwd = bool(ROUTE["bn_pair_bwd"])
        self.pair_apply = bool(ROUTE["pair_apply"])
        self.fin_batch = bool(ROUTE["fin_batch"])
        # presets with independent unshared blocks run them interleaved (hourglass_compare)
        self.pair_blocks = bool(ROUTE["pair_blocks"])
        self.n_fin_batched = 0
        self.wg_batch = bool(ROUTE["wg_batch"])
        self.defer_running = self.twin and training
        self._run_entries = []  # (bn module, fp64 record [2][C]) in reference call order
        self._run_hold = None   # down-branch records of the open twin chain
        # branch-parallel schedule (enable_branches): independent hourglass branches run on side
        # streams; stream 0 = the caller's current stream
        self.multi = False
        self._streams = [(torch.cuda.current_stream(device), self.stream)]
        self.sid = 0
        self._active = []      # side-stream indices held by open branches
        self._last = {}        # resource key -> (stream index, event) of its last writer
        self._hold = []        # every tensor a side-stream kernel may touch: freed at the end

    @staticmethod
    def debug_lifetime_default():
        """HGK_DEBUG_LIFETIME=1: every Ctx runs under the lifetime guard (a debug path)."""
        return os.environ.get("HGK_DEBUG_LIFETIME", "0") != "0"

    def enable_branches(self, on=True):
        """Run the up-branch of every hourglass level on a side stream, concurrently with the
        down-branch (which holds the latency-bound small levels). Ordering of the shared-weight
        read-modify-writes (BN running stats, dgamma/dbeta, weight-grad slabs, activation-grad
        accumulation) follows host issue order through per-resource events, so results are
        identical to the single-stream schedule."""
        self.multi = bool(on)
        if self.multi:
            self.twin = False
            self.defer_running = False
            self.fold_apply = False  # a pending apply would launch on whichever stream reads it
            self.fold_fin = False
        return self

    def branch_level(self, n):
        """fork the up-branch of hourglass level n (every level when branches are on)?"""
        return self.multi

    # ------------------------------------------------------------------ streams / ordering
    def _set_stream(self, sid):
        self.sid = sid
        self.stream = self._streams[sid][1]

    def _event(self):
        ev = torch.cuda.Event()
        ev.record(self._streams[self.sid][0])
        return ev

    def _wait(self, ev):
        self._streams[self.sid][0].wait_event(ev)

    def _dep(self, key):
        """Order this stream after the last writer of `key` (if it ran on another stream)."""
        if self.multi:
            last = self._last.get(key)
            if last is not None and last[0] != self.sid:
                self._wait(last[1])

    def _pub(self, key):
        if self.multi:
            self._last[key] = (self.sid, self._event())

    def _torch_sync(self):
        """torch ops (zeros / copy_) run on stream 0: make the current side stream wait."""
        if self.multi and self.sid != 0:
            ev = torch.cuda.Event()
            ev.record(self._streams[0][0])
            self._wait(ev)

    def _rec(self, fn):
        self.tape.append((self.sid, fn))

    def fork(self):
        """Start a branch on a free side stream (after everything issued so far on this one)."""
        if not self.multi:
            return None
        parent = self.sid
        child = 1
        while child in self._active:
            child += 1
        self._active.append(child)
        while len(self._streams) <= child:
            st = _side_stream(self.device, len(self._streams) - 1)
            self._streams.append((st, st.cuda_stream))
        ev = self._event()
        self._set_stream(child)
        self._wait(ev)
        self.tape.append(("fork", parent, child))
        return (parent, child)

    def back(self, br):
        """Continue on the parent stream (the branch keeps running on its side stream)."""
        if br is None:
            return
        self._set_stream(br[0])
        self.tape.append(("back", br[0], br[1]))

    def join(self, br):
        """The parent stream waits for the branch."""
        if br is None:
            return
        parent, child = br
        self._set_stream(child)
        ev = self._event()
        self._set_stream(parent)
        self._wait(ev)
        self._active.remove(child)
        self.tape.append(("join", parent, child))

    # ------------------------------------------------------------------ helpers
    def _alloc(self, shape, dtype):
        # buffers are allocated on stream 0 (torch's current stream); with side streams in use a
        # freed buffer could be handed to a stream-0 allocation while a side kernel still reads
        # it, so every buffer is held until the Ctx is done
        t = torch.empty(shape, dtype=dtype, device=self.device)
        if self.multi:
            self._hold.append(t)
        if self.guard is not None:
            self.guard.track(t)
        return t

    def _empty(self, *shape, dtype=None):
        return self._alloc(shape, dtype or self.dtype)

    def _f32(self, *shape):
        return self._alloc(shape, torch.float32)

    def _zeros_f32(self, *shape):
        t = torch.zeros(shape, dtype=torch.float32, device=self.device)
        if self.multi:
            self._hold.append(t)
        if self.guard is not None:
            self.guard.track(t)
        self._torch_sync()
        return t

    def workspace(self, nbytes):
        """conv split-K workspace: allocated zeroed (its head holds the split tiles' arrival
        counters, which every launch leaves zero)"""
        ws = self._ws.get(self.sid)
        if ws is None or ws.numel() < nbytes:
            ws = torch.zeros((max(nbytes, 1 << 20),), dtype=torch.uint8, device=self.device)
            if self.multi:
                self._hold.append(ws)
            if self.guard is not None:
                self.guard.track(ws)
            self._torch_sync()
            self._ws[self.sid] = ws
        return ws

    def pgrad(self, p):
        if id(p) in self.sealed:
            raise RuntimeError("gradient write into a parameter whose grad-ready group was sealed at "
                               "an earlier grad barrier (its all-reduce is already in flight): the "
                               "model's grad_ready_groups() do not match its dataflow")
        self.touched.add(id(p))
        g = self.pgrads.get(id(p))
        if g is None:
            g = torch.zeros(p.shape, dtype=torch.float32, device=self.device)
            if self.guard is not None:
                self.guard.track(g)
            if self.multi:  # zeroed by torch on stream 0
                self._hold.append(g)
                ev = torch.cuda.Event()
                ev.record(self._streams[0][0])
                self._last[("pg", id(p))] = (0, ev)
            self.pgrads[id(p)] = g
        self._dep(("pg", id(p)))
        return g

    def grad_slot(self, act):
        """(dst, accumulate, src) to write act's grad into: dst = src (+)= new grad. src is not
        dst when act's grad buffer is shared with a deferred weight-grad (copy on write: the
        accumulation is done out of place into a fresh dst). Call _pub(("g", id(act))) after."""
        if act.grad is None:
            act.grad = self._empty(act.N, act.H, act.W, act.C)
            return act.grad, 0, act.grad
        self._dep(("g", id(act)))
        if act.gshared:
            old = act.grad
            act.grad = self._empty(act.N, act.H, act.W, act.C)
            act.gshared = False
            return act.grad, 1, old
        return act.grad, 1, act.grad

    def grad_slot_inplace(self, act):
        """grad_slot for kernels that can only accumulate in place: a shared buffer is copied
        into the fresh one first."""
        dst, acc, src = self.grad_slot(act)
        if src is not dst:
            H.check(self.lib.hgk_add(self.stream, self.dt, src.data_ptr(), None, dst.data_ptr(),
                                     src.numel(), 0))
        return dst, acc

    def add_grad(self, act, g, shared=False):
        """act.grad += g; `shared`: g is also read by a deferred weight-grad (no aliasing writes)."""
        if not act.requires_grad:
            return
        if act.grad is None:
            act.grad = g  # alias: g's previous owner is already consumed (reverse order)
            act.gshared = shared
        else:
            dst, _, src = self.grad_slot(act)
            H.check(self.lib.hgk_add(self.stream, self.dt, g.data_ptr(),
                                     None if src is dst else src.data_ptr(), dst.data_ptr(),
                                     g.numel(), 1 if src is dst else 0))
        self._pub(("g", id(act)))

    def input(self, x_nchw, requires_grad=False):
        """NCHW fp32 -> NHWC engine dtype. Fewer channels than one 16-byte chunk (the RGB image)
        are zero-padded to one chunk, so the stem conv takes the small-Cin MFMA path."""
        N, C, Hh, W = x_nchw.shape
        vec = 8 if self.dtype == torch.bfloat16 else 4
        cs = vec if C < vec else C
        t = self._empty(N, Hh, W, cs)
        x32 = x_nchw.contiguous().float()
        H.check(self.lib.hgk_nchw_to_nhwc(self.stream, self.dt, x32.data_ptr(), t.data_ptr(), N, C,
                                          Hh, W, cs))
        return Act(t, N, Hh, W, cs, requires_grad=requires_grad, C_log=C)

    def output_nchw(self, a):
        out = self._alloc((a.N, a.C_log, a.H, a.W), torch.float32)
        H.check(self.lib.hgk_nhwc_to_nchw(self.stream, self.dt, a.t.data_ptr(), out.data_ptr(), a.N,
                                          a.C_log, a.H, a.W, a.C))
        return out

    def grad_from_nchw(self, a, g_nchw):
        g = self._empty(a.N, a.H, a.W, a.C)
        g32 = g_nchw.contiguous().float()
        H.check(self.lib.hgk_nchw_to_nhwc(self.stream, self.dt, g32.data_ptr(), g.data_ptr(), a.N,
                                          a.C_log, a.H, a.W, a.C))
        self.add_grad(a, g)

    def store_channels(self, C):
        """Stored channel count of a conv output: a multiple of the MFMA k-stage (64 bf16 / 32
        fp32) so consumers take the vectorised path; the 17/18-channel heatmaps get padded."""
        bk = 64 if self.dtype == torch.bfloat16 else 32
        return C if C % bk == 0 else (C + bk - 1) // bk * bk

    def _unit_affine(self, C):
        """[4, C] = (ones, zeros, zeros, zeros): scale=1/shift=0 rows and coef (1, 0, 0, 0)."""
        u = torch.zeros((4, C), dtype=torch.float32, device=self.device)
        u[0].fill_(1.0)
        if self.multi:
            self._hold.append(u)
        if self.guard is not None:
            self.guard.track(u)
        self._torch_sync()
        return u

    # ------------------------------------------------------------------ weights
    def _pack(self, conv, dgrad, cout_st, cin_st):
        key = (id(conv), cout_st, cin_st)
        cache = self.packed_dgrad if dgrad else self.packed
        hit = cache.get(key)
        if hit is not None:
            self._dep(("pk", dgrad) + key)  # packed on another stream by an earlier use
            return hit
        w = conv.weight
        Cout, Cin, KH, KW = w.shape
        rows = cin_st if dgrad else cout_st
        ld = self.lib.hgk_conv_w_ld(KH * KW * (cout_st if dgrad else cin_st))
        rows_pad = (rows + 127) // 128 * 128
        packed = self._empty(rows_pad, ld)
        w32 = w.detach().float().contiguous()
        H.check(self.lib.hgk_pack_conv_weight(self.stream, self.dt, w32.data_ptr(), packed.data_ptr(),
                                              ld, Cout, Cin, KH, KW, 1 if dgrad else 0, cout_st,
                                              cin_st))
        self._pub(("pk", dgrad) + key)
        cache[key] = (packed, ld)
        return packed, ld

    def pack_plan(self):
        """The weight layouts this context packed, as prepack() takes them."""
        plan = [(k[0], False, k[1], k[2]) for k in self.packed if k[0] != "bias"]
        plan += [(k[0], True, k[1], k[2]) for k in self.packed_dgrad]
        return plan

    def prepack(self, plan, convs):
        """Pack every layout of `plan` [(id(conv), dgrad, cout_st, cin_st)] in ONE multi-pack
        launch (hgk_pack_conv_weight_multi) and seed the caches that _pack() reads; `convs`
        maps id(conv) -> the nn.Conv2d."""
        descs, keep = [], []
        for cid, dgrad, cout_st, cin_st in plan:
            conv = convs[cid]
            key = (cid, cout_st, cin_st)
            cache = self.packed_dgrad if dgrad else self.packed
            if key in cache:
                continue
            w = conv.weight
            Cout, Cin, KH, KW = w.shape
            rows = cin_st if dgrad else cout_st
            ld = self.lib.hgk_conv_w_ld(KH * KW * (cout_st if dgrad else cin_st))
            packed = self._empty((rows + 127) // 128 * 128, ld)
            w32 = w.detach()
            assert w32.dtype == torch.float32 and w32.is_contiguous()
            descs.append(H.PackDesc(w32.data_ptr(), packed.data_ptr(), ld, Cout, Cin, KH, KW,
                                    1 if dgrad else 0, cout_st, cin_st, rows))
            keep.append(w32)
            cache[key] = (packed, ld)
        if descs:
            arr = (H.PackDesc * len(descs))(*descs)
            H.check(self.lib.hgk_pack_conv_weight_multi(self.stream, self.dt, arr, len(descs)))
        self._keep.extend(keep)

    def _bias(self, conv, cout_st):
        """the conv bias, zero-extended to the stored output channels"""
        b = conv.bias
        if b is None or cout_st == b.numel():
            return b
        key = ("bias", id(conv), cout_st)
        hit = self.packed.get(key)
        if hit is None:
            hit = torch.zeros(cout_st, dtype=torch.float32, device=self.device)
            hit[:b.numel()].copy_(b.detach())
            if self.multi:  # written by torch on stream 0
                ev = torch.cuda.Event()
                ev.record(self._streams[0][0])
                self._last[key] = (0, ev)
            self.packed[key] = hit
        self._dep(key)
        return hit

    # ------------------------------------------------------------------ BatchNorm (+ReLU), virtual
    def _fin_scratch(self, rows, C):
        """Scratch for the 64:1 partial merge of the finalisers (kept alive on the tape owner)."""
        nbytes = self.lib.hgk_bn_finalize_scratch(rows, C)
        if not nbytes:
            return None
        buf = self._f32(nbytes // 4)
        self._keep.append(buf)
        return buf.data_ptr()

    def bn_relu(self, x, bn, relu=True):
        """relu?(bn(x)) as a virtual activation consumed by convolutions' input staging."""
        assert x.bn is None
        C, M = x.C, x.M
        stat = self._f32(4, C)
        mean, invstd, scale, shift = stat[0], stat[1], stat[2], stat[3]
        training = self.training
        if training:
            if x.stats is None:
                rows_cap = min(2048, (M + 7) // 8 + 1)
                part = self._f32(rows_cap * 3 * C)
                H.check(self.lib.hgk_bn_stats(self.stream, self.dt, x.t.data_ptr(), M, C,
                                              part.data_ptr(), H.ctypes.byref(self._rows)))
                x.stats = (part, self._rows.value)
                self._pub(("st", id(x)))
            else:
                self._dep(("st", id(x)))
            part, rows = x.stats
            fold = self._can_fold_fin(x, rows)
            lazy = not fold and self.fin_batch and self.defer_running
            if not fold and not lazy:
                self._finalize(bn, part, rows, M, C, stat)
            mod_id = id(bn)
            prev = self.bn_uses.get(mod_id)
            self.bn_uses[mod_id] = (bn, 1 if prev is None else prev[1] + 1)
        else:
            H.check(self.lib.hgk_bn_finalize(self.stream, None, 0, M, C, bn.weight.data_ptr(),
                                             bn.bias.data_ptr(), bn.running_mean.data_ptr(),
                                             bn.running_var.data_ptr(), float(bn.momentum),
                                             float(bn.eps), 0, mean.data_ptr(), invstd.data_ptr(),
                                             scale.data_ptr(), shift.data_ptr(), None))
        use = BNUse(bn, x, stat, relu, training)
        if training and (fold or lazy):
            rec = self._alloc((2, C), torch.float64)
            self._run_entries.append((bn, rec))  # the record's place in the reference's call order
            use.batch = lazy
            self._defer_fin(use, part, rows, rec)
        v = Act(None, x.N, x.H, x.W, C, requires_grad=x.requires_grad)
        v.bn = use
        v.src = x
        if self.grad_enabled:
            self._rec(lambda: self._bn_relu_bwd(v))
        return v

    def _can_fold_fin(self, x, rows):
        return (self.fold_fin and self.defer_running and self.dt == H.BF16 and 0 < rows <= 32
                and rows % 4 == 0 and x.C <= 256)

    def _defer_fin(self, use, part, rows, rec):
        use.pending = (part, rows, rec)
        use.ctx = self
        self._pending_fin.append(use)

    def _resolve_fin(self, use):
        """launch a pending finalize (its consumer could not fold it); a lazy one (use.batch) goes
        out with every other lazy finalize pending now, in ONE hgk_bn_finalize_multi launch
        (bitwise each BN's own hgk_bn_finalize_deferred)"""
        if use.batch:
            group = [u for u in self._pending_fin if u.batch and u.pending is not None]
            if use not in group:
                group.append(use)
            jobs = []
            for u in group:
                part, rows, rec = u.pending
                bn = u.mod
                jobs.append(H.BnFinJob(part.data_ptr(), rows, u.x.M, u.x.C, H.ptr(bn.weight),
                                       H.ptr(bn.bias), float(bn.eps), rec.data_ptr(),
                                       u.stat.data_ptr()))
                u.pending = None
                u.ctx = None
            self.n_fin_batched += len(group)
            H.check(self.lib.hgk_bn_finalize_multi(self.stream, (H.BnFinJob * len(jobs))(*jobs),
                                                   len(jobs)))
            return
        part, rows, rec = use.pending
        use.pending = None
        use.ctx = None  # (no Ctx <-> BNUse cycle once resolved)
        bn = use.mod
        arr = (H.BnSeg * 1)(H.BnSeg(part.data_ptr(), rows, use.x.M, rec.data_ptr(), use.stat.data_ptr()))
        H.check(self.lib.hgk_bn_finalize_deferred(self.stream, arr, 1, use.x.C, H.ptr(bn.weight),
                                                  H.ptr(bn.bias), float(bn.eps)))

    def _fold_ok(self, as_, conv):
        """the conv launch over these inputs (1 or 2 segments) folds their pending finalizes"""
        w = conv.weight
        Cout, Cin, KH, KW = w.shape
        xs = [a.real for a in as_]
        if not all(a.bn is not None and a.bn.pending is not None and not a.bn.batch for a in as_):
            return False
        x1 = xs[1] if len(xs) > 1 else None
        return bool(self.lib.hgk_conv_fold_ok(
            self.dt, xs[0].N, xs[0].H, xs[0].W, 0 if x1 is None else x1.N, 0 if x1 is None else x1.H,
            0 if x1 is None else x1.W, xs[0].C, self.store_channels(Cout), KH, KW, conv.stride[0],
            conv.padding[0], conv.dilation[0], as_[0].bn.pending[1],
            0 if x1 is None else as_[1].bn.pending[1]))

    def _finalize(self, bn, part, rows, M, C, stat):
        if self.defer_running:
            self._finalize_deferred(bn, [(part, rows, M, stat)], C)
            return
        self._dep(("bn", id(bn)))  # running stats: updated in call order
        H.check(self.lib.hgk_bn_finalize(self.stream, part.data_ptr(), rows, M, C,
                                         bn.weight.data_ptr(), bn.bias.data_ptr(),
                                         bn.running_mean.data_ptr(), bn.running_var.data_ptr(),
                                         float(bn.momentum), float(bn.eps), 1, stat[0].data_ptr(),
                                         stat[1].data_ptr(), stat[2].data_ptr(), stat[3].data_ptr(),
                                         self._fin_scratch(rows, C)))
        self._pub(("bn", id(bn)))

    def _bn_relu_bwd(self, v):
        if v.grad is None or not v.src.requires_grad and not v.bn.mod.weight.requires_grad:
            return
        use, x = v.bn, v.src
        M, C = x.M, x.C
        if v.bwd_part is not None:
            part, rows = v.bwd_part  # reduced by the producing input-grad conv's epilogue
            v.bwd_part = None
        else:
            rows_cap = min(2048, (M + 7) // 8 + 1)
            part = self._f32(rows_cap * 2 * C)
            H.check(self.lib.hgk_bn_bwd_reduce(self.stream, self.dt, v.grad.data_ptr(),
                                               x.t.data_ptr(), M, C, use.scale.data_ptr(),
                                               use.shift.data_ptr(), 1 if use.relu else 0,
                                               use.mean.data_ptr(), use.invstd.data_ptr(),
                                               part.data_ptr(), H.ctypes.byref(self._rows)))
            rows = self._rows.value
        bn = use.mod
        if (x.requires_grad and self.fused_bwd_fin and rows <= self.lib.hgk_bn_bwd_fused_max_rows()
                and C % 8 == 0 and C <= 512 and 256 % (C // 2) == 0):
            has = x._grad is not None  # bn1: the skip gradient is already there (added by the fold)
            if (not has or self.fold_bwd_add) and self._can_defer_apply(x, fin_rows=(rows,), add=has):
                # finalize AND apply folded into the producing conv's input-gradient launch
                add = x._grad
                x._grad = self._empty(x.N, x.H, x.W, x.C)
                x.gshared = False
                x.pending = PendingApply(self, v.grad, x, use, None, x._grad, fin=(part, rows), add=add)
                self._fin_pending.append(x.pending)
                v.grad = None
                return
            # few partial rows (<= 16x16 levels): finalize + apply in one launch
            self._dep(("bnb", id(bn)))
            dst, acc, src = self.grad_slot(x)
            H.check(self.lib.hgk_bn_bwd_finalize_apply(
                self.stream, self.dt, part.data_ptr(), rows, M, C, use.scale.data_ptr(),
                use.shift.data_ptr(), 1 if use.relu else 0, use.mean.data_ptr(),
                use.invstd.data_ptr(), 1 if use.training else 0, self.pgrad(bn.weight).data_ptr(),
                self.pgrad(bn.bias).data_ptr(), v.grad.data_ptr(), x.t.data_ptr(),
                None if src is dst else src.data_ptr(), dst.data_ptr(), acc if src is dst else 0))
            self._pub(("bnb", id(bn)))
            self._pub(("g", id(x)))
            v.grad = None
            return
        coef = self._f32(4, C)
        self._dep(("bnb", id(bn)))  # dgamma / dbeta accumulate in call order
        H.check(self.lib.hgk_bn_bwd_finalize(self.stream, part.data_ptr(), rows, M, C,
                                             use.scale.data_ptr(), use.mean.data_ptr(),
                                             use.invstd.data_ptr(), 1 if use.training else 0,
                                             self.pgrad(bn.weight).data_ptr(),
                                             self.pgrad(bn.bias).data_ptr(), coef.data_ptr(),
                                             self._fin_scratch(rows, C)))
        self._pub(("bnb", id(bn)))
        if x.requires_grad and self._can_defer_apply(x):
            x._grad = self._empty(x.N, x.H, x.W, x.C)
            x.pending = PendingApply(self, v.grad, x, use, coef, x._grad)
        elif x.requires_grad:
            dst, acc, src = self.grad_slot(x)
            H.check(self.lib.hgk_bn_bwd_apply(self.stream, self.dt, v.grad.data_ptr(), x.t.data_ptr(),
                                              M, C, use.scale.data_ptr(), use.shift.data_ptr(),
                                              1 if use.relu else 0, coef.data_ptr(),
                                              None if src is dst else src.data_ptr(),
                                              dst.data_ptr(), acc if src is dst else 0))
            self._pub(("g", id(x)))
        v.grad = None

    # ------------------------------------------------------------------ convolution
    def conv(self, a, conv, res=None, inplace_res=False, post_relu=False, stats=True):
        """y = conv(a) + bias (+ res); `a` real or virtual (BN+ReLU fused into input staging)."""
        x = a.real
        a.uses += 1
        w = conv.weight
        Cout, Cin, KH, KW = w.shape
        assert Cin == a.C_log, (Cin, a.C_log)
        stride, pad, dil = conv.stride[0], conv.padding[0], conv.dilation[0]
        Ho = (x.H + 2 * pad - dil * (KH - 1) - 1) // stride + 1
        Wo = (x.W + 2 * pad - dil * (KW - 1) - 1) // stride + 1
        cout_st = self.store_channels(Cout)
        packed, ld = self._pack(conv, False, cout_st, x.C)
        if res is not None:
            assert res.C == cout_st
        if res is not None and inplace_res:
            y = res.t
        else:
            y = self._empty(x.N, Ho, Wo, cout_st)
        M = x.N * Ho * Wo
        part = None
        if stats:
            rows_cap = 2 * ((M + 63) // 64) + 2  # <= 2 partial rows per 128-row tile
            part = self._f32(rows_cap * 3 * cout_st)
        pre = a.bn
        bias = self._bias(conv, cout_st)
        ws_b = self.lib.hgk_conv_fwd_workspace(self.dt, x.N, x.H, x.W, x.C, cout_st, KH, KW,
                                               stride, pad, dil)
        ws = self.workspace(ws_b) if ws_b else None
        if pre is not None and pre.pending is not None and self._fold_ok((a,), conv):
            fd = pre.fold_desc()
            pre.pending = pre.ctx = None  # this launch computes and publishes the BN's statistics
            self.n_fin_folded += 1
            H.check(self.lib.hgk_conv_fwd_fold(
                self.stream, self.dt, x.t.data_ptr(), packed.data_ptr(), ld,
                None if bias is None else bias.data_ptr(),
                None if res is None else res.t.data_ptr(), y.data_ptr(), 1 if pre.relu else 0,
                1 if post_relu else 0, None if part is None else part.data_ptr(),
                H.ctypes.byref(self._rows), x.N, x.H, x.W, x.C, cout_st, KH, KW, stride, pad, dil,
                None if ws is None else ws.data_ptr(), 0 if ws is None else ws.numel(),
                H.ctypes.byref(fd)))
        else:
            H.check(self.lib.hgk_conv_fwd(
                self.stream, self.dt, x.t.data_ptr(), packed.data_ptr(), ld,
                None if bias is None else bias.data_ptr(),
                None if res is None else res.t.data_ptr(), y.data_ptr(),
                None if pre is None else pre.scale.data_ptr(),
                None if pre is None else pre.shift.data_ptr(),
                1 if (pre is not None and pre.relu) else 0, 1 if post_relu else 0,
                None if part is None else part.data_ptr(), H.ctypes.byref(self._rows),
                x.N, x.H, x.W, x.C, cout_st, KH, KW, stride, pad, dil,
                None if ws is None else ws.data_ptr(), 0 if ws is None else ws.numel()))
        out = Act(y, x.N, Ho, Wo, cout_st,
                  stats=(part, self._rows.value) if stats else None, C_log=Cout)
        if self.grad_enabled:
            out.producer = (((a,), conv, post_relu, (_oshape(out),)), 0)
            self._rec(lambda: self._conv_bwd(a, conv, res, out, post_relu))
        return out

    def _vg_ok(self, as_, conv, shapes, post_relu=False, fin_rows=None, add=False):
        """the input-gradient launch of this conv (single or twin) can fold its outputs' pending
        BN-backward applies (with fin_rows = the partial rows per output: their finalizes too):
        bf16 ring or image-tile kernel, fused BN-backward reduction of its own input.
        `shapes`: the outputs' (N, H, W, C)"""
        w = conv.weight
        Cout, Cin, KH, KW = w.shape
        if post_relu or conv.stride[0] != 1 or not all(a.requires_grad for a in as_):
            return False
        if not all(a.bn is not None and a.uses == 1 for a in as_):
            return False
        pad, dil = conv.padding[0], conv.dilation[0]
        (n0, h0, w0, c0), (n1, h1, w1, _) = shapes[0], (shapes[1] if len(shapes) > 1 else (0, 0, 0, 0))
        geo = (self.dt, n0, h0, w0, n1, h1, w1, c0, as_[0].real.C, KH, KW, 1, dil * (KH - 1) - pad, dil)
        if KH != 1 and H.KFAM.get(self.lib.hgk_conv_fwd_kernel_family(*geo)) != "img":
            # the row-streaming 3x3 input gradient can fold the apply too (hgk_conv_vgrad_ok,
            # tested bitwise), but measured -0.2 % img/s same-box (profiles/r03_row3_vg_ab.txt):
            # the kernel's slower rows cost what the apply launch did
            return False
        if fin_rows is not None:
            r0, r1 = fin_rows[0], (fin_rows[1] if len(fin_rows) > 1 else 0)
            return self.fold_bwd_fin and bool(
                self.lib.hgk_conv_vgrad_fin_ok(*geo, 1, r0, r1, 1 if add else 0))
        if add:
            return False
        return bool(self.lib.hgk_conv_vgrad_ok(*geo, 1))

    def _conv_bwd(self, a, conv, res, out, post_relu):
        pend = out.pending
        if pend is not None and self._vg_ok((a,), conv, (_oshape(out),), post_relu,
                                            None if pend.fin is None else (pend.fin[1],),
                                            pend.add is not None):
            out.pending = None  # this launch applies it (and writes pend.dst)
            dout = out._grad
        else:
            pend = None
            dout = out.grad
        if dout is None:
            return
        x = a.real
        if post_relu:
            # ReLU backward on the conv output: dout * [y > 0] (bn_bwd_apply with unit affine)
            one = self._unit_affine(out.C)
            masked = self._empty(out.N, out.H, out.W, out.C)
            H.check(self.lib.hgk_bn_bwd_apply(self.stream, self.dt, dout.data_ptr(), out.t.data_ptr(),
                                              out.M, out.C, one[0].data_ptr(), one[1].data_ptr(), 1,
                                              one.data_ptr(), None, masked.data_ptr(), 0))
            dout = masked
        w = conv.weight
        Cout, Cin, KH, KW = w.shape
        stride, pad, dil = conv.stride[0], conv.padding[0], conv.dilation[0]
        pre = a.bn
        # input grad (stride-1 conv == forward conv of dout with the flipped, transposed weight)
        if a.requires_grad:
            wd, ld = self._pack(conv, True, out.C, x.C)
            pad_t = dil * (KH - 1) - pad
            gin, Hg, Wg = dout, out.H, out.W
            if stride != 1:
                # strided conv (train.py:411-447): zero-insert dout to the stride-1 grid, then the
                # same stride-1 input-grad conv (sizes: Hz = H + 2 pad - dil (K-1))
                Hg = x.H + 2 * pad - dil * (KH - 1)
                Wg = x.W + 2 * pad - dil * (KW - 1)
                gin = self._empty(out.N, Hg, Wg, out.C)
                H.check(self.lib.hgk_zero_insert(self.stream, self.dt, dout.data_ptr(),
                                                 gin.data_ptr(), out.N, out.H, out.W, out.C,
                                                 stride, Hg, Wg))
            dst, acc, src = self.grad_slot(a)
            ws_b = self.lib.hgk_conv_fwd_workspace(self.dt, out.N, Hg, Wg, out.C, x.C, KH, KW,
                                                   1, pad_t, dil)
            ws = self.workspace(ws_b) if ws_b else None
            if pre is not None and a.uses == 1:
                # sole consumer of a BN(+ReLU) output: this launch produces the complete dA, so
                # the BN-backward reduction runs in its epilogue (no separate bn_bwd_reduce pass)
                rows_cap = 2 * ((x.M + 63) // 64) + 2
                part = self._f32(rows_cap * 2 * x.C)
                bnb = (None if ws is None else ws.data_ptr(), 0 if ws is None else ws.numel(),
                       x.t.data_ptr(), pre.scale.data_ptr(), pre.shift.data_ptr(),
                       1 if pre.relu else 0, pre.mean.data_ptr(), pre.invstd.data_ptr(),
                       part.data_ptr(), H.ctypes.byref(self._rows))
                if pend is not None:
                    self.n_folded += 1
                    STATS["folded"] += 1
                    STATS["fin_folded"] += pend.fin is not None
                    # the kernel reads the upstream gradient dA and applies out's BN backward
                    # while staging it; it also writes the applied dy (dout) for the weight grad
                    vg = pend.vgrad()
                    H.check(self.lib.hgk_conv_fwd_bnbwd_vg(
                        self.stream, self.dt, pend.dA.data_ptr(), wd.data_ptr(), ld,
                        src.data_ptr() if acc else None, dst.data_ptr(),
                        out.N, Hg, Wg, out.C, x.C, KH, KW, 1, pad_t, dil, *bnb, H.ctypes.byref(vg)))
                else:
                    H.check(self.lib.hgk_conv_fwd_bnbwd(
                        self.stream, self.dt, gin.data_ptr(), wd.data_ptr(), ld,
                        src.data_ptr() if acc else None, dst.data_ptr(),
                        out.N, Hg, Wg, out.C, x.C, KH, KW, 1, pad_t, dil, *bnb))
                a.bwd_part = (part, self._rows.value)
            else:
                H.check(self.lib.hgk_conv_fwd(
                    self.stream, self.dt, gin.data_ptr(), wd.data_ptr(), ld, None,
                    src.data_ptr() if acc else None, dst.data_ptr(), None, None, 0, 0, None, None,
                    out.N, Hg, Wg, out.C, x.C, KH, KW, 1, pad_t, dil,
                    None if ws is None else ws.data_ptr(), 0 if ws is None else ws.numel()))
            self._pub(("g", id(a)))
        self._conv_wgrad_res(a, conv, res, out, dout)

    def _conv_wgrad_res(self, a, conv, res, out, dout):
        """weight / bias grad of one use + the residual's grad (the tail of _conv_bwd)"""
        x = a.real
        w = conv.weight
        Cout, Cin, KH, KW = w.shape
        stride, pad, dil = conv.stride[0], conv.padding[0], conv.dilation[0]
        pre = a.bn
        # weight / bias grad: this use's split-K partials are ADDED into the weight's slab set;
        # one reduction per weight at the end of backward (finish_wgrads) — shared modules are
        # used up to 32 times per step (try_with_torch.py:217,224-237,268,286)
        if w.requires_grad:
            ent = self.wslabs.get(id(conv))
            if ent is None:
                cap = self.lib.hgk_conv_wgrad_max_splits()
                nbytes = self.lib.hgk_conv_wgrad_slab_bytes(x.C, out.C, KH, KW, cap)
                buf = self._alloc((nbytes,), torch.uint8)
                has_b = conv.bias is not None and conv.bias.requires_grad
                ent = [buf, 0, cap, conv, (x.C, out.C, KH, KW, Cin, Cout), has_b]
                self.wslabs[id(conv)] = ent
            assert ent[4][:2] == (x.C, out.C), "stored channel counts changed between uses"
            max_m = self.wdefer_max_m_1x1 if KH * KW == 1 else self.wdefer_max_m
            if (KH, KW, stride, pad, dil) == (3, 3, 1, 1, 1) and self.dt == H.BF16 and H.get_route("wg_halo_multi") > 0:
                # route wg_halo_multi: every use of a bf16 3x3 weight goes into ONE halo launch over
                # the uses' concatenated tiles (one slab read-modify-write instead of one per use)
                max_m = 1 << 30
            if out.M <= max_m and x.C % 64 == 0 and out.C % 8 == 0 and stride == 1:
                # batched with the weight's other uses into one launch at the end of backward
                # (finish_wgrads). A residual's grad aliases dout: marked shared, so later grads
                # accumulate into it out of place (grad_slot copy-on-write)
                src = (x.t.data_ptr(), dout.data_ptr(),
                       None if pre is None else pre.scale.data_ptr(),
                       None if pre is None else pre.shift.data_ptr(),
                       1 if (pre is not None and pre.relu) else 0, x.N, x.H, x.W)
                self.wdefer.setdefault(id(conv), []).append(
                    (src, (x.t, dout, None if pre is None else pre.stat)))
                if res is not None:
                    self.add_grad(res, dout, shared=True)
                out.grad = None
                return
            self._dep(("w", id(conv)))  # the weight's slabs: read-modify-write in call order
            H.check(self.lib.hgk_conv_wgrad_accum(
                self.stream, self.dt, x.t.data_ptr(), dout.data_ptr(),
                None if pre is None else pre.scale.data_ptr(),
                None if pre is None else pre.shift.data_ptr(),
                1 if (pre is not None and pre.relu) else 0,
                ent[0].data_ptr(), ent[2], ent[1], 1 if ent[5] else 0, H.ctypes.byref(self._rows),
                x.N, x.H, x.W, x.C, out.C, KH, KW, stride, pad, dil))
            ent[1] = max(ent[1], self._rows.value)
            self._pub(("w", id(conv)))
        if res is not None:
            self.add_grad(res, dout, shared=out.gshared and dout is out.grad)
        out.grad = None

    # ------------------------------------------------------------------ twin execution
    def twin_begin(self):
        """Open a twin chain: segment-1 (down-branch) running-statistics records are held back
        and appended after the chain's segment-0 (up-branch) records at twin_end — the
        reference runs the whole up-branch chain first (try_with_torch.py:224-228)."""
        assert self._run_hold is None, "twin chains do not nest"
        self._run_hold = []

    def twin_end(self):
        self._run_entries.extend(self._run_hold)
        self._run_hold = None

    def _finalize_deferred(self, bn, segs, C):
        """hgk_bn_finalize_deferred for 1-2 uses [(part, rows, M, stat)]; records queued."""
        recs = [self._alloc((2, C), torch.float64) for _ in segs]
        arr = (H.BnSeg * len(segs))(*[H.BnSeg(p.data_ptr(), rows, M, r.data_ptr(), st.data_ptr())
                                      for (p, rows, M, st), r in zip(segs, recs)])
        H.check(self.lib.hgk_bn_finalize_deferred(self.stream, arr, len(segs), C, H.ptr(bn.weight),
                                                  H.ptr(bn.bias), float(bn.eps)))
        self._run_entries.append((bn, recs[0]))
        if len(recs) == 2:
            (self._run_hold if self._run_hold is not None else self._run_entries).append((bn, recs[1]))

    def bn_relu_twin(self, xs, bn, relu=True):
        """bn_relu for the two segments of a twin chain: one finalize launch."""
        if not (self.training and self.defer_running):
            return tuple(self.bn_relu(x, bn, relu) for x in xs)
        C = xs[0].C
        segs = []
        for x in xs:
            assert x.bn is None and x.C == C
            if x.stats is None:
                rows_cap = min(2048, (x.M + 7) // 8 + 1)
                part = self._f32(rows_cap * 3 * C)
                H.check(self.lib.hgk_bn_stats(self.stream, self.dt, x.t.data_ptr(), x.M, C,
                                              part.data_ptr(), H.ctypes.byref(self._rows)))
                x.stats = (part, self._rows.value)
            part, rows = x.stats
            segs.append((part, rows, x.M, self._f32(4, C)))
        # both segments' finalizes folded into the consuming (twin) conv, or one launch for both
        fold = len(xs) == 2 and all(self._can_fold_fin(x, seg[1]) for x, seg in zip(xs, segs))
        recs = None
        if fold:
            # records in the reference's call order, as _finalize_deferred places them
            recs = [self._alloc((2, C), torch.float64) for _ in segs]
            self._run_entries.append((bn, recs[0]))
            (self._run_hold if self._run_hold is not None else self._run_entries).append((bn, recs[1]))
        else:
            self._finalize_deferred(bn, segs, C)
        prev = self.bn_uses.get(id(bn))
        self.bn_uses[id(bn)] = (bn, len(xs) if prev is None else prev[1] + len(xs))
        vs = []
        for i, (x, seg) in enumerate(zip(xs, segs)):
            v = Act(None, x.N, x.H, x.W, C, requires_grad=x.requires_grad)
            v.bn = BNUse(bn, x, seg[3], relu, True)
            if fold:
                self._defer_fin(v.bn, seg[0], seg[1], recs[i])
            v.src = x
            vs.append(v)
        if self.grad_enabled:
            self._rec(lambda: self._bn_relu_bwd_twin(vs))
        return tuple(vs)

    def _can_defer_apply(self, x, twin=False, fin_rows=None, add=False):
        """x's gradient is exactly one BN-backward apply (no other contribution so far) and the
        conv that produced x can fold it into its input-gradient launch: defer the apply
        (PendingApply). `twin`: x is one of the two outputs of a conv_twin call (both deferred).
        `fin_rows`: the finalize is deferred too (partial rows of each output of the producer);
        `add`: x already has a gradient contribution, added by the fold (with fin_rows only)."""
        prod = x.producer
        if not (self.fold_apply and self.dt == H.BF16 and (x._grad is None) != add and x.pending is None
                and x.src is None and x.bn is None and prod is not None
                and len(prod[0][3]) == (2 if twin else 1)):
            return False
        as_, conv, post_relu, shapes = prod[0]
        return self._vg_ok(as_, conv, shapes, post_relu, fin_rows, add)

    def _bn_relu_bwd_twin(self, vs):
        ok = all(v.grad is not None and v.bwd_part is not None and v.src.requires_grad for v in vs)
        if not ok:
            for v in vs:
                self._bn_relu_bwd(v)
            return
        use0 = vs[0].bn
        bn, C = use0.mod, vs[0].src.C
        p0, p1 = (vs[0].src.producer, vs[1].src.producer) if len(vs) == 2 else (None, None)
        if (p0 is not None and p1 is not None and p0[0] is p1[0] and (p0[1], p1[1]) == (0, 1)
                and all(self._can_defer_apply(v.src, twin=True) for v in vs)
                and max(v.bwd_part[1] for v in vs) > self.lib.hgk_bn_bwd_fused_max_rows()):
            # many partial rows: coefficients + dgamma / dbeta in one launch, the applies deferred
            # to the consuming input-gradient conv (PendingApply)
            parts = [v.bwd_part for v in vs]
            coef = self._f32(len(vs), 6, C)
            segs = []
            for v, (part, rows) in zip(vs, parts):
                v.bwd_part = None
                segs.append(H.BnbSeg(part.data_ptr(), rows, v.src.M, v.bn.stat.data_ptr(), None,
                                     None, None, None, 0))
            arr = (H.BnbSeg * len(segs))(*segs)
            H.check(self.lib.hgk_bn_bwd_twin(self.stream, self.dt, arr, len(segs), C,
                                             1 if use0.relu else 0, 1 if use0.training else 0,
                                             self.pgrad(bn.weight).data_ptr(),
                                             self.pgrad(bn.bias).data_ptr(), coef.data_ptr()))
            for q, v in enumerate(vs):
                x = v.src
                x._grad = self._empty(x.N, x.H, x.W, x.C)
                x.pending = PendingApply(self, v.grad, x, v.bn, coef[q], x._grad)
                v.grad = None
            return
        has = [v.src._grad is not None for v in vs]
        if (p0 is not None and p1 is not None and p0[0] is p1[0] and (p0[1], p1[1]) == (0, 1)
                and self.fused_bwd_fin and has[0] == has[1] and (not has[0] or self.fold_bwd_add)
                and max(v.bwd_part[1] for v in vs) <= self.lib.hgk_bn_bwd_fused_max_rows()
                and all(self._can_defer_apply(v.src, twin=True, fin_rows=tuple(u.bwd_part[1] for u in vs),
                                              add=has[0]) for v in vs)):
            # few partial rows: finalize AND apply deferred to the consuming twin input-gradient
            # launch (its segment-0 first workgroup accumulates both segments' dgamma / dbeta)
            for v in vs:
                x = v.src
                add = x._grad
                x._grad = self._empty(x.N, x.H, x.W, x.C)
                x.gshared = False
                x.pending = PendingApply(self, v.grad, x, v.bn, None, x._grad, fin=v.bwd_part, add=add)
                self._fin_pending.append(x.pending)
                v.bwd_part = None
                v.grad = None
            return
        segs = []
        # every segment's partials stay referenced until the launch: a buffer freed here could
        # be handed to the next grad_slot allocation, which the same kernel writes
        parts = [v.bwd_part for v in vs]
        hold = []
        for v, (part, rows) in zip(vs, parts):
            x = v.src
            v.bwd_part = None
            dst, acc, src = self.grad_slot(x)
            segs.append(H.BnbSeg(part.data_ptr(), rows, x.M, v.bn.stat.data_ptr(), v.grad.data_ptr(),
                                 x.t.data_ptr(), None if src is dst else src.data_ptr(),
                                 dst.data_ptr(), acc if src is dst else 0))
            hold.append(src)  # a copy-on-write source loses its last owner here
        coef = self._f32(len(vs), 6, C)  # unfused path (many partial rows) only
        arr = (H.BnbSeg * len(segs))(*segs)
        H.check(self.lib.hgk_bn_bwd_twin(self.stream, self.dt, arr, len(segs), C,
                                         1 if use0.relu else 0, 1 if use0.training else 0,
                                         self.pgrad(bn.weight).data_ptr(),
                                         self.pgrad(bn.bias).data_ptr(), coef.data_ptr()))
        for v in vs:
            self._pub(("g", id(v.src)))
            v.grad = None

    def _twin_geom_ok(self, as_, conv):
        w = conv.weight
        Cout, Cin, KH, KW = w.shape
        xs = [a.real for a in as_]
        pres = [a.bn for a in as_]
        return (self.twin and conv.stride[0] == 1 and xs[0].C == xs[1].C and xs[0].N == xs[1].N
                and (pres[0] is None) == (pres[1] is None)
                and (pres[0] is None or pres[0].relu == pres[1].relu))

    def conv_twin(self, as_, conv, res=(None, None)):
        """conv for the two segments of a twin chain (same module, independent inputs)."""
        if not self._twin_geom_ok(as_, conv):
            return tuple(self.conv(a, conv, res=r) for a, r in zip(as_, res))
        xs = [a.real for a in as_]
        for a in as_:
            a.uses += 1
        w = conv.weight
        Cout, Cin, KH, KW = w.shape
        assert Cin == as_[0].C_log, (Cin, as_[0].C_log)
        stride, pad, dil = conv.stride[0], conv.padding[0], conv.dilation[0]
        cout_st = self.store_channels(Cout)
        packed, ld = self._pack(conv, False, cout_st, xs[0].C)
        bias = self._bias(conv, cout_st)
        rows_c = [H.ctypes.c_int(0), H.ctypes.c_int(0)]
        segs, outs = [], []
        for i, (a, x, r) in enumerate(zip(as_, xs, res)):
            Ho = (x.H + 2 * pad - dil * (KH - 1) - 1) // stride + 1
            Wo = (x.W + 2 * pad - dil * (KW - 1) - 1) // stride + 1
            if r is not None:
                assert r.C == cout_st
            y = self._empty(x.N, Ho, Wo, cout_st)
            M = x.N * Ho * Wo
            part = self._f32((2 * ((M + 63) // 64) + 2) * 3 * cout_st)
            pre = a.bn
            # the stat tensor's pointers (valid before a folded finalize has written them)
            segs.append(H.ConvSeg(x.t.data_ptr(), None if r is None else r.t.data_ptr(), y.data_ptr(),
                                  None if pre is None else pre.stat[2].data_ptr(),
                                  None if pre is None else pre.stat[3].data_ptr(), part.data_ptr(),
                                  H.ctypes.pointer(rows_c[i]), x.N, x.H, x.W, None, None, None,
                                  None, None, None, 0, None))
            outs.append((y, x.N, Ho, Wo, part))
        pre0 = as_[0].bn
        ws_b = self.lib.hgk_conv_fwd_twin_workspace(self.dt, xs[0].N, xs[0].H, xs[0].W, xs[1].N,
                                                    xs[1].H, xs[1].W, xs[0].C, cout_st, KH, KW,
                                                    stride, pad, dil)
        ws = self.workspace(ws_b) if ws_b else None
        if pre0 is not None and self._fold_ok(as_, conv):
            # the twin launch folds both segments' pending finalizes
            folds = [a.bn.fold_desc() for a in as_]
            for seg, fd in zip(segs, folds):
                seg.fold = H.ctypes.pointer(fd)
                seg.pre_scale = None
                seg.pre_shift = None
            for a in as_:
                a.bn.pending = a.bn.ctx = None
            self.n_fin_folded += 2
        else:
            for a in as_:
                if a.bn is not None:
                    a.bn.resolve()  # the segments read stat: its finalize must run first
        arr = (H.ConvSeg * 2)(*segs)
        H.check(self.lib.hgk_conv_fwd_twin(
            self.stream, self.dt, packed.data_ptr(), ld, None if bias is None else bias.data_ptr(),
            1 if (pre0 is not None and pre0.relu) else 0, 0, xs[0].C, cout_st, KH, KW, stride, pad,
            dil, arr, None if ws is None else ws.data_ptr(), 0 if ws is None else ws.numel()))
        acts = tuple(Act(y, N, Ho, Wo, cout_st, stats=(part, rc.value), C_log=Cout)
                     for (y, N, Ho, Wo, part), rc in zip(outs, rows_c))
        if self.grad_enabled:
            core = (tuple(as_), conv, False, tuple(_oshape(o) for o in acts))
            for i, o in enumerate(acts):
                o.producer = (core, i)
            self._rec(lambda: self._conv_bwd_twin(as_, conv, res, acts))
        return acts

    def _conv_bwd_twin(self, as_, conv, res, outs):
        fused = [a.bn is not None and a.uses == 1 for a in as_]
        pends = [o.pending for o in outs]
        # a pending apply counts as a gradient here: it is either folded into the twin launch
        # below or materialised by _conv_bwd (reading .grad) on the per-segment route
        ok = (all(o._grad is not None for o in outs) and all(a.requires_grad for a in as_)
              and fused[0] == fused[1])
        fins = [None if p is None else p.fin for p in pends]
        vg = ok and all(p is not None for p in pends) and (fins[0] is None) == (fins[1] is None) and \
            (pends[0].add is None) == (pends[1].add is None) and \
            self._vg_ok(as_, conv, tuple(_oshape(o) for o in outs),
                        fin_rows=None if fins[0] is None else (fins[0][1], fins[1][1]),
                        add=pends[0].add is not None)
        if vg:
            self.n_folded += len(outs)
            STATS["folded"] += len(outs)
            STATS["fin_folded"] += len(outs) if fins[0] is not None else 0
            for o in outs:
                o.pending = None  # the twin launch applies both (and writes their dst)
        if not ok:
            for a, r, o in zip(as_, res, outs):
                self._conv_bwd(a, conv, r, o, False)
            return
        xs = [a.real for a in as_]
        w = conv.weight
        Cout, Cin, KH, KW = w.shape
        pad, dil = conv.padding[0], conv.dilation[0]
        pad_t = dil * (KH - 1) - pad
        o0, o1 = outs
        wd, ld = self._pack(conv, True, o0.C, xs[0].C)
        rows_c = [H.ctypes.c_int(0), H.ctypes.c_int(0)]
        segs, parts = [], []
        hold = []  # every operand referenced until the launch (see _bn_relu_bwd_twin)
        for i, (a, x, o) in enumerate(zip(as_, xs, outs)):
            dst, acc, src = self.grad_slot(a)
            hold.append(src)
            if fused[i]:
                pre = a.bn
                part = self._f32((2 * ((x.M + 63) // 64) + 2) * 2 * x.C)
                parts.append(part)
                vgp = None
                if vg:
                    vgs = pends[i].vgrad()
                    hold.append(vgs)
                    vgp = H.ctypes.pointer(vgs)
                segs.append(H.ConvSeg((pends[i].dA if vg else o.grad).data_ptr(),
                                      src.data_ptr() if acc else None,
                                      dst.data_ptr(), None, None, None, None, o.N, o.H, o.W,
                                      x.t.data_ptr(), pre.scale.data_ptr(), pre.shift.data_ptr(),
                                      pre.mean.data_ptr(), pre.invstd.data_ptr(), part.data_ptr(),
                                      1 if pre.relu else 0, H.ctypes.pointer(rows_c[i]), vgp))
            else:
                parts.append(None)
                segs.append(H.ConvSeg(o.grad.data_ptr(), src.data_ptr() if acc else None,
                                      dst.data_ptr(), None, None, None, None, o.N, o.H, o.W, None,
                                      None, None, None, None, None, 0, None))
        ws_b = self.lib.hgk_conv_fwd_twin_workspace(self.dt, o0.N, o0.H, o0.W, o1.N, o1.H, o1.W,
                                                    o0.C, xs[0].C, KH, KW, 1, pad_t, dil)
        ws = self.workspace(ws_b) if ws_b else None
        arr = (H.ConvSeg * 2)(*segs)
        H.check(self.lib.hgk_conv_fwd_twin(self.stream, self.dt, wd.data_ptr(), ld, None, 0, 0, o0.C,
                                           xs[0].C, KH, KW, 1, pad_t, dil, arr,
                                           None if ws is None else ws.data_ptr(),
                                           0 if ws is None else ws.numel()))
        for i, a in enumerate(as_):
            if fused[i]:
                a.bwd_part = (parts[i], rows_c[i].value)
            self._pub(("g", id(a)))
        for a, r, o in zip(as_, res, outs):
            self._conv_wgrad_res(a, conv, r, o, o.grad)

    # ------------------------------------------------------------------ pooling / upsampling
    def maxpool2(self, x):
        assert x.bn is None
        Ho, Wo = x.H // 2, x.W // 2
        y = self._empty(x.N, Ho, Wo, x.C)
        stats = None
        if self.training and self.stats_ops:
            # the output feeds a train-mode BN (the next residual block's bn1): its statistics
            # come out of this kernel instead of a separate hgk_bn_stats pass
            M = x.N * Ho * Wo
            part = self._f32(min(2048, (M + 7) // 8 + 1) * 3 * x.C)
            H.check(self.lib.hgk_maxpool2_fwd_stats(self.stream, self.dt, x.t.data_ptr(),
                                                    y.data_ptr(), x.N, x.H, x.W, x.C,
                                                    part.data_ptr(), H.ctypes.byref(self._rows)))
            stats = (part, self._rows.value)
        else:
            H.check(self.lib.hgk_maxpool2_fwd(self.stream, self.dt, x.t.data_ptr(), y.data_ptr(),
                                              x.N, x.H, x.W, x.C))
        out = Act(y, x.N, Ho, Wo, x.C, stats=stats, requires_grad=x.requires_grad)
        if self.grad_enabled:
            self._rec(lambda: self._maxpool2_bwd(x, out))
        return out

    def _maxpool2_bwd(self, x, out):
        if out.grad is None or not x.requires_grad:
            return
        dst, acc = self.grad_slot_inplace(x)
        H.check(self.lib.hgk_maxpool2_bwd(self.stream, self.dt, x.t.data_ptr(), out.grad.data_ptr(),
                                          dst.data_ptr(), x.N, x.H, x.W, x.C, acc))
        self._pub(("g", id(x)))
        out.grad = None

    def upsample2_add(self, low, skip, mode):
        """x2 up-sampling of `low` (+ skip; skip None: the plain F.interpolate of train.py:531)"""
        assert low.bn is None and (skip is None or skip.bn is None)
        y = self._empty(low.N, 2 * low.H, 2 * low.W, low.C)
        stats = None
        if self.training and self.stats_ops and skip is not None:
            M = low.N * 4 * low.H * low.W
            part = self._f32(min(2048, (M + 7) // 8 + 1) * 3 * low.C)
            H.check(self.lib.hgk_upsample2_add_fwd_stats(
                self.stream, self.dt, mode, low.t.data_ptr(), skip.t.data_ptr(), y.data_ptr(),
                low.N, low.H, low.W, low.C, part.data_ptr(), H.ctypes.byref(self._rows)))
            stats = (part, self._rows.value)
        else:
            H.check(self.lib.hgk_upsample2_add_fwd(self.stream, self.dt, mode, low.t.data_ptr(),
                                                   None if skip is None else skip.t.data_ptr(),
                                                   y.data_ptr(), low.N, low.H, low.W, low.C))
        out = Act(y, low.N, 2 * low.H, 2 * low.W, low.C, stats=stats)
        if self.grad_enabled:
            self._rec(lambda: self._upsample2_bwd(low, skip, out, mode))
        return out

    def _upsample2_bwd(self, low, skip, out, mode):
        if out.grad is None:
            return
        if low.requires_grad:
            dst, acc = self.grad_slot_inplace(low)
            H.check(self.lib.hgk_upsample2_bwd(self.stream, self.dt, mode, out.grad.data_ptr(),
                                               dst.data_ptr(), low.N, low.H, low.W, low.C, acc))
            self._pub(("g", id(low)))
        if skip is not None:
            self.add_grad(skip, out.grad, shared=out.gshared)
        out.grad = None

    def spatial_mean(self, x):
        """nn.AdaptiveAvgPool2d((1, 1)) of a real activation -> [N, 1, 1, C] (the live ASPP's
        image-pool branch, try_more_layer.py:266); backward broadcasts grad / (H W)."""
        assert x.bn is None
        HW = x.H * x.W
        y = self._empty(x.N, 1, 1, x.C)
        H.check(self.lib.hgk_spatial_sum(self.stream, self.dt, x.t.data_ptr(), y.data_ptr(), x.N,
                                         HW, x.C, 1.0 / HW, 0))
        out = Act(y, x.N, 1, 1, x.C, C_log=x.C_log, requires_grad=x.requires_grad)
        if self.grad_enabled:
            def bwd():
                if out.grad is None or not x.requires_grad:
                    return
                dst, acc = self.grad_slot_inplace(x)
                H.check(self.lib.hgk_spatial_broadcast(self.stream, self.dt, out.grad.data_ptr(),
                                                       dst.data_ptr(), x.N, HW, x.C, 1.0 / HW, acc))
                self._pub(("g", id(x)))
                out.grad = None
            self._rec(bwd)
        return out

    def broadcast(self, x, Hh, W):
        """F.interpolate of a [N, 1, 1, C] activation to Hh x W, bilinear, align_corners=True
        (source coordinate 0 for every output pixel: a broadcast; try_more_layer.py:287);
        backward sums grad over the positions."""
        assert x.bn is None and x.H == 1 and x.W == 1
        y = self._empty(x.N, Hh, W, x.C)
        H.check(self.lib.hgk_spatial_broadcast(self.stream, self.dt, x.t.data_ptr(), y.data_ptr(),
                                               x.N, Hh * W, x.C, 1.0, 0))
        out = Act(y, x.N, Hh, W, x.C, C_log=x.C_log, requires_grad=x.requires_grad)
        if self.grad_enabled:
            def bwd():
                if out.grad is None or not x.requires_grad:
                    return
                dst, acc = self.grad_slot_inplace(x)
                H.check(self.lib.hgk_spatial_sum(self.stream, self.dt, out.grad.data_ptr(),
                                                 dst.data_ptr(), x.N, Hh * W, x.C, 1.0, acc))
                self._pub(("g", id(x)))
                out.grad = None
            self._rec(bwd)
        return out

    def add(self, a, b):
        """a + b of two real activations (hourglass_compare's BN-ed residual branch + BN-ed
        projection, its stage re-injection; hourglass_compare.py:437-440,621)."""
        assert a.bn is None and b.bn is None and (a.N, a.H, a.W, a.C) == (b.N, b.H, b.W, b.C)
        y = self._empty(a.N, a.H, a.W, a.C)
        H.check(self.lib.hgk_add(self.stream, self.dt, a.t.data_ptr(), b.t.data_ptr(), y.data_ptr(),
                                 y.numel(), 0))
        out = Act(y, a.N, a.H, a.W, a.C, C_log=a.C_log,
                  requires_grad=a.requires_grad or b.requires_grad)
        if self.grad_enabled:
            def bwd():
                if out.grad is None:
                    return
                # both operands receive the same gradient buffer (copy-on-write if either
                # accumulates into it later)
                self.add_grad(a, out.grad, shared=True)
                self.add_grad(b, out.grad, shared=True)
                out.grad = None
            self._rec(bwd)
        return out

    def concat(self, parts):
        """torch.cat(parts, dim=1) of real activations (the progressive heads' re-injection,
        try_with_aspp.py:327-334). Logical channels stay contiguous: every part but the last
        must be unpadded; the last part's channel padding becomes the result's."""
        p0 = parts[0]
        for p in parts:
            assert p.bn is None and (p.N, p.H, p.W) == (p0.N, p0.H, p0.W)
        for p in parts[:-1]:
            assert p.C == p.C_log, "only the last concatenated part may be channel-padded"
        C_st = sum(p.C for p in parts)
        C_log = sum(p.C_log for p in parts)
        y = self._empty(p0.N, p0.H, p0.W, C_st)
        offs, off = [], 0
        for p in parts:
            H.check(self.lib.hgk_channel_copy(self.stream, self.dt, p.t.data_ptr(), p.C, 0,
                                              y.data_ptr(), C_st, off, p.C, p.M, 0))
            offs.append(off)
            off += p.C
        out = Act(y, p0.N, p0.H, p0.W, C_st, C_log=C_log,
                  requires_grad=any(p.requires_grad for p in parts))
        if self.grad_enabled:
            def bwd():
                if out.grad is None:
                    return
                for p, o in zip(parts, offs):
                    if not p.requires_grad:
                        continue
                    dst, acc = self.grad_slot_inplace(p)
                    H.check(self.lib.hgk_channel_copy(self.stream, self.dt, out.grad.data_ptr(),
                                                      C_st, o, dst.data_ptr(), p.C, 0, p.C, p.M,
                                                      acc))
                    self._pub(("g", id(p)))
                out.grad = None
            self._rec(bwd)
        return out

    def bn_add(self, va, vb):
        """relu?(bn_a(ya)) + relu?(bn_b(yb)) of two virtual activations, materialised in ONE pass
        (hgk_bn_apply2_add: bitwise materialize x2 + add, and the sum's BN statistics for its
        consumer without a bn_stats pass); backward: both BNs' reductions over the common
        gradient in one pass (hgk_bn_bwd_reduce2), then each BN's finalize / apply as usual.
        hourglass_compare.py:437-440 (bn4(conv3(..)) + downsaple(x)), train.py:444-447."""
        assert va.bn is not None and vb.bn is not None
        xa, xb = va.src, vb.src
        assert (xa.N, xa.H, xa.W, xa.C) == (xb.N, xb.H, xb.W, xb.C)
        va.uses += 1
        vb.uses += 1
        ua, ub = va.bn, vb.bn
        M, C = xa.M, xa.C
        y = self._empty(xa.N, xa.H, xa.W, C)
        part = None
        if self.training:
            part = self._f32(min(2048, (M + 7) // 8 + 1) * 3 * C)
        sa = H.BnSide(xa.t.data_ptr(), ua.scale.data_ptr(), ua.shift.data_ptr(), None, None,
                      1 if ua.relu else 0, None)
        sb = H.BnSide(xb.t.data_ptr(), ub.scale.data_ptr(), ub.shift.data_ptr(), None, None,
                      1 if ub.relu else 0, None)
        H.check(self.lib.hgk_bn_apply2_add(self.stream, self.dt, H.ctypes.byref(sa),
                                           H.ctypes.byref(sb), y.data_ptr(), M, C,
                                           None if part is None else part.data_ptr(),
                                           H.ctypes.byref(self._rows)))
        out = Act(y, xa.N, xa.H, xa.W, C, stats=None if part is None else (part, self._rows.value),
                  C_log=xa.C_log, requires_grad=va.requires_grad or vb.requires_grad)
        if self.grad_enabled:
            def bwd():
                g = out.grad
                if g is None:
                    return
                if (va.requires_grad and vb.requires_grad and va is not vb
                        and va.uses == 1 and vb.uses == 1
                        and va._grad is None and vb._grad is None
                        and va.pending is None and vb.pending is None
                        and va.bwd_part is None and vb.bwd_part is None):
                    # the reductions _bn_relu_bwd would launch for each side, sharing g's reads;
                    # only when g is each side's WHOLE gradient (sole consumer, nothing
                    # accumulated yet): precomputed sums over g alone would otherwise miss the
                    # other consumers' contributions
                    # (a second consumer: tests/test_gpu_bn_pair.py::test_bn_add_shared_operand)
                    rows_cap = min(2048, (M + 7) // 8 + 1)
                    pa, pb = self._f32(rows_cap * 2 * C), self._f32(rows_cap * 2 * C)
                    da = H.BnSide(xa.t.data_ptr(), ua.scale.data_ptr(), ua.shift.data_ptr(),
                                  ua.mean.data_ptr(), ua.invstd.data_ptr(), 1 if ua.relu else 0,
                                  pa.data_ptr())
                    db = H.BnSide(xb.t.data_ptr(), ub.scale.data_ptr(), ub.shift.data_ptr(),
                                  ub.mean.data_ptr(), ub.invstd.data_ptr(), 1 if ub.relu else 0,
                                  pb.data_ptr())
                    H.check(self.lib.hgk_bn_bwd_reduce2(self.stream, self.dt, g.data_ptr(), M, C,
                                                        H.ctypes.byref(da), H.ctypes.byref(db),
                                                        H.ctypes.byref(self._rows)))
                    va.bwd_part = (pa, self._rows.value)
                    vb.bwd_part = (pb, self._rows.value)
                    if self.bn_pair_bwd and self._bn_pair_bwd(va, vb, g):
                        out.grad = None
                        return
                self.add_grad(va, g, shared=True)
                self.add_grad(vb, g, shared=True)
                out.grad = None
            self._rec(bwd)
        return out

    def _bn_pair_bwd(self, va, vb, g):
        """Both sides of bn_add backward in ONE hgk_bn_bwd_pair launch (g read once): each side's
        finalize in-kernel (few partial rows) or by its own hgk_bn_bwd_finalize, the applies
        writing xa / xb's fresh gradients — what the two _bn_relu_bwd calls would do when neither
        apply can fold into its producer's input gradient (else False: that path runs instead)."""
        xa, xb = va.src, vb.src
        (pa, rows), (pb, _) = va.bwd_part, vb.bwd_part
        M, C = xa.M, xa.C
        if not (va.uses == 1 and vb.uses == 1 and va.grad is None and vb.grad is None
                and xa.requires_grad and xb.requires_grad and xa._grad is None and xb._grad is None
                and xa.pending is None and xb.pending is None and xa is not xb):
            return False
        fused = (self.fused_bwd_fin and rows <= self.lib.hgk_bn_bwd_fused_max_rows()
                 and C % 8 == 0 and C <= 512 and 256 % (C // 2) == 0)
        if fused:
            if any(self._can_defer_apply(x, fin_rows=(rows,)) for x in (xa, xb)):
                return False
        elif any(self._can_defer_apply(x) for x in (xa, xb)):
            return False
        sides, keep = [], []  # keep: both coefficient arrays alive until the pair launch is queued
        multi = (not fused and self.fin_batch
                 and rows >= self.lib.hgk_bn_bwd_finalize_multi_min_rows())
        fins = []
        for v, part in ((va, pa), (vb, pb)):
            use, x = v.bn, v.src
            bn = use.mod
            self._dep(("bnb", id(bn)))
            dg, db = self.pgrad(bn.weight), self.pgrad(bn.bias)
            coef = None
            if not fused:
                coef = self._f32(4, C)
                keep.append(coef)
                if multi:  # both sides' finalizes in one launch, below
                    fins.append(H.BnbFinJob(part.data_ptr(), rows, M, C, use.scale.data_ptr(),
                                            use.mean.data_ptr(), use.invstd.data_ptr(),
                                            1 if use.training else 0, dg.data_ptr(), db.data_ptr(),
                                            coef.data_ptr()))
                else:
                    H.check(self.lib.hgk_bn_bwd_finalize(
                        self.stream, part.data_ptr(), rows, M, C, use.scale.data_ptr(),
                        use.mean.data_ptr(), use.invstd.data_ptr(), 1 if use.training else 0,
                        dg.data_ptr(), db.data_ptr(), coef.data_ptr(), self._fin_scratch(rows, C)))
            dst, acc, _ = self.grad_slot(x)
            assert acc == 0
            sides.append(H.BnbSide(
                x.t.data_ptr(), use.scale.data_ptr(), use.shift.data_ptr(), use.mean.data_ptr(),
                use.invstd.data_ptr(), 1 if use.relu else 0, part.data_ptr() if fused else None,
                rows, None if fused else coef.data_ptr(), dg.data_ptr() if fused else None,
                db.data_ptr() if fused else None, dst.data_ptr()))
            v.bwd_part = None
        if fins:
            H.check(self.lib.hgk_bn_bwd_finalize_multi(self.stream, (H.BnbFinJob * 2)(*fins), 2))
        if fused or self.pair_apply:
            H.check(self.lib.hgk_bn_bwd_pair(self.stream, self.dt, g.data_ptr(), M, C,
                                             1 if va.bn.training else 0, H.ctypes.byref(sides[0]),
                                             H.ctypes.byref(sides[1])))
        else:
            # route pair_apply off: two apply launches (3 streams each) — bitwise the same values
            for sd in sides:
                H.check(self.lib.hgk_bn_bwd_apply(self.stream, self.dt, g.data_ptr(), sd.y, M, C,
                                                  sd.scale, sd.shift, sd.relu, sd.coef, None, sd.dy,
                                                  0))
        for v in (va, vb):
            self._pub(("bnb", id(v.bn.mod)))
            self._pub(("g", id(v.src)))
        return True

    def materialize(self, a):
        """A real activation for `a` (runs BN(+ReLU) apply for a virtual one)."""
        if a.bn is None:
            return a
        a.uses += 1
        x, use = a.src, a.bn
        y = self._empty(x.N, x.H, x.W, x.C)
        H.check(self.lib.hgk_bn_apply(self.stream, self.dt, x.t.data_ptr(), x.M, x.C,
                                      use.scale.data_ptr(), use.shift.data_ptr(),
                                      1 if use.relu else 0, y.data_ptr()))
        out = Act(y, x.N, x.H, x.W, x.C, requires_grad=a.requires_grad)
        if self.grad_enabled:
            def bwd():
                if out.grad is not None:
                    self.add_grad(a, out.grad, shared=out.gshared)
                    out.grad = None
            self._rec(bwd)
        return out

    # ------------------------------------------------------------------ finish
    def grad_barrier(self, tag):
        """Forward-time marker. When the reverse tape reaches it, every weight used AFTER it in
        forward has had its last gradient contribution: the deferred weight-grads are flushed
        (finish_wgrads) so those grads are complete in HBM, then on_grads_ready(tag) runs."""
        if self.grad_enabled:
            self._rec(lambda: self._grads_ready(tag))

    def _flush_fin_pending(self):
        """Launch every deferred BN-backward finalize+apply no conv has taken yet: it accumulates
        dgamma / dbeta, which must happen before a grad barrier seals their group (and before
        backward ends, whether or not anything reads the input gradient)."""
        for p in self._fin_pending:
            if p.x.pending is p:
                p.x.pending = None
                p.materialize()
        self._fin_pending = []

    def _grads_ready(self, tag):
        self._flush_fin_pending()
        self.finish_wgrads()
        if self.seal_groups is not None and len(self.barriers_passed) < len(self.seal_groups):
            self.sealed |= self.seal_groups[len(self.barriers_passed)]
        self.barriers_passed.append(tag)
        if self.on_grads_ready is not None:
            self.on_grads_ready(tag)

    def finish_forward(self):
        for use in self._pending_fin:
            use.resolve()  # finalizes no conv folded (their records must exist)
        self._pending_fin = []
        if self._run_entries:
            # the deferred running-statistics updates, in the reference's call order
            ents = [H.BnRunning(bn.running_mean.data_ptr(), bn.running_var.data_ptr(),
                                rec.data_ptr(), bn.num_features, float(bn.momentum))
                    for bn, rec in self._run_entries if bn.running_mean is not None]
            if ents:
                arr = (H.BnRunning * len(ents))(*ents)
                H.check(self.lib.hgk_bn_running_update(self.stream, arr, len(ents)))
            self._keep.append([rec for _, rec in self._run_entries])
            self._run_entries = []
        # num_batches_tracked += uses (PyTorch increments it on every train-mode call); the
        # Trainer keeps every counter in one flat buffer and adds the per-step counts in ONE op
        if self.nbt_batch is not None:
            flat, counts = self.nbt_batch
            flat.add_(counts)
            return
        for bn, count in self.bn_uses.values():
            if bn.num_batches_tracked is not None:
                bn.num_batches_tracked.add_(count)

    def finish_wgrads(self):
        # weights with ONE deferred use (the unshared blocks of hourglass_compare / train.py): their
        # launches batched across weights (hgk_conv_wgrad_accum_batch, bitwise the single calls)
        singles = [k for k, uses in self.wdefer.items() if len(uses) == 1] if self.wg_batch else []
        if len(singles) > 1:
            jobs = []
            for key in singles:
                ent = self.wslabs[key]
                buf, cap, conv, (cin_st, cout_st, KH, KW, _, _), has_b = ent[0], ent[2], ent[3], ent[4], ent[5]
                self._dep(("w", key))
                jobs.append(H.WgradJob(H.WgradSrc(*self.wdefer[key][0][0]), buf.data_ptr(), cap, ent[1],
                                       1 if has_b else 0, cin_st, cout_st, KH, KW, conv.stride[0],
                                       conv.padding[0], conv.dilation[0]))
            splits = (H.ctypes.c_int * len(jobs))()
            H.check(self.lib.hgk_conv_wgrad_accum_batch(self.stream, self.dt, (H.WgradJob * len(jobs))(*jobs),
                                                        len(jobs), splits))
            for key, sp in zip(singles, splits):
                self.wslabs[key][1] = max(self.wslabs[key][1], sp)
                self._pub(("w", key))
                self._keep.append(self.wdefer.pop(key))
        for key, uses in self.wdefer.items():
            ent = self.wslabs[key]
            buf, cap, conv, (cin_st, cout_st, KH, KW, _, _), has_b = ent[0], ent[2], ent[3], ent[4], ent[5]
            # (branch schedule: backward() has joined every side stream into stream 0 by now)
            self._dep(("w", key))
            arr = (H.WgradSrc * len(uses))(*[H.WgradSrc(*u[0]) for u in uses])
            H.check(self.lib.hgk_conv_wgrad_accum_multi(
                self.stream, self.dt, arr, len(uses), buf.data_ptr(), cap, ent[1],
                1 if has_b else 0, H.ctypes.byref(self._rows), cin_st, cout_st, KH, KW,
                conv.stride[0], conv.padding[0], conv.dilation[0]))
            ent[1] = max(ent[1], self._rows.value)
            self._pub(("w", key))
            self._keep.append(uses)
        self.wdefer = {}
        # every weight's slab reduction in one launch (hgk_conv_wgrad_finish_multi)
        fins = []
        for buf, nslabs, cap, conv, (cin_st, cout_st, KH, KW, Cin, Cout), has_b in self.wslabs.values():
            if nslabs == 0:
                continue
            db = self.pgrad(conv.bias).data_ptr() if has_b else None
            fins.append(H.WgradFin(buf.data_ptr(), cap, nslabs, self.pgrad(conv.weight).data_ptr(), db,
                                   cin_st, cout_st, KH, KW, Cin, Cout))
        if fins:
            arr = (H.WgradFin * len(fins))(*fins)
            H.check(self.lib.hgk_conv_wgrad_finish_multi(self.stream, arr, len(fins)))
        self.wslabs = {}

    def backward(self):
        """Replay the tape in reverse. Branch markers mirror the forward schedule: a forward
        join becomes the point where the branch's backward may start (it waits for its grads),
        a forward fork the point where the parent waits for the branch's backward."""
        for ent in reversed(self.tape):
            if isinstance(ent[0], str):
                kind, parent, child = ent
                if kind == "join":
                    self._set_stream(parent)
                    ev = self._event()
                    self._set_stream(child)
                    self._wait(ev)
                elif kind == "fork":
                    self._set_stream(child)
                    ev = self._event()
                    self._set_stream(parent)
                    self._wait(ev)
                continue
            sid, fn = ent
            self._set_stream(sid)
            fn()
        self._set_stream(0)
        self.tape = []
        self._flush_fin_pending()
        self.finish_wgrads()
