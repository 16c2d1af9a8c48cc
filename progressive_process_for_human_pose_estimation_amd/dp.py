"""Data-parallel plumbing: one process per GPU, torch.distributed over RCCL ("nccl" on ROCm).

SURVEY.md §8(e): pure data parallel. Rank r trains on samples [r*n, (r+1)*n) of the global batch,
weights are replicated, BatchNorm uses each rank's LOCAL batch statistics (the reference has no
SyncBN, so this equals running the reference on each shard), and the only exchange is the SUM
all-reduce of the weight gradients (the loss gradient is pre-scaled by 1/world, so SUM == mean).

Overlap with backward (GradSync): the hourglass, residual4, lin and head modules are shared by all
stacks (try_with_torch.py:268,286-297), so their gradients become final only when stack 0's
backward has run — but that is BEFORE the stem's backward (residual3, residual2, max_pool1,
residual1, conv1: :276-281), which still has to run. The flat gradient is therefore laid out in
grad-ready order, [trunk | stem | never-grad tail]: the trunk segment's all-reduce is launched on a
side stream as soon as backward passes the stem (engine.Ctx.grad_barrier) and runs concurrently
with the stem's backward; the stem segment follows; the optimizer waits for both. Parameters no
forward reads (conv4 of square blocks) sit in the tail and are never reduced or updated, as
torch.optim.Adam skips parameters whose grad is None.
"""
import os
import time

import torch
import torch.distributed as dist

BUCKET_BYTES = 8 << 20  # xGMI ring: a few MB per call amortises the per-call latency


def world_info():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init_from_env(backend=None):
    """Initialise the default process group from torchrun's env (no-op for world size 1)."""
    rank, world, local = world_info()
    if world == 1 or (dist.is_available() and dist.is_initialized()):
        return rank, world, local
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    kw = {}
    if backend == "nccl":
        torch.cuda.set_device(local)
        kw["device_id"] = torch.device("cuda", local)
    dist.init_process_group(backend, **kw)
    return rank, world, local


def shard_bounds(global_batch, rank, world):
    """Sample range of this rank: [rank*n, (rank+1)*n) with n = global_batch // world."""
    if global_batch % world:
        raise ValueError(f"global batch {global_batch} not divisible by world size {world}")
    n = global_batch // world
    return rank * n, (rank + 1) * n


def broadcast_flat(flat, src=0, group=None):
    """Make every rank start from rank src's weights (seeded init is identical anyway)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.broadcast(flat, src=src, group=group)


def allreduce_flat(flat, group=None, bucket_bytes=BUCKET_BYTES):
    """SUM all-reduce of a contiguous fp32 buffer in fixed-size buckets (in place)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return flat
    per = max(1, bucket_bytes // flat.element_size())
    for off in range(0, flat.numel(), per):
        dist.all_reduce(flat[off:off + per], op=dist.ReduceOp.SUM, group=group)
    return flat


def _allreduce(flat, group, bucket_bytes):
    per = max(1, bucket_bytes // flat.element_size())
    for off in range(0, flat.numel(), per):
        dist.all_reduce(flat[off:off + per], op=dist.ReduceOp.SUM, group=group)


class GradSync:
    """Bucketed SUM all-reduce of a flat fp32 gradient, one segment per grad-ready group.

    launch(i) enqueues segment i's all-reduce behind everything issued so far on the current
    stream — on a side stream for GPU tensors, so it overlaps whatever the current stream runs
    next (with RCCL the collective runs on the communicator's stream, ordered after the side
    stream); wait() makes the current stream wait for every launched segment. CPU tensors (gloo)
    are reduced synchronously."""

    def __init__(self, grad, segments, group=None, bucket_bytes=BUCKET_BYTES):
        self.grad = grad
        self.segments = list(segments)
        self.group = group
        self.bucket_bytes = bucket_bytes
        # a process group of any size (world 1 included) runs the collectives: a 1-rank RCCL
        # group exercises the side-stream / graph-cut schedule of the multi-GPU step
        self.grouped = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if self.grouped else 1
        self.stream = torch.cuda.Stream(device=grad.device) if grad.is_cuda and self.grouped else None
        self.launched = []
        # comm accounting (bench.py's `comm` object): off by default, no events in a timed step
        self.timing = False
        self._marks = []     # per launched segment: (start, end) events on the side stream
        self._steps = []     # per wait(): (main-stream-ready event, that step's segment marks)
        self._host_s = []    # synchronous (CPU / gloo) path: seconds per wait()
        self._host_acc = 0.0

    def buckets(self):
        """Number of all_reduce calls per step over the active segments."""
        per = max(1, self.bucket_bytes // self.grad.element_size())
        return sum(-(-(hi - lo) // per) for lo, hi in self.segments if hi > lo)

    def reduced_bytes(self):
        return sum(hi - lo for lo, hi in self.segments) * self.grad.element_size()

    def launch(self, i):
        lo, hi = self.segments[i]
        self.launched.append(i)
        if not self.grouped or hi <= lo:
            return
        if self.stream is None:
            t0 = time.perf_counter()
            _allreduce(self.grad[lo:hi], self.group, self.bucket_bytes)
            self._host_acc += time.perf_counter() - t0
            return
        self.stream.wait_stream(torch.cuda.current_stream(self.grad.device))
        with torch.cuda.stream(self.stream):
            if self.timing:
                e0 = torch.cuda.Event(enable_timing=True)
                e0.record(self.stream)
            _allreduce(self.grad[lo:hi], self.group, self.bucket_bytes)
            if self.timing:
                e1 = torch.cuda.Event(enable_timing=True)
                e1.record(self.stream)
                self._marks.append((e0, e1))

    def wait(self):
        if self.stream is not None:
            cur = torch.cuda.current_stream(self.grad.device)
            if self.timing:
                ready = torch.cuda.Event(enable_timing=True)
                ready.record(cur)   # the main stream has issued everything before the optimizer
                self._steps.append((ready, self._marks))
                self._marks = []
            cur.wait_stream(self.stream)
        elif self.timing:
            self._host_s.append(self._host_acc)
        self._host_acc = 0.0
        done, self.launched = self.launched, []
        return done

    def comm_stats(self):
        """Per-step means over the waits recorded while `timing` was on, then cleared:
        `allreduce_ms` = time the collectives ran (sum over segments, side stream), `exposed_ms` =
        how long after the main stream reached the optimizer the last collective ended (0 when
        the overlap hid it). Synchronous (gloo / CPU) reductions are fully exposed."""
        if self.stream is not None:
            torch.cuda.synchronize(self.grad.device)
            busy, exposed = [], []
            for ready, marks in self._steps:
                busy.append(sum(a.elapsed_time(b) for a, b in marks))
                exposed.append(max(0.0, ready.elapsed_time(marks[-1][1])) if marks else 0.0)
            self._steps = []
        else:
            busy = [s * 1e3 for s in self._host_s]
            exposed = list(busy)
            self._host_s = []
        n = max(1, len(busy))
        return {"steps": len(busy), "allreduce_ms": round(sum(busy) / n, 4),
                "exposed_ms": round(sum(exposed) / n, 4)}
