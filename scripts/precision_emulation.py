"""Where does a reduced-precision training step lose the gradient? CPU emulation (fp64 arithmetic
with rounding at the points where the HIP engine stores or feeds the MFMA with a narrow type) of
the batch-32 headline step (4-stack, 256x256, N=32, the inputs of tests/golden/primary_s4_n32_256),
compared with the reference's own fp64 gradients (the fixture's strided samples).

Rounding points, as the engine has them: every STORED activation — conv outputs
(incl. the residual add of the epilogue), maxpool and upsample+add outputs, the input — rounds its
value (forward) and its gradient (backward) to the storage type; the conv's MFMA operands (the
BN+ReLU-transformed input, applied in staging and never stored, and the weight) round to the
operand type in the forward; the gradient w.r.t. a conv's input (the stored dA the BN backward
reads) rounds to the storage type. All arithmetic between those points is fp64 (the kernels
accumulate in fp32 — far finer than bf16).

Modes (storage / operand): fp64 (none: reproduces the fixture), fp32/fp32 (the fp32 engine),
bf16/bf16 (the bf16 engine), fp32/bf16 (bf16 MFMA operands, fp32 storage of every activation and
gradient: the verdict's O1-like split), fp16/fp16 (apex O1's storage type; range ignored), and
the bf16 engine with only the forward or only the backward rounded.

  python scripts/precision_emulation.py [--modes bf16,fp32xbf16] [--threads 8] [--device cuda]
Writes one table (per-parameter cosine with fp64, grouped along the backward chain) to stdout.
"""
import argparse
import os
import sys
import time

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle.hourglass_oracle import OracleModel  # noqa: E402
from progressive_process_for_human_pose_estimation_amd.data import gaussian_targets, synthetic_images  # noqa: E402

DT = {"fp64": None, "fp32": torch.float32, "bf16": torch.bfloat16, "fp16": torch.float16}
# name -> (forward storage, forward operand, backward storage)
MODES = {
    "fp64": ("fp64", "fp64", "fp64"),
    "fp32": ("fp32", "fp32", "fp32"),
    "bf16": ("bf16", "bf16", "bf16"),
    "fp32xbf16": ("fp32", "bf16", "fp32"),
    "fp16": ("fp16", "fp16", "fp16"),
    "bf16fwd": ("bf16", "bf16", "fp32"),
    "bf16bwd": ("fp32", "fp32", "bf16"),
    "bf16op": ("bf16", "fp32", "bf16"),
}


def rnd(t, name):
    d = DT[name]
    return t if d is None else t.to(d).to(t.dtype)


class Q(torch.autograd.Function):
    """forward: round to `fwd`; backward: round the incoming gradient to `bwd`"""

    @staticmethod
    def forward(ctx, x, fwd, bwd):
        ctx.bwd = bwd
        return rnd(x, fwd)

    @staticmethod
    def backward(ctx, g):
        return rnd(g, ctx.bwd), None, None


class Emu:
    def __init__(self, store, op, bstore):
        self.store, self.op, self.bstore = store, op, bstore

    def stored(self, t):
        return Q.apply(t, self.store, self.bstore)

    def operand(self, t):
        # forward: the staged MFMA operand; backward: the conv's input gradient is stored
        return Q.apply(t, self.op, self.bstore)


def install(emu):
    """Patch the functional ops the oracle uses (restored by the returned undo)."""
    conv0, mp0, interp0 = F.conv2d, F.max_pool2d, F.interpolate

    def conv(x, w, b=None, stride=1, padding=0, dilation=1, groups=1):
        y = conv0(emu.operand(x), rnd(w, emu.op) if emu.op != "fp64" else w, b, stride, padding,
                  dilation, groups)
        return emu.stored(y)

    def mp(*a, **k):
        return emu.stored(mp0(*a, **k))

    def interp(*a, **k):
        return interp0(*a, **k)  # the add that follows is stored (see OracleHourglass patch)

    F.conv2d, F.max_pool2d, F.interpolate = conv, mp, interp
    nn.modules.conv.F.conv2d = conv
    nn.modules.pooling.F.max_pool2d = mp

    def undo():
        F.conv2d, F.max_pool2d, F.interpolate = conv0, mp0, interp0
        nn.modules.conv.F.conv2d = conv0
        nn.modules.pooling.F.max_pool2d = mp0
    return undo


def run(mode, x, t, dev, eval_mode=False):
    store, op, bstore = MODES[mode]
    emu = Emu(store, op, bstore)
    torch.manual_seed(0)
    m = OracleModel().double().to(dev)
    if eval_mode:
        m.eval()  # BN from running statistics (init: mean 0, var 1) — no batch-statistics coupling
    # the residual add and upsample+add results are stored activations too
    import oracle.hourglass_oracle as O
    res_fwd, hg_fwd = O.OracleResidual.forward, O.OracleHourglass.forward

    def res_forward(self, xx):
        return emu.stored(res_fwd(self, xx))

    def hg_forward(self, xx):
        return emu.stored(hg_fwd(self, xx))
    O.OracleResidual.forward, O.OracleHourglass.forward = res_forward, hg_forward
    undo = install(emu)
    try:
        outs = m(emu.stored(x.double().to(dev)))
        loss = sum(F.mse_loss(o, t.double().to(dev)) for o in outs)
        loss.backward()
    finally:
        undo()
        O.OracleResidual.forward, O.OracleHourglass.forward = res_fwd, hg_fwd
    rows = []
    for k, p in m.named_parameters():
        if p.grad is None:
            continue
        rows.append((k, p.grad.detach().reshape(-1)[::97].cpu().numpy()))
    return float(loss.detach()), rows


def group(name):
    if name.startswith(("conv1.", "residual1.", "residual2.", "residual3.")):
        return "stem (conv1, residual1-3)"
    if name.startswith("hourglass1."):
        depth = name.count("hourglass1.")
        return f"hourglass level {depth} ({64 >> (depth - 1)}x{64 >> (depth - 1)})"
    return "heads (residual4, lin, conv2-4)"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="fp64,fp32,bf16,fp32xbf16,fp16,bf16fwd,bf16bwd,bf16op")
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--n", type=int, default=32)
    ap.add_argument("--device", default="cpu", help="cpu, or cuda (fp64 on the GPU box: N=32 needs ~60 GB)")
    ap.add_argument("--eval", action="store_true",
                    help="eval-mode BN (running statistics): reference = this script's fp64 mode "
                         "(the fixture holds train-mode gradients only)")
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    g = np.load(os.path.join(ROOT, "tests", "golden", "primary_s4_n32_256.npz"))
    x = synthetic_images(a.n, 256, 256, seed=1234)
    t = gaussian_targets(a.n, 17, 64, 64, seed=1)[0]
    r64 = g["grad_sample64"]
    modes = a.modes.split(",")
    if a.eval:
        _, rows64 = run("fp64", x, t, a.device, True)
        r64 = np.concatenate([r for _, r in rows64])
    res = {}
    for mode in modes:
        t0 = time.time()
        loss, rows = run(mode, x, t, a.device, a.eval)
        flat = np.concatenate([r for _, r in rows])
        assert len(flat) == len(r64), (len(flat), len(r64))
        cos = float((flat * r64).sum() / (np.linalg.norm(flat) * np.linalg.norm(r64)))
        res[mode] = (loss, rows, cos)
        print(f"[{mode}] loss {loss:.6f} (ref64 {float(g['loss64']):.6f}) overall grad cosine with fp64 "
              f"{cos:.4f}  ({time.time() - t0:.0f} s)", flush=True)
    names = [k for k, _ in res[modes[0]][1]]
    off = 0
    per = {m: [] for m in modes}
    slices = []
    for i, k in enumerate(names):
        n = len(res[modes[0]][1][i][1])
        slices.append((k, off, off + n))
        off += n
    print("\nper-parameter cosine with the reference's fp64 gradient (median per group; groups in "
          "backward order: heads first, stem last)")
    hdr = "%-36s %5s " % ("group", "params") + " ".join("%10s" % m for m in modes)
    print(hdr)
    order = ["heads (residual4, lin, conv2-4)"] + [f"hourglass level {d} ({64 >> (d - 1)}x{64 >> (d - 1)})"
                                                   for d in range(1, 5)] + ["stem (conv1, residual1-3)"]
    for gname in order:
        cols = []
        cnt = 0
        for m in modes:
            cs = []
            for i, (k, lo, hi) in enumerate(slices):
                if group(k) != gname:
                    continue
                r = r64[lo:hi]
                s = res[m][1][i][1]
                if np.linalg.norm(r) < 1e-9:
                    continue
                cs.append(float((s * r).sum() / (np.linalg.norm(s) * np.linalg.norm(r) + 1e-300)))
            cnt = len(cs)
            cols.append(np.median(cs) if cs else float("nan"))
        print("%-36s %5d " % (gname, cnt) + " ".join("%10.4f" % c for c in cols))
    print("%-36s %5s " % ("overall (all samples)", "") + " ".join("%10.4f" % res[m][2] for m in modes))
    rb = g["grad_samplebf16"].astype(np.float64)
    r32 = g["grad_sample32"].astype(np.float64)
    print("reference's own runs: fp32 %.4f, bf16 %.4f" % (
        float((r32 * r64).sum() / (np.linalg.norm(r32) * np.linalg.norm(r64))),
        float((rb * r64).sum() / (np.linalg.norm(rb) * np.linalg.norm(r64)))))


if __name__ == "__main__":
    main()
