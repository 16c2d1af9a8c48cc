"""Generate the golden fixtures in tests/golden/ from the REFERENCE's own model classes.

Run in the build container only (needs /root/reference):  python tests/golden/make_golden.py
The reference classes are loaded by AST extraction (tools/ref_loader.py); this
script is committed next to its outputs so the vectors can be regenerated. Nothing here ships to or
runs on the GPU box; the .npz files are data (inputs + expected outputs), not reference source.

Per case we record, for torch.manual_seed(0) construction and seeded synthetic inputs:
  sd_sha256            hash of the initial state_dict (keys, shapes, bytes)
  eval32_*             eval-mode fp32 heatmaps (fresh model, running stats at init)
  train32_* / train64_* train-mode heatmaps in fp32 and fp64 (tolerance gate of SURVEY §8(c):
                       |build - ref64| <= 1e-3 + 2 |ref32 - ref64|)
  loss32 / loss64      sum of per-stack MSE vs Gaussian targets
  grad_norm_*          per-parameter grad L2 norms (None grads recorded as -1)
  grad_sample_*        strided samples of every grad
  bn_running_*         BN running_mean / running_var / num_batches_tracked after one train step
"""
import hashlib
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, ROOT)

from ref_loader import load_reference  # noqa: E402
from progressive_process_for_human_pose_estimation_amd.data import (  # noqa: E402
    class_maps, gaussian_targets, synthetic_images)
from ref_loader import MODEL_CLASSES  # noqa: E402

GRAD_STRIDE = 97


def sd_hash(model):
    h = hashlib.sha256()
    for k, v in model.state_dict().items():
        h.update(k.encode())
        h.update(str(tuple(v.shape)).encode())
        h.update(v.detach().cpu().contiguous().numpy().tobytes())
    return h.hexdigest()


def build(file, overrides):
    ns = load_reference(file, overrides=overrides)
    torch.manual_seed(0)
    return ns["creatModel"]()


def run_train(model, x, t):
    model.train()
    model.zero_grad(set_to_none=True)
    outs = model(x)
    loss = sum(torch.nn.functional.mse_loss(o, t) for o in outs)
    loss.backward()
    return outs, loss


def load_image_batch(names, size=256):
    from PIL import Image
    arrs = []
    for n in names:
        im = Image.open(os.path.join("/root/reference/test_img", n)).convert("RGB").resize([size, size])
        arrs.append(np.asarray(im, dtype=np.uint8))
    return np.stack(arrs)  # [N, H, W, 3] uint8


def images_to_input(u8):
    x = torch.from_numpy(u8).permute(0, 3, 1, 2).double() / 255.0
    return ((x - 0.5) / 0.5).float()


def make_case(name, file, overrides, n, h, w, full_outputs, image_names=None, sample_stride=16):
    nout = overrides.get("nOutChannels", 17) if overrides else None
    ns_probe = load_reference(file, overrides=overrides)
    nout = ns_probe["nOutChannels"]
    rec = {}
    if image_names:
        u8 = load_image_batch(image_names, h)
        rec["images_u8"] = u8
        x = images_to_input(u8)
    else:
        x = synthetic_images(n, h, w, seed=1234)
    t, xs, ys, vis = gaussian_targets(n, nout, h // 4, w // 4, seed=1)
    rec["x"] = x.numpy()
    rec["target"] = t.numpy()

    m32 = build(file, overrides)
    rec["sd_sha256"] = np.array(sd_hash(m32))
    keys = [k for k, _ in m32.named_parameters()]
    rec["param_names"] = np.array(keys)

    # eval mode, fresh model
    meval = build(file, overrides).eval()
    with torch.no_grad():
        ev = meval(x)
    # train mode fp32 and fp64
    outs32, loss32 = run_train(m32, x, t)
    m64 = build(file, overrides).double()
    outs64, loss64 = run_train(m64, x.double(), t.double())

    def put_outputs(tag, outs):
        arr = torch.stack([o.detach() for o in outs]).numpy()  # [S, N, K, Hm, Wm]
        if full_outputs:
            rec[tag] = arr
        else:
            rec[tag + "_sample"] = arr.reshape(-1)[::sample_stride].copy()
        s, nn_, k = arr.shape[:3]
        flat = arr.reshape(s, nn_, k, -1)
        rec[tag + "_sum"] = flat.sum(-1)
        rec[tag + "_sumsq"] = (flat.astype(np.float64) ** 2).sum(-1)
        rec[tag + "_argmax"] = flat.argmax(-1)
        srt = np.sort(flat, axis=-1)
        rec[tag + "_gap"] = srt[..., -1] - srt[..., -2]

    put_outputs("eval32", ev)
    put_outputs("train32", outs32)
    put_outputs("train64", outs64)
    rec["loss32"] = np.array(float(loss32))
    rec["loss64"] = np.array(float(loss64))

    gn32, gn64, gs32, gs64 = [], [], [], []
    for (k, p32), (_, p64) in zip(m32.named_parameters(), m64.named_parameters()):
        if p32.grad is None:
            gn32.append(-1.0)
            gn64.append(-1.0)
            continue
        gn32.append(float(p32.grad.norm()))
        gn64.append(float(p64.grad.norm()))
        gs32.append(p32.grad.reshape(-1)[::GRAD_STRIDE])
        gs64.append(p64.grad.reshape(-1)[::GRAD_STRIDE])
    rec["grad_norm32"] = np.array(gn32)
    rec["grad_norm64"] = np.array(gn64)
    rec["grad_sample32"] = torch.cat(gs32).numpy()
    rec["grad_sample64"] = torch.cat(gs64).numpy()

    rm, rv, nbt, rm64, rv64 = [], [], [], [], []
    for (k, b), (_, b64) in zip(m32.named_buffers(), m64.named_buffers()):
        if k.endswith("running_mean"):
            rm.append(b.reshape(-1)); rm64.append(b64.reshape(-1))
        elif k.endswith("running_var"):
            rv.append(b.reshape(-1)); rv64.append(b64.reshape(-1))
        elif k.endswith("num_batches_tracked"):
            nbt.append(int(b))
    rec["bn_running_mean32"] = torch.cat(rm).numpy()
    rec["bn_running_var32"] = torch.cat(rv).numpy()
    rec["bn_running_mean64"] = torch.cat(rm64).numpy()
    rec["bn_running_var64"] = torch.cat(rv64).numpy()
    rec["bn_num_batches_tracked"] = np.array(nbt)

    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **rec)
    print(name, "->", path, os.path.getsize(path), "bytes; loss32", float(loss32))


def make_progressive_case(name, file, n, h, w, full_outputs):
    """Progressive-head presets (try_with_aspp.py / try_different_stack.py): 3 outputs with 2 / 20
    / 17 channels, loss = CE(out0, bg) + CE(out1, skeleton) + MSE(out2, keypoints)
    (try_with_aspp.py:356-396). Targets: class maps seeds 2 / 3, Gaussian keypoints seed 1."""
    classes = MODEL_CLASSES + ("_ASPPModule",)

    def mk():
        ns = load_reference(file, class_names=classes)
        torch.manual_seed(0)
        return ns["creatModel"]()

    x = synthetic_images(n, h, w, seed=1234)
    hm, wm = h // 4, w // 4
    bg = class_maps(n, 2, hm, wm, seed=2)
    sk = class_maps(n, 20, hm, wm, seed=3)
    kp = gaussian_targets(n, 17, hm, wm, seed=1)[0]
    rec = {"x": x.numpy(), "bg": bg.numpy(), "skeleton": sk.numpy(), "keypoints": kp.numpy()}
    m32 = mk()
    rec["sd_sha256"] = np.array(sd_hash(m32))
    rec["param_names"] = np.array([k for k, _ in m32.named_parameters()])
    meval = mk().eval()
    with torch.no_grad():
        ev = meval(x)

    def train(m, dt):
        m.train()
        outs = m(x.to(dt))
        loss = (torch.nn.functional.cross_entropy(outs[0], bg)
                + torch.nn.functional.cross_entropy(outs[1], sk)
                + torch.nn.functional.mse_loss(outs[2], kp.to(dt)))
        loss.backward()
        return outs, loss

    outs32, loss32 = train(m32, torch.float32)
    m64 = mk().double()
    outs64, loss64 = train(m64, torch.float64)
    for tag, outs in (("eval32", ev), ("train32", outs32), ("train64", outs64)):
        for i, o in enumerate(outs):
            arr = o.detach().numpy()
            if full_outputs:
                rec[f"{tag}_{i}"] = arr
            else:
                rec[f"{tag}_{i}_sample"] = arr.reshape(-1)[::16].copy()
            flat = arr.reshape(arr.shape[0], arr.shape[1], -1)
            rec[f"{tag}_{i}_argmax"] = flat.argmax(-1)
            srt = np.sort(flat, axis=-1)
            rec[f"{tag}_{i}_gap"] = srt[..., -1] - srt[..., -2]
            # per-pixel class argmax (the segmentation decision of the CE heads)
            rec[f"{tag}_{i}_clsmax"] = arr.argmax(1)
    rec["loss32"] = np.array(float(loss32))
    rec["loss64"] = np.array(float(loss64))
    gn32, gn64 = [], []
    for (k, p32), (_, p64) in zip(m32.named_parameters(), m64.named_parameters()):
        gn32.append(-1.0 if p32.grad is None else float(p32.grad.norm()))
        gn64.append(-1.0 if p64.grad is None else float(p64.grad.norm()))
    rec["grad_norm32"] = np.array(gn32)
    rec["grad_norm64"] = np.array(gn64)
    for tag, mm in (("32", m32), ("64", m64)):
        rm, rv, nbt = [], [], []
        for k, b in mm.named_buffers():
            if k.endswith("running_mean"):
                rm.append(b.reshape(-1))
            elif k.endswith("running_var"):
                rv.append(b.reshape(-1))
            elif k.endswith("num_batches_tracked"):
                nbt.append(int(b))
        rec["bn_running_mean" + tag] = torch.cat(rm).numpy()
        rec["bn_running_var" + tag] = torch.cat(rv).numpy()
    rec["bn_num_batches_tracked"] = np.array(nbt)
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **rec)
    print(name, "->", path, os.path.getsize(path), "bytes; loss32", float(loss32))


def make_cmp_case(name, n, h, w):
    """hourglass_compare.py preset (4 unshared stages, 16 outputs, always-on projection + bn4,
    nearest up-sampling, stem BN): sum of per-stage MSE vs 16-channel Gaussian targets."""
    def mk():
        ns = load_reference("hourglass_compare.py")
        torch.manual_seed(0)
        return ns["creatModel"]()

    x = synthetic_images(n, h, w, seed=1234)
    t = gaussian_targets(n, 16, h // 4, w // 4, seed=1)[0]
    rec = {"x": x.numpy(), "target": t.numpy()}
    m32 = mk()
    rec["sd_sha256"] = np.array(sd_hash(m32))
    with torch.no_grad():
        ev = mk().eval()(x)
    outs32, loss32 = run_train(m32, x, t)
    m64 = mk().double()
    outs64, loss64 = run_train(m64, x.double(), t.double())
    for tag, outs in (("eval32", ev), ("train32", outs32), ("train64", outs64)):
        arr = torch.stack([o.detach() for o in outs]).numpy()
        rec[tag] = arr
        flat = arr.reshape(arr.shape[0], arr.shape[1], arr.shape[2], -1)
        rec[tag + "_argmax"] = flat.argmax(-1)
        srt = np.sort(flat, axis=-1)
        rec[tag + "_gap"] = srt[..., -1] - srt[..., -2]
    rec["loss32"] = np.array(float(loss32))
    rec["loss64"] = np.array(float(loss64))
    rec["grad_norm32"] = np.array([-1.0 if p.grad is None else float(p.grad.norm())
                                   for p in m32.parameters()])
    rec["grad_norm64"] = np.array([-1.0 if p.grad is None else float(p.grad.norm())
                                   for p in m64.parameters()])
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **rec)
    print(name, "->", path, os.path.getsize(path), "bytes; loss32", float(loss32))


def main_compare():
    torch.set_num_threads(8)
    make_cmp_case("hgcompare_s4_n2_128", 2, 128, 128)


def main_progressive():
    torch.set_num_threads(8)
    make_progressive_case("aspp_s3_n2_128", "try_with_aspp.py", 2, 128, 128, True)
    make_progressive_case("diffstack_s3_n2_128", "try_different_stack.py", 2, 128, 128, True)


def main_morelayer():
    """try_more_layer.py (§8 a14, live ASPP at the innermost 2x2 level; 4 stacks, 4 outputs, the
    loss on outputs 0-2 as the reference's training loop, :398-401)."""
    torch.set_num_threads(8)
    make_progressive_case("morelayer_s4_n2_128", "try_more_layer.py", 2, 128, 128, True)


def make_trainpy_case(name, n, h, w, fraction=0.5):
    """train.py preset (stride-2 residual blocks, unshared hourglass with live ASPP_Block, nearest
    x2 + concat, 3 stages): loss = the reference's own Costomer_CrossEntropyLoss (bootstrapped
    top-k CE) + CrossEntropyLoss on outputs 1 and 2 (train.py:886-890), fraction 0.5."""
    classes = ("ResidualBlock", "_ASPPModule", "ASPP_Block", "hourglass", "creatModel",
               "Costomer_CrossEntropyLoss")

    ns = load_reference("train.py", class_names=classes)

    def mk():
        torch.manual_seed(0)
        return ns["creatModel"]()

    x = synthetic_images(n, h, w, seed=1234)
    hm, wm = h // 4, w // 4
    sk = class_maps(n, 16, hm, wm, seed=3)
    kp = class_maps(n, 17, hm, wm, seed=4)
    rec = {"x": x.numpy(), "skeleton": sk.numpy(), "keypoints": kp.numpy(),
           "fraction": np.array(fraction)}
    m32 = mk()
    rec["sd_sha256"] = np.array(sd_hash(m32))
    rec["param_names"] = np.array([k for k, _ in m32.named_parameters()])
    with torch.no_grad():
        ev = mk().eval()(x)
    boot = ns["Costomer_CrossEntropyLoss"]()
    ce = torch.nn.CrossEntropyLoss()

    def train(m, dt):
        m.train()
        outs = m(x.to(dt))
        loss = (boot.forward(outs[1], sk, fraction) + ce(outs[1], sk)
                + boot.forward(outs[2], kp, fraction) + ce(outs[2], kp))
        loss.backward()
        return outs, loss

    outs32, loss32 = train(m32, torch.float32)
    m64 = mk().double()
    outs64, loss64 = train(m64, torch.float64)
    for tag, outs in (("eval32", ev), ("train32", outs32), ("train64", outs64)):
        for i, o in enumerate(outs):
            arr = o.detach().numpy()
            rec[f"{tag}_{i}"] = arr
            flat = arr.reshape(arr.shape[0], arr.shape[1], -1)
            srt = np.sort(flat, axis=-1)
            rec[f"{tag}_{i}_argmax"] = flat.argmax(-1)
            rec[f"{tag}_{i}_gap"] = srt[..., -1] - srt[..., -2]
    rec["loss32"] = np.array(float(loss32))
    rec["loss64"] = np.array(float(loss64))
    gn32, gn64 = [], []
    for (k, p32), (_, p64) in zip(m32.named_parameters(), m64.named_parameters()):
        gn32.append(-1.0 if p32.grad is None else float(p32.grad.norm()))
        gn64.append(-1.0 if p64.grad is None else float(p64.grad.norm()))
    rec["grad_norm32"] = np.array(gn32)
    rec["grad_norm64"] = np.array(gn64)
    for tag, mm in (("32", m32), ("64", m64)):
        rm, rv, nbt = [], [], []
        for k, b in mm.named_buffers():
            if k.endswith("running_mean"):
                rm.append(b.reshape(-1))
            elif k.endswith("running_var"):
                rv.append(b.reshape(-1))
            elif k.endswith("num_batches_tracked"):
                nbt.append(int(b))
        rec["bn_running_mean" + tag] = torch.cat(rm).numpy()
        rec["bn_running_var" + tag] = torch.cat(rv).numpy()
    rec["bn_num_batches_tracked"] = np.array(nbt)
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **rec)
    print(name, "->", path, os.path.getsize(path), "bytes; loss32", float(loss32))


def main_losses():
    """train.py:343-408's four loss classes, executed from the reference, on seeded inputs: loss
    values and input gradients (fp64, so the GPU fp32 kernels are judged against exact values)."""
    torch.set_num_threads(8)
    names = ("Costomer_CrossEntropyLoss", "Costomer_CrossEntropyLoss_with_mask",
             "Costomer_MSELoss_with_mask", "Costomer_MSELoss")
    ns = load_reference("train.py", class_names=names)
    g = torch.Generator().manual_seed(11)
    N, K, C, h, w = 2, 16, 17, 16, 16
    logits = torch.randn(N, K, h, w, generator=g, dtype=torch.float64) * 2
    cls = torch.randint(0, K, (N, h, w), generator=g)
    mask = (torch.rand(N, h, w, generator=g) > 0.4).to(torch.int64)
    x = torch.randn(N, C, h, w, generator=g, dtype=torch.float64)
    tgt = torch.rand(N, C, h, w, generator=g, dtype=torch.float64)
    rec = {"logits": logits.float().numpy(), "cls": cls.numpy(), "mask": mask.numpy(),
           "x": x.float().numpy(), "tgt": tgt.float().numpy()}
    # the fp32-rounded inputs, evaluated in fp64
    logits, x, tgt = logits.float().double(), x.float().double(), tgt.float().double()
    cases = [("ce_boot_0.5", names[0], "logits", lambda m, a: m.forward(a, cls, 0.5)),
             ("ce_boot_0.05", names[0], "logits", lambda m, a: m.forward(a, cls, 0.05)),
             ("ce_mask", names[1], "logits", lambda m, a: m.forward(a, cls, mask)),
             ("mse_mask", names[2], "x", lambda m, a: m.forward(a, tgt, mask)),
             ("mse_boot_0.5", names[3], "x", lambda m, a: m.forward(a, tgt, 0.5)),
             ("mse_boot_0.1", names[3], "x", lambda m, a: m.forward(a, tgt, 0.1))]
    for tag, cname, which, fn in cases:
        a = (logits if which == "logits" else x).clone().requires_grad_()
        loss = fn(ns[cname](), a)
        loss.backward()
        rec[tag + "_loss"] = np.array(float(loss))
        rec[tag + "_grad"] = a.grad.numpy()
    path = os.path.join(HERE, "losses_trainpy.npz")
    np.savez_compressed(path, **rec)
    print("losses ->", path, os.path.getsize(path), "bytes")


def main_trainpy():
    torch.set_num_threads(8)
    make_trainpy_case("trainpy_s3_n2_128", 2, 128, 128)


def main_stress():
    """BASELINE configs[4]: 8-stack hourglass at 384x384 (fp32); N=1 keeps the CPU reference run
    to seconds (the GPU bench runs N=16). Summaries + samples only."""
    torch.set_num_threads(8)
    make_case("primary_s8_n1_384", "try_with_torch.py", {"nStack": 8}, 1, 384, 384, False)
    # inputs / targets are regenerated from their seeds by the test (keeps the fixture small)
    path = os.path.join(HERE, "primary_s8_n1_384.npz")
    rec = dict(np.load(path))
    del rec["x"], rec["target"]
    np.savez_compressed(path, **rec)


def main_batch32():
    """BASELINE configs[1]/[2] at their own batch: 4-stack, 256x256, N=32 (the bench's kernel
    routing: M = 131072 at 64x64, two-stage finalisers, split-K plans, halo tile counts). Outputs
    sampled every 61st element; inputs / targets regenerated from their seeds by the test."""
    torch.set_num_threads(8)
    name = "primary_s4_n32_256"
    make_case(name, "try_with_torch.py", None, 32, 256, 256, False, sample_stride=61)
    path = os.path.join(HERE, name + ".npz")
    rec = dict(np.load(path))
    del rec["x"], rec["target"]
    rec["sample_stride"] = np.array(61)
    np.savez_compressed(path, **rec)
    print(name, "final size", os.path.getsize(path))


def main_batch32_bf16():
    """bf16 noise floor of the reference at N=32: the reference classes run in bfloat16 on the
    CPU (bf16 parameters and activations, as the engine's bf16 path stores them), eval and train
    mode from the same seeded init; added to primary_s4_n32_256.npz. The engine's bf16 path is
    gated against 2x this noise (the fp32 path's rule, SURVEY §8(c), at bf16 precision)."""
    torch.set_num_threads(8)
    name = "primary_s4_n32_256"
    path = os.path.join(HERE, name + ".npz")
    rec = dict(np.load(path))
    st = int(rec["sample_stride"])
    x = synthetic_images(32, 256, 256, seed=1234)
    t = gaussian_targets(32, 17, 64, 64, seed=1)[0]
    with torch.no_grad():
        ev = build("try_with_torch.py", None).to(torch.bfloat16).eval()(x.to(torch.bfloat16))
    rec["evalbf16_sample"] = torch.stack([o.float() for o in ev]).numpy().reshape(-1)[::st].copy()
    m = build("try_with_torch.py", None).to(torch.bfloat16)
    outs, loss = run_train(m, x.to(torch.bfloat16), t.to(torch.bfloat16))
    arr = torch.stack([o.detach().float() for o in outs]).numpy()
    rec["trainbf16_sample"] = arr.reshape(-1)[::st].copy()
    rec["trainbf16_argmax"] = arr.reshape(4, 32, 17, -1).argmax(-1)
    rec["lossbf16"] = np.array(float(loss))
    rec["grad_normbf16"] = np.array([-1.0 if p.grad is None else float(p.grad.float().norm())
                                     for p in m.parameters()])
    rec["grad_samplebf16"] = torch.cat([p.grad.float().reshape(-1)[::GRAD_STRIDE]
                                        for p in m.parameters() if p.grad is not None]).numpy()
    np.savez_compressed(path, **rec)
    print(name, "+ bf16 noise floor:", os.path.getsize(path), "bytes; lossbf16", float(loss))


def main_eval32():
    """Eval-mode gradients of the batch-32 headline step (4-stack, 256x256, N=32): BN from the
    running statistics, so the forward is well-conditioned (fp32 vs fp64 heatmaps 1.7e-6; the
    CPU precision emulation gives bf16 gradients cosine 0.9999 with fp64, where the train-mode
    step decorrelates: scripts/precision_emulation.py --eval). The engine's bf16 backward is
    gated tightly against these (tests/test_gpu_parity.py). Added to primary_s4_n32_256.npz:
    loss / per-parameter grad norms / strided grad samples in fp64 and fp32."""
    torch.set_num_threads(8)
    name = "primary_s4_n32_256"
    path = os.path.join(HERE, name + ".npz")
    rec = dict(np.load(path))
    x = synthetic_images(32, 256, 256, seed=1234)
    t = gaussian_targets(32, 17, 64, 64, seed=1)[0]
    for dt, tag in ((torch.float64, "64"), (torch.float32, "32")):
        m = build("try_with_torch.py", None).to(dt).eval()
        m.zero_grad(set_to_none=True)
        outs = m(x.to(dt))
        loss = sum(torch.nn.functional.mse_loss(o, t.to(dt)) for o in outs)
        loss.backward()
        rec["evalloss" + tag] = np.array(float(loss))
        rec["evalgrad_norm" + tag] = np.array([-1.0 if p.grad is None else float(p.grad.double().norm())
                                               for p in m.parameters()])
        rec["evalgrad_sample" + tag] = torch.cat([p.grad.double().reshape(-1)[::GRAD_STRIDE]
                                                  for p in m.parameters() if p.grad is not None]).numpy()
        del m, outs, loss
    np.savez_compressed(path, **rec)
    print(name, "+ eval-mode grads:", os.path.getsize(path), "bytes")


def main_stress8():
    """BASELINE configs[4] at a production-like batch: 8-stack, 384x384, N=8 (the largest batch
    whose fp64 reference run fits this container's 64 GB: ~4 GB per image in fp64). Outputs
    sampled every 61st element; inputs / targets regenerated from their seeds by the test."""
    torch.set_num_threads(8)
    name = "primary_s8_n8_384"
    make_case(name, "try_with_torch.py", {"nStack": 8}, 8, 384, 384, False, sample_stride=61)
    path = os.path.join(HERE, name + ".npz")
    rec = dict(np.load(path))
    del rec["x"], rec["target"]
    rec["sample_stride"] = np.array(61)
    np.savez_compressed(path, **rec)
    print(name, "final size", os.path.getsize(path))


def run_train_ckpt(model, x, t):
    """run_train with every ResidualBlock call checkpointed (torch.utils.checkpoint: its interior
    is recomputed in backward, only its input is kept) so a batch-16 fp64 run of the 8-stack
    384x384 model fits the container; the recomputation re-runs the train-mode BatchNorms, so
    their buffers are restored to the forward's values afterwards (outputs, loss and gradients
    are those of the plain run: the recomputed forward uses the same batch statistics)."""
    from torch.utils.checkpoint import checkpoint
    model.train()
    model.zero_grad(set_to_none=True)
    wrapped = []
    for mod in model.modules():
        if type(mod).__name__ == "ResidualBlock":
            f = mod.forward
            mod.forward = (lambda f: (lambda *a: checkpoint(f, *a, use_reentrant=False)))(f)
            wrapped.append(mod)
    outs = model(x)
    loss = sum(torch.nn.functional.mse_loss(o, t) for o in outs)
    bufs = {k: b.detach().clone() for k, b in model.named_buffers()}
    loss.backward()
    with torch.no_grad():
        for k, b in model.named_buffers():
            b.copy_(bufs[k])
    for mod in wrapped:
        del mod.forward
    return outs, loss


def main_stress16():
    """BASELINE configs[4] at its own batch: 8-stack, 384x384, N=16 (fp64 and fp32 reference runs
    with checkpointed ResidualBlocks, run_train_ckpt). Same records as stress8."""
    global run_train
    torch.set_num_threads(8)
    run_train = run_train_ckpt
    name = "primary_s8_n16_384"
    make_case(name, "try_with_torch.py", {"nStack": 8}, 16, 384, 384, False, sample_stride=61)
    path = os.path.join(HERE, name + ".npz")
    rec = dict(np.load(path))
    del rec["x"], rec["target"]
    rec["sample_stride"] = np.array(61)
    np.savez_compressed(path, **rec)
    print(name, "final size", os.path.getsize(path))


def main_twin():
    """Per-parameter fp32 rounding noise of the reference at the twin-schedule test's shape
    (1 stack, 128x128, N=8: every hourglass level 32..2 runs a twin chain in the engine). Records
    ||g32 - g64|| / ||g64|| per parameter (`grad_noise32`), the fp64 grad norms, loss and sampled
    heatmaps; inputs regenerated from their seeds by the test."""
    torch.set_num_threads(8)
    name = "primary_s1_n8_128"
    make_case(name, "try_with_torch.py", {"nStack": 1}, 8, 128, 128, False, sample_stride=7)
    path = os.path.join(HERE, name + ".npz")
    rec = dict(np.load(path))
    x = torch.from_numpy(rec.pop("x"))
    t = torch.from_numpy(rec.pop("target"))
    m32 = build("try_with_torch.py", {"nStack": 1})
    run_train(m32, x, t)
    m64 = build("try_with_torch.py", {"nStack": 1}).double()
    run_train(m64, x.double(), t.double())
    noise = []
    for p32, p64 in zip(m32.parameters(), m64.parameters()):
        if p64.grad is None:
            noise.append(-1.0)
            continue
        d = (p32.grad.double() - p64.grad).norm() / max(float(p64.grad.norm()), 1e-300)
        noise.append(float(d))
    rec["grad_noise32"] = np.array(noise)
    rec["sample_stride"] = np.array(7)
    np.savez_compressed(path, **rec)
    print(name, "final size", os.path.getsize(path))


def make_progressive_batch_case(name, file, n, h, w, stride=61):
    """A progressive-head preset at its BASELINE batch (configs[3]: try_with_aspp.py, 256x256,
    N=16): same records as make_progressive_case but outputs as strided samples, the CE heads'
    per-pixel class decision + top-1/top-2 gap of the fp64 run, loss components, grad samples;
    inputs and targets are regenerated from their seeds by the test."""
    classes = MODEL_CLASSES + ("_ASPPModule",)

    def mk():
        ns = load_reference(file, class_names=classes)
        torch.manual_seed(0)
        return ns["creatModel"]()

    x = synthetic_images(n, h, w, seed=1234)
    hm, wm = h // 4, w // 4
    bg = class_maps(n, 2, hm, wm, seed=2)
    sk = class_maps(n, 20, hm, wm, seed=3)
    kp = gaussian_targets(n, 17, hm, wm, seed=1)[0]
    rec = {"sample_stride": np.array(stride)}
    m32 = mk()
    rec["sd_sha256"] = np.array(sd_hash(m32))
    rec["param_names"] = np.array([k for k, _ in m32.named_parameters()])
    meval = mk().eval()
    with torch.no_grad():
        ev = meval(x)
    del meval

    def train(m, dt):
        m.train()
        outs = m(x.to(dt))
        parts = (torch.nn.functional.cross_entropy(outs[0], bg),
                 torch.nn.functional.cross_entropy(outs[1], sk),
                 torch.nn.functional.mse_loss(outs[2], kp.to(dt)))
        loss = parts[0] + parts[1] + parts[2]
        loss.backward()
        return [o.detach() for o in outs], loss, parts

    outs32, loss32, parts32 = train(m32, torch.float32)
    m64 = mk().double()
    outs64, loss64, parts64 = train(m64, torch.float64)
    for tag, outs in (("eval32", ev), ("train32", outs32), ("train64", outs64)):
        for i, o in enumerate(outs):
            arr = o.numpy()
            rec[f"{tag}_{i}_sample"] = arr.reshape(-1)[::stride].copy()
            flat = arr.reshape(arr.shape[0], arr.shape[1], -1)
            rec[f"{tag}_{i}_argmax"] = flat.argmax(-1)
            srt = np.sort(flat, axis=-1)
            rec[f"{tag}_{i}_gap"] = (srt[..., -1] - srt[..., -2]).astype(np.float32)
    for i in (0, 1):
        for tag, outs in (("train32", outs32), ("train64", outs64)):
            arr = outs[i].numpy()
            srt = np.sort(arr, axis=1)
            rec[f"{tag}_{i}_cls"] = arr.argmax(1).astype(np.int8)
            rec[f"{tag}_{i}_clsgap"] = (srt[:, -1] - srt[:, -2]).astype(np.float32)
    rec["loss32"] = np.array(float(loss32))
    rec["loss64"] = np.array(float(loss64))
    rec["loss_parts32"] = np.array([float(v) for v in parts32])
    rec["loss_parts64"] = np.array([float(v) for v in parts64])
    gn32, gn64, gs32, gs64 = [], [], [], []
    for p32, p64 in zip(m32.parameters(), m64.parameters()):
        if p64.grad is None:
            gn32.append(-1.0)
            gn64.append(-1.0)
            continue
        gn32.append(float(p32.grad.norm()))
        gn64.append(float(p64.grad.norm()))
        gs32.append(p32.grad.reshape(-1)[::GRAD_STRIDE])
        gs64.append(p64.grad.reshape(-1)[::GRAD_STRIDE])
    rec["grad_norm32"] = np.array(gn32)
    rec["grad_norm64"] = np.array(gn64)
    rec["grad_sample32"] = torch.cat(gs32).numpy()
    rec["grad_sample64"] = torch.cat(gs64).numpy()
    for tag, mm in (("32", m32), ("64", m64)):
        rm, rv, nbt = [], [], []
        for k, b in mm.named_buffers():
            if k.endswith("running_mean"):
                rm.append(b.reshape(-1))
            elif k.endswith("running_var"):
                rv.append(b.reshape(-1))
            elif k.endswith("num_batches_tracked"):
                nbt.append(int(b))
        rec["bn_running_mean" + tag] = torch.cat(rm).numpy()
        rec["bn_running_var" + tag] = torch.cat(rv).numpy()
    rec["bn_num_batches_tracked"] = np.array(nbt)
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **rec)
    print(name, "->", path, os.path.getsize(path), "bytes; loss32", float(loss32))


def main_aspp256():
    """BASELINE configs[3] at its own size: try_with_aspp.py, 256x256, N=16."""
    torch.set_num_threads(8)
    make_progressive_batch_case("aspp_s3_n16_256", "try_with_aspp.py", 16, 256, 256)


# Extra fp32 draws of the reference: the same classes, seeds and inputs, with a different CPU
# reduction order (oneDNN / aten partition their sums by thread count and memory format), so the
# production-batch gradient gates can be set against the SPREAD of several equally valid fp32
# runs instead of one draw (round-4 verdict, "What's weak" 1). (name, threads, channels_last)
# avx2 / sse41: oneDNN restricted to that vector ISA (ONEDNN_MAX_CPU_ISA, set in the process's
# environment before torch loads: `ONEDNN_MAX_CPU_ISA=AVX2 python make_golden.py draws s8n16 avx2`)
# -> other convolution blockings / summation orders, NCHW. t1 / t3 turned out bit-identical to the
# original run at N = 16 and N = 32 (oneDNN's partition does not follow the thread count there),
# so they add no distinct draw; the ISA variants do.
DRAWS = (("t1", 1, False), ("t3", 3, False), ("cl8", 8, True), ("nomkl", 8, "nomkl"),
         ("avx2", 8, False), ("sse41", 8, False))
DRAW_ISA = {"avx2": "AVX2", "sse41": "SSE41"}


def _draw(file, overrides, n, res, stride, threads, channels_last, ckpt):
    torch.set_num_threads(threads)
    # "nomkl": NCHW with oneDNN off -> aten's own (im2col + GEMM) convolutions, a different
    # summation order in the same memory format as the reference script
    torch.backends.mkldnn.enabled = channels_last != "nomkl"
    channels_last = channels_last is True
    x = synthetic_images(n, res, res, seed=1234)
    nout = 17
    t = gaussian_targets(n, nout, res // 4, res // 4, seed=1)[0]
    m = build(file, overrides)
    if channels_last:
        m = m.to(memory_format=torch.channels_last)
        x = x.contiguous(memory_format=torch.channels_last)
    outs, loss = (run_train_ckpt if ckpt else run_train)(m, x, t)
    arr = torch.stack([o.detach().contiguous() for o in outs]).numpy()
    norms = np.array([-1.0 if p.grad is None else float(p.grad.norm()) for p in m.parameters()])
    samp = torch.cat([p.grad.contiguous().reshape(-1)[::GRAD_STRIDE]
                      for p in m.parameters() if p.grad is not None]).numpy()
    torch.backends.mkldnn.enabled = True
    return arr.reshape(-1)[::stride].copy(), float(loss.detach()), norms, samp


def main_draws(which, only=None):
    """Adds `draw32_<name>_{train_sample,loss,grad_norm,grad_sample}` to the production-batch
    fixtures: primary_s8_n16_384 (configs[4] at N=16, checkpointed as stress16),
    primary_s8_n8_384 and primary_s4_n32_256 (configs[1])."""
    cases = {"s8n16": ("primary_s8_n16_384", {"nStack": 8}, 16, 384, True),
             "s8n8": ("primary_s8_n8_384", {"nStack": 8}, 8, 384, True),
             "s4n32": ("primary_s4_n32_256", None, 32, 256, False)}
    name, ov, n, res, ckpt = cases[which]
    path = os.path.join(HERE, name + ".npz")
    for tag, threads, cl in DRAWS:
        if (only is None and tag in DRAW_ISA) or (only is not None and tag != only):
            continue
        if os.environ.get("ONEDNN_MAX_CPU_ISA") != DRAW_ISA.get(tag):
            raise SystemExit(f"draw {tag} needs ONEDNN_MAX_CPU_ISA={DRAW_ISA.get(tag)} in the environment")
        rec = dict(np.load(path))
        if f"draw32_{tag}_loss" in rec:
            continue
        st = int(rec["sample_stride"])
        samp, loss, norms, gs = _draw("try_with_torch.py", ov, n, res, st, threads, cl, ckpt)
        rec[f"draw32_{tag}_train_sample"] = samp
        rec[f"draw32_{tag}_loss"] = np.array(loss)
        rec[f"draw32_{tag}_grad_norm"] = norms
        rec[f"draw32_{tag}_grad_sample"] = gs
        tmp = path[:-4] + ".tmp.npz"   # atomic: a snapshot of the tree never sees a partial file
        np.savez_compressed(tmp, **rec)
        os.replace(tmp, path)
        g64 = rec["grad_sample64"].astype(np.float64)
        c = float((gs * g64).sum() / (np.linalg.norm(gs) * np.linalg.norm(g64)))
        print(name, "draw", tag, "loss", loss, "grad cosine with fp64 %.4f" % c, flush=True)


def main_eval8s16():
    """Eval-mode gradients of configs[4] at its own batch (8-stack, 384x384, N=16): BN from the
    running statistics at init, so no batch-statistics coupling amplifies rounding (the train-mode
    gradient's direction spreads over 0.85-0.89 across equally valid fp32 runs, gates.py): the
    engine's fp32 BACKWARD is pinned tightly here. fp64 and fp32 runs (ResidualBlocks
    checkpointed, run_train_ckpt's recipe in eval mode); added to primary_s8_n16_384.npz as
    evalloss*, evalgrad_norm*, evalgrad_sample*."""
    from torch.utils.checkpoint import checkpoint
    torch.set_num_threads(8)
    name = "primary_s8_n16_384"
    path = os.path.join(HERE, name + ".npz")
    x = synthetic_images(16, 384, 384, seed=1234)
    t = gaussian_targets(16, 17, 96, 96, seed=1)[0]
    out = {}
    for dt, tag in ((torch.float64, "64"), (torch.float32, "32")):
        m = build("try_with_torch.py", {"nStack": 8}).to(dt).eval()
        for mod in m.modules():
            if type(mod).__name__ == "ResidualBlock":
                f = mod.forward
                mod.forward = (lambda f: (lambda *a: checkpoint(f, *a, use_reentrant=False)))(f)
        m.zero_grad(set_to_none=True)
        outs = m(x.to(dt))
        loss = sum(torch.nn.functional.mse_loss(o, t.to(dt)) for o in outs)
        loss.backward()
        out["evalloss" + tag] = np.array(float(loss.detach()))
        out["evalgrad_norm" + tag] = np.array([-1.0 if p.grad is None else float(p.grad.double().norm())
                                               for p in m.parameters()])
        out["evalgrad_sample" + tag] = torch.cat([p.grad.double().reshape(-1)[::GRAD_STRIDE]
                                                  for p in m.parameters() if p.grad is not None]).numpy()
        print(name, "eval", tag, "loss", float(loss.detach()), flush=True)
        del m, outs, loss
    rec = dict(np.load(path))
    rec.update(out)
    tmp = path[:-4] + ".tmp.npz"
    np.savez_compressed(tmp, **rec)
    os.replace(tmp, path)
    print(name, "+ eval-mode grads:", os.path.getsize(path), "bytes")


def main_onestack256():
    """BASELINE configs[0] at its own size: only_one_hourgless.py (1 stack, 18 outputs), 256x256,
    N=2 — eval and train mode in fp32 / fp64, full outputs (2 x 18 x 64 x 64 per stack)."""
    torch.set_num_threads(8)
    make_case("oneStack_s1_n2_256", "only_one_hourgless.py", None, 2, 256, 256, True)


# Convergence fixture (round-5 verdict, next-round item 1): the reference's own training loop
# (try_with_torch.py:330-344: model(x) -> sum of per-stack nn.MSELoss -> zero_grad -> backward ->
# Adam.step) on a fixed learnable synthetic pose batch (data.keypoint_task), K steps from the
# seeded init, in fp32 under several CPU reduction orders (DRAWS: the train-mode step is chaotic,
# so one fp32 run cannot tell rounding from a defect); per step the loss, every CONV_EVERY steps the
# PCKh curve of the reference's own PCKh class (train.py:759-791) on the train-mode forward's last
# stack, for head boxes of CONV_BOXES heatmap pixels, and at the end the per-joint predictions.
# N = 2 distinct crops: the 4-stack model learns them in ~1000 Adam steps (round-6 GPU probe,
# scripts/converge_probe.py: N = 8 / 32 stay near the all-zero-heatmap plateau for > 1500 steps). The
# GPU test trains the bench's N = 32 configuration on 16 copies of these 2 crops: BN batch statistics
# and the mean MSE (hence every gradient and Adam step) are unchanged by duplicating a batch, so it
# is the same training run at the bench's batch and kernel routing.
CONV_N, CONV_STEPS, CONV_EVERY, CONV_LR = 2, 1200, 100, 4e-4
CONV_BOXES = (4.0, 8.0)


def main_converge(tag):
    threads, cl = {d[0]: (d[1], d[2]) for d in DRAWS}.get(tag, (8, False)) if tag != "orig" else (8, False)
    if os.environ.get("ONEDNN_MAX_CPU_ISA") != DRAW_ISA.get(tag):
        raise SystemExit(f"draw {tag} needs ONEDNN_MAX_CPU_ISA={DRAW_ISA.get(tag)} in the environment")
    torch.set_num_threads(threads)
    torch.backends.mkldnn.enabled = cl != "nomkl"
    from progressive_process_for_human_pose_estimation_amd.data import keypoint_task
    name = f"converge_s4_n{CONV_N}_256"
    path = os.path.join(HERE, name + ".npz")
    rec = dict(np.load(path)) if os.path.exists(path) else {}
    if f"{tag}_loss" in rec:
        print(name, tag, "already recorded")
        return
    ns = load_reference("try_with_torch.py")
    pk = load_reference("train.py", class_names=("PCKh",))["PCKh"]()
    x, t, lab = keypoint_task(CONV_N, 17, 64, seed=5)
    torch.manual_seed(0)
    m = ns["creatModel"]()
    opt = torch.optim.Adam(m.parameters(), lr=CONV_LR)
    crit = torch.nn.MSELoss()
    rects = {b: np.tile(np.array([0.0, 0.0, b, b]), (CONV_N, 1)) for b in CONV_BOXES}
    losses, curves, preds = [], [], None
    for step in range(1, CONV_STEPS + 1):
        m.train()
        outs = m(x)
        loss = sum(crit(o, t) for o in outs)
        opt.zero_grad()
        loss.backward()
        opt.step()
        losses.append(float(loss.detach()))
        if step % CONV_EVERY == 0:
            with torch.no_grad():
                hm = m(x)[-1]
            row = []
            for b in CONV_BOXES:
                acc, pr, _ = pk(hm, lab, rects[b])
                row.append(np.nanmean(np.asarray(acc, np.float64), axis=0))
                preds = np.stack([np.asarray(q, np.float64) for q in pr]).astype(np.int16)
            curves.append(np.stack(row))
            print(name, tag, "step", step, "loss %.6f" % losses[-1], "PCKh@0.5",
                  " ".join("%.3f" % r[10] for r in row), flush=True)
    rec = dict(np.load(path)) if os.path.exists(path) else {}
    rec.update({"n": np.array(CONV_N), "steps": np.array(CONV_STEPS), "every": np.array(CONV_EVERY),
                "lr": np.array(CONV_LR), "boxes": np.array(CONV_BOXES), "labels": lab.numpy(),
                "sd_sha256": np.array(sd_hash(build("try_with_torch.py", None))),
                f"{tag}_loss": np.array(losses), f"{tag}_pckh": np.stack(curves),
                f"{tag}_preds": preds})
    tmp = path[:-4] + ".tmp.npz"
    np.savez_compressed(tmp, **rec)
    os.replace(tmp, path)
    torch.backends.mkldnn.enabled = True
    print(name, tag, "->", path, os.path.getsize(path), "bytes")


def main():
    torch.set_num_threads(8)
    # primary 4-stack (try_with_torch.py), small input -> full outputs
    make_case("primary_s4_n2_64", "try_with_torch.py", None, 2, 64, 64, True)
    # primary 4-stack at the real resolution -> summaries + samples
    make_case("primary_s4_n2_256", "try_with_torch.py", None, 2, 256, 256, False)
    # 1-stack / 18 outputs (only_one_hourgless.py), config 1
    make_case("oneStack_s1_n2_128", "only_one_hourgless.py", None, 2, 128, 128, True)
    # real images from the reference's test_img/ (2 crops resized to 256^2)
    make_case("primary_s4_img2_256", "try_with_torch.py", None, 2, 256, 256, False,
              image_names=["images_3.jpeg", "im0026.jpg"])


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "progressive":
        main_progressive()
    elif len(sys.argv) > 1 and sys.argv[1] == "stress":
        main_stress()
    elif len(sys.argv) > 1 and sys.argv[1] == "losses":
        main_losses()
    elif len(sys.argv) > 1 and sys.argv[1] == "trainpy":
        main_trainpy()
    elif len(sys.argv) > 1 and sys.argv[1] == "morelayer":
        main_morelayer()
    elif len(sys.argv) > 1 and sys.argv[1] == "compare":
        main_compare()
    elif len(sys.argv) > 1 and sys.argv[1] == "stress8":
        main_stress8()
    elif len(sys.argv) > 1 and sys.argv[1] == "stress16":
        main_stress16()
    elif len(sys.argv) > 1 and sys.argv[1] == "twin":
        main_twin()
    elif len(sys.argv) > 1 and sys.argv[1] == "aspp256":
        main_aspp256()
    elif len(sys.argv) > 1 and sys.argv[1] == "eval32":
        main_eval32()
    elif len(sys.argv) > 1 and sys.argv[1] == "draws":
        main_draws(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
    elif len(sys.argv) > 1 and sys.argv[1] == "eval8s16":
        main_eval8s16()
    elif len(sys.argv) > 1 and sys.argv[1] == "converge":
        main_converge(sys.argv[2] if len(sys.argv) > 2 else "orig")
    elif len(sys.argv) > 1 and sys.argv[1] == "onestack256":
        main_onestack256()
    elif len(sys.argv) > 1 and sys.argv[1] == "batch32":
        main_batch32()
        main_batch32_bf16()
    else:
        main()
