"""Pin the CPU oracle (oracle/hourglass_oracle.py) to the reference's own outputs.

The fixtures were produced by tests/golden/make_golden.py from the reference classes
(/root/reference/try_with_torch.py:179-298, only_one_hourgless.py:215-254). This is what makes the
oracle trustworthy as the parity checker for the HIP engine."""
import hashlib
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle.hourglass_oracle import OracleModel, OracleProgressive, progressive_loss, stack_mse
from oracle.hourglass_oracle import OracleTrainModel, trainpy_loss

CASES = {
    "primary_s4_n2_64": dict(nStack=4, nOutChannels=17),
    "oneStack_s1_n2_128": dict(nStack=1, nOutChannels=18),
    "primary_s4_n2_256": dict(nStack=4, nOutChannels=17),
}


def sd_hash(model):
    h = hashlib.sha256()
    for k, v in model.state_dict().items():
        h.update(k.encode())
        h.update(str(tuple(v.shape)).encode())
        h.update(v.detach().cpu().contiguous().numpy().tobytes())
    return h.hexdigest()


def load(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz")))


def build(cfg, dtype=torch.float32):
    torch.manual_seed(0)
    return OracleModel(**cfg).to(dtype)


@pytest.mark.parametrize("name", list(CASES))
def test_state_dict_identical(name):
    g = load(name)
    m = build(CASES[name])
    assert sd_hash(m) == str(g["sd_sha256"])
    assert [k for k, _ in m.named_parameters()] == list(g["param_names"])


@pytest.mark.parametrize("name", ["primary_s4_n2_64", "oneStack_s1_n2_128"])
def test_oracle_matches_reference_train_and_eval(name):
    torch.set_num_threads(8)
    g = load(name)
    cfg = CASES[name]
    x = torch.from_numpy(g["x"])
    t = torch.from_numpy(g["target"])
    m = build(cfg).eval()
    with torch.no_grad():
        ev = torch.stack(m(x)).numpy()
    np.testing.assert_allclose(ev, g["eval32"], rtol=0, atol=1e-5)

    m = build(cfg).train()
    outs = m(x)
    loss = stack_mse(outs, t)
    loss.backward()
    o = torch.stack([q.detach() for q in outs]).numpy()
    # same aten ops in the same order -> agreement at the fp32 noise floor
    np.testing.assert_allclose(o, g["train32"], rtol=0, atol=2e-4)
    assert abs(float(loss.detach()) - float(g["loss32"])) < 1e-5 * max(1.0, float(g["loss32"]))
    norms = np.array([-1.0 if p.grad is None else float(p.grad.norm()) for p in m.parameters()])
    ref = g["grad_norm32"]
    assert np.array_equal(norms < 0, ref < 0), "set of params without grad differs"
    np.testing.assert_allclose(norms[norms >= 0], ref[ref >= 0], rtol=2e-3, atol=1e-6)
    rm = torch.cat([b.reshape(-1) for k, b in m.named_buffers() if k.endswith("running_mean")])
    rv = torch.cat([b.reshape(-1) for k, b in m.named_buffers() if k.endswith("running_var")])
    nbt = [int(b) for k, b in m.named_buffers() if k.endswith("num_batches_tracked")]
    np.testing.assert_allclose(rm.detach().numpy(), g["bn_running_mean32"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(rv.detach().numpy(), g["bn_running_var32"], rtol=1e-4, atol=1e-5)
    assert nbt == list(g["bn_num_batches_tracked"])


def test_oracle_256_summary():
    torch.set_num_threads(8)
    g = load("primary_s4_n2_256")
    x = torch.from_numpy(g["x"])
    m = build(CASES["primary_s4_n2_256"]).train()
    o = torch.stack([q.detach() for q in m(x)]).numpy()
    np.testing.assert_allclose(o.reshape(-1)[::16], g["train32_sample"], rtol=0, atol=1e-3)
    am = o.reshape(o.shape[0], o.shape[1], o.shape[2], -1).argmax(-1)
    sure = g["train32_gap"] > 1e-3
    assert np.array_equal(am[sure], g["train32_argmax"][sure])


@pytest.mark.parametrize("name,aspp", [("aspp_s3_n2_128", True), ("diffstack_s3_n2_128", False)])
def test_progressive_oracle_matches_reference(name, aspp):
    """oracle OracleProgressive (try_with_aspp.py:299-343 / try_different_stack.py:282-330)
    against fixtures from the reference classes themselves"""
    torch.set_num_threads(8)
    g = load(name)
    torch.manual_seed(0)
    m = OracleProgressive(aspp=aspp)
    assert sd_hash(m) == str(g["sd_sha256"])
    x = torch.from_numpy(g["x"])
    m.train()
    outs = m(x)
    loss = progressive_loss(outs, torch.from_numpy(g["bg"]), torch.from_numpy(g["skeleton"]),
                            torch.from_numpy(g["keypoints"]))
    loss.backward()
    for i, o in enumerate(outs):
        np.testing.assert_allclose(o.detach().numpy(), g[f"train32_{i}"], rtol=0, atol=2e-4)
    assert abs(float(loss.detach()) - float(g["loss32"])) < 1e-5 * max(1.0, float(g["loss32"]))
    norms = np.array([-1.0 if p.grad is None else float(p.grad.norm()) for p in m.parameters()])
    ref = g["grad_norm32"]
    assert np.array_equal(norms < 0, ref < 0)
    np.testing.assert_allclose(norms[norms >= 0], ref[ref >= 0], rtol=2e-3, atol=1e-6)


def test_morelayer_oracle_matches_reference():
    """try_more_layer.py (live innermost ASPP: dilated 3x3s, image-pool branch with BN over the N
    pooled rows, bilinear-ac broadcast, 1280 -> 256 conv1; 4 stacks, `elif i >= 2`): oracle vs the
    reference's own outputs / loss / grad norms"""
    torch.set_num_threads(8)
    g = load("morelayer_s4_n2_128")
    torch.manual_seed(0)
    m = OracleProgressive(nStack=4, aspp=True, aspp_live=True, late_heads=True)
    assert sd_hash(m) == str(g["sd_sha256"])
    x = torch.from_numpy(g["x"])
    m.train()
    outs = m(x)
    assert len(outs) == 4
    loss = progressive_loss(outs, torch.from_numpy(g["bg"]), torch.from_numpy(g["skeleton"]),
                            torch.from_numpy(g["keypoints"]))
    loss.backward()
    for i, o in enumerate(outs):
        np.testing.assert_allclose(o.detach().numpy(), g[f"train32_{i}"], rtol=0, atol=2e-4)
    assert abs(float(loss.detach()) - float(g["loss32"])) < 1e-5 * max(1.0, float(g["loss32"]))
    norms = np.array([-1.0 if p.grad is None else float(p.grad.norm()) for p in m.parameters()])
    ref = g["grad_norm32"]
    assert np.array_equal(norms < 0, ref < 0)
    np.testing.assert_allclose(norms[norms >= 0], ref[ref >= 0], rtol=2e-3, atol=1e-6)
    torch.manual_seed(0)
    m = OracleProgressive(nStack=4, aspp=True, aspp_live=True, late_heads=True).eval()
    with torch.no_grad():
        ev = m(x)
    for i, o in enumerate(ev):
        np.testing.assert_allclose(o.numpy(), g[f"eval32_{i}"], rtol=0, atol=1e-4)


def test_trainpy_oracle_matches_reference():
    """train.py (stride-2 residual blocks, unshared hourglass with the live ASPP_Block, nearest x2
    + concat, 3 stages; bootstrapped top-k CE + CE): oracle vs the reference's own outputs, loss
    (its Costomer_CrossEntropyLoss), grad norms"""
    torch.set_num_threads(8)
    g = load("trainpy_s3_n2_128")
    torch.manual_seed(0)
    m = OracleTrainModel()
    assert sd_hash(m) == str(g["sd_sha256"])
    x = torch.from_numpy(g["x"])
    outs = m.train()(x)
    loss = trainpy_loss(outs, torch.from_numpy(g["skeleton"]), torch.from_numpy(g["keypoints"]),
                        float(g["fraction"]))
    loss.backward()
    for i, o in enumerate(outs):
        np.testing.assert_allclose(o.detach().numpy(), g[f"train32_{i}"], rtol=0, atol=2e-4)
    assert abs(float(loss.detach()) - float(g["loss32"])) < 1e-5 * max(1.0, float(g["loss32"]))
    norms = np.array([-1.0 if p.grad is None else float(p.grad.norm()) for p in m.parameters()])
    ref = g["grad_norm32"]
    assert np.array_equal(norms < 0, ref < 0)
    np.testing.assert_allclose(norms[norms >= 0], ref[ref >= 0], rtol=2e-3, atol=1e-6)
    torch.manual_seed(0)
    with torch.no_grad():
        ev = OracleTrainModel().eval()(x)
    for i, o in enumerate(ev):
        np.testing.assert_allclose(o.numpy(), g[f"eval32_{i}"], rtol=0, atol=1e-4)


LOSS_CASES = [("ce_boot_0.5", "logits"), ("ce_boot_0.05", "logits"), ("ce_mask", "logits"),
              ("mse_mask", "x"), ("mse_boot_0.5", "x"), ("mse_boot_0.1", "x")]


@pytest.mark.parametrize("tag,which", LOSS_CASES)
def test_loss_oracles_match_reference(tag, which):
    """train.py:343-408 loss restatements vs the reference's own loss classes (fp64 values and
    input gradients, tests/golden/losses_trainpy.npz)"""
    from oracle.hourglass_oracle import bootstrapped_ce, bootstrapped_mse, masked_ce, masked_mse
    g = load("losses_trainpy")
    cls, mask = torch.from_numpy(g["cls"]), torch.from_numpy(g["mask"])
    tgt = torch.from_numpy(g["tgt"]).double()
    a = torch.from_numpy(g[which]).double().requires_grad_()
    fn = {"ce_boot_0.5": lambda: bootstrapped_ce(a, cls, 0.5),
          "ce_boot_0.05": lambda: bootstrapped_ce(a, cls, 0.05),
          "ce_mask": lambda: masked_ce(a, cls, mask),
          "mse_mask": lambda: masked_mse(a, tgt, mask),
          "mse_boot_0.5": lambda: bootstrapped_mse(a, tgt, 0.5),
          "mse_boot_0.1": lambda: bootstrapped_mse(a, tgt, 0.1)}[tag]
    loss = fn()
    loss.backward()
    assert abs(float(loss.detach()) - float(g[tag + "_loss"])) < 1e-12
    np.testing.assert_allclose(a.grad.numpy(), g[tag + "_grad"], rtol=0, atol=1e-14)


def test_oracle_8stack_384_summary():
    """BASELINE configs[4] shape (8 stacks, 384x384) at N=1: oracle vs the reference's outputs."""
    from progressive_process_for_human_pose_estimation_amd.data import synthetic_images
    torch.set_num_threads(8)
    g = load("primary_s8_n1_384")
    x = synthetic_images(1, 384, 384, seed=1234)
    m = build(dict(nStack=8, nOutChannels=17)).train()
    o = torch.stack([q.detach() for q in m(x)]).numpy()
    np.testing.assert_allclose(o.reshape(-1)[::16], g["train32_sample"], rtol=0, atol=1e-3)
    am = o.reshape(8, 1, 17, -1).argmax(-1)
    sure = g["train32_gap"] > 1e-3
    assert np.array_equal(am[sure], g["train32_argmax"][sure])


def test_hgcompare_oracle_matches_reference():
    """OracleHGCompare (hourglass_compare.py:405-638) against the reference classes' outputs"""
    from oracle.hourglass_oracle import OracleHGCompare
    torch.set_num_threads(8)
    g = load("hgcompare_s4_n2_128")
    torch.manual_seed(0)
    m = OracleHGCompare()
    assert sd_hash(m) == str(g["sd_sha256"])
    m.train()
    outs = m(torch.from_numpy(g["x"]))
    loss = stack_mse(outs, torch.from_numpy(g["target"]))
    loss.backward()
    np.testing.assert_allclose(torch.stack([o.detach() for o in outs]).numpy(), g["train32"],
                               rtol=0, atol=2e-4)
    assert abs(float(loss.detach()) - float(g["loss32"])) < 1e-5 * max(1.0, float(g["loss32"]))
    norms = np.array([-1.0 if p.grad is None else float(p.grad.norm()) for p in m.parameters()])
    ref = g["grad_norm32"]
    assert np.array_equal(norms < 0, ref < 0)
    np.testing.assert_allclose(norms[norms >= 0], ref[ref >= 0], rtol=2e-3, atol=1e-6)
