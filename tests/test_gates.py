"""CPU checks of the production-batch gradient gates (tests/gates.py) on the fixtures themselves:
every fp32 draw of the reference inside the envelope passes, and a gradient with a real error —
one large parameter's gradient scaled beyond the draws' spread, or the direction rotated — fails. Test
infrastructure only (no GPU)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from gates import NCHW_DRAWS, eval_grad_gate, fp32_draws, grad_spread_gate, grad_spread_median

FIXTURES = ["primary_s4_n32_256", "primary_s8_n8_384", "primary_s8_n16_384"]


def load(name):
    path = os.path.join(GOLDEN, name + ".npz")
    if not os.path.exists(path):
        pytest.skip(f"{name} missing")
    return dict(np.load(path))


@pytest.mark.parametrize("name", FIXTURES)
def test_fixture_holds_reference_draws(name):
    g = load(name)
    names = [d[0] for d in fp32_draws(g)]
    assert names[0] == "orig" and len(names) >= 3, names
    for d in names[1:]:
        assert g[f"draw32_{d}_grad_norm"].shape == g["grad_norm32"].shape
        assert g[f"draw32_{d}_grad_sample"].shape == g["grad_sample32"].shape
        assert np.array_equal(g[f"draw32_{d}_grad_norm"] < 0, g["grad_norm64"] < 0)


@pytest.mark.parametrize("name", FIXTURES)
def test_reference_draws_pass_their_own_gate(name):
    g = load(name)
    for d, n, s in fp32_draws(g):
        grad_spread_gate(n.copy(), s.astype(np.float64), g, f"{name} {d}")


# a factor the reference's own draws never show on one parameter: batch 32 draws stay within 3 %,
# the 8-stack ones reach 23.5 % (N=8, one thread) - the 8-stack gates only catch gross errors
@pytest.mark.parametrize("name,scale", [("primary_s4_n32_256", 1.1), ("primary_s8_n8_384", 1.5),
                                        ("primary_s8_n16_384", 1.5)])
def test_gate_catches_a_scaled_parameter_gradient(name, scale):
    g = load(name)
    n = g["grad_norm32"].copy()
    big = int(np.argmax(n))
    n[big] *= scale
    with pytest.raises(AssertionError):
        grad_spread_gate(n, g["grad_sample32"].astype(np.float64), g, name)


def test_gate_catches_a_wrong_direction():
    g = load("primary_s4_n32_256")
    s = g["grad_sample32"].astype(np.float64)
    rng = np.random.default_rng(0)
    noise = rng.standard_normal(s.shape) * np.linalg.norm(s) / np.sqrt(s.size)
    with pytest.raises(AssertionError):
        grad_spread_gate(g["grad_norm32"].copy(), s + 0.3 * noise, g, "rotated")


def test_envelope_is_the_nchw_family():
    assert set(NCHW_DRAWS) == {"t1", "t3", "nomkl", "avx2", "sse41"}


def test_eval_mode_gate_passes_the_reference_fp32_and_catches_errors():
    g = load("primary_s8_n16_384")
    if "evalgrad_norm64" not in g:
        pytest.skip("no eval-mode gradients (make_golden.py eval8s16)")
    n32, s32 = g["evalgrad_norm32"].copy(), g["evalgrad_sample32"].astype(np.float64)
    eval_grad_gate(n32, s32, g, "reference fp32")
    bad = n32.copy()
    bad[int(np.argmax(bad))] *= 1.002  # 0.2 % on one parameter
    with pytest.raises(AssertionError):
        eval_grad_gate(bad, s32, g, "scaled")
    rng = np.random.default_rng(1)
    with pytest.raises(AssertionError):
        eval_grad_gate(n32, s32 + 3e-3 * np.abs(s32).max() * rng.standard_normal(s32.shape), g, "rotated")


def test_n16_train_median_record_numbers():
    """the N=16 strict-xfail record compares against the worst NCHW draw's median (0.032, round 5)"""
    g = load("primary_s8_n16_384")
    med, med_w = grad_spread_median(g["grad_norm32"], g)
    assert med <= med_w and 0.02 < med_w < 0.05, (med, med_w)


def test_bf16_out_close_catches_small_element_errors():
    """the per-element bf16 bound passes RNE-rounded outputs (and a flipped stored intermediate)
    but catches a wrong value on a small-magnitude element that a 1e-2 max|ref| bound accepts"""
    import torch
    from gates import bf16_out_close
    g = torch.Generator().manual_seed(0)
    ref = torch.randn(4096, generator=g, dtype=torch.float64) * torch.logspace(-3, 1, 4096, dtype=torch.float64)
    y = ref.to(torch.bfloat16)
    bf16_out_close(y, ref)
    bad = y.clone()
    i = int(ref.abs().argmin())
    bad[i] = bad[i] + 0.05 * float(ref.abs().max()) * 1e-1   # well under 1e-2 max|ref|
    assert (bad.double() - ref).abs().max() <= 1e-2 * ref.abs().max()
    with pytest.raises(AssertionError):
        bf16_out_close(bad, ref)
    # residual after a stored conv output: one ulp of the conv may flip
    conv = torch.full((8,), 2.0 + 2 ** -7, dtype=torch.float64)  # a bf16 rounding midpoint
    res = torch.full((8,), -1.9, dtype=torch.float64)
    exact = conv + res
    stored_other = torch.full((8,), 2.0 + 2 ** -6, dtype=torch.float64)  # rounded up instead
    bf16_out_close((stored_other + res).to(torch.bfloat16), exact, stored=conv)


def test_ulp_perturbed_moves_exactly_count_elements_by_one_ulp():
    import torch
    from gates import ulp_perturbed
    x = torch.rand(2, 3, 16, 16) * 2 - 1
    y = ulp_perturbed(x, 7, count=50)
    moved = (y != x).reshape(-1)
    assert int(moved.sum()) == 50
    a, b = x.reshape(-1)[moved], y.reshape(-1)[moved]
    assert torch.equal(torch.nextafter(a, b), b)  # exactly one representable step
    assert torch.equal(ulp_perturbed(x, 7, count=50), y)  # seeded


def test_draw_ensemble_gate_uses_the_worst_reference_draw():
    from gates import _norm_stats, draw_ensemble_median_gate
    path = os.path.join(GOLDEN, "primary_s8_n16_384.npz")
    g = np.load(path)
    worst = max(_norm_stats(n, g["grad_norm64"])[0] for _, n, _ in fp32_draws(g))
    draw_ensemble_median_gate([worst, worst + 1e-3], g, "at the bound")
    with pytest.raises(AssertionError):
        draw_ensemble_median_gate([worst + 2.5e-3] * 3, g, "over the bound")
