"""Shared parity gates for the production-batch fixtures (SURVEY.md §8(c) rules at strided
samples). Test infrastructure only."""
import numpy as np


def sample_bound(r32, r64):
    """b = 1e-3 + 2 max|ref32 - ref64| over one stack's / head's share of the samples."""
    return 1e-3 + 2 * float(np.abs(r32 - r64).max())


def grad_norm_gate(norms, n32, n64, what=""):
    """Per-parameter grad L2 norms against the fp64 reference, on the reference's own fp32 noise:

    * the set of parameters without a gradient must match exactly;
    * each parameter within 1e-3 + 4x its noise, the noise floored at the MEDIAN relative noise of
      the live parameters (one parameter's |n32 - n64| is a single draw of the step's rounding
      noise: by chance it can be ~1e-6 relative where the median is ~1e-2), and never below the
      reference's own largest relative noise on a live parameter;
    * the median relative error within 2x the reference's median (+1e-3), and the 90th percentile
      within 2x the reference's 90th percentile (+1e-3): a real error of a few percent on a
      handful of parameters cannot hide under the floor.
    Returns (median rel err, reference median) for the log."""
    assert np.array_equal(norms < 0, n64 < 0), f"{what}: parameters with / without a gradient"
    ok = n64 >= 0
    a, a32, a64 = norms[ok], n32[ok], n64[ok]
    err = np.abs(a - a64)
    # conv biases feeding a train-mode BN have a mathematically zero grad: pure rounding noise
    floor = 1e-5 * a64.max()
    live = a64 > floor
    rel_ref = np.abs(a32 - a64) / np.maximum(a64, 1e-30)
    med_ref = float(np.median(rel_ref[live]))
    noise = np.maximum(np.abs(a32 - a64), med_ref * a64)
    # ... and never tighter than the largest relative noise the reference itself shows on a live
    # parameter: each parameter's noise is one draw from that (heavy-tailed: 8 train-mode stacks)
    # distribution, so an implementation with the same noise lands there on some parameter too
    max_ref = float(rel_ref[live].max())
    bound = np.maximum(1e-3 * a64 + 4 * noise, max_ref * a64) + floor
    worst = int(np.argmax(err / bound))
    assert np.all(err <= bound), (what, worst, float(err[worst]), float(bound[worst]),
                                  float(a64[worst]))
    rel = err[live] / a64[live]
    med = float(np.median(rel))
    print(f"{what}: grad-norm rel err median {med:.4f} p90 {np.percentile(rel, 90):.4f} max "
          f"{rel.max():.4f}; reference fp32 median {med_ref:.4f} p90 "
          f"{np.percentile(rel_ref[live], 90):.4f} max {max_ref:.4f}")
    assert med <= 2 * med_ref + 1e-3, (what, med, med_ref)
    p90, p90_ref = float(np.percentile(rel, 90)), float(np.percentile(rel_ref[live], 90))
    assert p90 <= 2 * p90_ref + 1e-3, (what, p90, p90_ref)
    return med, med_ref


def grad_cosine_gate(gs, r32, r64, slack=0.01):
    """Gradient direction over the strided samples: the engine's distance from the fp64 direction,
    1 - cosine, at most twice the reference's own fp32 distance (+ `slack`) — the rule the norm
    gate applies to the median. The reference's fp32 cosine is one draw of the step's rounding
    noise: at 8 train-mode stacks it is 0.74 (N=8) / 0.89 (N=16), so a one-draw comparison
    (cosine >= reference - 0.01, the rule before the N=16 fixture existed) measured the draw,
    not the implementation; where the reference is well-conditioned (cosine ~1) both rules agree."""
    r32 = r32.astype(np.float64)

    def cos(a, b):
        return float((a * b).sum() / (np.linalg.norm(a) * np.linalg.norm(b)))
    c, c_ref = cos(gs, r64), cos(r32, r64)
    assert 1.0 - c <= 2.0 * (1.0 - c_ref) + slack, (c, c_ref)
    return c, c_ref


def running_stats_gate(named_buffers, g):
    """BN running stats per module: noise = the module's max |ref32 - ref64|."""
    for suffix, k in (("running_mean", "bn_running_mean"), ("running_var", "bn_running_var")):
        r32_, r64_ = g[k + "32"], g[k + "64"]
        off = 0
        for name, b in named_buffers:
            if not name.endswith(suffix):
                continue
            n = b.numel()
            got = b.reshape(-1).cpu().numpy()
            a32, a64 = r32_[off:off + n], r64_[off:off + n]
            tol = 1e-4 + 1e-4 * np.abs(a64) + 4 * np.abs(a32 - a64).max()
            bad = np.abs(got - a64) > tol
            assert not bad.any(), (name, float(np.abs(got - a64).max()), float(tol.max()))
            off += n
        assert off == r64_.size
