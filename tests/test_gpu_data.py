"""GPU: Gaussian target and PCKh kernels (csrc/hgk_data.hip) against the golden vectors produced
by executing the reference's code (tools/make_golden_data.py) — bit-exact — and against the
oracle (oracle/data_oracle.py) on larger random cases."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle.data_oracle import gauss_targets, pckh
from progressive_process_for_human_pose_estimation_amd.targets import PCKh, render_gaussian_targets

pytestmark = pytest.mark.gpu
D = np.load(os.path.join(GOLDEN, "data_targets_pckh.npz"))


def test_gauss_targets_bit_exact_vs_reference():
    out = render_gaussian_targets(torch.from_numpy(D["g_kps"]), torch.from_numpy(D["g_counts"]),
                                  torch.from_numpy(D["g_wh"]))
    assert np.array_equal(out.cpu().numpy(), D["g_maps"])


def test_gauss_targets_random_vs_oracle():
    rng = np.random.default_rng(3)
    B, P, K = 16, 4, 17
    wh = rng.integers(32, 1500, (B, 2)).astype(np.float32)
    kps = np.zeros((B, P, K, 3), np.float32)
    kps[..., 0] = rng.uniform(-5, 1, (B, P, K)) * wh[:, None, None, 0]   # incl. negative x
    kps[..., 1] = rng.uniform(0, 1.05, (B, P, K)) * wh[:, None, None, 1]
    kps[..., 2] = rng.integers(0, 3, (B, P, K))
    counts = rng.integers(0, P + 1, B).astype(np.int32)                 # incl. no annotation
    out = render_gaussian_targets(torch.from_numpy(kps), torch.from_numpy(counts),
                                  torch.from_numpy(wh)).cpu().numpy()
    for b in range(B):
        ref = gauss_targets(kps[b], int(counts[b]), float(wh[b, 0]), float(wh[b, 1]))
        assert np.array_equal(out[b], ref), b


def test_pckh_bit_exact_vs_reference():
    acc, preds, labels = PCKh()(torch.from_numpy(D["p_x"]), torch.from_numpy(D["p_target"]),
                                D["p_rect64"])
    np.testing.assert_array_equal(acc, D["p_acc"])
    np.testing.assert_array_equal(np.stack(preds), D["p_pred"])
    np.testing.assert_array_equal(np.stack(labels), D["p_label"])


def test_pckh_random_vs_oracle():
    rng = np.random.default_rng(5)
    B, C, Hh, W = 32, 18, 64, 64
    x = rng.standard_normal((B, C, Hh, W)).astype(np.float32)
    x[:, :, ::7, ::5] = np.round(x[:, :, ::7, ::5])  # ties
    target = np.zeros((B, Hh, W), np.int32)
    for b in range(B):
        for j in range(C - 1):
            if rng.uniform() < 0.8:
                target[b, rng.integers(0, Hh), rng.integers(0, W)] = j + 1
    rect = rng.uniform(0, 64, (B, 4))
    acc, preds, labels = PCKh()(torch.from_numpy(x), torch.from_numpy(target), rect)
    racc, rpreds, rlabels = pckh(x, target, rect)
    np.testing.assert_array_equal(acc, racc)
    np.testing.assert_array_equal(np.stack(preds), rpreds)
    np.testing.assert_array_equal(np.stack(labels), rlabels)
