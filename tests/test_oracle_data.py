"""CPU: the data-side oracle (Gaussian targets, PCKh) against golden vectors produced by running
the reference's own code (tools/make_golden_data.py)."""
import os

import numpy as np

from conftest import GOLDEN
from oracle.data_oracle import gauss_targets, pckh

D = np.load(os.path.join(GOLDEN, "data_targets_pckh.npz"))


def test_gauss_targets_match_reference_dataset():
    for i in range(len(D["g_counts"])):
        w, h = D["g_wh"][i]
        got = gauss_targets(D["g_kps"][i], int(D["g_counts"][i]), float(w), float(h))
        assert np.array_equal(got, D["g_maps"][i]), i


def test_pckh_matches_reference_module():
    acc, preds, labels = pckh(D["p_x"], D["p_target"], D["p_rect64"])
    np.testing.assert_array_equal(acc, D["p_acc"])
    np.testing.assert_array_equal(preds, D["p_pred"])
    np.testing.assert_array_equal(labels, D["p_label"])
