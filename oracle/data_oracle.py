"""CPU ORACLE — test infrastructure only, never the product path.

numpy restatements of the two components either side of the hot path.
Imported only by tests/ as the checker of the HIP kernels in csrc/hgk_data.hip.

Parity pin: tests/golden/data_targets_pckh.npz was produced by EXECUTING the reference's code
(tools/make_golden_data.py: `myImageDataset_COCO.__getitem__` with a stub annotation object on the
reference's test images, and `PCKh.forward`); tests/test_oracle_data.py checks this restatement
against it bit for bit.
"""
import numpy as np


def gauss_targets(kps, count, w, h, hm=64, wm=64, sigma=1.0, k=17):
    """try_with_torch.py:104-130. kps [P][k][3] = (x, y, v) in original-image pixels.

    * `Gauss_map` is re-created inside the per-annotation loop (:113), so only the LAST
      annotation's joints survive;
    * joint coordinates are truncated toward zero after scaling to the 64-wide map (:110-111,
      `np.array(kp/w*64).astype(np.int)`; the map size is hard-wired to 64 there);
    * a joint with v == 0 leaves an all-zero map (:115);
    * map[k][row][col] = exp(-((col-x)^2 + (row-y)^2) / (2 sigma^2)) in float64 (:117-128), returned
      as float32 (`torch.Tensor`, :130)."""
    out = np.zeros((k, hm, wm), np.float64)
    if count <= 0:
        return out.astype(np.float32)
    kp = np.asarray(kps[count - 1], np.float64)
    x = (kp[:, 0] / w * wm).astype(np.int64)
    y = (kp[:, 1] / h * hm).astype(np.int64)
    col = np.tile(np.arange(wm), (hm, 1))
    row = np.tile(np.arange(hm), (wm, 1)).T
    for j in range(k):
        if kp[j, 2] > 0:
            out[j] = np.exp(-(((col - x[j]) ** 2 + (row - y[j]) ** 2) / (2 * sigma ** 2)))
    return out.astype(np.float32)


THRESHOLDS = np.arange(0, 0.55, 0.05)  # train.py:784


def pckh(x, target, rect):
    """train.py:759-791. x [B][C][H][W] float32 heatmaps (channel j+1 <-> joint j), target
    [B][H][W] int label map (value j+1 marks joint j), rect [B][4] head box (float64).

    Per joint j: label = first row-major pixel with target == j+1 (joint skipped if none);
    prediction = first row-major pixel of channel j+1 at its maximum; distance (float32 tensor
    arithmetic in the reference) = sqrt(dy^2 + dx^2) / (0.6 * |head diagonal|); correct at
    threshold k iff distance < k. Returns (accuracy [B][11], predicts [B][C][2] (x, y),
    labels [B][C][2]) — accuracy = correct / total per image (nan when no joint is labelled)."""
    B, C, H, W = x.shape
    acc = np.zeros((B, len(THRESHOLDS)))
    preds = np.zeros((B, C, 2), np.int64)
    labels = np.zeros((B, C, 2), np.int64)
    for i in range(B):
        correct = np.zeros(len(THRESHOLDS))
        total = np.zeros(len(THRESHOLDS))
        standard = np.sqrt((rect[i][0] - rect[i][2]) ** 2 + (rect[i][1] - rect[i][3]) ** 2) * 0.6
        for j in range(C):
            hit = np.flatnonzero(target[i].reshape(-1) == j + 1)
            if len(hit) == 0:
                continue
            ly, lx = divmod(int(hit[0]), W)
            ch = x[i, j + 1].reshape(-1)
            py, px = divmod(int(np.flatnonzero(ch >= ch.max())[0]), W)
            d2 = (ly - py) ** 2 + (lx - px) ** 2
            with np.errstate(divide="ignore", invalid="ignore"):
                dist = np.float32(np.sqrt(np.float32(d2))) / np.float32(standard)
            for s, k in enumerate(THRESHOLDS):
                if dist < np.float32(k):
                    correct[s] += 1
                total[s] += 1
            preds[i, j] = (px, py)
            labels[i, j] = (lx, ly)
        with np.errstate(divide="ignore", invalid="ignore"):
            acc[i] = correct / total
    return acc, preds, labels
