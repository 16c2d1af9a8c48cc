"""GPU Gaussian heatmap targets (try_with_torch.py:104-130) and PCKh (train.py:759-791).

Drop-in for the two steps either side of the training path: the
reference renders targets with numpy on data-loader workers and evaluates PCKh with per-joint
Python loops; here both are HIP kernels (csrc/hgk_data.hip) with the reference's exact semantics
(tests/test_gpu_data.py pins them bit for bit against vectors produced by running the reference).
"""
import numpy as np
import torch
import torch.nn as nn

from . import hgk as H


def render_gaussian_targets(kps, counts, wh, hm=64, wm=64, sigma=1.0):
    """kps [B, P, K, 3] (x, y, v) in original-image pixels, counts [B] annotations per image,
    wh [B, 2] original image (w, h) -> float32 heatmaps [B, K, hm, wm] on the GPU.
    Reference semantics: only the last annotation of an image survives (:113)."""
    L = H.lib()
    kps = kps.to("cuda", torch.float32).contiguous()
    counts = counts.to("cuda", torch.int32).contiguous()
    wh = wh.to("cuda", torch.float32).contiguous()
    B, P, K, _ = kps.shape
    out = torch.empty(B, K, hm, wm, dtype=torch.float32, device="cuda")
    H.check(L.hgk_gauss_targets(H.stream_handle(), kps.data_ptr(), counts.data_ptr(), wh.data_ptr(),
                                B, P, K, hm, wm, float(sigma), out.data_ptr()))
    return out


def pckh_gpu(x, target, rect):
    """(acc [B, 11] float64, preds [B, C, 2] int32 (x, y), labels [B, C, 2] int32), on the GPU."""
    L = H.lib()
    x = x.detach().to("cuda", torch.float32).contiguous()
    target = target.to("cuda", torch.int32).contiguous()
    rect = torch.as_tensor(np.asarray(rect, np.float64)).to("cuda").contiguous()
    B, C, Hh, W = x.shape
    preds = torch.empty(B, C, 2, dtype=torch.int32, device="cuda")
    labels = torch.empty_like(preds)
    scratch = torch.empty(B, C, dtype=torch.int32, device="cuda")
    acc = torch.empty(B, 11, dtype=torch.float64, device="cuda")
    H.check(L.hgk_pckh(H.stream_handle(), x.data_ptr(), target.data_ptr(), rect.data_ptr(), B, C,
                       Hh, W, preds.data_ptr(), labels.data_ptr(), scratch.data_ptr(),
                       acc.data_ptr()))
    return acc, preds, labels


class PCKh(nn.Module):
    """train.py:759-791 surface: forward(x, target, rect) -> (accuracy ndarray [B, 11],
    predicts list of [C, 2] arrays (x, y), labels list of [C, 2] arrays)."""

    def forward(self, x, target, rect):
        acc, preds, labels = pckh_gpu(x, target, rect)
        preds = preds.cpu().numpy().astype(np.float64)
        labels = labels.cpu().numpy().astype(np.float64)
        return acc.cpu().numpy(), list(preds), list(labels)
