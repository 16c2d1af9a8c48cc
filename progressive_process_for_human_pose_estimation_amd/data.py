"""Synthetic batches shaped like the reference's training data.

* images: the reference feeds `Normalize(mean=0.5, std=0.5)` RGB crops in [-1, 1]
  (try_with_torch.py:310-313) -> here `rand(N,3,H,W) * 2 - 1` from a seeded generator;
* targets: K Gaussian heatmaps at H/4 x W/4, sigma = 1, peak 1, as rendered by
  `myImageDataset_COCO.__getitem__` (try_with_torch.py:104-130):
  map[k, row, col] = exp(-((col - x_k)^2 + (row - y_k)^2) / 2), integer (x_k, y_k), an
  all-zero map for an invisible joint (v_k == 0, :115).
There is no network and no MPII/COCO here, so these stand in for the crops.
"""
import torch


def synthetic_images(n, h=256, w=256, seed=1234, dtype=torch.float32):
    g = torch.Generator().manual_seed(seed)
    return (torch.rand(n, 3, h, w, generator=g, dtype=torch.float64) * 2 - 1).to(dtype)


def gaussian_targets(n, k=17, hm=64, wm=None, seed=1, visible_prob=1.0, sigma=1.0,
                     dtype=torch.float32):
    """Reference-style Gaussian heatmaps [n, k, hm, wm] (try_with_torch.py:114-130)."""
    wm = hm if wm is None else wm
    g = torch.Generator().manual_seed(seed)
    xs = torch.randint(0, wm, (n, k), generator=g)
    ys = torch.randint(0, hm, (n, k), generator=g)
    vis = torch.rand(n, k, generator=g) < visible_prob
    col = torch.arange(wm, dtype=torch.float64).view(1, 1, 1, wm)
    row = torch.arange(hm, dtype=torch.float64).view(1, 1, hm, 1)
    d2 = (col - xs.view(n, k, 1, 1).double()) ** 2 + (row - ys.view(n, k, 1, 1).double()) ** 2
    maps = torch.exp(-d2 / (2 * sigma ** 2)) * vis.view(n, k, 1, 1).double()
    return maps.to(dtype), xs, ys, vis


def class_maps(n, classes, hm=64, wm=None, seed=2):
    """Integer class maps [n, hm, wm] (int64) for the progressive heads' CrossEntropy targets
    (background 2 classes, skeleton 20: try_with_aspp.py:356-395), uniform over the classes."""
    wm = hm if wm is None else wm
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, classes, (n, hm, wm), generator=g)
