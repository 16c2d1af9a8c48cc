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


def joint_colors(k):
    """k distinct RGB codes from {-1, 0, 1}^3 \\ {0} (k <= 26), in a fixed order."""
    codes = [(r, g, b) for r in (1, -1, 0) for g in (1, -1, 0) for b in (1, -1, 0) if (r, g, b) != (0, 0, 0)]
    if k > len(codes):
        raise ValueError(f"at most {len(codes)} joint colours")
    return torch.tensor(codes[:k], dtype=torch.float64)


def keypoint_task(n, k=17, hm=64, seed=5, margin=2, background=0.25):
    """A learnable synthetic pose batch for short-training (convergence / PCKh) runs. Per image,
    k distinct joint positions (row, col) on the hm x hm heatmap grid in [margin, hm - margin);
    the image (4 hm square, [-1, 1] like the reference's Normalize(0.5, 0.5) crops) is uniform
    noise of amplitude `background` with joint j drawn as the 4x4 input-pixel cell over its
    heatmap pixel in colour joint_colors(k)[j] — so the joints are visible and the task is
    learnable in a few hundred images' worth of steps (random keypoints on pure-noise images are
    only memorised: the MSE stalls at the all-zero heatmap). Returns (images [n, 3, 4hm, 4hm]
    fp32, sigma = 1 Gaussian heatmaps [n, k, hm, hm] fp32 as gaussian_targets, PCKh label map
    [n, hm, hm] int32 holding j at joint j's pixel for j = 1 .. k-1: train.py:775 reads channel
    j + 1 for label j + 1, so channel 0 is trained but not scored)."""
    g = torch.Generator().manual_seed(seed)
    side = hm - 2 * margin
    pos = torch.stack([torch.randperm(side * side, generator=g)[:k] for _ in range(n)])
    ys, xs = pos // side + margin, pos % side + margin
    col = torch.arange(hm, dtype=torch.float64).view(1, 1, 1, hm)
    row = torch.arange(hm, dtype=torch.float64).view(1, 1, hm, 1)
    d2 = (col - xs.view(n, k, 1, 1).double()) ** 2 + (row - ys.view(n, k, 1, 1).double()) ** 2
    maps = torch.exp(-d2 / 2.0).float()
    labels = torch.zeros(n, hm, hm, dtype=torch.int32)
    for j in range(1, k):
        labels[torch.arange(n), ys[:, j], xs[:, j]] = j
    img = (torch.rand(n, 3, 4 * hm, 4 * hm, generator=g, dtype=torch.float64) * 2 - 1) * background
    colors = joint_colors(k)
    for i in range(n):
        for j in range(k):
            r, c = 4 * int(ys[i, j]), 4 * int(xs[i, j])
            img[i, :, r:r + 4, c:c + 4] = colors[j].view(3, 1, 1)
    return img.float(), maps, labels


def class_maps(n, classes, hm=64, wm=None, seed=2):
    """Integer class maps [n, hm, wm] (int64) for the progressive heads' CrossEntropy targets
    (background 2 classes, skeleton 20: try_with_aspp.py:356-395), uniform over the classes."""
    wm = hm if wm is None else wm
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, classes, (n, hm, wm), generator=g)
