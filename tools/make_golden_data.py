"""Golden vectors for the two components either side of the hot path,
produced by EXECUTING the reference's own code (build container only; tools/ never ships):

* Gaussian heatmap targets: `myImageDataset_COCO.__getitem__` (try_with_torch.py:93-130), run on
  the reference's own test images with a stub annotation object (pycocotools is absent) that
  serves synthetic keypoints. numpy 2 no longer has `np.int` (used at :110-111): the namespace
  gets a numpy proxy with `int` mapped to the builtin (what `np.int` was: an alias).
* PCKh@{0,0.05..0.5}: `PCKh.forward` (train.py:759-791) on synthetic predictions with exact
  ties, label maps with missing joints and head rectangles.

Writes tests/golden/data_targets_pckh.npz.
"""
import os
import sys
import types

import numpy as np
import numpy.matlib  # noqa: F401  (the reference calls np.matlib.repmat)
import torch
import torch.utils.data as tdata
from PIL import Image, ImageDraw

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from ref_loader import REF_ROOT, load_reference  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                   "data_targets_pckh.npz")


class _NumpyProxy(types.ModuleType):
    def __getattr__(self, name):
        if name == "int":
            return int
        return getattr(np, name)


class _StubCOCO:
    """what __getitem__ asks of pycocotools.COCO: loadImgs / getAnnIds / loadAnns"""

    def __init__(self, files, anns):
        self.files, self.anns = files, anns

    def loadImgs(self, i):
        return [{"file_name": self.files[i]}]

    def getAnnIds(self, i):
        return i

    def loadAnns(self, i):
        return self.anns[i]


def gaussian_cases(rng):
    files = sorted(os.listdir(os.path.join(REF_ROOT, "test_img")))
    cases = []
    for i, f in enumerate(files):
        w, h = Image.open(os.path.join(REF_ROOT, "test_img", f)).size
        n_people = [1, 2, 3, 1, 2, 1, 3][i % 7]
        anns = []
        for p in range(n_people):
            kp = np.zeros(17 * 3)
            kp[0::3] = rng.uniform(0, w, 17)
            kp[1::3] = rng.uniform(0, h, 17)
            kp[2::3] = rng.integers(0, 3, 17)           # v in {0,1,2}
            if i == 2 and p == n_people - 1:            # edges: exactly at w / h and 0
                kp[0:6] = [w, h, 2, 0.0, 0.0, 1]
            kp = kp.astype(np.float32).astype(np.float64)  # what the float32 fixture holds
            anns.append({"keypoints": kp.tolist()})
        cases.append((f, w, h, anns))
    return cases


def make_gauss(rng):
    ns = load_reference("try_with_torch.py", class_names=("myImageDataset_COCO",),
                        pre={"data": tdata})
    ns.update({"np": _NumpyProxy("numpy"), "Image": Image, "ImageDraw": ImageDraw,
               "path": os.path, "keypoints": 17})
    Dataset = ns["myImageDataset_COCO"]
    cases = gaussian_cases(rng)
    ds = Dataset.__new__(Dataset)  # __init__ needs COCO(anno_file)
    ds.anno = _StubCOCO([c[0] for c in cases], [c[3] for c in cases])
    ds.image_dir = os.path.join(REF_ROOT, "test_img")
    ds.lists = list(range(len(cases)))
    ds.transform = lambda im: im
    maps, kps, counts, whs = [], [], [], []
    maxp = max(len(c[3]) for c in cases)
    for i, (f, w, h, anns) in enumerate(cases):
        _, target = ds[i]
        maps.append(target.numpy())
        k = np.zeros((maxp, 17, 3), np.float32)
        for p, a in enumerate(anns):
            k[p] = np.asarray(a["keypoints"], np.float32).reshape(17, 3)
        kps.append(k)
        counts.append(len(anns))
        whs.append((w, h))
    return {"g_maps": np.stack(maps).astype(np.float32), "g_kps": np.stack(kps),
            "g_counts": np.asarray(counts, np.int32), "g_wh": np.asarray(whs, np.float32)}


def make_pckh(rng):
    ns = load_reference("train.py", class_names=("PCKh",))
    pckh = ns["PCKh"]()
    B, C, H, W = 6, 17, 64, 64
    x = rng.standard_normal((B, C, H, W)).astype(np.float32)
    x[0, 3] = 0.0                                  # all-equal channel: first index wins
    x[1, 5, 10, 10] = x[1, 5, 20, 7] = x[1, 5].max() + 1.0   # exact tie
    target = np.zeros((B, H, W), np.int64)
    for b in range(B):
        for j in range(C - 1):
            if rng.uniform() < 0.15:
                continue                            # joint absent -> skipped
            r, c = rng.integers(0, H), rng.integers(0, W)
            target[b, r, c] = j + 1
            if rng.uniform() < 0.2:                 # duplicate label: first row-major counts
                target[b, rng.integers(0, H), rng.integers(0, W)] = j + 1
    # about 60 % of the labelled joints get their prediction peak within a few pixels of the
    # label, so the 11 thresholds are all exercised
    for b in range(B):
        for j in range(C - 1):
            hit = np.argwhere(target[b] == j + 1)
            if len(hit) and rng.uniform() < 0.6 and not (b == 0 and j + 1 == 3):
                r, c = hit[0] + rng.integers(-4, 5, 2)
                x[b, j + 1, min(max(r, 0), H - 1), min(max(c, 0), W - 1)] = 10.0
    rect = rng.uniform(0, 64, (B, 4)).astype(np.float64)
    rect[2] = [10.0, 10.0, 10.0, 10.0]              # zero-size head: distance = inf / nan
    acc, preds, labels = pckh(torch.from_numpy(x), torch.from_numpy(target), rect)
    return {"p_x": x, "p_target": target.astype(np.int32), "p_rect": rect.astype(np.float32),
            "p_rect64": rect, "p_acc": np.asarray(acc, np.float64),
            "p_pred": np.stack(preds).astype(np.int32), "p_label": np.stack(labels).astype(np.int32)}


def main():
    rng = np.random.default_rng(7)
    out = make_gauss(rng)
    out.update(make_pckh(rng))
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
