"""Per-module-group comparison of the configs[4] N=16 train-mode fp32 gradients against fp64:
the engine's routings (scripts/engine_draws.py output) next to every reference fp32 draw of the
fixture (tests/golden/make_golden.py draws). Cosine over the strided grad samples and the median
relative norm error, per group of parameters (stem blocks, each hourglass depth, heads).
usage: python scripts/draw_compare.py profiles/r05_draws/engine_draws_s8_n16.npz"""
import collections
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
from gates import NCHW_DRAWS, OTHER_DRAWS, _cos, fp32_draws  # noqa: E402


def group_of(name):
    parts = name.split(".")
    if parts[0].startswith("hourglass"):
        depth = sum(1 for q in parts if q in ("low2", "hg"))
        return f"hourglass depth {depth}"
    return parts[0]


def main():
    g = np.load(os.path.join(ROOT, "tests", "golden", "primary_s8_n16_384.npz"))
    e = np.load(sys.argv[1])
    n64, s64, names = g["grad_norm64"], g["grad_sample64"], list(g["param_names"])
    import progressive_process_for_human_pose_estimation_amd as P
    sizes = [p.numel() for p in P.creatModel(nStack=8).parameters()]
    ok = n64 >= 0
    lens = [len(range(0, nm, 97)) for nm, o in zip(sizes, ok) if o]
    offs = np.cumsum([0] + lens)
    live = [k for k, o in zip(names, ok) if o]
    cols = [(f"engine {k[:-12]}", e[k], e[k[:-12] + "_grad_norm"]) for k in e.files if k.endswith("_grad_sample")]
    cols += [(f"ref {d}", s, nn) for d, nn, s in fp32_draws(g, NCHW_DRAWS + OTHER_DRAWS)]
    grp = collections.defaultdict(list)
    for i, k in enumerate(live):
        grp[group_of(k)].append(i)
    print("overall: " + "  ".join(f"{c}: cos {_cos(s, s64):.4f}" for c, s, _ in cols))
    print(f"{'group':24s} " + " ".join(f"{c[:14]:>14s}" for c, _, _ in cols))
    w = n64[ok]
    for key, idx in sorted(grp.items()):
        row = []
        for _, s, nn in cols:
            cs, ws = [], []
            for i in idx:
                a, b = s[offs[i]:offs[i + 1]], s64[offs[i]:offs[i + 1]]
                if np.linalg.norm(b) > 0 and np.linalg.norm(a) > 0:
                    cs.append(_cos(a, b))
                    ws.append(w[i])
            big = [i for i in idx if w[i] > 1e-5 * w.max()]  # not the mathematically-zero biases
            rel = np.abs(nn[ok][big] - w[big]) / w[big]
            row.append(f"{np.average(cs, weights=ws):.3f}/{np.median(rel):.3f}")
        print(f"{key:24s} " + " ".join(f"{r:>14s}" for r in row))
    print("(cells: norm-weighted mean per-parameter cosine with fp64 / median relative norm error)")


if __name__ == "__main__":
    main()
