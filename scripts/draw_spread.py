"""Whole-model gate statistics of every engine draw (scripts/engine_draws.py output) next to every
reference fp32 draw of the configs[4] N=16 fixture: gradient direction (cosine with fp64 over the
strided samples), median / p90 / max relative grad-norm error (tests/gates.py _norm_stats).
usage: python scripts/draw_spread.py profiles/r06_draws/engine_draws_s8_n16.npz"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from gates import NCHW_DRAWS, OTHER_DRAWS, _cos, _norm_stats, fp32_draws  # noqa: E402


def main():
    g = np.load(os.path.join(ROOT, "tests", "golden", "primary_s8_n16_384.npz"))
    e = np.load(sys.argv[1])
    n64, s64 = g["grad_norm64"], g["grad_sample64"]
    rows = [(f"ref {d}", nn, s) for d, nn, s in fp32_draws(g, NCHW_DRAWS + OTHER_DRAWS)]
    rows += [(f"engine {k[:-10]}", e[k], e[k[:-10] + "_grad_sample"])
             for k in e.files if k.endswith("_grad_norm")]
    print(f"{'draw':34s} {'cos':>7s} {'median':>7s} {'p90':>7s} {'max':>7s}")
    meds = {}
    for name, nn, s in rows:
        med, p90, rel = _norm_stats(nn, n64)
        meds[name] = med
        print(f"{name:34s} {_cos(s, s64):7.4f} {med:7.4f} {p90:7.4f} {rel.max():7.4f}")
    env = [meds["ref orig"]] + [meds[f"ref {d}"] for d in NCHW_DRAWS if f"ref {d}" in meds]
    eng = [v for k, v in meds.items() if k.startswith("engine")]
    print(f"reference NCHW draws: median error {min(env):.4f} .. {max(env):.4f} (mean {np.mean(env):.4f}, "
          f"{len(env)} draws)")
    print(f"engine draws:         median error {min(eng):.4f} .. {max(eng):.4f} (mean {np.mean(eng):.4f}, "
          f"{len(eng)} draws)")


if __name__ == "__main__":
    main()
