"""Build libhgk.so (all HIP kernels + the C-ABI) for gfx950, in-tree.

`python -m progressive_process_for_human_pose_estimation_amd.build_ext` or
`__graft_entry__.build()`. Objects compile in parallel; the .so lands next to this file so it
travels to the GPU box with the repo snapshot (it is git-ignored, not gpurun-ignored).
"""
import concurrent.futures as cf
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
# ablation builds (scripts only): HGK_EXTRA_FLAGS="-DHGK_ABL_..." HGK_OUT=scratch/abl/x.so
OUT = os.environ.get("HGK_OUT") or os.path.join(PKG, "libhgk.so")
EXTRA = os.environ.get("HGK_EXTRA_FLAGS", "").split()
BUILD = os.path.join(ROOT, "build", "hgk" + ("-" + str(abs(hash(" ".join(EXTRA)))) if EXTRA else ""))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("HGK_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I" + os.path.join(ROOT, "include"),
         "-Wno-unused-result"] + EXTRA


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC)
                  if f.endswith(".hip") or f.endswith(".cpp"))


def _compile(src):
    obj = os.path.join(BUILD, os.path.basename(src) + ".o")
    deps = [src] + [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".h")]
    deps.append(os.path.join(ROOT, "include", "hgk.h"))
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(d) for d in deps):
        return obj
    cmd = [HIPCC] + FLAGS + ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
    return obj


def build(verbose=True):
    os.makedirs(BUILD, exist_ok=True)
    srcs = sources()
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(_compile, srcs))
    if os.path.exists(OUT) and os.path.getmtime(OUT) >= max(os.path.getmtime(o) for o in objs):
        return OUT
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", OUT] + objs
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("link failed:\n" + r.stderr)
    if verbose:
        print("built", OUT)
    return OUT


if __name__ == "__main__":
    build()
    sys.exit(0)
