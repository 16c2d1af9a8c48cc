"""Fixture-generation helper: load the reference's model classes by AST extraction.

TEST INFRASTRUCTURE ONLY. Runs in the survey/build container (where /root/reference exists);
never shipped to or executed on the GPU box (tools/ is listed in .gpurunignore).

`import try_with_torch` fails with an ordinary ModuleNotFoundError (torchvision / pycocotools are
absent, /root/reference/try_with_torch.py:8,12), so — as SURVEY.md Appendix A describes — we parse
the file, keep only the `ClassDef` nodes and simple module-level constants, and exec them into a
namespace holding torch / nn / F / np. Module globals (nStack, nOutChannels ...) can be overridden
before the classes are instantiated because the class bodies read them at call time.
"""
import ast
import os

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

REF_ROOT = os.environ.get("HG_REFERENCE_ROOT", "/root/reference")

_SIMPLE_VALUE_NODES = (ast.Constant, ast.BinOp, ast.Name, ast.List, ast.UnaryOp)


MODEL_CLASSES = ("ResidualBlock", "hourglass", "lin", "creatModel")


def load_reference(filename, overrides=None, class_names=MODEL_CLASSES, pre=None):
    """Return a namespace dict holding the reference file's classes and scalar globals.
    `pre`: names the class bodies need at definition time (e.g. a base class module)."""
    path = os.path.join(REF_ROOT, filename)
    with open(path, "r") as fh:
        tree = ast.parse(fh.read(), filename=path)
    ns = {"torch": torch, "nn": nn, "F": F, "np": np,
          "loss": torch.nn.modules.loss, "__name__": "hg_reference_" + filename[:-3]}
    if pre:
        ns.update(pre)
    for node in tree.body:
        keep = False
        if isinstance(node, ast.ClassDef):
            keep = class_names is None or node.name in class_names
        elif isinstance(node, ast.Assign) and isinstance(node.value, _SIMPLE_VALUE_NODES):
            keep = all(isinstance(t, ast.Name) for t in node.targets)
        if not keep:
            continue
        mod = ast.Module(body=[node], type_ignores=[])
        try:
            exec(compile(mod, path, "exec"), ns)
        except Exception:
            # e.g. a constant that references a name we did not import (file paths etc.)
            # classes outside the model (datasets needing torchvision / pycocotools) are skipped
            pass
    if overrides:
        ns.update(overrides)
    return ns
