import os
import sys

import pytest


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs via gpurun)")
    config.addinivalue_line("markers", "slow: long-running CPU test")
    # torch references of the GPU kernel tests: exact fp32 (no reduced-precision convolution or
    # matmul modes), so the per-element bf16 bounds (tests/gates.py) compare against fp32 math
    try:
        import torch
        torch.backends.cudnn.allow_tf32 = False
        torch.backends.cuda.matmul.allow_tf32 = False
    except Exception:  # noqa: BLE001 (CPU-only collection works without torch)
        pass


def pytest_collection_modifyitems(config, items):
    # GPU tests are skipped (not failed) when no GPU is visible, so `-m "not gpu"` and a bare
    # `pytest` both work on the CPU-only build container.
    try:
        import torch
        have_gpu = torch.cuda.is_available()
    except Exception:
        have_gpu = False
    if have_gpu:
        return
    skip = pytest.mark.skip(reason="no GPU visible")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture
def routes():
    """routes(name=value, ...): set engine routes (engine.ROUTE: twin, fold_apply, fold_fin, fold_bwd_fin) and
    library routes (hgk.ROUTES, set through the hgk_set_route ABI) for this test; every value
    is restored afterwards. Routing is never read from the environment."""
    from progressive_process_for_human_pose_estimation_amd import engine as E
    from progressive_process_for_human_pose_estimation_amd import hgk as H
    saved_eng = dict(E.ROUTE)
    saved_lib = {}

    def set_(**kw):
        for k, v in kw.items():
            if k in E.ROUTE:
                E.ROUTE[k] = bool(int(v))
            else:
                prev = H.set_route(k, int(v))
                saved_lib.setdefault(k, prev)
    yield set_
    E.ROUTE.update(saved_eng)
    for k, v in saved_lib.items():
        H.set_route(k, v)

