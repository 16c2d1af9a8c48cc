"""CPU-side checks of the C-ABI boundary: libhgk.so loads and exports exactly what include/hgk.h
declares (no compute calls: there is no GPU here)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "hgk.h")
LIB = os.path.join(ROOT, "progressive_process_for_human_pose_estimation_amd", "libhgk.so")


def header_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(hgk_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        from progressive_process_for_human_pose_estimation_amd import build_ext
        build_ext.build(verbose=False)
    import torch  # noqa: F401  (HIP runtime from torch)
    return ctypes.CDLL(LIB)


def test_header_declares_symbols():
    syms = header_symbols()
    assert "hgk_conv_fwd" in syms and "hgk_conv_wgrad" in syms and len(syms) >= 20


def test_library_exports_every_header_symbol(lib):
    missing = [s for s in header_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_python_binding_matches_header(lib):
    from progressive_process_for_human_pose_estimation_amd import hgk
    assert sorted(hgk.SIGNATURES) == header_symbols()
    hgk.load_library()
    assert hgk.lib().hgk_abi_version() == hgk.ABI_VERSION


def test_host_side_queries(lib):
    from progressive_process_for_human_pose_estimation_amd import hgk
    L = hgk.load_library()
    assert L.hgk_conv_w_ld(147) == 192 and L.hgk_conv_w_ld(1152) == 1152
    ws = L.hgk_conv_wgrad_workspace(0, 2, 64, 64, 128, 128, 3, 3, 1, 1, 1)
    assert ws > 128 * 1152 * 4
    # argument validation happens on the host before any launch
    rc = L.hgk_conv_fwd(None, 0, None, None, 64, None, None, None, None, None, 0, 0, None, None,
                        1, 8, 8, 64, 64, 1, 1, 1, 0, 1, None, 0)
    assert rc == -1 and b"null" in L.hgk_last_error()
    # split-K only for small-M launches: 4x4 level at N=32 asks for a workspace, 64x64 does not
    assert L.hgk_conv_fwd_workspace(1, 32, 4, 4, 128, 128, 3, 3, 1, 1, 1) > 0
    assert L.hgk_conv_fwd_workspace(1, 32, 64, 64, 128, 128, 3, 3, 1, 1, 1) == 0
    assert rc == -1 and b"null" in L.hgk_last_error()
    rc = L.hgk_add(None, 7, 1, None, 1, 4, 0)
    assert rc == -1
