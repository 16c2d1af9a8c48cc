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


def test_routing_is_explicit_not_environment(lib):
    """Kernel routing: compiled defaults, changed only through hgk_set_route (no getenv in the
    library's sources, no HGK_* routing variables read by the engine)."""
    from progressive_process_for_human_pose_estimation_amd import engine, hgk
    csrc = os.path.join(ROOT, "progressive_process_for_human_pose_estimation_amd", "csrc")
    for f in os.listdir(csrc):
        src = open(os.path.join(csrc, f)).read()
        assert "getenv" not in src, f
    eng = open(engine.__file__).read()
    assert re.findall(r"environ\.get\(\"(HGK_\w+)\"", eng) == ["HGK_DEBUG_LIFETIME"]
    hgk.load_library()
    defaults = {"ring_nw": 4, "ring_minm": 16384, "ring_small": 1, "row3": 2, "splitk_fixup": 1,
                "img": 8192, "wg_ring": 65536, "wg_halo_multi": 128}
    os.environ["HGK_ROW3"] = "0"  # a stray variable changes nothing
    try:
        assert {k: hgk.get_route(k) for k in defaults} == defaults
    finally:
        del os.environ["HGK_ROW3"]
    with hgk.route(row3=0, ring_minm=0):
        assert hgk.get_route("row3") == 0 and hgk.get_route("ring_minm") == 0
    assert {k: hgk.get_route(k) for k in defaults} == defaults
    assert hgk.set_route("ring_nw", 8) == 4 and hgk.set_route("ring_nw", -1) == 8
    assert hgk.get_route("ring_nw") == 4
    assert hgk.lib().hgk_set_route(99, 1) == -1 and b"unknown knob" in hgk.lib().hgk_last_error()
    with pytest.raises(hgk.HgkError):
        hgk.set_route("nope", 1)
    with engine.routing(twin=False):
        assert engine.ROUTE["twin"] is False
    assert engine.ROUTE == {"twin": True, "fold_apply": True, "fold_fin": True, "fold_bwd_fin": True,
                            "fold_bwd_add": False,
                            "bn_add": True, "bn_pair_bwd": True, "pair_apply": True, "fin_batch": True, "pair_blocks": True, "wg_batch": True,
                            "mse_heads": True}
    cms = engine.apply_route_spec("twin=0,row3=1")
    assert engine.ROUTE["twin"] is False and hgk.get_route("row3") == 1
    for cm in reversed(cms):
        cm.__exit__(None, None, None)
    assert engine.ROUTE["twin"] is True and hgk.get_route("row3") == 2


def test_kernel_family_routing(lib):
    """Host-side routing of the forward convolutions (no launch): the headline step's shapes take
    the kernel families DESIGN.md §4 describes, and a route switch moves them."""
    from progressive_process_for_human_pose_estimation_amd import hgk
    L = hgk.load_library()

    def fam(N, H, cin, cout, k, N1=0, H1=0, dt=hgk.BF16):
        pad = k // 2
        return hgk.KFAM[L.hgk_conv_fwd_kernel_family(dt, N, H, H, N1, H1, H1, cin, cout, k, k, 1, pad, 1)]
    assert fam(32, 64, 256, 128, 1) == "ring"
    assert fam(32, 32, 128, 256, 1) == "ring"
    assert fam(16, 32, 128, 256, 1) == "ring" and fam(16, 32, 256, 128, 1) == "ring"  # try_with_aspp
    assert fam(32, 64, 128, 128, 3) == "row3"
    assert fam(32, 64, 128, 128, 3, 32, 32) == "row3"
    assert fam(32, 32, 128, 128, 3) == "halo"
    for h in (16, 8, 4):
        assert fam(32, h, 128, 256, 1) == "img", h
    for h in (8, 4):
        assert fam(32, h, 128, 128, 3) == "img", h
    assert fam(32, 16, 128, 128, 3) == "halo"  # 16x16 strips: the halo kernel is faster
    assert fam(16, 16, 128, 128, 3) == "img"   # ... except in one round of workgroups (N = 16)
    assert fam(32, 8, 128, 128, 3, 32, 4) == "img"
    assert fam(32, 16, 128, 128, 3, 32, 8) == "split"
    assert fam(32, 16, 128, 256, 1, 32, 8) == "img"
    assert fam(32, 2, 128, 128, 3) == "implicit"  # 16 images of 2x2 per tile: halo too large
    assert fam(32, 8, 128, 128, 3, dt=hgk.F32) == "implicit"
    with hgk.route(img=0):
        assert fam(32, 8, 128, 128, 3) == "implicit"
        assert fam(32, 16, 128, 128, 3) == "halo"
    with hgk.route(img=2048):
        assert fam(32, 16, 128, 256, 1) == "implicit" and fam(32, 8, 128, 256, 1) == "img"


def test_route_key_tracks_changes_from_the_compiled_defaults():
    from progressive_process_for_human_pose_estimation_amd import hgk
    """modules._signature keys captured hipGraphs on hgk.route_key(): empty at the compiled
    defaults, the changed knobs inside hgk.route(), empty again once restored."""
    hgk.load_library()
    assert hgk.route_key() == ()
    with hgk.route(img=0, wg_full=65536):
        assert dict(hgk.route_key()) == {"img": 0, "wg_full": 65536}
    assert hgk.route_key() == ()
    prev = hgk.set_route("ring_minm", 0)
    assert dict(hgk.route_key()) == {"ring_minm": 0}
    hgk.set_route("ring_minm", -1)   # back to the default
    assert hgk.route_key() == () and hgk.get_route("ring_minm") == prev
