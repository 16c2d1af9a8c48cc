"""engine.LifetimeGuard mechanics on the CPU (a stand-in library object records the calls): the
launch-time check refuses pointers into a buffer whose last owner is gone, scans c_void_p fields
of descriptor arrays, and ignores sizes and untracked pointers. The GPU test
(tests/test_gpu_lifetime.py) runs it over real training steps."""
import ctypes

import pytest
import torch

from progressive_process_for_human_pose_estimation_amd.engine import LifetimeGuard


class _Seg(ctypes.Structure):
    _fields_ = [("a", ctypes.c_void_p), ("n", ctypes.c_int), ("b", ctypes.c_void_p)]


class _Lib:
    def __init__(self):
        self.calls = []

    def hgk_copy(self, *args):
        self.calls.append(args)
        return 0

    def not_a_kernel(self):
        return "plain"


def test_guard_live_released_and_descriptors():
    lib = _Lib()
    g = LifetimeGuard(lib)
    x = g.track(torch.empty(1024))
    y = g.track(torch.empty(1024))
    g.hgk_copy(0, x.data_ptr() + 64, y.data_ptr(), 1 << 20)  # interior pointer, a size
    assert g.checked == 2 and len(lib.calls) == 1
    assert g.not_a_kernel() == "plain"
    px = x.data_ptr()
    del x
    with pytest.raises(RuntimeError, match="hgk_copy arg 1 reads a buffer with no owner"):
        g.hgk_copy(0, px, y.data_ptr(), 16)
    assert len(lib.calls) == 1  # refused before the call
    segs = (_Seg * 2)(_Seg(y.data_ptr(), 3, None), _Seg(px + 128, 4, y.data_ptr()))
    with pytest.raises(RuntimeError, match=r"arg 0\[1\]\.a"):
        g.hgk_copy(segs)
    view = y[100:]
    py = y.data_ptr()
    del y
    g.hgk_copy(py, view.data_ptr())  # a view still owns the storage
    other = torch.empty(8)
    g.hgk_copy(other.data_ptr())  # untracked: not checked
    assert len(lib.calls) == 3
