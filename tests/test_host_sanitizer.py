"""Host-side sanitizer build: libhgk's HOST code compiled with AddressSanitizer +
UndefinedBehaviorSanitizer (-Xarch_host; GPU sanitizers are not available on this pool) and driven
by scripts/asan_host_check.cpp through argument validation, launch planning, twin / multi-entry
descriptor packing and the running-statistics grouping. CPU only: without a GPU every launch fails
cleanly after the host work that precedes it. The first build takes ~2 minutes (objects cached in
build/asan)."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT


@pytest.mark.skipif(shutil.which("/opt/rocm/bin/hipcc") is None, reason="hipcc not available")
def test_host_code_is_asan_ubsan_clean():
    if os.environ.get("HGK_SKIP_ASAN"):
        pytest.skip("HGK_SKIP_ASAN set")
    r = subprocess.run(["bash", os.path.join(ROOT, "scripts", "asan_host.sh")], capture_output=True,
                       text=True, timeout=900, env=dict(os.environ, HIP_VISIBLE_DEVICES=""))
    tail = (r.stdout + r.stderr)[-3000:]
    assert r.returncode == 0, tail
    assert "asan host check: ok" in r.stdout, tail
