"""Host sanitizers over the C++ codec core: builds csrc/core with
AddressSanitizer + UndefinedBehaviorSanitizer together with tools/native/sanitize_core.cpp
(golden encoder -> oracle decoder round trip with deblocking/SAO, MP4 mux/demux, AV1 range
coder, CDEF direction search) and requires a clean run.  CPU only."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(600)
def test_core_clean_under_asan_ubsan(tmp_path):
    if shutil.which(os.environ.get("CXX", "g++")) is None:
        pytest.skip("no host C++ compiler")
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "sanitize_core.sh"), str(tmp_path)],
                       capture_output=True, text=True, timeout=600)
    out = r.stdout + r.stderr
    if r.returncode != 0 and "cannot find" in out and "asan" in out:
        pytest.skip("sanitizer runtime not installed")
    assert r.returncode == 0, out[-4000:]
    assert "sanitize_core: ok" in out
    assert "runtime error" not in out
