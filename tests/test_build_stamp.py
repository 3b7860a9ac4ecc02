"""Build staleness is decided by content: the libraries embed the hash of the sources they
were built from and the loader refuses a library built from other sources."""
import shutil

import pytest

from thinvids_amd import _build, _native


def test_libraries_embed_current_source_hash():
    _native.core_lib()
    for name, which in (("libtvcore.so", "core"), ("libtvgpu.so", "gpu")):
        p = _build.LIBDIR / name
        if not p.exists():
            pytest.skip("library not built")
        assert _native._embedded_ok(p, _build.expected_hash(which))
    assert _native.build_hash(_native.core_lib(), "core") == _build.expected_hash("core")


def test_stale_library_is_refused(tmp_path, monkeypatch):
    lib = tmp_path / "libtvcore.so"
    shutil.copy(_build.LIBDIR / "libtvcore.so", lib)
    monkeypatch.setattr(_native, "LIBDIR", tmp_path)
    monkeypatch.setattr(_build, "expected_hash", lambda which: "0" * 64)  # sources "changed"
    monkeypatch.setenv("TV_NO_AUTOBUILD", "1")
    with pytest.raises(RuntimeError, match="stale"):
        _native._ensure_built("libtvcore.so")


def test_hash_tracks_flags_and_headers(monkeypatch):
    h0 = _build.expected_hash("gpu")
    monkeypatch.setattr(_build, "HIPFLAGS", _build.HIPFLAGS + ["-DTV_TEST_FLAG"])
    assert _build.expected_hash("gpu") != h0
    assert _build.expected_hash("core") == _build.expected_hash("core")
