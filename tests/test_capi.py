"""The C ABI library loads and exports every symbol include/abcgpu.h declares
(no compute calls: this runs on the CPU-only build host)."""
import ctypes
import os
import re

from conftest import ROOT


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "abcgpu.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(abc_[a-z0-9_]+)\s*\(", src)))


def test_header_matches_binding_table():
    from pyabc_amd import _native
    assert sorted(_native.SIGNATURES) == declared_symbols()


def test_library_exports_all_symbols():
    from pyabc_amd import _native
    lib = ctypes.CDLL(_native.LIB_PATH)
    for name in declared_symbols():
        assert hasattr(lib, name), name
    _native.load()
    assert _native.load().abc_version() == 1


def test_size_queries_are_pure_host():
    from pyabc_amd import _native as nat
    assert nat.query("abc_mvn_packed_bytes", 1000, 10, nat.ABC_PREC_F64) == \
        63 * 64 * 3 * 8
    assert nat.query("abc_mvn_logpdf_workspace", 4096, 4096, 10, 0) > 0
    # the x3 call at c3 (M = N = 1e6, r = 10): the main plan (candidate
    # image, 32 chunks of partials) plus the nested rescue pass capped at
    # 16384 rows -- not a nested plan sized for all M (~4 GB)
    nb = nat.query("abc_mvn_logpdf_workspace", 10 ** 6, 10 ** 6, 10, nat.ABC_PREC_X3)
    assert 0.5e9 < nb < 0.8e9, nb
    assert nat.query("abc_sort_pairs_workspace", 10 ** 6) > 32 * 10 ** 6
    # LocalTransition fit: d <= 5 carries the deferred collect's queue (256
    # row indices per particle) beside the dense moments' buffers
    n = 10 ** 5
    for d in (1, 5):
        assert nat.query("abc_local_fit_workspace", n, d) > n * 256 * 4
    assert nat.query("abc_local_fit_workspace", 2 * n, 5) > \
        nat.query("abc_local_fit_workspace", n, 5)


def test_invalid_arguments_raise_without_device():
    import pytest
    from pyabc_amd import _native as nat
    with pytest.raises(ValueError):
        nat.call("abc_pnorm", None, 10, 0, None, None, 2.0, None, None)
    assert "pnorm" in nat.load().abc_last_error().decode()


def test_store_library_exports_abcstore_h():
    """libabcstore.so (host code) exports every symbol include/abcstore.h
    declares, and reports errors through abc_store_last_error."""
    from pyabc_amd import build
    from pyabc_amd.storage import sqlite_store
    build.build_store(verbose=False)
    src = open(os.path.join(ROOT, "include", "abcstore.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = sorted(set(re.findall(r"\b(abc_store_[a-z0-9_]+)\s*\(", src)))
    assert len(names) == 5
    lib = sqlite_store.load()
    for name in names:
        assert hasattr(lib, name), name
    h = ctypes.c_void_p()
    assert lib.abc_store_open(b"/nonexistent-dir/x.db", ctypes.byref(h)) != 0
    assert b"open" in lib.abc_store_last_error()


def test_comm_unique_id_and_argument_checks():
    """The RCCL wrappers (abc_comm_*): RCCL is opened on first use; a unique
    id needs no GPU; bad ranks are rejected before RCCL is touched."""
    import pytest
    from pyabc_amd import _native as nat
    a = ctypes.create_string_buffer(nat.ABC_COMM_ID_BYTES)
    b = ctypes.create_string_buffer(nat.ABC_COMM_ID_BYTES)
    nat.call("abc_comm_unique_id", a)
    nat.call("abc_comm_unique_id", b)
    assert a.raw != b.raw
    h = ctypes.c_void_p()
    with pytest.raises(ValueError):
        nat.call("abc_comm_init", ctypes.addressof(h), 2, 2, a)
    assert nat.load().abc_comm_destroy(None) == 0
