"""The C-ABI library loads and exports every entry point include/zdl.h declares
(no compute calls: no GPU needed)."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared():
    txt = open(os.path.join(ROOT, "include", "zdl.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(zdl_[a-z_0-9]+)\s*\(", txt)))


def test_header_declares_entry_points():
    names = declared()
    for n in ("zdl_create", "zdl_put_spans", "zdl_link", "zdl_merge_links", "zdl_set_window"):
        assert n in names


def test_library_exports_every_declared_symbol():
    from zipkin_amd import _native
    lib = ctypes.CDLL(_native.LIB_PATH)
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing
    assert set(declared()) <= set(_native.EXPORTS)


def test_abi_version():
    from zipkin_amd import _native
    assert _native.lib().zdl_abi_version() == _native.ZDL_ABI_VERSION == 7


def test_create_rejects_bad_config_without_device():
    from zipkin_amd import _native
    L = _native.lib()
    cfg = _native.Config(0, 0, 0, 0)  # n_services = 0 is rejected before any device call
    assert not L.zdl_create(ctypes.byref(cfg))
    assert b"n_services" in L.zdl_create_error()


def test_product_does_not_import_oracle():
    pkg = os.path.join(ROOT, "zipkin_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".cpp", ".h")):
                src = open(os.path.join(dirpath, f), encoding="utf-8").read()
                assert "import oracle" not in src and "from oracle" not in src, f
                assert "dl_ref" not in src and "liboracle" not in src, f


def test_group_config_rejects_duplicate_devices_without_device():
    """A device group is checked before any device call: RCCL takes one rank per device."""
    from zipkin_amd import _native
    L = _native.lib()
    ids = (ctypes.c_int32 * 2)(0, 0)
    cfg = _native.Config(0, 50, 0, 0, 2, ctypes.cast(ids, ctypes.POINTER(ctypes.c_int32)))
    assert not L.zdl_create(ctypes.byref(cfg))
    assert b"twice" in L.zdl_create_error()
    cfg = _native.Config(0, 50, _native.ZDL_FLAG_INSERTION_ORDER, 0, 1, ctypes.cast(ids, ctypes.POINTER(ctypes.c_int32)))
    assert not L.zdl_create(ctypes.byref(cfg))
    assert b"INSERTION_ORDER" in L.zdl_create_error()


def test_native_shard_of_matches_python_partition():
    """The device group's host-side sharding (zdl_shard_of, C++) equals shard.shard_of, which
    the multi-process bench and partition_columns use: the same trace lands on the same GPU."""
    import numpy as np
    from zipkin_amd import _native, shard
    rng = np.random.default_rng(1)
    lo = rng.integers(0, 2 ** 63, 100_000, dtype=np.int64).astype(np.uint64) * np.uint64(2) + np.uint64(1)
    for n in (1, 2, 3, 8):
        assert np.array_equal(_native.shard_of(lo, n).astype(np.int64), shard.shard_of(lo, n))
