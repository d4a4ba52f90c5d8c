"""CPU tests of the C-ABI library: it builds for gfx950, loads, exports every symbol the
public header declares, and its host-only entry points behave without a GPU."""
import ctypes
import os
import re

import numpy as np
import pytest

import netflow_amd as nf

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(nf.LIB_PATH):
        nf.build()
    return nf.lib()


def declared_symbols():
    hdr = open(os.path.join(ROOT, "include", "nfcs.h")).read()
    return sorted(set(re.findall(r"NFCS_API\s+[\w\s\*]+?\b(nfcs_\w+)\s*\(", hdr)))


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ("nfcs_update_device", "nfcs_update_host", "nfcs_ctx_create", "nfcs_ctx_destroy"):
        assert s in syms
    assert len(syms) >= 19


def test_library_exports_every_declared_symbol(lib):
    raw = ctypes.CDLL(nf.LIB_PATH)
    missing = [s for s in declared_symbols() if not hasattr(raw, s)]
    assert not missing, missing


def test_library_contains_gfx950_code_object():
    blob = open(nf.LIB_PATH, "rb").read()
    assert b"gfx950" in blob
    assert b"update_rows_kernel" in blob


def test_error_conventions_without_gpu(lib):
    assert lib.nfcs_abi_version() == 2
    assert lib.nfcs_strerror(0) == b"ok"
    assert lib.nfcs_strerror(-1) == b"invalid argument"
    # null context / arguments are rejected, never crash
    assert lib.nfcs_update_device(None, None, 0, None, 0, None, None, None) == -1
    assert lib.nfcs_update_host(None, None, 0, None, 0, None, 0) == -1
    assert lib.nfcs_update_host_frames(None, None, None, 0, None, 0) == -1
    assert lib.nfcs_ctx_create(0, None) == -1
    assert lib.nfcs_ctx_set_slot_bytes(None, 128) == -1
    c = ctypes.c_void_p()
    rc = lib.nfcs_ctx_create(0, ctypes.byref(c))
    if not os.path.exists("/dev/kfd"):
        assert rc == -4 and not c.value  # ENODEV: no silent CPU fallback
    elif rc == 0:
        lib.nfcs_ctx_destroy(c)


def test_host_layout(lib):
    d, nb = nf.layout_config(nf.CFG_C1, 1, 0, 1000)
    assert (d["len"] == 1500).all() and np.all(np.diff(d["off16"].astype(np.int64)) == 94)
    assert nb == 1000 * 1504
    d, nb = nf.layout_config(nf.CFG_C3, 1, 0, 0)
    assert nb == 0 and len(d) == 0
    with pytest.raises(nf.NfcsError):
        nf.layout_config(7, 1, 0, 10)


def test_no_cpu_fallback_when_library_missing(monkeypatch, tmp_path):
    monkeypatch.setattr(nf, "LIB_PATH", str(tmp_path / "missing.so"))
    monkeypatch.setattr(nf, "_lib", None)
    with pytest.raises(nf.NfcsError):
        nf.lib()
