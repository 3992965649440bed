"""libspg.so loads on a CPU-only host and exports every entry point include/spg.h declares; without a
gfx950 device spg_init must fail loudly (no CPU fallback)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "spartan-parallel_amd", "lib", "libspg.so")
HDR = os.path.join(ROOT, "include", "spg.h")


def declared_symbols():
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(spg_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    assert "spg_init" in syms and "spg_msm" in syms and "spg_commit_rows" in syms


def test_library_exports_all_symbols():
    assert os.path.exists(LIB), "run __graft_entry__.build() first"
    lib = ctypes.CDLL(LIB)
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_init_without_device_fails_loudly():
    import torch

    if torch.cuda.is_available():
        pytest.skip("a device is present")
    lib = ctypes.CDLL(LIB)
    h = ctypes.c_void_p()
    assert lib.spg_init(0, ctypes.byref(h)) == -5  # SPG_E_NODEVICE
