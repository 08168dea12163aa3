"""CPU-side checks of the drop-in boundary: libfaasbal.so loads and exports every
symbol include/faasbal.h declares (no compute calls without a GPU)."""
import ctypes
import os
import re

import pytest

from faasbal import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    txt = open(os.path.join(REPO, "include", "faasbal.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char \*)\s*(fb_\w+)\s*\(", txt, re.M)))


def test_library_exports_every_header_symbol():
    lib = ctypes.CDLL(_lib.LIB_PATH)
    syms = header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(lib, s), s
    assert sorted(_lib.EXPORTS) == syms


def test_binding_prototypes_load():
    lib = _lib.load()
    for s in _lib.EXPORTS:
        assert getattr(lib, s).argtypes is not None


def test_create_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from faasbal import GpuBalancer, FaasbalError
    with pytest.raises(FaasbalError):
        GpuBalancer(16, 16)


def test_missing_library_is_loud(tmp_path):
    with pytest.raises(ImportError):
        _lib.load.__wrapped__(str(tmp_path / "nope.so")) if hasattr(_lib.load, "__wrapped__") else \
            _lib_load_fresh(str(tmp_path / "nope.so"))


def _lib_load_fresh(path):
    saved = _lib._LIB
    _lib._LIB = None
    try:
        return _lib.load(path)
    finally:
        _lib._LIB = saved
