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


def test_env_paths_parse_defensively():
    """FAASBAL_PATHS (same-box A/B runs): malformed entries and layout-changing knobs are
    ignored with a warning, never fatal to the import."""
    import warnings
    from faasbal.balancer import _env_paths
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        got = _env_paths("cmix=0, wtiles=2,bogus,xplan=0,n=abc,=3")
    assert got == {"cmix": 0, "wtiles": 2}
    assert len(w) == 4


def test_iter_compact_matches_round_expansion():
    """CompactAssignments / iter_compact (the dispatcher's lazy expansion) against a plain
    round-by-round expansion of the closed form: round r serves, in LRU
    order, the positions with min(c, L + 1) > r; the last round only its first p."""
    import numpy as np
    from faasbal.balancer import CompactAssignments, iter_compact
    rng = np.random.default_rng(0)
    for trial in range(50):
        Q = int(rng.integers(0, 400))
        L = int(rng.integers(0, 20))
        slot = rng.integers(-1, 10_000, Q).astype(np.int32)
        c = rng.integers(0, L + 2, Q).astype(np.uint8)
        ref = []
        for r in range(L + 1):
            ref.extend(int(s) for s, x in zip(slot, c) if x > r)
        total = len(ref)
        n = int(rng.integers(0, total + 1))
        got = np.concatenate(list(iter_compact(slot, c, n))) if n else np.zeros(0, np.int32)
        assert got.tolist() == ref[:n]
        ca = CompactAssignments(slot, c, n)
        assert list(ca) == ref[:n] and len(ca) == n and ca.array().tolist() == ref[:n]
