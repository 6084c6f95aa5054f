"""CPU suite: the C-ABI library loads and exports every symbol include/ttmpc.h declares.
No compute calls here (no GPU in the CPU suite)."""
import ctypes
import re

import pytest

from conftest import PKG, REPO


def _declared():
    hdr = (REPO / "include" / "ttmpc.h").read_text()
    return sorted(set(re.findall(r"^\s*(?:int|void|long long|const char\*)\s+(tt_\w+)\s*\(", hdr, flags=re.M)))


def test_header_declares_the_boundary():
    names = _declared()
    for n in ("tt_create", "tt_solve_batch", "tt_solve_batch_device", "tt_plan_batch", "tt_destroy", "tt_last_error"):
        assert n in names


def test_library_exports_every_declared_symbol():
    so = PKG / "ttmpc" / "libttmpc.so"
    if not so.exists():
        pytest.skip("libttmpc.so not built (run __graft_entry__.build())")
    L = ctypes.CDLL(str(so))
    for n in _declared():
        assert hasattr(L, n), n
    from ttmpc import _lib
    assert set(_lib.EXPORTED_SYMBOLS) == set(_declared())


def test_introspection_without_gpu():
    so = PKG / "ttmpc" / "libttmpc.so"
    if not so.exists():
        pytest.skip("libttmpc.so not built")
    from ttmpc import lib
    L = lib()
    assert L.tt_max_horizon() >= 60
    assert L.tt_lds_bytes(20) == 8 * (118 * 21 + 256)
    assert 4 * L.tt_lds_bytes(40) <= 160 * 1024   # C3: four N = 40 instances per CU
    assert b"gfx950" in L.tt_version()


def test_product_fails_loudly_without_gpu():
    """No CPU fallback: without a usable gfx950 device tt_create must fail."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    so = PKG / "ttmpc" / "libttmpc.so"
    if not so.exists():
        pytest.skip("libttmpc.so not built")
    import numpy as np
    import ttmpc
    with pytest.raises(ttmpc.TTError):
        ttmpc.BatchSolver(10, {"dt": 0.05, "L1": 7.05, "L2": 12.45, "M": 0.15}, np.eye(6), np.eye(2),
                          [-1e20] * 6, [1e20] * 6, [-5, -1], [5, 1])
