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


def test_small_host_calls_marshal_like_the_general_path():
    """BatchSolver.solve's cached small-batch marshalling (B <= 64: per-shape arrays, pointers made once) hands
    tt_solve_batch the same bytes as the general path, returns fresh arrays each call, and leaves shape errors to
    the general path.  A recording stand-in replaces the library (no GPU here)."""
    import ctypes as C

    import numpy as np

    from ttmpc import _lib

    N = 20
    seen = []

    class Rec:
        def tt_solve_batch(self, h, B, x0, xr, ur, w, zg, X, U, st, it, kk):
            def arr(p, n, t=C.c_double):
                return None if p is None else np.ctypeslib.as_array(C.cast(p, C.POINTER(t)), (n,)).copy()
            seen.append((B, arr(x0, 6 * B), arr(xr, 6 * (N + 1) * B), arr(ur, 2 * N * B), arr(w, 8 * B),
                         arr(zg, (8 * N + 6) * B)))
            o = np.ctypeslib.as_array(C.cast(X, C.POINTER(C.c_double)), (6 * (N + 1) * B,))
            o[:] = len(seen)
            np.ctypeslib.as_array(C.cast(st, C.POINTER(C.c_int)), (B,))[:] = len(seen)
            return 0

        def tt_last_error(self, h):
            return b""

    s = object.__new__(_lib.BatchSolver)
    s.N, s._L, s._h = N, Rec(), None
    rng = np.random.default_rng(5)
    for B in (1, 3, 64, 65):
        x0, xr, ur = rng.normal(size=(B, 6)), rng.normal(size=(B, N + 1, 6)), rng.normal(size=(B, N, 2))
        w, zg = rng.normal(size=(B, 8)), rng.normal(size=(B, 8 * N + 6))
        for kw in ({}, {"wq_wr": w}, {"z_guess": zg}, {"wq_wr": w, "z_guess": zg}):
            r1 = s.solve(x0, xr.tolist() if B == 3 else xr, ur, **kw)
            got = seen[-1]
            assert got[0] == B
            for a, b in zip(got[1:], (x0, xr, ur, kw.get("wq_wr"), kw.get("z_guess"))):
                assert (a is None and b is None) or np.array_equal(a, np.ravel(b))
            r2 = s.solve(x0, xr, ur, **kw)
            assert r1[0].shape == (B, N + 1, 6) and r1[2].dtype == np.int32
            assert r1[0][0, 0, 0] == len(seen) - 1 and r2[0][0, 0, 0] == len(seen)  # fresh arrays, not the cache
    with pytest.raises(ValueError):
        s.solve(np.zeros((2, 6)), np.zeros((1, N + 1, 6)), np.zeros((2, N, 2)))
