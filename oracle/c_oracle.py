"""ctypes wrapper over oracle/build/libttoracle.so (CPU ORACLE: test infrastructure + cpu_baseline).

Never imported by the product package.  Layout of z is the reference's interleaved vector
[x0,u0,...,x_{N-1},u_{N-1},x_N] (python-files/trajectory_planning.py:38-58).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
# TTO_ORACLE_LIB: another build of the oracle (the ASan/UBSan one of `make -C oracle sanitize`)
LIB_PATH = Path(os.environ["TTO_ORACLE_LIB"]).resolve() if os.environ.get("TTO_ORACLE_LIB") else _HERE / "build" / "libttoracle.so"


class TTOProblem(C.Structure):
    _fields_ = [("N", C.c_int), ("dt", C.c_double), ("L1", C.c_double), ("L2", C.c_double), ("Mh", C.c_double),
                ("Q", C.c_double * 36), ("R", C.c_double * 4), ("xlb", C.c_double * 6), ("xub", C.c_double * 6),
                ("ulb", C.c_double * 2), ("uub", C.c_double * 2), ("tol", C.c_double), ("acc_tol", C.c_double),
                ("max_iter", C.c_int), ("acc_iter", C.c_int)]


_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", str(_HERE)])


def lib():
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build()
        _lib = C.CDLL(str(LIB_PATH))
        dp = C.POINTER(C.c_double)
        ip = C.POINTER(C.c_int)
        _lib.tto_solve_batch.argtypes = [C.POINTER(TTOProblem), C.c_int, dp, dp, dp, dp, dp, dp, dp, ip, ip, dp, C.c_int]
        _lib.tto_solve_batch.restype = C.c_int
    return _lib


def _fin(a):
    a = np.asarray(a, dtype=np.float64).copy()
    a[np.isposinf(a)] = 1e300
    a[np.isneginf(a)] = -1e300
    return a


def make_problem(N, params, Q, R, xlb, xub, ulb, uub, tol=1e-8, acc_tol=1e-6, max_iter=3000, acc_iter=15):
    P = TTOProblem()
    P.N = int(N)
    P.dt, P.L1, P.L2, P.Mh = params["dt"], params["L1"], params["L2"], params["M"]
    P.Q[:] = list(np.asarray(Q, float).reshape(36))
    P.R[:] = list(np.asarray(R, float).reshape(4))
    P.xlb[:] = list(_fin(xlb)); P.xub[:] = list(_fin(xub))
    P.ulb[:] = list(_fin(ulb)); P.uub[:] = list(_fin(uub))
    P.tol, P.acc_tol, P.max_iter, P.acc_iter = tol, acc_tol, max_iter, acc_iter
    return P


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.POINTER(C.c_double))


def solve_batch(P, x0, xref, uref, wq=None, wr=None, z_guess=None, nthreads=0):
    """x0 (B,6), xref (B,N+1,6), uref (B,N,2) -> (z (B,n), status, iters, kkt)."""
    N = P.N
    n = 8 * N + 6
    x0 = np.ascontiguousarray(x0, dtype=np.float64)
    B = x0.shape[0]
    xref = np.ascontiguousarray(xref, dtype=np.float64).reshape(B, N + 1, 6)
    uref = np.ascontiguousarray(uref, dtype=np.float64).reshape(B, N, 2)
    wq = None if wq is None else np.ascontiguousarray(wq, dtype=np.float64).reshape(B, 6)
    wr = None if wr is None else np.ascontiguousarray(wr, dtype=np.float64).reshape(B, 2)
    zg = None if z_guess is None else np.ascontiguousarray(z_guess, dtype=np.float64).reshape(B, n)
    z = np.zeros((B, n))
    st = np.zeros(B, dtype=np.int32)
    it = np.zeros(B, dtype=np.int32)
    kk = np.zeros(B)
    rc = lib().tto_solve_batch(C.byref(P), B, _ptr(x0), _ptr(xref), _ptr(uref), _ptr(wq), _ptr(wr), _ptr(zg),
                               _ptr(z), st.ctypes.data_as(C.POINTER(C.c_int)), it.ctypes.data_as(C.POINTER(C.c_int)),
                               _ptr(kk), int(nthreads))
    if rc != 0:
        raise RuntimeError(f"tto_solve_batch failed: {rc}")
    return z, st, it, kk


def split(z, N):
    """(B,n) -> X (B,N+1,6), U (B,N,2)."""
    z = np.asarray(z)
    B = z.shape[0]
    body = z[:, : 8 * N].reshape(B, N, 8)
    X = np.concatenate([body[:, :, :6], z[:, None, 8 * N:]], axis=1)
    return X, body[:, :, 6:].copy()


os.environ.setdefault("OMP_PROC_BIND", "false")


# ------------------------------------------------------------------------------------------------
# OBCA NLPs (tt_obca.c): TrajectoryOptimization.plan / MPCTrackingControlObs.solve restated
# ------------------------------------------------------------------------------------------------
MAXM = 16
OBCA_PLAN, OBCA_TRACK = 0, 1
# tt_obca.h switches: IPOPT defaults off (round 2's PD block test, no iterative refinement) and oracle-only opt-in
# IPOPT features (kappa_d damping, line-search watchdog, rows-first elimination of indefinite blocks)
OPT_PD_BLOCKS, OPT_NO_REFINE = 32, 64
OPT_KAPPA_D, OPT_WATCHDOG, OPT_BLOCK_MW, OPT_GLOBAL_INERTIA = 8, 16, 128, 256
OPT_R3_PERTURB = 512  # round 3's delta_x-only inertia correction instead of IPOPT's perturbation handler (A/B)


class TTOObcaProblem(C.Structure):
    _fields_ = [("N", C.c_int), ("M", C.c_int), ("mode", C.c_int),
                ("dt", C.c_double), ("L1", C.c_double), ("L2", C.c_double), ("Mh", C.c_double),
                ("W1", C.c_double), ("W2", C.c_double),
                ("Q", C.c_double * 36), ("R", C.c_double * 4), ("xlb", C.c_double * 6), ("xub", C.c_double * 6),
                ("ulb", C.c_double * 2), ("uub", C.c_double * 2), ("obs", C.c_double * (4 * MAXM)),
                ("dmin", C.c_double), ("eq_tol", C.c_double), ("fin_tol", C.c_double), ("tfac", C.c_double),
                ("tol", C.c_double), ("acc_tol", C.c_double), ("max_iter", C.c_int), ("acc_iter", C.c_int),
                ("dual_init", C.c_int), ("opts", C.c_int)]


def make_obca_problem(N, params, Q, R, xlb, xub, ulb, uub, obstacles, mode=OBCA_PLAN, tol=1e-8, acc_tol=1e-6,
                      max_iter=5000, acc_iter=15, dual_init=0, opts=0):
    """obstacles: (M,4) array of (cx, cy, w, h) (get_obstacles.py format)."""
    ob = np.asarray(obstacles, dtype=np.float64).reshape(-1, 4)
    if not 1 <= ob.shape[0] <= MAXM:
        raise ValueError("1 <= M <= 16 obstacles")
    P = TTOObcaProblem()
    P.N, P.M, P.mode = int(N), ob.shape[0], int(mode)
    P.dt, P.L1, P.L2, P.Mh = params["dt"], params["L1"], params["L2"], params["M"]
    P.W1, P.W2 = params["W1"], params["W2"]
    P.Q[:] = list(np.asarray(Q, float).reshape(36))
    P.R[:] = list(np.asarray(R, float).reshape(4))
    P.xlb[:] = list(_fin(xlb)); P.xub[:] = list(_fin(xub))
    P.ulb[:] = list(_fin(ulb)); P.uub[:] = list(_fin(uub))
    P.obs[: ob.size] = list(ob.reshape(-1))
    P.dmin, P.eq_tol, P.fin_tol = 0.2, 1e-5, 1e-2
    P.tfac = 100.0 if mode == OBCA_PLAN else 1.0
    P.tol, P.acc_tol, P.max_iter, P.acc_iter = tol, acc_tol, max_iter, acc_iter
    P.dual_init = int(dual_init)
    P.opts = int(opts)
    return P


def obca_n(N, M):
    return N * (8 + 16 * M) + 6 + 16 * M


def _obca_lib():
    L = lib()
    if not hasattr(L, "_obca_ready"):
        dp = C.POINTER(C.c_double)
        ip = C.POINTER(C.c_int)
        L.tto_obca_solve_batch_it.argtypes = [C.POINTER(TTOObcaProblem), C.c_int, dp, dp, dp, dp, dp, dp, ip, ip, dp,
                                              dp, C.c_int]
        L.tto_obca_solve_batch_it.restype = C.c_int
        L.tto_obca_iterate_len.argtypes = [C.c_int, C.c_int]
        L.tto_obca_iterate_len.restype = C.c_longlong
        L.tto_obca_eval_iterate.argtypes = [C.POINTER(TTOObcaProblem), dp, dp, dp, dp, dp, dp]
        L.tto_obca_eval_iterate.restype = C.c_int
        L._obca_ready = True
    return L


def obca_iterate_len(N, M):
    """Length of the primal-dual iterate export (include/ttmpc.h tt_obca_iterate_len; tt_obca.c pack_iterate)."""
    return 30 * (N + 1) + 64 * M * (N + 1) + 24


def obca_solve_batch(P, x0, x_goal=None, xref=None, uref=None, z_guess=None, nthreads=0, iterate=False):
    """-> (z (B,n), status, iters, kkt) [+ the final primal-dual iterates (B, obca_iterate_len) with iterate=True].
    plan mode needs x_goal (B,6); track mode xref/uref."""
    L = _obca_lib()
    N, M = P.N, P.M
    n = obca_n(N, M)
    x0 = np.ascontiguousarray(x0, dtype=np.float64).reshape(-1, 6)
    B = x0.shape[0]
    cv = lambda a, shp: None if a is None else np.ascontiguousarray(a, dtype=np.float64).reshape(shp)  # noqa: E731
    xg = cv(x_goal, (B, 6))
    xr = cv(xref, (B, N + 1, 6))
    ur = cv(uref, (B, N, 2))
    zg = cv(z_guess, (B, n))
    z = np.zeros((B, n))
    st = np.zeros(B, dtype=np.int32)
    it = np.zeros(B, dtype=np.int32)
    kk = np.zeros(B)
    I = np.zeros((B, obca_iterate_len(N, M))) if iterate else None
    rc = L.tto_obca_solve_batch_it(C.byref(P), B, _ptr(x0), _ptr(xg), _ptr(xr), _ptr(ur), _ptr(zg), _ptr(z),
                                   st.ctypes.data_as(C.POINTER(C.c_int)), it.ctypes.data_as(C.POINTER(C.c_int)),
                                   _ptr(kk), _ptr(I), int(nthreads))
    if rc != 0:
        raise RuntimeError(f"tto_obca_solve_batch failed: {rc}")
    return (z, st, it, kk, I) if iterate else (z, st, it, kk)


def obca_eval_iterate(P, x0, iterate, x_goal=None, xref=None, uref=None):
    """IPOPT's optimality error at a given primal-dual point (tto_obca_eval_iterate), one instance per row:
    -> dict of arrays E0 (scaled, IPOPT eq. (5)), dinf (unscaled dual infeasibility), pinf, compl (max |z s|), sd, sc,
    converged / acceptable (IPOPT's convergence check at P.tol / P.acc_tol), interior (the slacks inside the bounds)."""
    L = _obca_lib()
    N = P.N
    x0 = np.ascontiguousarray(x0, dtype=np.float64).reshape(-1, 6)
    B = x0.shape[0]
    I = np.ascontiguousarray(iterate, dtype=np.float64).reshape(B, obca_iterate_len(N, P.M))
    cv = lambda a, shp: None if a is None else np.ascontiguousarray(a, dtype=np.float64).reshape(shp)  # noqa: E731
    xg, xr, ur = cv(x_goal, (B, 6)), cv(xref, (B, N + 1, 6)), cv(uref, (B, N, 2))
    out = np.zeros((B, 8))
    ok = np.zeros(B, dtype=bool)
    for b in range(B):
        o = np.zeros(8)
        rc = L.tto_obca_eval_iterate(C.byref(P), _ptr(x0[b]), None if xg is None else _ptr(xg[b]),
                                     None if xr is None else _ptr(xr[b]), None if ur is None else _ptr(ur[b]),
                                     _ptr(I[b]), _ptr(o))
        out[b] = o
        ok[b] = rc == 0
    keys = ("E0", "dinf", "pinf", "compl", "sd", "sc")
    r = {k: out[:, i] for i, k in enumerate(keys)}
    r["converged"] = out[:, 6] != 0
    r["acceptable"] = out[:, 7] != 0
    r["interior"] = ok
    return r


def obca_split(z, N, M):
    """_split_decision_variables (trajectory_optimization.py:277-309): (B,n) -> X (B,N+1,6), U (B,N,2),
    mu (B,N+1,8M), lam (B,N+1,8M)."""
    z = np.asarray(z).reshape(z.shape[0], -1)
    B = z.shape[0]
    st = 8 + 16 * M
    body = z[:, : N * st].reshape(B, N, st)
    last = z[:, N * st:]
    X = np.concatenate([body[:, :, :6], last[:, None, :6]], axis=1)
    U = body[:, :, 6:8].copy()
    mu = np.concatenate([body[:, :, 8:8 + 8 * M], last[:, None, 6:6 + 8 * M]], axis=1)
    lam = np.concatenate([body[:, :, 8 + 8 * M:], last[:, None, 6 + 8 * M:]], axis=1)
    return X, U, mu, lam
