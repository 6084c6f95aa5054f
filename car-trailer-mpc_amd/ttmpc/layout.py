"""Decision-vector layout of the reference NLP (python-files/trajectory_planning.py:38-84).

z = [x_0, u_0, x_1, u_1, ..., x_{N-1}, u_{N-1}, x_N]   (n = 8N + 6)
"""
from __future__ import annotations

import numpy as np

NX, NU = 6, 2


def pack(X, U):
    """X (B,N+1,6), U (B,N,2) -> z (B,8N+6)."""
    X = np.asarray(X, dtype=np.float64)
    U = np.asarray(U, dtype=np.float64)
    B, N = U.shape[0], U.shape[1]
    body = np.concatenate([X[:, :N], U], axis=2).reshape(B, 8 * N)
    return np.ascontiguousarray(np.concatenate([body, X[:, N]], axis=1))


def unpack(z, N):
    """z (B,8N+6) -> X (B,N+1,6), U (B,N,2)  (_split_decision_variables, trajectory_planning.py:62-84)."""
    z = np.asarray(z, dtype=np.float64)
    B = z.shape[0]
    body = z[:, : 8 * N].reshape(B, N, 8)
    X = np.concatenate([body[:, :, :NX], z[:, None, 8 * N:]], axis=1)
    return X, body[:, :, NX:].copy()


def shift(z, N, bug_compatible=True):
    """Warm-start shift of mpc_control_nmpc.py:69-88 (also mpc_control_fuzzy.py, same code).

    The reference builds the last stage from ``z[-step:-nu]`` and ``z[-nu:]`` (step = 8), i.e.
    x_{N-1} <- [u_{N-1}, x_N[0:4]], u_{N-1} <- x_N[4:6], x_N <- the same 6 values.  With
    ``bug_compatible=False`` the intended x_N / u_{N-1} are used instead."""
    z = np.asarray(z, dtype=np.float64)
    B = z.shape[0]
    step = NX + NU
    body = z[:, step: step * N]  # stages 1..N-1 -> slots 0..N-2
    if bug_compatible:
        last_state = z[:, -step:-NU]
        last_input = z[:, -NU:]
    else:
        X, U = unpack(z, N)
        last_state, last_input = X[:, -1], U[:, -1]
    return np.ascontiguousarray(np.concatenate([body, last_state, last_input, last_state], axis=1).reshape(B, -1))
