"""Mirror of python-files/mpc_control_fuzzy.py (MPCTrackingControlFuzzy) on the GPU solver.

Per-instance fuzzy weights (mpc_control_fuzzy.py:90-119) enter the cost squared,
Q_w = diag(w_q) Q diag(w_q), R_w = diag(w_r) R diag(w_r) (23-24); one retry with unit weights on
failure (145-159); (None, None) if both fail (160-161); shift warm start as in the NMPC class.
"""
from __future__ import annotations

import numpy as np

from . import layout
from ._lib import TT_VARIANT_FUZZY
from .trajectory_planning import TrajectoryPlanning


def fuzzy_weights(current_state, reference_states):
    """mpc_control_fuzzy.py:90-119 (hitch-angle / reversing rules, clipped to [1, 3.5])."""
    psi = float(current_state[3])
    v = float(current_state[5])
    reference_states = np.asarray(reference_states)
    ref_v = float(reference_states[5, 0]) if reference_states.size > 0 else 0.0
    h = min(abs(psi) / 0.35, 1.0)
    reversing = (ref_v < -0.1) or (v < -0.1)
    hitch, steer, steer_rate = 1.0 + 2.0 * h, 1.0 + 1.2 * h, 1.0 + 1.5 * h
    if reversing:
        hitch, steer, steer_rate = hitch * 1.1, steer * 1.1, steer_rate * 1.2
    q = np.ones(6)
    r = np.ones(2)
    q[2] = max(1.0, steer)
    q[3] = max(1.0, hitch)
    q[4] = max(1.0, steer)
    r[1] = max(1.0, steer_rate)
    return np.clip(q, 1.0, 3.5), np.clip(r, 1.0, 3.5)


class MPCTrackingControlFuzzy(TrajectoryPlanning):
    _variant = TT_VARIANT_FUZZY
    _ipopt = {"max_iter": 2000, "tol": 1e-3, "acc_tol": 1e-2, "acc_iter": 5}

    def __init__(self, dynamics, params, Q, R, state_bound, input_bound, device=None, bug_compatible=True):
        super().__init__(dynamics, params, Q, R, state_bound, input_bound, device=device)
        self._last_solution = None
        self._bug_compatible = bug_compatible

    def _compute_fuzzy_weights(self, current_state, reference_states):
        return fuzzy_weights(current_state, reference_states)

    def solve_batch(self, initial_states, reference_states, reference_inputs):
        x0, xr, ur = self._batch_inputs(initial_states, reference_states, reference_inputs)
        B, N = x0.shape[0], self._horizon
        guess = layout.pack(xr, ur)
        if self._last_solution is not None and self._last_solution.shape[0] == B:
            have = np.all(np.isfinite(self._last_solution), axis=1)
            if have.any():
                guess[have] = layout.shift(self._last_solution[have], N, self._bug_compatible)
        w = np.empty((B, 8))
        for b in range(B):
            q, r = fuzzy_weights(x0[b], xr[b].T)
            w[b, :6], w[b, 6:] = q, r
        X, U, st, _, _ = self._solver.solve(x0, xr, ur, wq_wr=w, z_guess=guess)
        bad = ~self._success(st)
        if bad.any():  # retry with unit weights, same guess (mpc_control_fuzzy.py:145-159)
            idx = np.where(bad)[0]
            X2, U2, st2, _, _ = self._solver.solve(x0[idx], xr[idx], ur[idx], wq_wr=np.ones((idx.size, 8)),
                                                   z_guess=guess[idx])
            X[idx], U[idx], st[idx] = X2, U2, st2
        ok = self._success(st)
        if self._last_solution is None or self._last_solution.shape[0] != B:
            self._last_solution = np.full((B, 8 * N + 6), np.nan)
        self._last_solution[ok] = layout.pack(X[ok], U[ok])
        return X.transpose(0, 2, 1).copy(), U.transpose(0, 2, 1).copy(), st

    def solve(self, initial_state, reference_states, reference_inputs):
        X, U, st = self.solve_batch(np.asarray(initial_state)[None], np.asarray(reference_states)[None],
                                    np.asarray(reference_inputs)[None])
        if not self._success(st[0]):
            return None, None
        return X[0], U[0]
