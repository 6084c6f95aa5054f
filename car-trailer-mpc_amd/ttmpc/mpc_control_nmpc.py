"""Mirror of python-files/mpc_control_nmpc.py (TruckTrailerNMPC) on the GPU solver.

IPOPT options (mpc_control_nmpc.py:36-45): max_iter 2000, tol 1e-3, acceptable 1e-2 x 5.
Warm start: the previous optimum shifted by one stage (mpc_control_nmpc.py:69-88), including the
reference's last-stage slicing (``bug_compatible=True``, default).  Failure -> (None, None) and the
previous solution is kept (mpc_control_nmpc.py:107-111).
"""
from __future__ import annotations

import numpy as np

from . import layout
from ._lib import TT_VARIANT_NMPC
from .trajectory_planning import TrajectoryPlanning


class TruckTrailerNMPC(TrajectoryPlanning):
    _variant = TT_VARIANT_NMPC
    _ipopt = {"max_iter": 2000, "tol": 1e-3, "acc_tol": 1e-2, "acc_iter": 5}

    def __init__(self, dynamics, params, Q, R, state_bound, input_bound, device=None, bug_compatible=True):
        super().__init__(dynamics, params, Q, R, state_bound, input_bound, device=device)
        self._last_solution = None  # (B, 8N+6) per instance, NaN rows = none yet
        self._bug_compatible = bug_compatible

    def _shift_solution(self, vars_opt):
        return layout.shift(np.asarray(vars_opt, dtype=np.float64).reshape(1, -1), self._horizon,
                            self._bug_compatible)[0]

    def _guess(self, Xr, Ur):
        B = Xr.shape[0]
        guess = layout.pack(Xr, Ur)
        if self._last_solution is not None and self._last_solution.shape[0] == B:
            have = np.all(np.isfinite(self._last_solution), axis=1)
            if have.any():
                guess[have] = layout.shift(self._last_solution[have], self._horizon, self._bug_compatible)
        return guess

    def solve_batch(self, initial_states, reference_states, reference_inputs):
        x0, xr, ur = self._batch_inputs(initial_states, reference_states, reference_inputs)
        B = x0.shape[0]
        X, U, st, it, _ = self._solver.solve(x0, xr, ur, z_guess=self._guess(xr, ur))
        ok = self._success(st)
        if self._last_solution is None or self._last_solution.shape[0] != B:
            self._last_solution = np.full((B, 8 * self._horizon + 6), np.nan)
        self._last_solution[ok] = layout.pack(X[ok], U[ok])
        return X.transpose(0, 2, 1).copy(), U.transpose(0, 2, 1).copy(), st

    def solve(self, initial_state, reference_states, reference_inputs):
        X, U, st = self.solve_batch(np.asarray(initial_state)[None], np.asarray(reference_states)[None],
                                    np.asarray(reference_inputs)[None])
        if not self._success(st[0]):
            return None, None
        return X[0], U[0]
