"""Mirror of python-files/mpc_control.py (MPCTrackingControl) on the GPU solver.

IPOPT options of the reference (mpc_control.py:35-39): max_iter 5000, tol 1e-8 (default),
acceptable 1e-6 x 15 (defaults).
"""
from __future__ import annotations

import numpy as np

from ._lib import TT_VARIANT_TRACK
from .trajectory_planning import TrajectoryPlanning


class MPCTrackingControl(TrajectoryPlanning):
    _variant = TT_VARIANT_TRACK
    _ipopt = {"max_iter": 5000}

    def __init__(self, dynamics, params, Q, R, state_bound, input_bound, device=None):
        super().__init__(dynamics, params, Q, R, state_bound, input_bound, device=device)
        self.last_status = None
        self.last_iters = None

    def solve(self, initial_state, reference_states, reference_inputs):
        """mpc_control.py:67-110: returns (states (6,N+1), inputs (2,N)); on failure prints
        "Cannot find a solution!" and still returns the last iterate (mpc_control.py:106-110)."""
        X, U, st = self.solve_batch(np.asarray(initial_state)[None], np.asarray(reference_states)[None],
                                    np.asarray(reference_inputs)[None])
        if not self._success(st[0]):
            print("Cannot find a solution!")
        return X[0], U[0]

    def solve_batch(self, initial_states, reference_states, reference_inputs):
        """B instances at once: (B,6), (B,6,N+1), (B,2,N) -> (B,6,N+1), (B,2,N), status (B,)."""
        x0, xr, ur = self._batch_inputs(initial_states, reference_states, reference_inputs)
        X, U, st, it, _ = self._solver.solve(x0, xr, ur)
        self.last_status, self.last_iters = st, it
        return X.transpose(0, 2, 1).copy(), U.transpose(0, 2, 1).copy(), st
