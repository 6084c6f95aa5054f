"""Mirror of python-files/mpc_control_obs.py (MPCTrackingControlObs): tracking NMPC with OBCA collision
rows on the GPU solver (TT_VARIANT_TRACK_OBCA of libttmpc.so).

Same constructor and solve(initial_state, reference_states, reference_inputs) -> (states, inputs),
"Cannot find a solution!" + last iterate on failure (mpc_control_obs.py:318-322), _last_solution kept.
IPOPT options (mpc_control_obs.py:189-193): max_iter 5000, defaults otherwise.  With an empty obstacle
list the reference NLP is the plain tracking NLP of mpc_control.py; the mirror then runs the
tracking kernel.
"""
from __future__ import annotations

import numpy as np

from ._lib import TT_VARIANT_TRACK, TT_VARIANT_TRACK_OBCA, BatchSolver, ObcaSolver
from . import scenarios
from .trajectory_planning import TrajectoryPlanning


class MPCTrackingControlObs(TrajectoryPlanning):
    _ipopt = {"max_iter": 5000}

    def __init__(self, dynamics, params, Q, R, state_bound, input_bound, obstacle_list=None, dual_init=False,
                 device=None):
        self.obstacle_list = list(obstacle_list) if obstacle_list is not None else []
        self._obstacles = scenarios.obstacles_array(self.obstacle_list) if self.obstacle_list else None
        self._variant = TT_VARIANT_TRACK_OBCA if self.obstacle_list else TT_VARIANT_TRACK
        self._dual_init = bool(dual_init)
        super().__init__(dynamics, params, Q, R, state_bound, input_bound, device=device)
        self._last_solution = None
        self.last_status = None
        self.last_iters = None

    def _make_solver(self):
        lb, ub = self._state_bound["lb"], self._state_bound["ub"]
        ulb, uub = self._input_bound["lb"], self._input_bound["ub"]
        if self._obstacles is None:
            return BatchSolver(self._horizon, self._params, self._Q, self._R, lb, ub, ulb, uub,
                               variant=TT_VARIANT_TRACK, device=self._device, **self._ipopt)
        return ObcaSolver(self._horizon, self._params, self._Q, self._R, lb, ub, ulb, uub, self._obstacles,
                          variant=TT_VARIANT_TRACK_OBCA, dual_init=self._dual_init, device=self._device,
                          **self._ipopt)

    def solve(self, initial_state, reference_states, reference_inputs):
        """mpc_control_obs.py:284-322."""
        X, U, st = self.solve_batch(np.asarray(initial_state)[None], np.asarray(reference_states)[None],
                                    np.asarray(reference_inputs)[None])
        if not self._success(st[0]):
            print("Cannot find a solution!")
        return X[0], U[0]

    def solve_batch(self, initial_states, reference_states, reference_inputs):
        """(B,6), (B,6,N+1), (B,2,N) -> (B,6,N+1), (B,2,N), status (B,)."""
        x0, xr, ur = self._batch_inputs(initial_states, reference_states, reference_inputs)
        if self._obstacles is None:
            X, U, st, it, _ = self._solver.solve(x0, xr, ur)
            Z = None
        else:
            X, U, Z, st, it, _ = self._solver.solve(x0, xref=xr, uref=ur)
        self._last_solution = Z if Z is not None else None
        self.last_status, self.last_iters = st, it
        return X.transpose(0, 2, 1).copy(), U.transpose(0, 2, 1).copy(), st
