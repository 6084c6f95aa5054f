"""Mirror of python-files/trajectory_planning.py: the direct-multiple-shooting base class.

Same constructor signature; the CasADi symbols are replaced by one GPU solver handle
(libttmpc.so) that every subclass configures with its IPOPT options.
"""
from __future__ import annotations

import numpy as np

from . import layout
from ._lib import TT_ACCEPTABLE, BatchSolver


def _vec(b, n):
    v = np.asarray(b, dtype=np.float64).reshape(-1)  # accepts ca.DM, lists, numpy
    if v.size != n:
        raise ValueError(f"expected {n} bound entries, got {v.size}")
    return v


class TrajectoryPlanning:
    """trajectory_planning.py:3-25 (dynamics, params, Q, R, state_bound, input_bound)."""

    _variant = 0
    _ipopt = {}

    def __init__(self, dynamics, params, Q, R, state_bound, input_bound, device=None):
        self._dynamics = dynamics
        self._params = dict(params)
        self._horizon = int(params["horizon"])
        self._num_state = dynamics.num_state
        self._num_input = dynamics.num_input
        if (self._num_state, self._num_input) != (6, 2):
            raise ValueError("the truck-trailer model has 6 states and 2 inputs (truck_trailer_model.py:4-5)")
        self._state_bound = {"lb": _vec(state_bound["lb"], 6), "ub": _vec(state_bound["ub"], 6)}
        self._input_bound = {"lb": _vec(input_bound["lb"], 2), "ub": _vec(input_bound["ub"], 2)}
        self._Q = np.asarray(Q, dtype=np.float64).reshape(6, 6)
        self._R = np.asarray(R, dtype=np.float64).reshape(2, 2)
        self._device = device
        self._solver = self._make_solver()

    def _make_solver(self):
        return BatchSolver(self._horizon, self._params, self._Q, self._R, self._state_bound["lb"],
                           self._state_bound["ub"], self._input_bound["lb"], self._input_bound["ub"],
                           variant=self._variant, device=self._device, **self._ipopt)

    # trajectory_planning.py:62-84
    def _split_decision_variables(self, vars):
        X, U = layout.unpack(np.asarray(vars, dtype=np.float64).reshape(1, -1), self._horizon)
        return X[0].T.copy(), U[0].T.copy()

    # mpc_control.py:58-65
    def _get_initial_guess(self, reference_states, reference_inputs):
        Xr = np.asarray(reference_states, dtype=np.float64).T[None]
        Ur = np.asarray(reference_inputs, dtype=np.float64).T[None]
        return layout.pack(Xr, Ur)[0]

    # ---- batched core shared by the subclasses ----
    def _batch_inputs(self, initial_states, reference_states, reference_inputs):
        """(B,6), (B,6,N+1), (B,2,N) in the reference orientation -> instance-major device layout."""
        N = self._horizon
        x0 = np.ascontiguousarray(np.asarray(initial_states, dtype=np.float64).reshape(-1, 6))
        B = x0.shape[0]
        Xr = np.asarray(reference_states, dtype=np.float64).reshape(B, 6, N + 1)
        Ur = np.asarray(reference_inputs, dtype=np.float64).reshape(B, 2, N)
        return x0, np.ascontiguousarray(Xr.transpose(0, 2, 1)), np.ascontiguousarray(Ur.transpose(0, 2, 1))

    @staticmethod
    def _success(status):
        return np.asarray(status) <= TT_ACCEPTABLE
