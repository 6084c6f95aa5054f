"""Mirror of python-files/trajectory_optimization.py (TrajectoryOptimization, the OBCA planner) on the
GPU solver (TT_VARIANT_OBCA_PLAN of libttmpc.so).

Same constructor (dynamics, params, Q, R, state_bound, input_bound, obstacle_list) and
plan(initial_state, goal_state) -> (states (6,N+1), inputs (2,N)); plan_batch() solves B scenarios in
one launch.  IPOPT options of the reference (trajectory_optimization.py:196-199): max_iter 5000, the
rest IPOPT defaults (tol 1e-8, acceptable 1e-6 x 15).

Initial guess: like the reference, plan() always builds it from initialize.json
(_hybrid_a_star_initial_trajectory, trajectory_optimization.py:227-274, reading ../initialize.json at
232-234), ignoring plan()'s arguments for the guess.  The file is ``initialize_path`` if given, else
$TTMPC_INITIALIZE, else ../initialize.json (the reference's location relative to python-files/, the
directory its scripts run from), else ./initialize.json; a missing file raises FileNotFoundError as the
reference's open() does.  Duals start at the reference's mu = 100, lam = kron(1_M, [100, 105, 110, 115,
...]) (222, 260-261); dual_init=True opts into the separating-axis certificate start instead.
Like the reference (326-331) plan() does not check success; ``last_status`` exposes it.
``optimize`` is an alias of ``plan`` (the entry point name BASELINE.json's north star uses).
"""
from __future__ import annotations

import os

import numpy as np

from ._lib import TT_VARIANT_OBCA_PLAN, ObcaSolver
from . import scenarios
from .trajectory_planning import TrajectoryPlanning


class TrajectoryOptimization(TrajectoryPlanning):
    _variant = TT_VARIANT_OBCA_PLAN
    _ipopt = {"max_iter": 5000}

    def __init__(self, dynamics, params, Q, R, state_bound, input_bound, obstacle_list, initialize_path=None,
                 dual_init=False, device=None):
        self.obstacle_list = list(obstacle_list)
        if len(self.obstacle_list) == 0:
            raise ValueError("TrajectoryOptimization needs at least one obstacle (trajectory_optimization.py:25-26)")
        self._obstacles = scenarios.obstacles_array(self.obstacle_list)
        self._dual_init = bool(dual_init)
        self._initialize_path = initialize_path or os.environ.get("TTMPC_INITIALIZE")
        super().__init__(dynamics, params, Q, R, state_bound, input_bound, device=device)
        self.last_status = None
        self.last_iters = None

    def _make_solver(self):
        return ObcaSolver(self._horizon, self._params, self._Q, self._R, self._state_bound["lb"],
                          self._state_bound["ub"], self._input_bound["lb"], self._input_bound["ub"], self._obstacles,
                          variant=self._variant, dual_init=self._dual_init, device=self._device, **self._ipopt)

    # trajectory_optimization.py:32-53
    def _obstacle_Hrep(self, obstacle):
        A = np.array([[1.0, 0.0], [0.0, 1.0], [-1.0, 0.0], [0.0, -1.0]])
        w, h = obstacle["width"], obstacle["height"]
        b = np.array([w / 2.0, h / 2.0, w / 2.0, h / 2.0]) + A @ np.asarray(obstacle["center"], dtype=np.float64)
        return A, b.reshape(4, 1)

    # trajectory_optimization.py:209-225
    def _generate_initial_trajectory_guess(self, initial_state, goal_state):
        N, M = self._horizon, len(self.obstacle_list)
        st = 8 + 16 * M
        z = np.zeros(N * st + 6 + 16 * M)
        duals = np.concatenate([np.full(8 * M, 100.0), np.tile(scenarios.LAM_PATTERN, M)])
        x0 = np.asarray(initial_state, dtype=np.float64)
        xg = np.asarray(goal_state, dtype=np.float64)
        for k in range(N):
            t = k / N
            z[k * st:k * st + 6] = (1 - t) * x0 + t * xg
            z[k * st + 8:(k + 1) * st] = duals
        z[N * st:N * st + 6] = xg
        z[N * st + 6:] = duals
        return z

    def _initialize_file(self, initialize_path=None):
        for cand in (initialize_path, self._initialize_path, os.path.join(os.pardir, "initialize.json"), "initialize.json"):
            if cand and os.path.exists(cand):
                return cand
        raise FileNotFoundError("initialize.json not found (trajectory_optimization.py:232 reads ../initialize.json); "
                                "pass initialize_path= or set TTMPC_INITIALIZE")

    # trajectory_optimization.py:227-274
    def _hybrid_a_star_initial_trajectory(self, initialize_path=None):
        pos, hd, hi = scenarios.load_initialize(self._initialize_file(initialize_path))
        return scenarios.obca_guess(pos, hd, hi, self._horizon, len(self.obstacle_list))

    # trajectory_optimization.py:277-309
    def _split_decision_variables(self, vars):
        N, M = self._horizon, len(self.obstacle_list)
        z = np.asarray(vars, dtype=np.float64).reshape(-1)
        st = 8 + 16 * M
        body = z[:N * st].reshape(N, st)
        last = z[N * st:]
        states = np.vstack([body[:, :6], last[None, :6]]).T.copy()
        inputs = body[:, 6:8].T.copy()
        mus = np.vstack([body[:, 8:8 + 8 * M], last[None, 6:6 + 8 * M]]).T.copy()
        lams = np.vstack([body[:, 8 + 8 * M:], last[None, 6 + 8 * M:]]).T.copy()
        return states, inputs, mus, lams

    def plan(self, initial_state, goal_state):
        """trajectory_optimization.py:311-331 -> (states (6,N+1), inputs (2,N)); the guess comes from
        initialize.json (312), never from the arguments."""
        guess = self._hybrid_a_star_initial_trajectory()
        X, U, _ = self.plan_batch(np.asarray(initial_state)[None], np.asarray(goal_state)[None], guess[None])
        return X[0], U[0]

    optimize = plan

    def plan_batch(self, initial_states, goal_states, z_guess=None):
        """B scenarios at once: (B,6), (B,6), z_guess (B,n)|None -> (B,6,N+1), (B,2,N), z (B,n)."""
        x0 = np.asarray(initial_states, dtype=np.float64).reshape(-1, 6)
        xg = np.asarray(goal_states, dtype=np.float64).reshape(-1, 6)
        X, U, Z, st, it, _ = self._solver.solve(x0, x_goal=xg, z_guess=z_guess)
        self.last_status, self.last_iters = st, it
        return X.transpose(0, 2, 1).copy(), U.transpose(0, 2, 1).copy(), Z
