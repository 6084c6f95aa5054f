"""OBCA plan -> MPC reference hand-off.

File format of the reference: trajectory_animation.py:108-110 writes ``np.savetxt`` of the (6, N+1) state
plan and the (2, N) input plan (data/state_traj.txt, data/input_traj.txt, '%.18e', space separated);
simulation.py:445-449 reads them back and resamples dt 0.1 -> 0.05 with do_interpolation
(simulation.py:201-218: linear states, zero-order-hold inputs).

Batched path: plan_batch_to_references() takes the device outputs of an OBCA launch (B plans,
X (B,N+1,6), U (B,N,2)) and resamples all of them on the GPU (interp_kernel), so config-C4 plans feed a
ClosedLoop / tracking batch without leaving HBM.
"""
from __future__ import annotations

from pathlib import Path

import numpy as np

from .simulation import interpolate


def save_plan(states, inputs, state_path, input_path):
    """np.savetxt of states (6, N+1) and inputs (2, N) as trajectory_animation.py:108-110 does."""
    np.savetxt(state_path, np.asarray(states, dtype=np.float64))
    np.savetxt(input_path, np.asarray(inputs, dtype=np.float64))


def load_plan(state_path, input_path):
    """np.loadtxt of the two plan files (simulation.py:445-446) -> states (6, N+1), inputs (2, N)."""
    S = np.loadtxt(Path(state_path), dtype=np.float64, ndmin=2)
    U = np.loadtxt(Path(input_path), dtype=np.float64, ndmin=2)
    if S.shape[0] != 6 or U.shape[0] != 2 or S.shape[1] != U.shape[1] + 1:
        raise ValueError(f"plan files must hold (6, N+1) states and (2, N) inputs, got {S.shape} and {U.shape}")
    return S, U


def plan_batch_to_references(X, U, dt_plan=0.1, dt_mpc=0.05):
    """Device OBCA outputs X (B,N+1,6), U (B,N,2) (torch, cuda) -> per-instance MPC references
    (B, n N + 1, 6), (B, n N, 2) with n = floor(dt_plan / dt_mpc), on the GPU (do_interpolation)."""
    return interpolate(X.contiguous(), U.contiguous(), dt_plan, dt_mpc)
