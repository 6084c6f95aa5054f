"""LQR terminal score on the GPU -- python-files/LQR_cost.py:7-41, batched.

lqr_riccati(params, dynamics, Q, R, x_goal, u_goal) -> P          LQR_cost.py:7-34
lqr_distance(x_current, x_goal, params, dynamics, Q, R, u_goal)   LQR_cost.py:37-41
lqr_scores(x_cur, x_goal, params, Q, R) -> (scores, P, doublings) batched, device tensors or arrays

The DARE is solved per instance by the doubling algorithm in csrc/tt_lqr.hip (the reference calls
scipy.linalg.solve_discrete_are; tests/test_gpu_lqr.py compares the two).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from ._lib import TTError, lib
from .simulation import plant


def lqr_scores(x_cur, x_goal, params, Q, R, u_goal=None, stream=None):
    """Batched lqr_distance: x_cur, x_goal (B,6) -> score (B,), P (B,6,6), doublings (B,) as torch tensors
    on the GPU (inputs may be numpy or device tensors)."""
    dev = x_goal.device if torch.is_tensor(x_goal) and x_goal.is_cuda else torch.device("cuda", torch.cuda.current_device())
    t = lambda a: (a if torch.is_tensor(a) else torch.as_tensor(np.ascontiguousarray(a, dtype=np.float64))  # noqa: E731
                   ).to(dev, torch.float64).reshape(-1, 6).contiguous()
    xc, xg = t(x_cur), t(x_goal)
    B = xg.shape[0]
    P = torch.empty((B, 6, 6), dtype=torch.float64, device=dev)
    score = torch.empty(B, dtype=torch.float64, device=dev)
    it = torch.empty(B, dtype=torch.int32, device=dev)
    q = np.ascontiguousarray(np.asarray(Q, dtype=np.float64).reshape(36))
    r = np.ascontiguousarray(np.asarray(R, dtype=np.float64).reshape(4))
    dp = C.POINTER(C.c_double)
    s = stream if stream is not None else torch.cuda.current_stream(dev)
    p = plant(params)
    rc = lib().tt_lqr_score_device(B, C.byref(p), q.ctypes.data_as(dp), r.ctypes.data_as(dp), xc.data_ptr(),
                                   xg.data_ptr(), None, P.data_ptr(), score.data_ptr(), it.data_ptr(),
                                   C.c_void_p(s.cuda_stream))
    if rc != 0:
        raise TTError(f"tt_lqr_score_device failed ({rc})")
    return score, P, it


def lqr_riccati(params, dynamics, Q, R, x_goal, u_goal):
    """LQR_cost.py:7-34 (dynamics is accepted for signature parity; the model is the built-in one)."""
    _, P, _ = lqr_scores(np.asarray(x_goal, dtype=np.float64), np.asarray(x_goal, dtype=np.float64), params, Q, R)
    return P.cpu().numpy()[0]


def lqr_distance(x_current, x_goal, params, dynamics, Q, R, u_goal):
    """LQR_cost.py:37-41."""
    s, _, _ = lqr_scores(np.asarray(x_current, dtype=np.float64), np.asarray(x_goal, dtype=np.float64), params, Q, R)
    return float(s.cpu()[0])
