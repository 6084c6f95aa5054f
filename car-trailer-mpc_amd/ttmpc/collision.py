"""Batched separating-axis collision checks of the truck and trailer rectangles against axis-aligned
obstacles -- the reference's MPC-switch test (python-files/simulation.py:224-385), vectorised over poses.

check_state_collision(state, params, obstacle_list)   simulation.py:337-361 (one pose)
check_trajectory_collision(states, params, obstacles) simulation.py:363-385 ((6, K) trajectory)
collision_mask(poses, params, obstacles)              batched: poses (..., >=4) -> bool (...)
sat_gap(poses, params, obstacles)                     batched: largest separating gap over the four SAT
                                                      axes per (pose, body, obstacle); > 0 = separated
Body geometry: truck_trailer_model.py:58-72 (centres), 31-56 (half extents L/2, W/2).
"""
from __future__ import annotations

import numpy as np


def _obstacles(obstacle_list):
    if isinstance(obstacle_list, np.ndarray):
        return np.asarray(obstacle_list, dtype=np.float64).reshape(-1, 4)
    return np.array([[o["center"][0], o["center"][1], o["width"], o["height"]] for o in obstacle_list],
                    dtype=np.float64).reshape(-1, 4)


def _bodies(poses, params):
    """-> centres (..., 2 bodies, 2), headings (..., 2), half lengths (2,), half widths (2,)."""
    p = np.asarray(poses, dtype=np.float64)
    x, y, th, psi = p[..., 0], p[..., 1], p[..., 2], p[..., 3]
    L1, L2, M = params["L1"], params["L2"], params["M"]
    vc = np.stack([x + np.cos(th) * L1 / 2, y + np.sin(th) * L1 / 2], axis=-1)
    hx, hy = x - np.cos(th) * M, y - np.sin(th) * M
    tc = np.stack([hx - np.cos(th + psi) * L2 / 2, hy - np.sin(th + psi) * L2 / 2], axis=-1)
    centres = np.stack([vc, tc], axis=-2)
    heads = np.stack([th, th + psi], axis=-1)
    hl = np.array([L1 / 2, L2 / 2])
    hw = np.array([params["W1"] / 2, params["W2"] / 2])
    return centres, heads, hl, hw


def sat_gap(poses, params, obstacle_list):
    """Largest gap between the projections of body and obstacle over the SAT axes (obstacle x, y and the
    body's two edge normals).  Shape (..., 2, M); positive = a separating axis exists (no collision)."""
    ob = _obstacles(obstacle_list)
    centres, heads, hl, hw = _bodies(poses, params)
    c, s = np.cos(heads), np.sin(heads)
    # body half-projections on an axis a: hl |a . e_l| + hw |a . e_w|, e_l = (c, s), e_w = (-s, c)
    axes = [np.broadcast_to(np.array([1.0, 0.0]), c.shape + (2,)), np.broadcast_to(np.array([0.0, 1.0]), c.shape + (2,)),
            np.stack([-s, c], axis=-1), np.stack([c, s], axis=-1)]
    best = None
    for ax in axes:
        ax = ax[..., None, :]                                                     # (..., 2, 1, 2)
        el = np.stack([c, s], axis=-1)[..., None, :]
        ew = np.stack([-s, c], axis=-1)[..., None, :]
        rb = hl[:, None] * np.abs((ax * el).sum(-1)) + hw[:, None] * np.abs((ax * ew).sum(-1))   # (..., 2, 1)
        ro = 0.5 * ob[:, 2] * np.abs(ax[..., 0]) + 0.5 * ob[:, 3] * np.abs(ax[..., 1])           # (..., 2, M)
        dist = np.abs(((centres[..., None, :] - ob[:, :2]) * ax).sum(-1))                        # (..., 2, M)
        gap = dist - rb - ro
        best = gap if best is None else np.maximum(best, gap)
    return best


def collision_mask(poses, params, obstacle_list):
    """True where the truck or the trailer overlaps any obstacle (simulation.py:337-361 semantics:
    touching projections count as overlap)."""
    if len(_obstacles(obstacle_list)) == 0:
        return np.zeros(np.asarray(poses).shape[:-1], dtype=bool)
    return np.any(sat_gap(poses, params, obstacle_list) <= 0.0, axis=(-1, -2))


def check_state_collision(state, params, obstacle_list):
    return bool(collision_mask(np.asarray(state, dtype=np.float64)[:4], params, obstacle_list))


def check_trajectory_collision(states, params, obstacle_list):
    """states (6, K) as the reference passes them."""
    if len(_obstacles(obstacle_list)) == 0:
        return False
    return bool(np.any(collision_mask(np.asarray(states, dtype=np.float64).T, params, obstacle_list)))
