"""Deterministic synthetic MPC batches and scenario I/O helpers.

Instances are independent tracking problems of the reference controller
(python-files/mpc_control.py) with the reference's params/weights/bounds
(python-files/simulation.py:391-414):

* reference: xr_0 random feasible pose, ur_k random inputs, xr_{k+1} = xr_k + dt f(xr_k, ur_k)
  (forward Euler, truck_trailer_model.py:26-29), regenerated while any bound is violated;
* x0 = xr_0 + N(0, diag(.5,.5,.05,.05,.02,.2)^2), clipped into the bounds.

All arrays are instance-major, C-contiguous float64:
x0 (B,6), xref (B,N+1,6), uref (B,N,2) -- the stage-major layout of the reference parameter vector
(mpc_control.py:45-52, 86-88) per instance.
"""
from __future__ import annotations

import json
import math
from pathlib import Path

import numpy as np

NX, NU = 6, 2
PARAMS = {"M": 0.15, "L1": 7.05, "L2": 12.45, "W1": 3.05, "W2": 2.95, "dt": 0.05}
XLB = np.array([-np.inf, -np.inf, -np.pi, -np.pi / 3.0, -np.pi / 4.0, -10.0])
XUB = np.array([np.inf, np.inf, np.pi, np.pi / 3.0, np.pi / 4.0, 10.0])
ULB = np.array([-5.0, -np.pi / 2])
UUB = np.array([5.0, np.pi / 2])


def _f(q, u, p):
    L1, L2, M = p["L1"], p["L2"], p["M"]
    th, psi, phi, v = q[:, 2], q[:, 3], q[:, 4], q[:, 5]
    t = np.tan(phi)
    out = np.empty_like(q)
    out[:, 0] = v * np.cos(th)
    out[:, 1] = v * np.sin(th)
    out[:, 2] = v * t / L1
    out[:, 3] = -v * t / L1 * (1 + M / L2 * np.cos(psi)) - v * np.sin(psi) / L2
    out[:, 4] = u[:, 1]
    out[:, 5] = u[:, 0]
    return out


def synthetic_batch(B: int, N: int, seed: int = 0, psi_range: float = 0.3, params=None,
                    xlb=XLB, xub=XUB, ulb=ULB, uub=UUB):
    """SURVEY.md §8(d) generator.  psi_range=0.9 is the C3 hitch-stress variant."""
    p = dict(PARAMS if params is None else params)
    rng = np.random.default_rng(seed)
    x0 = np.empty((B, NX))
    xref = np.empty((B, N + 1, NX))
    uref = np.empty((B, N, NU))
    todo = np.arange(B)
    lo = np.where(np.isfinite(xlb), xlb, -np.inf)
    hi = np.where(np.isfinite(xub), xub, np.inf)
    while todo.size:
        nb = todo.size
        xr = np.empty((nb, N + 1, NX))
        xr[:, 0, 0:2] = rng.uniform(0.0, 60.0, (nb, 2))
        xr[:, 0, 2] = rng.uniform(-np.pi / 2, np.pi / 2, nb)
        xr[:, 0, 3] = rng.uniform(-psi_range, psi_range, nb)
        xr[:, 0, 4] = rng.uniform(-0.3, 0.3, nb)
        xr[:, 0, 5] = rng.uniform(-3.0, 3.0, nb)
        ur = np.empty((nb, N, NU))
        ur[:, :, 0] = rng.uniform(-1.0, 1.0, (nb, N))
        ur[:, :, 1] = rng.uniform(-0.3, 0.3, (nb, N))
        for k in range(N):
            xr[:, k + 1] = xr[:, k] + p["dt"] * _f(xr[:, k], ur[:, k], p)
        ok = np.all((xr >= lo) & (xr <= hi), axis=(1, 2)) & np.all((ur >= ulb) & (ur <= uub), axis=(1, 2))
        noise = rng.normal(0.0, 1.0, (nb, NX)) * np.array([0.5, 0.5, 0.05, 0.05, 0.02, 0.2])
        xi = np.clip(xr[:, 0] + noise, lo, hi)
        good = todo[ok]
        x0[good] = xi[ok]
        xref[good] = xr[ok]
        uref[good] = ur[ok]
        todo = todo[~ok]
    return np.ascontiguousarray(x0), np.ascontiguousarray(xref), np.ascontiguousarray(uref)


# ----------------------------------------------------------------------------------------------
# reference scenario files -- read-only helpers over the reference formats
# ----------------------------------------------------------------------------------------------
def load_initialize(path):
    """initialize.json -> (positions (W,2), headings+pi/2 (W,), hitch (W,)),
    get_initial_goal_states.py:5-26 / trajectory_optimization.py:232-239."""
    with open(path) as fh:
        d = json.load(fh)
    pos = np.asarray(d["Positions"], dtype=np.float64)
    hd = np.asarray(d["Headings"], dtype=np.float64) + np.pi / 2
    hi = np.asarray(d["HitchAngles"], dtype=np.float64)
    return pos, hd, hi


def load_obstacles(path):
    """obstacles.json corner format -> [{'center': (cx, cy), 'width': w, 'height': h}] rounded to 4 dp
    (get_obstacles.py:5-32)."""
    with open(path) as fh:
        data = json.load(fh)
    out = []
    for ob in data:
        FL, FR, BL, BR = ob["FL"], ob["FR"], ob["BL"], ob["BR"]
        cx = round((FL["X"] + FR["X"] + BL["X"] + BR["X"]) / 4, 4)
        cy = round((FL["Y"] + FR["Y"] + BL["Y"] + BR["Y"]) / 4, 4)
        out.append({"center": (cx, cy), "width": round(abs(FR["X"] - FL["X"]), 4),
                    "height": round(abs(BL["Y"] - FL["Y"]), 4)})
    return out


def straight_line_reference(start, goal, N):
    """C5 reference: straight-line pose interpolation start -> goal over the horizon, zero inputs."""
    start = np.asarray(start, dtype=np.float64)
    goal = np.asarray(goal, dtype=np.float64)
    t = np.linspace(0.0, 1.0, N + 1)[:, None]
    return (1 - t) * start[None, :] + t * goal[None, :], np.zeros((N, NU))


def test_case_batch(cases, B: int, N: int, seed: int = 0, pos_sigma=0.5, ang_sigma=0.05):
    """C5 generator: mixed test_cases.json scenarios x Monte-Carlo start perturbations.
    ``cases`` is the parsed test_cases.json ``cases`` list (heading convention of
    initialize.json, +pi/2 applied as in get_initial_goal_states.py:13)."""
    rng = np.random.default_rng(seed)
    x0 = np.empty((B, NX))
    xref = np.empty((B, N + 1, NX))
    uref = np.zeros((B, N, NU))
    for b in range(B):
        c = cases[b % len(cases)]
        s = np.array([c["start"]["x"], c["start"]["y"], c["start"]["heading_rad"] + np.pi / 2,
                      c["start"]["hitch_angle_rad"], 0.0, 0.0])
        g = np.array([c["goal"]["x"], c["goal"]["y"], c["goal"]["heading_rad"] + np.pi / 2,
                      c["goal"]["hitch_angle_rad"], 0.0, 0.0])
        s[2] = math.remainder(s[2], 2 * math.pi)
        g[2] = s[2] + math.remainder(g[2] - s[2], 2 * math.pi)
        g[2] = float(np.clip(g[2], -np.pi + 1e-3, np.pi - 1e-3))
        xr, _ = straight_line_reference(s, g, N)
        xref[b] = xr
        pert = np.concatenate([rng.normal(0, pos_sigma, 2), rng.normal(0, ang_sigma, 2), [0.0, 0.0]])
        x0[b] = np.clip(s + pert, np.where(np.isfinite(XLB), XLB + 1e-6, -np.inf),
                        np.where(np.isfinite(XUB), XUB - 1e-6, np.inf))
    return x0, xref, uref


def default_data_dir() -> Path:
    return Path(__file__).resolve().parent / "data"
