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
MPC_Q = np.eye(NX)           # simulation.py:400-405
MPC_R = 10.0 * np.eye(NU)    # simulation.py:406-409


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
        return obstacles_from_corners(json.load(fh))


def obstacles_from_corners(data):
    """Corner-format list (obstacles.json) -> centre / width / height dicts (get_obstacles.py:5-32)."""
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


# ----------------------------------------------------------------------------------------------
# OBCA planning scenarios (BASELINE config C4; trajectory_optimization.py / trajectory_animation.py)
# ----------------------------------------------------------------------------------------------
OBCA_PARAMS = {"M": 0.15, "L1": 7.05, "L2": 12.45, "W1": 3.05, "W2": 2.95, "dt": 0.1}  # trajectory_animation.py:48-52
# trajectory_animation.py:77-80 (theta free, v in [-5, 10])
OBCA_XLB = np.array([-np.inf, -np.inf, -np.inf, -np.pi / 3.0, -np.pi / 4.0, -5.0])
OBCA_XUB = np.array([np.inf, np.inf, np.inf, np.pi / 3.0, np.pi / 4.0, 10.0])
OBCA_ULB = np.array([-5.0, -np.pi / 2])
OBCA_UUB = np.array([5.0, np.pi / 2])
OBCA_Q = np.eye(NX)                      # trajectory_animation.py:63-69
OBCA_R = 10.0 * np.eye(NU)               # trajectory_animation.py:70-72
LAM_PATTERN = np.array([100.0, 105.0, 110.0, 115.0, 100.0, 105.0, 110.0, 115.0])  # trajectory_optimization.py:222


def obstacles_array(obstacle_list):
    """[{'center': (cx, cy), 'width': w, 'height': h}] -> (M,4) float64 (cx, cy, w, h)."""
    return np.array([[o["center"][0], o["center"][1], o["width"], o["height"]] for o in obstacle_list],
                    dtype=np.float64).reshape(-1, 4)


def interpolate_waypoints(waypoints, num_output_nodes):
    """interpolate_waypoints.py:5-26: scipy CubicSpline over linspace(0,1,W) sampled at
    linspace(0,1,num_output_nodes).  Returns the array (the reference wraps it in a 1-list)."""
    from scipy.interpolate import CubicSpline
    w = np.asarray(waypoints, dtype=np.float64)
    sp = CubicSpline(np.linspace(0.0, 1.0, len(w)), w)
    return sp(np.linspace(0.0, 1.0, num_output_nodes))


def complete_speed_steering(X, dt, L1, vlim=(-5.0, 10.0), philim=np.pi / 4):
    """Fill the speed / steering columns the reference leaves at 0 ("has to be implemented later",
    trajectory_optimization.py:251-252): v_k from the position increment along the heading, phi_k from
    the heading increment (theta_dot = v tan(phi) / L1, truck_trailer_model.py:19), both clipped to 90%
    of their bounds; v_N = phi_N = 0.  X (N+1, 6) -> copy."""
    X = np.array(X, dtype=np.float64)
    d = X[1:, :2] - X[:-1, :2]
    v = (d[:, 0] * np.cos(X[:-1, 2]) + d[:, 1] * np.sin(X[:-1, 2])) / dt
    v = np.clip(v, 0.9 * vlim[0], 0.9 * vlim[1])
    with np.errstate(divide="ignore", invalid="ignore"):
        phi = np.where(np.abs(v) > 1e-3, np.arctan(L1 * (X[1:, 2] - X[:-1, 2]) / (dt * v)), 0.0)
    X[:-1, 5] = v
    X[:-1, 4] = np.clip(phi, -0.9 * philim, 0.9 * philim)
    X[-1, 4:6] = 0.0
    return X


def obca_guess(positions, headings, hitch, N, M, complete=False, dt=0.1, L1=7.05):
    """_hybrid_a_star_initial_trajectory (trajectory_optimization.py:227-274): waypoint splines to N
    nodes, x_k = (p_k, theta_k, psi_k, 0, 0) for k < N, x_N = last node, u = 0, mu = 100,
    lam = kron(1_M, [100,105,110,115,100,105,110,115]).  ``headings`` already carry the +pi/2 shift
    (trajectory_optimization.py:238).  complete=True fills the speed/steering placeholders
    (complete_speed_steering).  Returns the reference's interleaved z (n = N(8+16M)+6+16M)."""
    P = interpolate_waypoints(positions, N)
    H = interpolate_waypoints(headings, N)
    S = interpolate_waypoints(hitch, N)
    X = np.zeros((N + 1, NX))
    X[:N, 0:2] = P
    X[:N, 2] = H
    X[:N, 3] = S
    X[N, 0:2] = P[-1]
    X[N, 2] = H[-1]
    X[N, 3] = S[-1]
    if complete:
        X = complete_speed_steering(X, dt, L1)
    st = 8 + 16 * M
    z = np.zeros(N * st + 6 + 16 * M)
    duals = np.concatenate([np.full(8 * M, 100.0), np.tile(LAM_PATTERN, M)])
    for k in range(N):
        z[k * st:k * st + 6] = X[k]
        z[k * st + 8:(k + 1) * st] = duals
    z[N * st:N * st + 6] = X[N]
    z[N * st + 6:] = duals
    return z


def obca_case_batch(cases, B: int, N: int, M: int, seed: int = 0, pos_sigma=0.5, ang_sigma=0.05, complete=False,
                    obstacles=None, params=None):
    """C4 generator: test_cases.json cases x Monte-Carlo start perturbations.  Each instance is the
    2-waypoint initialize.json of its case (apply_case.py:16-34) with a perturbed start; the guess is
    built from those waypoints (obca_guess) and (x_init, x_goal) as get_initial_goal_states.py:5-26 +
    trajectory_animation.py:83-92 (speed and steering appended as 0).

    ``obstacles`` given: only cases whose exact start and goal poses are collision-free against them are
    used, and a perturbed start that lands inside an obstacle is redrawn (an OBCA NLP pinned to a pose in
    collision is infeasible, blocked_poses).
    Returns x0 (B,6), x_goal (B,6), z_guess (B,n)."""
    rng = np.random.default_rng(seed)
    x0 = np.empty((B, NX))
    xg = np.empty((B, NX))
    st = 8 + 16 * M
    zg = np.empty((B, N * st + 6 + 16 * M))

    def waypoints(c):
        pos = np.array([[c["start"]["x"], c["start"]["y"]], [c["goal"]["x"], c["goal"]["y"]]], dtype=np.float64)
        hd = np.array([c["start"]["heading_rad"], c["goal"]["heading_rad"]], dtype=np.float64) + np.pi / 2
        hi = np.array([c["start"]["hitch_angle_rad"], c["goal"]["hitch_angle_rad"]], dtype=np.float64)
        return pos, hd, hi

    def blocked(pos, hd, hi):
        poses = np.array([[pos[i, 0], pos[i, 1], hd[i], hi[i]] for i in range(2)])
        return obstacles is not None and bool(blocked_poses(poses, obstacles, params).any())

    cases = [c for c in cases if not blocked(*waypoints(c))]
    if not cases:
        raise ValueError("no test case has a collision-free start and goal")
    for b in range(B):
        pos, hd, hi = waypoints(cases[b % len(cases)])
        if b >= len(cases):  # instance 0..len-1 are the exact cases, the rest Monte-Carlo perturbed
            base = (pos.copy(), hd.copy(), hi.copy())
            for _ in range(100):
                pos, hd, hi = base[0].copy(), base[1].copy(), base[2].copy()
                pos[0] += rng.normal(0.0, pos_sigma, 2)
                hd[0] += rng.normal(0.0, ang_sigma)
                hi[0] = float(np.clip(hi[0] + rng.normal(0.0, ang_sigma), -0.5, 0.5))
                if not blocked(pos, hd, hi):
                    break
            else:  # every redraw blocked: the exact (collision-free) case start keeps the promise
                pos, hd, hi = base
        x0[b] = [pos[0, 0], pos[0, 1], hd[0], hi[0], 0.0, 0.0]
        xg[b] = [pos[1, 0], pos[1, 1], hd[1], hi[1], 0.0, 0.0]
        zg[b] = obca_guess(pos, hd, hi, N, M, complete=complete)
    return x0, xg, zg


def obca_replan_batch(base_states, B: int, N: int, M: int, seed: int = 0, n_waypoints: int = 8,
                      pos_sigma=0.5, ang_sigma=0.05, complete=True):
    """C4 generator: Monte-Carlo re-plans around a collision-free OBCA plan.

    ``base_states`` (6, N+1) is a plan such as the reference's committed IPOPT solution
    (python-files/data/state_traj.txt).  Each instance subsamples it to ``n_waypoints`` waypoints
    (the shape of a Hybrid-A* initialize.json, trajectory_optimization.py:227-274), perturbs the
    start pose (instance 0 unperturbed) and builds the reference's guess from those waypoints
    (obca_guess; complete=True fills its speed/steering placeholders).  x_init = first waypoint,
    x_goal = last waypoint with zero steering and speed (get_initial_goal_states.py +
    trajectory_animation.py:83-92).
    Returns x0 (B,6), x_goal (B,6), z_guess (B,n)."""
    S = np.asarray(base_states, dtype=np.float64)
    rng = np.random.default_rng(seed)
    idx = np.linspace(0, S.shape[1] - 1, n_waypoints).round().astype(int)
    st = 8 + 16 * M
    x0 = np.empty((B, NX))
    xg = np.empty((B, NX))
    zg = np.empty((B, N * st + 6 + 16 * M))
    for b in range(B):
        pos = S[0:2, idx].T.copy()
        hd = S[2, idx].copy()
        hi = S[3, idx].copy()
        if b > 0:
            pos[0] += rng.normal(0.0, pos_sigma, 2)
            hd[0] += rng.normal(0.0, ang_sigma)
            hi[0] += rng.normal(0.0, ang_sigma)
        x0[b] = [pos[0, 0], pos[0, 1], hd[0], hi[0], 0.0, 0.0]
        xg[b] = [pos[-1, 0], pos[-1, 1], hd[-1], hi[-1], 0.0, 0.0]
        zg[b] = obca_guess(pos, hd, hi, N, M, complete=complete)
    return x0, xg, zg


def interpolate_plan(state_traj, input_traj, dt_1, dt_2):
    """do_interpolation (simulation.py:201-218): OBCA plan at dt_1 -> MPC reference at dt_2
    (linear states, zero-order-hold inputs)."""
    N = input_traj.shape[1]
    n = int(math.floor(dt_1 / dt_2))
    S = np.zeros((state_traj.shape[0], n * N + 1))
    U = np.zeros((input_traj.shape[0], n * N))
    for k in range(N):
        for m in range(n):
            t = m / n
            S[:, k * n + m] = (1 - t) * state_traj[:, k] + t * state_traj[:, k + 1]
            U[:, k * n + m] = input_traj[:, k]
    S[:, -1] = state_traj[:, -1]
    return S, U


def reference_window(ref_states, ref_inputs, k, horizon):
    """Reference windowing with end padding (simulation.py:485-499): (6, H+1), (2, H)."""
    N = ref_inputs.shape[1]
    Xr = np.zeros((NX, horizon + 1))
    Ur = np.zeros((NU, horizon))
    if k + horizon <= N:
        Xr[:, :] = ref_states[:, k:k + horizon + 1]
        Ur[:, :] = ref_inputs[:, k:k + horizon]
    elif k < N:
        Xr[:, :N + 1 - k] = ref_states[:, k:]
        Xr[:, N + 1 - k:] = ref_states[:, -1:]
        Ur[:, :N - k] = ref_inputs[:, k:]
        Ur[:, N - k:] = ref_inputs[:, -1:]
    else:
        Xr[:, :] = ref_states[:, -1:]
        Ur[:, :] = 0.0
    return Xr, Ur


def mpc_obs_batch(state_traj, input_traj, B: int, horizon: int, seed: int = 0, dt_plan=0.1, dt=0.05,
                  pos_sigma=0.2, ang_sigma=0.02, obstacles=None, min_gap=0.2):
    """MPC+OBCA batch (mpc_control_obs.py, driven as simulation.py:417-424, 484-522): the OBCA plan is
    interpolated to the MPC step (do_interpolation), instance b tracks the window starting at an evenly
    spread step index, x0 = window start + Gaussian perturbation.  Returns x0 (B,6), xref (B,H+1,6),
    uref (B,H,2) in the stage-major parameter layout (mpc_control_obs.py:290-301).

    With ``obstacles`` ((M,4) cx, cy, w, h) a perturbed start whose truck or trailer lies closer than
    ``min_gap`` (d_min, trajectory_optimization.py:95) to an obstacle under the reference's SAT test is
    redrawn: x_0 = x_init is a constraint of the NLP, so such a start makes it infeasible by construction
    (a closed loop never measures a pose inside an obstacle)."""
    from .collision import sat_gap
    rng = np.random.default_rng(seed)
    S, U = interpolate_plan(np.asarray(state_traj, float), np.asarray(input_traj, float), dt_plan, dt)
    ks = np.linspace(0, U.shape[1] - 1, B).round().astype(int)
    x0 = np.empty((B, NX))
    xref = np.empty((B, horizon + 1, NX))
    uref = np.empty((B, horizon, NU))
    lo = np.where(np.isfinite(XLB), XLB + 1e-6, -np.inf)
    hi = np.where(np.isfinite(XUB), XUB - 1e-6, np.inf)
    for b, k in enumerate(ks):
        Xr, Ur = reference_window(S, U, int(k), horizon)
        xref[b] = Xr.T
        uref[b] = Ur.T
        for _ in range(1000):
            pert = np.concatenate([rng.normal(0, pos_sigma, 2), rng.normal(0, ang_sigma, 2), [0.0, 0.0]])
            x0[b] = np.clip(Xr[:, 0] + pert, lo, hi)
            if obstacles is None or sat_gap(x0[b, :4], PARAMS, obstacles).min() >= min_gap:
                break
        else:  # every redraw too close: fall back to the window's own (plan) start, which must itself keep the gap
            x0[b] = np.clip(Xr[:, 0], lo, hi)
            if sat_gap(x0[b, :4], PARAMS, obstacles).min() < min_gap:
                raise ValueError(f"mpc_obs_batch: instance {b}: neither 1000 perturbed draws nor the window's own start "
                                 f"keep the gap {min_gap} to the obstacles (the NLP would be infeasible)")
            import warnings
            warnings.warn(f"mpc_obs_batch: instance {b}: no perturbed start at >= {min_gap} from the obstacles in "
                          "1000 draws; using the unperturbed window start", RuntimeWarning, stacklevel=2)
    return x0, xref, uref


def blocked_poses(poses, obstacles, params=None):
    """True where a pose (..., >=4) puts the truck or the trailer inside an obstacle (SAT gap < 0, the
    reference's check_state_collision, simulation.py:337-361): an OBCA NLP pinned to such a start or goal is
    infeasible."""
    from .collision import sat_gap
    return sat_gap(np.asarray(poses)[..., :4], params or PARAMS, obstacles).min(axis=(-1, -2)) < 0.0


# ----------------------------------------------------------------------------------------------
# scenario generators / writers of the reference
# ----------------------------------------------------------------------------------------------
STALL_WIDTH, STRIPE_WIDTH, WALL_WIDTH, N_STALLS = 5.0, 1.0, 30.0, 10


def _rect(x0, x1, y0, y1):
    """corner format of obstacles.json: FL/FR at the far edge y1, BL/BR at y0."""
    return {"FL": {"X": x0, "Y": y1}, "FR": {"X": x1, "Y": y1}, "BL": {"X": x0, "Y": y0}, "BR": {"X": x1, "Y": y0}}


def build_parking_obstacles(open_spot: int, depth: float = 20.0):
    """One-sided parking row (make_parking_obstacles.py:6-51): two 30 m walls bounding 10 stalls of
    5 m separated by 1 m stripes, every stall blocked except ``open_spot`` (1-based).  Returns the
    obstacles.json corner-format list (walls first, then stalls in x order)."""
    if not 1 <= open_spot <= N_STALLS:
        raise ValueError("open_spot must be between 1 and 10 (inclusive)")
    pitch = STALL_WIDTH + STRIPE_WIDTH
    span_end = STRIPE_WIDTH + N_STALLS * pitch - STRIPE_WIDTH
    out = [_rect(-WALL_WIDTH, 0.0, 0.0, depth), _rect(span_end, span_end + WALL_WIDTH, 0.0, depth)]
    for i in range(N_STALLS):
        if i + 1 != open_spot:
            x0 = STRIPE_WIDTH + i * pitch
            out.append(_rect(x0, x0 + STALL_WIDTH, 0.0, depth))
    return out


def parking_goal(open_spot: int):
    """Goal the reference writes for the open stall (make_parking_obstacles.py:83-87): stall centre x,
    y = 12.45 (parked flush at the trailer length)."""
    return STRIPE_WIDTH + (open_spot - 1) * (STALL_WIDTH + STRIPE_WIDTH) + STALL_WIDTH / 2.0, 12.45


def initialize_doc(case: dict) -> dict:
    """The 2-waypoint initialize.json of a test_cases.json case (apply_case.py:16-34)."""
    s, g = case["start"], case["goal"]
    return {"Positions": [[s["x"], s["y"]], [g["x"], g["y"]]],
            "Headings": [s["heading_rad"], g["heading_rad"]],
            "HitchAngles": [s["hitch_angle_rad"], g["hitch_angle_rad"]]}


def write_initialize(case: dict, output_path) -> None:
    """apply_case.write_initialize: json.dump(indent=2) of initialize_doc(case)."""
    with open(output_path, "w") as fh:
        json.dump(initialize_doc(case), fh, indent=2)


def load_test_cases(path) -> dict:
    """test_cases.json -> {name: case} (apply_case.py:10-13)."""
    with open(path) as fh:
        return {c["name"]: c for c in json.load(fh)["cases"]}
