"""CPU ORACLE (test infrastructure only) -- KKT certificate of a given OBCA plan (X, U).

THIS IS A CHECKER.  Only tests/ import it.

The reference commits one IPOPT optimum of its OBCA NLP: python-files/data/state_traj.txt (6 x 201) and
input_traj.txt (2 x 200), written by trajectory_animation.py:108-111 from TrajectoryOptimization.plan
(trajectory_optimization.py:311-331, N = 200, dt = 0.1).  Only the states and inputs are stored: the OBCA
duals mu/lam (primal variables of the NLP), the goal x_goal (a parameter) and every multiplier are not.
``certify_plan`` rebuilds them and reports how well (X, U) satisfies the first-order conditions of the
restated NLP (the statement tt_obca.c / tt_obca.hip solve; trajectory_optimization.py:93-183):

  * mu/lam of every (stage, obstacle, body) block: the exact dual certificate of the rectangle-rectangle
    distance (closest points of the two polygons; lam = A-facet weights of the unit normal n, mu = body
    facet weights of -R'n), so G'mu + R'A'lam = 0, ||A'lam|| = 1 and d1 = d_min - dist(body, obstacle);
  * blocks with dist - d_min <= act_tol are active: their 4 row multipliers (y1 >= 0, y2 / y3 free for the
    +-1e-5 range rows, y4 >= 0) and the mu/lam bound multipliers of zero entries (>= 0) are unknowns;
  * x_goal, the dynamics multipliers, the final-box multipliers and the multipliers of active variable
    bounds are unknowns;
  * stationarity of the Lagrangian in (x, u, mu, lam) is linear in all unknowns: bounded least squares
    (scipy lsq_linear, bounded=True), as oracle/obca_nlp.ObcaNLP.kkt_check does, or plain least squares
    with every multiplier free (bounded=False) -- a lower bound of the bounded residual, seconds instead
    of minutes when many blocks are active.

Checked on the oracle's own optima (tests/test_obca_oracle.py): stat_rel ~1e-8.  On the reference's
committed plan the free fit already leaves stat_rel 1.06e-2, concentrated in the input rows
2 R u_k - dt y_{k+1}[(5, 4)] of stages 0-14 ("KKT certificate").
Row Jacobians come from the C oracle's block linearisation (tto_obca_block_lin, itself checked against
finite differences in tests/test_obca_oracle.py).
"""
from __future__ import annotations

import ctypes as C

import numpy as np


def _poly(center, ang, hl, hw):
    c, s = np.cos(ang), np.sin(ang)
    ex, ey = np.array([c, s]), np.array([-s, c])
    return np.array([center + hl * ex + hw * ey, center - hl * ex + hw * ey, center - hl * ex - hw * ey,
                     center + hl * ex - hw * ey])


def _seg_point(a, b, p):
    d = b - a
    t = np.clip(np.dot(p - a, d) / np.dot(d, d), 0.0, 1.0)
    return a + t * d


def polygon_distance(P, Q):
    """Distance and closest points (on P, on Q) of two disjoint convex polygons (vertex lists)."""
    best = (np.inf, None, None)
    for A, B, flip in ((P, Q, False), (Q, P, True)):
        for v in A:
            for i in range(len(B)):
                q = _seg_point(B[i], B[(i + 1) % len(B)], v)
                d = np.linalg.norm(v - q)
                if d < best[0]:
                    best = (d, q, v) if flip else (d, v, q)
    return best


def _body(x, b, p):
    """centre, angle, half length, half width of body b (0 truck, 1 trailer) at state x
    (truck_trailer_model.py:31-72)."""
    X, Y, th, ps = x[:4]
    if b == 0:
        return np.array([X + 0.5 * p["L1"] * np.cos(th), Y + 0.5 * p["L1"] * np.sin(th)]), th, 0.5 * p["L1"], 0.5 * p["W1"]
    hx, hy = X - p["M"] * np.cos(th), Y - p["M"] * np.sin(th)
    return (np.array([hx - 0.5 * p["L2"] * np.cos(th + ps), hy - 0.5 * p["L2"] * np.sin(th + ps)]), th + ps,
            0.5 * p["L2"], 0.5 * p["W2"])


def certify_plan(X, U, obstacles, params, Q, R, xlb, xub, ulb, uub, dmin=0.2, tfac=100.0, act_tol=1e-6,
                 bound_tol=1e-6, bounded=True):
    """X (N+1, 6), U (N, 2) -> dict(stat_rel, stat, n_active, x_goal, residual, ...).  The final-box rows
    |x_N - x_goal| <= 1e-2 get free multipliers (either side may be active)."""
    from scipy.optimize import lsq_linear
    from scipy.sparse import coo_matrix

    from . import c_oracle as co
    X, U = np.asarray(X, float), np.asarray(U, float)
    N = U.shape[0]
    ob = np.asarray(obstacles, float).reshape(-1, 4)
    M = ob.shape[0]
    dt = params["dt"]
    P = co.make_obca_problem(N, params, Q, R, xlb, xub, ulb, uub, ob)
    P.dmin = dmin
    L = co.lib()
    dp = C.POINTER(C.c_double)
    L.tto_obca_block_lin.argtypes = [C.POINTER(co.TTOObcaProblem), dp, C.c_int, dp, dp, dp, dp, dp, dp, dp, dp]
    ptr = lambda a: a.ctypes.data_as(dp)  # noqa: E731
    Qs, Rs = 0.5 * (Q + Q.T), 0.5 * (R + R.T)

    rows, cols, vals = [], [], []
    nrow_x = 6 * (N + 1)
    nrow_u = 2 * N
    rhs = []
    # unknown columns
    col = 0
    c_g = col; col += 6
    c_y = col; col += 6 * (N + 1)
    c_f = col; col += 6
    lo, hi = [-np.inf] * (6 + 6 * (N + 1) + 6), [np.inf] * (6 + 6 * (N + 1) + 6)

    def add(r, c, v):
        rows.append(r); cols.append(c); vals.append(v)

    # --- gradient of the cost (constant part) and its x_goal part; dynamics multipliers
    b = np.zeros(nrow_x + nrow_u)   # right-hand side = -(x-dependent constant part of the gradient)
    for k in range(N + 1):
        sc = tfac if k == N else 1.0
        gk = 2.0 * sc * Qs @ X[k]
        b[6 * k:6 * k + 6] -= gk
        for i in range(6):
            for j in range(6):
                add(6 * k + i, c_g + j, -2.0 * sc * Qs[i, j])
            add(6 * k + i, c_y + 6 * k + i, 1.0)                     # row c_k = x_k - ...: +y_k
        if k < N:
            th, psi, phi, v = X[k, 2], X[k, 3], X[k, 4], X[k, 5]
            L1, L2, Mh = params["L1"], params["L2"], params["M"]
            t, cphi = np.tan(phi), np.cos(phi)
            kk = 1.0 + Mh / L2 * np.cos(psi)
            A = np.eye(6)
            A[0, 2] += dt * (-v * np.sin(th)); A[0, 5] += dt * np.cos(th)
            A[1, 2] += dt * (v * np.cos(th)); A[1, 5] += dt * np.sin(th)
            A[2, 4] += dt * (v / cphi ** 2 / L1); A[2, 5] += dt * (t / L1)
            A[3, 3] += dt * (v * t * Mh * np.sin(psi) / (L1 * L2) - v * np.cos(psi) / L2)
            A[3, 4] += dt * (-v / cphi ** 2 / L1 * kk)
            A[3, 5] += dt * (-t / L1 * kk - np.sin(psi) / L2)
            for i in range(6):
                for r in range(6):
                    if A[r, i] != 0.0:
                        add(6 * k + i, c_y + 6 * (k + 1) + r, -A[r, i])  # row c_{k+1} = x_{k+1} - x_k - dt f
            for i in range(2):
                b[nrow_x + 2 * k + i] -= 2.0 * (Rs[i] @ U[k])
                add(nrow_x + 2 * k + i, c_y + 6 * (k + 1) + (5 if i == 0 else 4), -dt)
    for i in range(6):
        add(6 * N + i, c_f + i, 1.0)                                      # final box rows x_N - g
    # --- active variable bounds
    for k in range(N + 1):
        for i in range(6):
            for bnd, sgn in ((xlb[i], -1.0), (xub[i], 1.0)):
                if np.isfinite(bnd) and abs(X[k, i] - bnd) <= bound_tol * max(1.0, abs(bnd)):
                    add(6 * k + i, col, sgn); lo.append(0.0); hi.append(np.inf); col += 1
        if k < N:
            for i in range(2):
                for bnd, sgn in ((ulb[i], -1.0), (uub[i], 1.0)):
                    if np.isfinite(bnd) and abs(U[k, i] - bnd) <= bound_tol * max(1.0, abs(bnd)):
                        add(nrow_x + 2 * k + i, col, sgn); lo.append(0.0); hi.append(np.inf); col += 1
    # --- OBCA blocks
    n_active, r_w = 0, nrow_x + nrow_u
    dists = np.full((N + 1, M, 2), np.inf)
    for k in range(N + 1):
        for i in range(M):
            cx, cy, w, h = ob[i]
            O = np.array([[cx + w / 2, cy + h / 2], [cx - w / 2, cy + h / 2], [cx - w / 2, cy - h / 2], [cx + w / 2, cy - h / 2]])
            for bd in range(2):
                cen, ang, hl, hw = _body(X[k], bd, params)
                d, cb, cq = polygon_distance(_poly(cen, ang, hl, hw), O)
                dists[k, i, bd] = d
                if d - dmin > act_tol:
                    continue                                              # inactive: y = 0
                n_active += 1
                nrm = (cb - cq) / d
                m = -np.array([np.cos(ang) * nrm[0] + np.sin(ang) * nrm[1], -np.sin(ang) * nrm[0] + np.cos(ang) * nrm[1]])
                wv = np.array([max(m[0], 0), max(m[1], 0), max(-m[0], 0), max(-m[1], 0),
                               max(nrm[0], 0), max(nrm[1], 0), max(-nrm[0], 0), max(-nrm[1], 0)])
                out = [np.zeros(n_) for n_ in (4, 16, 32, 16, 32, 16)]
                L.tto_obca_block_lin(C.byref(P), ptr(np.ascontiguousarray(X[k])), 2 * i + bd, ptr(wv), None, *[ptr(o) for o in out])
                Jx, Jw = out[1].reshape(4, 4), out[2].reshape(4, 8)
                cy_ = col
                for r in range(4):
                    lo.append(0.0 if r in (0, 3) else -np.inf); hi.append(np.inf)
                    for q in range(4):
                        add(6 * k + q, cy_ + r, Jx[r, q])
                    for a in range(8):
                        add(r_w + a, cy_ + r, Jw[r, a])
                col += 4
                for a in range(8):                                         # bound multipliers of zero duals
                    if wv[a] <= 1e-14:
                        add(r_w + a, col, -1.0); lo.append(0.0); hi.append(np.inf); col += 1
                r_w += 8
    nrows = r_w
    b = np.concatenate([b, np.zeros(nrows - nrow_x - nrow_u)])
    Am = coo_matrix((vals, (rows, cols)), shape=(nrows, col)).toarray()
    if bounded:
        sol = lsq_linear(Am, b, bounds=(np.array(lo), np.array(hi)), method="bvls", tol=1e-15, max_iter=20000).x
    else:
        sol = np.linalg.lstsq(Am, b, rcond=None)[0]
    r = Am @ sol - b
    grad_scale = max(1.0, np.max(np.abs(b)))
    xg = sol[c_g:c_g + 6]
    return {"stat": float(np.max(np.abs(r))), "stat_rel": float(np.max(np.abs(r)) / grad_scale), "n_active": n_active,
            "x_goal": xg, "final_offset": X[N] - xg, "min_dist": float(dists.min()), "grad_scale": grad_scale,
            "residual": r, "nrow_x": nrow_x, "nrow_u": nrow_u}
