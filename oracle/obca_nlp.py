"""CPU ORACLE (test infrastructure only) -- numpy restatement of the OBCA NLPs for independent checks.

THIS IS THE CHECKER, NOT THE PRODUCT.  Only tests/ and fixture scripts import it.

Restates, directly from the reference (python-files/), as plain vectorised numpy functions of the
reference's decision vector z (layout trajectory_optimization.py:55-91):
  * g(z) = [g_dyn; g_col; g_fin] with lbg/ubg       trajectory_planning.py:28-36,
                                                    trajectory_optimization.py:93-166 (OBCA rows),
                                                    168-174 (final box); mpc_control_obs.py:65-138
  * lbx/ubx                                         trajectory_optimization.py:55-91
  * J(z) = cost                                     trajectory_optimization.py:176-183 (plan),
                                                    mpc_control_obs.py:31-41 (track)
Derivatives are by central finite differences (no shared code with tt_obca.c), so kkt_check() is an
independent optimality certificate for a solution returned by the C oracle or the GPU.
"""
from __future__ import annotations

import numpy as np


class ObcaNLP:
    def __init__(self, N, M, params, Q, R, xlb, xub, ulb, uub, obstacles, mode="plan", dmin=0.2, eq_tol=1e-5,
                 fin_tol=1e-2):
        self.N, self.M, self.p = int(N), int(M), dict(params)
        self.Q, self.R = np.asarray(Q, float), np.asarray(R, float)
        self.xlb, self.xub, self.ulb, self.uub = (np.asarray(v, float) for v in (xlb, xub, ulb, uub))
        self.ob = np.asarray(obstacles, float).reshape(-1, 4)[:M]
        self.mode, self.dmin, self.eq_tol, self.fin_tol = mode, dmin, eq_tol, fin_tol
        self.st = 8 + 16 * self.M
        self.n = self.N * self.st + 6 + 16 * self.M

    # ---- layout (trajectory_optimization.py:55-91, 277-309) ----
    def split(self, z):
        N, M, st = self.N, self.M, self.st
        z = np.asarray(z, float)
        body = z[:N * st].reshape(N, st)
        last = z[N * st:]
        X = np.vstack([body[:, :6], last[None, :6]])
        U = body[:, 6:8]
        mu = np.vstack([body[:, 8:8 + 8 * M], last[None, 6:6 + 8 * M]])
        lam = np.vstack([body[:, 8 + 8 * M:], last[None, 6 + 8 * M:]])
        return X, U, mu, lam

    def bounds(self):
        N, M = self.N, self.M
        lb_k = np.concatenate([self.xlb, self.ulb, np.zeros(16 * M)])
        ub_k = np.concatenate([self.xub, self.uub, np.full(16 * M, np.inf)])
        lb = np.concatenate([np.tile(lb_k, N), self.xlb, np.zeros(16 * M)])
        ub = np.concatenate([np.tile(ub_k, N), self.xub, np.full(16 * M, np.inf)])
        return lb, ub

    # ---- model (truck_trailer_model.py:8-29) ----
    def f(self, X, U):
        L1, L2, Mh = self.p["L1"], self.p["L2"], self.p["M"]
        th, psi, phi, v = X[:, 2], X[:, 3], X[:, 4], X[:, 5]
        return np.stack([v * np.cos(th), v * np.sin(th), v * np.tan(phi) / L1,
                         -v * np.tan(phi) / L1 * (1 + Mh / L2 * np.cos(psi)) - v * np.sin(psi) / L2,
                         U[:, 1], U[:, 0]], axis=1)

    # ---- constraints ----
    def g(self, z, x_init, x_goal=None):
        X, U, mu, lam = self.split(z)
        dyn = [X[0] - x_init, (X[1:] - (X[:-1] + self.p["dt"] * self.f(X[:-1], U))).reshape(-1)]
        L1, L2, W1, W2, Mh = self.p["L1"], self.p["L2"], self.p["W1"], self.p["W2"], self.p["M"]
        x, y, th, psi = X[:, 0], X[:, 1], X[:, 2], X[:, 3]
        pv = np.stack([x + np.cos(th) * L1 / 2, y + np.sin(th) * L1 / 2], axis=1)          # truck_trailer_model.py:58-61
        hx, hy = x - np.cos(th) * Mh, y - np.sin(th) * Mh                                    # 63-72
        pt = np.stack([hx - np.cos(th + psi) * L2 / 2, hy - np.sin(th + psi) * L2 / 2], axis=1)
        gv = np.array([L1 / 2, W1 / 2, L1 / 2, W1 / 2])
        gt = np.array([L2 / 2, W2 / 2, L2 / 2, W2 / 2])
        K = self.N + 1
        R = np.zeros((K, self.M, 8))
        for i, (cx, cy, w, h) in enumerate(self.ob):
            b = np.array([w / 2 + cx, h / 2 + cy, w / 2 - cx, h / 2 - cy])               # trajectory_optimization.py:32-53
            mv, mt = mu[:, 8 * i:8 * i + 4], mu[:, 8 * i + 4:8 * i + 8]
            lv, lt = lam[:, 8 * i:8 * i + 4], lam[:, 8 * i + 4:8 * i + 8]
            Apv = np.stack([pv[:, 0], pv[:, 1], -pv[:, 0], -pv[:, 1]], axis=1)             # A p, A = [I; -I]
            Apt = np.stack([pt[:, 0], pt[:, 1], -pt[:, 0], -pt[:, 1]], axis=1)
            R[:, i, 0] = mv @ gv - ((Apv - b) * lv).sum(1) + self.dmin
            R[:, i, 1] = mt @ gt - ((Apt - b) * lt).sum(1) + self.dmin
            av, cv = lv[:, 0] - lv[:, 2], lv[:, 1] - lv[:, 3]                                 # A' lam
            at, ct = lt[:, 0] - lt[:, 2], lt[:, 1] - lt[:, 3]
            c1, s1, c2, s2 = np.cos(th), np.sin(th), np.cos(th + psi), np.sin(th + psi)
            R[:, i, 2] = mv[:, 0] - mv[:, 2] + c1 * av + s1 * cv                              # G'mu + R'A'lam
            R[:, i, 3] = mv[:, 1] - mv[:, 3] - s1 * av + c1 * cv
            R[:, i, 4] = mt[:, 0] - mt[:, 2] + c2 * at + s2 * ct
            R[:, i, 5] = mt[:, 1] - mt[:, 3] - s2 * at + c2 * ct
            R[:, i, 6] = np.hypot(av, cv) - 1.0
            R[:, i, 7] = np.hypot(at, ct) - 1.0
        rows = R.reshape(-1)
        lo = np.tile([-np.inf, -np.inf] + [-self.eq_tol] * 4 + [-np.inf, -np.inf], K * self.M)
        hi = np.tile([0.0, 0.0] + [self.eq_tol] * 4 + [0.0, 0.0], K * self.M)
        out = [np.concatenate(dyn), rows]
        lbg = [np.zeros(6 * (self.N + 1)), np.array(lo)]
        ubg = [np.zeros(6 * (self.N + 1)), np.array(hi)]
        if self.mode == "plan":
            out.append(X[-1] - x_goal)
            lbg.append(np.full(6, -self.fin_tol))
            ubg.append(np.full(6, self.fin_tol))
        return np.concatenate(out), np.concatenate(lbg), np.concatenate(ubg)

    def cost(self, z, x_goal=None, xref=None, uref=None):
        X, U, _, _ = self.split(z)
        if self.mode == "plan":
            E = X - x_goal
            return float(np.einsum("ki,ij,kj->", U, self.R, U) + np.einsum("ki,ij,kj->", E[:-1], self.Q, E[:-1])
                         + E[-1] @ (100.0 * self.Q) @ E[-1])
        E, F = X - xref, U - uref
        return float(np.einsum("ki,ij,kj->", E, self.Q, E) + np.einsum("ki,ij,kj->", F, self.R, F))

    # ---- independent KKT certificate ----
    def kkt_check(self, z, x_init, x_goal=None, xref=None, uref=None, act_tol=1e-5, h=1e-6):
        """Finite-difference Jacobians, multipliers by bounded least squares on the active set.
        Returns dict(stat, prim, bviol): stationarity residual (inf-norm), constraint violation,
        bound violation (both against the reference's unrelaxed bounds)."""
        from scipy.optimize import lsq_linear
        z = np.asarray(z, float)
        n = z.size
        F = lambda zz: self.cost(zz, x_goal, xref, uref)  # noqa: E731
        G = lambda zz: self.g(zz, x_init, x_goal)[0]      # noqa: E731
        g0, lbg, ubg = self.g(z, x_init, x_goal)
        grad = np.empty(n)
        J = np.empty((g0.size, n))
        for j in range(n):
            e = np.zeros(n)
            e[j] = h * max(1.0, abs(z[j]))
            grad[j] = (F(z + e) - F(z - e)) / (2 * e[j])
            J[:, j] = (G(z + e) - G(z - e)) / (2 * e[j])
        lb, ub = self.bounds()
        prim = float(max(0.0, np.max(lbg - g0), np.max(g0 - ubg)))
        bviol = float(max(0.0, np.max(np.where(np.isfinite(lb), lb - z, -1.0)), np.max(np.where(np.isfinite(ub), z - ub, -1.0))))
        # active sets: equality rows free sign; active upper rows >= 0, active lower rows <= 0
        eq = np.isclose(lbg, ubg)
        scale = np.maximum(1.0, np.abs(g0))
        act_u = ~eq & np.isfinite(ubg) & (ubg - g0 <= act_tol * scale)
        act_l = ~eq & np.isfinite(lbg) & (g0 - lbg <= act_tol * scale)
        actL = np.isfinite(lb) & (z - lb <= act_tol * np.maximum(1.0, np.abs(lb)))
        actU = np.isfinite(ub) & (ub - z <= act_tol * np.maximum(1.0, np.abs(ub)))
        cols = [J[eq].T, J[act_u].T, -J[act_l].T, -np.eye(n)[:, actL], np.eye(n)[:, actU]]
        Am = np.hstack(cols)
        lo = np.concatenate([np.full(eq.sum(), -np.inf), np.zeros(act_u.sum() + act_l.sum() + actL.sum() + actU.sum())])
        res = lsq_linear(Am, -grad, bounds=(lo, np.full(Am.shape[1], np.inf)), method="bvls", tol=1e-14)
        r = grad + Am @ res.x
        return {"stat": float(np.max(np.abs(r))), "stat_rel": float(np.max(np.abs(r)) / max(1.0, np.max(np.abs(grad)))),
                "prim": prim, "bviol": bviol}
