"""CPU ORACLE (test infrastructure only) -- numpy restatement of the reference NLPs.

THIS IS THE CHECKER, NOT THE PRODUCT.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import it.  The product path
(``car-trailer-mpc_amd/ttmpc`` -> ``libttmpc.so`` -> HIP kernels) never calls into it.

What is restated here (all citations are ``path:line`` under the reference repo
Avan1ko/car-trailer-mpc, ``python-files/``):

* kinematic model ``f`` ............ truck_trailer_model.py:8-24 (numpy twin simulation.py:34-48)
* forward-Euler step ................ truck_trailer_model.py:26-29
* DMS variable layout / bounds ...... trajectory_planning.py:38-60
* dynamics equalities ............... trajectory_planning.py:28-36  (c_0 = x_0 - x_init)
* splitter .......................... trajectory_planning.py:62-84
* tracking cost (no 1/2, Q_f = Q) ... mpc_control.py:17-25
* parameter vector layout ........... mpc_control.py:45-52, 86-88
* reference-copy initial guess ...... mpc_control.py:58-65
* NMPC shift warm start (index bug) . mpc_control_nmpc.py:69-88 / mpc_control_fuzzy.py:69-88 (185-201 in file)
* fuzzy weights (weights act squared) mpc_control_fuzzy.py:23-24, 90-119
* do_interpolation .................. simulation.py:201-218

The reference solves these NLPs with CasADi ``nlpsol('ipopt')`` (mpc_control.py:53).  CasADi /
IPOPT are not installed in this image, so optimality is pinned by solving the SAME restated NLP
with two independent scipy solvers (SLSQP, trust-constr) plus the KKT residual checker below;
the model / data-format pieces are pinned against the reference's own numpy code (imported
behind a never-called ``casadi`` stub by ``tests/golden/make_golden.py``) and committed data.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

NX = 6
NU = 2

# simulation.py:391-395 / trajectory_animation.py:48-52
DEFAULT_PARAMS = {"M": 0.15, "L1": 7.05, "L2": 12.45, "W1": 3.05, "W2": 2.95, "dt": 0.05, "horizon": 20}
# simulation.py:400-409
DEFAULT_Q = np.eye(NX)
DEFAULT_R = 10.0 * np.eye(NU)
# simulation.py:411-414
MPC_XLB = np.array([-np.inf, -np.inf, -np.pi, -np.pi / 3.0, -np.pi / 4.0, -10.0])
MPC_XUB = np.array([np.inf, np.inf, np.pi, np.pi / 3.0, np.pi / 4.0, 10.0])
MPC_ULB = np.array([-5.0, -np.pi / 2])
MPC_UUB = np.array([5.0, np.pi / 2])
# trajectory_animation.py:77-80 (OBCA: theta free, v in [-5, 10])
OBCA_XLB = np.array([-np.inf, -np.inf, -np.inf, -np.pi / 3.0, -np.pi / 4.0, -5.0])
OBCA_XUB = np.array([np.inf, np.inf, np.inf, np.pi / 3.0, np.pi / 4.0, 10.0])


# ----------------------------------------------------------------------------------------------
# model
# ----------------------------------------------------------------------------------------------
def f(q, u, p):
    """Continuous kinematics, truck_trailer_model.py:8-24.  q (...,6), u (...,2)."""
    q = np.asarray(q, dtype=np.float64)
    u = np.asarray(u, dtype=np.float64)
    L1, L2, M = p["L1"], p["L2"], p["M"]
    th, psi, phi, v = q[..., 2], q[..., 3], q[..., 4], q[..., 5]
    out = np.empty(np.broadcast_shapes(q.shape, u.shape[:-1] + (NX,)))
    tphi = np.tan(phi)
    out[..., 0] = v * np.cos(th)
    out[..., 1] = v * np.sin(th)
    out[..., 2] = v * tphi / L1
    out[..., 3] = -v * tphi / L1 * (1 + M / L2 * np.cos(psi)) - v * np.sin(psi) / L2
    out[..., 4] = u[..., 1]
    out[..., 5] = u[..., 0]
    return out


def step(q, u, p):
    """Forward Euler, truck_trailer_model.py:26-29."""
    return np.asarray(q, dtype=np.float64) + f(q, u, p) * p["dt"]


def jac_f(q, p):
    """df/dq (6x6) of truck_trailer_model.py:8-24 (9 non-trivial entries; df/du is constant)."""
    L1, L2, M = p["L1"], p["L2"], p["M"]
    th, psi, phi, v = q[2], q[3], q[4], q[5]
    J = np.zeros((NX, NX))
    c2 = 1.0 / math.cos(phi) ** 2
    t = math.tan(phi)
    J[0, 2] = -v * math.sin(th)
    J[0, 5] = math.cos(th)
    J[1, 2] = v * math.cos(th)
    J[1, 5] = math.sin(th)
    J[2, 4] = v * c2 / L1
    J[2, 5] = t / L1
    J[3, 3] = v * t * M * math.sin(psi) / (L1 * L2) - v * math.cos(psi) / L2
    J[3, 4] = -v * c2 / L1 * (1 + M / L2 * math.cos(psi))
    J[3, 5] = -t / L1 * (1 + M / L2 * math.cos(psi)) - math.sin(psi) / L2
    return J


B_F = np.zeros((NX, NU))
B_F[5, 0] = 1.0  # v_dot = a
B_F[4, 1] = 1.0  # phi_dot = omega


def hess_f_contract(q, w, p):
    """sum_i w_i * d^2 f_i / dq^2 (6x6, symmetric).  f is linear in u, so only the q-block."""
    L1, L2, M = p["L1"], p["L2"], p["M"]
    th, psi, phi, v = q[2], q[3], q[4], q[5]
    H = np.zeros((NX, NX))
    s, c = math.sin(th), math.cos(th)
    t = math.tan(phi)
    c2 = 1.0 / math.cos(phi) ** 2
    sp, cp = math.sin(psi), math.cos(psi)
    # f0 = v cos th, f1 = v sin th
    H[2, 2] += w[0] * (-v * c) + w[1] * (-v * s)
    H[2, 5] += w[0] * (-s) + w[1] * c
    # f2 = v tan(phi)/L1
    H[4, 4] += w[2] * (2 * v * t * c2 / L1)
    H[4, 5] += w[2] * (c2 / L1)
    # f3 = -v t/L1 (1 + M/L2 cos psi) - v sin psi / L2
    k = 1 + M / L2 * cp
    H[3, 3] += w[3] * (v * t * M * cp / (L1 * L2) + v * sp / L2)
    H[3, 4] += w[3] * (v * c2 * M * sp / (L1 * L2))
    H[3, 5] += w[3] * (t * M * sp / (L1 * L2) - cp / L2)
    H[4, 4] += w[3] * (-2 * v * t * c2 * k / L1)
    H[4, 5] += w[3] * (-c2 * k / L1)
    # symmetrise the upper entries
    for (i, j) in ((2, 5), (3, 4), (3, 5), (4, 5)):
        H[j, i] = H[i, j]
    return H


# ----------------------------------------------------------------------------------------------
# tracking NLP (MPCTrackingControl / TruckTrailerNMPC / MPCTrackingControlFuzzy share it)
# ----------------------------------------------------------------------------------------------
@dataclass
class TrackingNLP:
    """The NLP built by mpc_control.py:27-56 on top of trajectory_planning.py:28-60."""

    N: int
    params: dict = field(default_factory=lambda: dict(DEFAULT_PARAMS))
    Q: np.ndarray = field(default_factory=lambda: DEFAULT_Q.copy())
    R: np.ndarray = field(default_factory=lambda: DEFAULT_R.copy())
    xlb: np.ndarray = field(default_factory=lambda: MPC_XLB.copy())
    xub: np.ndarray = field(default_factory=lambda: MPC_XUB.copy())
    ulb: np.ndarray = field(default_factory=lambda: MPC_ULB.copy())
    uub: np.ndarray = field(default_factory=lambda: MPC_UUB.copy())

    @property
    def n(self):  # decision variables, trajectory_planning.py:38-58
        return (NX + NU) * self.N + NX

    @property
    def m(self):  # equality rows, trajectory_planning.py:28-36
        return NX * (self.N + 1)

    # --- layout ------------------------------------------------------------------------------
    def unpack(self, z):
        """z = [x0,u0,...,x_{N-1},u_{N-1},x_N] -> X (N+1,6), U (N,2)  (trajectory_planning.py:38-58)."""
        z = np.asarray(z, dtype=np.float64).reshape(-1)
        N = self.N
        body = z[: (NX + NU) * N].reshape(N, NX + NU)
        X = np.vstack([body[:, :NX], z[(NX + NU) * N:][None, :]])
        U = body[:, NX:].copy()
        return X, U

    def pack(self, X, U):
        X = np.asarray(X, dtype=np.float64).reshape(self.N + 1, NX)
        U = np.asarray(U, dtype=np.float64).reshape(self.N, NU)
        return np.concatenate([np.hstack([X[:-1], U]).reshape(-1), X[-1]])

    def bounds(self):
        """lbx/ubx as built by trajectory_planning.py:46-58 (x_0 is bounded too)."""
        lb = np.concatenate([np.tile(np.concatenate([self.xlb, self.ulb]), self.N), self.xlb])
        ub = np.concatenate([np.tile(np.concatenate([self.xub, self.uub]), self.N), self.xub])
        return lb, ub

    def split(self, z):
        """_split_decision_variables, trajectory_planning.py:62-84 -> (states (6,N+1), inputs (2,N))."""
        X, U = self.unpack(z)
        return X.T.copy(), U.T.copy()

    # --- pieces of mpc_control.py ------------------------------------------------------------
    def initial_guess(self, Xref, Uref):
        """mpc_control.py:58-65: x_k <- Xref[:,k] (incl. k=0!), u_k <- Uref[:,k]. Xref (6,N+1)."""
        return self.pack(np.asarray(Xref).T, np.asarray(Uref).T)

    def shift_solution(self, z, bug_compatible=True):
        """mpc_control_nmpc.py:69-88.  With bug_compatible the reference's slice
        ``z[-step:-nu]`` (= [u_{N-1}, x_N[0:4]]) / ``z[-nu:]`` (= x_N[4:6]) is reproduced."""
        z = np.asarray(z, dtype=np.float64).reshape(-1)
        step_ = NX + NU
        N = self.N
        parts = [z[(k + 1) * step_:(k + 2) * step_] for k in range(N - 1)]
        if bug_compatible:
            last_state = z[-step_:-NU]
            last_input = z[-NU:]
        else:
            X, U = self.unpack(z)
            last_state, last_input = X[-1], U[-1]
        return np.concatenate(parts + [last_state, last_input, last_state])

    def weights(self, wq=None, wr=None):
        """Q_w = diag(w)Q diag(w), R_w likewise (mpc_control_fuzzy.py:23-24)."""
        Qs = 0.5 * (self.Q + self.Q.T)
        Rs = 0.5 * (self.R + self.R.T)
        if wq is not None:
            Qs = np.diag(wq) @ Qs @ np.diag(wq)
        if wr is not None:
            Rs = np.diag(wr) @ Rs @ np.diag(wr)
        return Qs, Rs

    def cost(self, z, Xref, Uref, wq=None, wr=None):
        """mpc_control.py:17-25 (no 1/2 factor, Q_f = Q)."""
        X, U = self.unpack(z)
        Qw, Rw = self.weights(wq, wr)
        dX = X - np.asarray(Xref).T
        dU = U - np.asarray(Uref).T
        return float(np.einsum("ki,ij,kj->", dX, Qw, dX) + np.einsum("ki,ij,kj->", dU, Rw, dU))

    def grad(self, z, Xref, Uref, wq=None, wr=None):
        X, U = self.unpack(z)
        Qw, Rw = self.weights(wq, wr)
        gX = 2.0 * (X - np.asarray(Xref).T) @ Qw
        gU = 2.0 * (U - np.asarray(Uref).T) @ Rw
        return self.pack(gX, gU)

    def constraints(self, z, x_init):
        """g = [x_0 - x_init; x_{k+1} - (x_k + dt f(x_k,u_k))], trajectory_planning.py:28-36."""
        X, U = self.unpack(z)
        c = np.empty((self.N + 1, NX))
        c[0] = X[0] - np.asarray(x_init, dtype=np.float64)
        c[1:] = X[1:] - step(X[:-1], U, self.params)
        return c.reshape(-1)

    def jacobian(self, z):
        """dense d g / d z (m x n)."""
        X, U = self.unpack(z)
        N, dt = self.N, self.params["dt"]
        Jc = np.zeros((self.m, self.n))
        off = lambda k: (NX + NU) * k  # noqa: E731
        Jc[0:NX, 0:NX] = np.eye(NX)
        for k in range(N):
            r = NX * (k + 1)
            A = np.eye(NX) + dt * jac_f(X[k], self.params)
            Jc[r:r + NX, off(k):off(k) + NX] = -A
            Jc[r:r + NX, off(k) + NX:off(k) + NX + NU] = -dt * B_F
            Jc[r:r + NX, off(k + 1):off(k + 1) + NX] = np.eye(NX)
        return Jc

    def param_vector(self, Xref, Uref, x_init, wq=None, wr=None):
        """p = [vec(Xref) stage-major; vec(Uref) stage-major; (w_q; w_r;) x_init] (mpc_control.py:45-52,
        86-88; fuzzy mpc_control_fuzzy.py:54-58)."""
        parts = [np.asarray(Xref).T.reshape(-1), np.asarray(Uref).T.reshape(-1)]
        if wq is not None:
            parts += [np.asarray(wq, float), np.asarray(wr, float)]
        parts.append(np.asarray(x_init, float))
        return np.concatenate(parts)

    # --- optimality checker -----------------------------------------------------------------
    def kkt_residual(self, z, x_init, Xref, Uref, wq=None, wr=None, act_tol=1e-6, relax=1e-8):
        """Primal-only KKT check: estimate (y, zL, zU >= 0) by bounded least squares on
        grad F + J^T y - zL + zU = 0 with bound duals allowed only on (near-)active bounds.
        Returns dict(stat=||grad L||_inf, prim=||g||_inf, bviol=max bound violation)."""
        from scipy.optimize import lsq_linear

        z = np.asarray(z, dtype=np.float64)
        g = self.grad(z, Xref, Uref, wq, wr)
        Jc = self.jacobian(z)
        c = self.constraints(z, x_init)
        lb, ub = self.bounds()
        lbr = lb - relax * np.maximum(1.0, np.abs(lb))
        ubr = ub + relax * np.maximum(1.0, np.abs(ub))
        actL = np.where(np.isfinite(lb) & (z - lb <= act_tol * np.maximum(1.0, np.abs(lb))))[0]
        actU = np.where(np.isfinite(ub) & (ub - z <= act_tol * np.maximum(1.0, np.abs(ub))))[0]
        cols = [Jc.T]
        if len(actL):
            EL = np.zeros((self.n, len(actL)))
            EL[actL, np.arange(len(actL))] = -1.0
            cols.append(EL)
        if len(actU):
            EU = np.zeros((self.n, len(actU)))
            EU[actU, np.arange(len(actU))] = 1.0
            cols.append(EU)
        Amat = np.hstack(cols)
        lo = np.concatenate([np.full(self.m, -np.inf), np.zeros(len(actL) + len(actU))])
        hi = np.full(Amat.shape[1], np.inf)
        res = lsq_linear(Amat, -g, bounds=(lo, hi), method="bvls", tol=1e-14, lsmr_tol="auto")
        r = g + Amat @ res.x
        bviol = float(max(0.0, np.max(np.nan_to_num(lbr - z, neginf=-1.0)),
                          np.max(np.nan_to_num(z - ubr, neginf=-1.0))))
        return {"stat": float(np.max(np.abs(r))), "prim": float(np.max(np.abs(c))), "bviol": bviol,
                "y": res.x[: self.m]}

    # --- independent solvers (fixture generation) -------------------------------------------
    def solve_scipy(self, x_init, Xref, Uref, z0=None, method="SLSQP", wq=None, wr=None,
                    maxiter=2000, tol=1e-12):
        from scipy.optimize import Bounds, NonlinearConstraint, minimize

        if z0 is None:
            z0 = self.initial_guess(Xref, Uref)
        lb, ub = self.bounds()
        z0 = np.clip(z0, np.where(np.isfinite(lb), lb, -1e20), np.where(np.isfinite(ub), ub, 1e20))
        fun = lambda z: self.cost(z, Xref, Uref, wq, wr)  # noqa: E731
        jac = lambda z: self.grad(z, Xref, Uref, wq, wr)  # noqa: E731
        Qw, Rw = self.weights(wq, wr)
        H = np.zeros((self.n, self.n))
        for k in range(self.N + 1):
            o = (NX + NU) * k
            H[o:o + NX, o:o + NX] = 2 * Qw
            if k < self.N:
                H[o + NX:o + NX + NU, o + NX:o + NX + NU] = 2 * Rw
        if method == "SLSQP":
            cons = {"type": "eq", "fun": lambda z: self.constraints(z, x_init), "jac": self.jacobian}
            res = minimize(fun, z0, jac=jac, bounds=Bounds(lb, ub), constraints=[cons], method="SLSQP",
                           options={"maxiter": maxiter, "ftol": tol})
        else:
            def chess(z, v):
                X, _ = self.unpack(z)
                Hc = np.zeros((self.n, self.n))
                dt = self.params["dt"]
                for k in range(self.N):
                    o = (NX + NU) * k
                    w = v[NX * (k + 1):NX * (k + 2)]
                    Hc[o:o + NX, o:o + NX] -= dt * hess_f_contract(X[k], w, self.params)
                return Hc
            nlc = NonlinearConstraint(lambda z: self.constraints(z, x_init), 0.0, 0.0, jac=self.jacobian,
                                      hess=chess)
            res = minimize(fun, z0, jac=jac, hess=lambda z: H, bounds=Bounds(lb, ub), constraints=[nlc],
                           method="trust-constr",
                           options={"maxiter": maxiter, "gtol": 1e-12, "xtol": 1e-14, "barrier_tol": 1e-12})
        return res


# ----------------------------------------------------------------------------------------------
# host-side helpers of the reference classes / harness
# ----------------------------------------------------------------------------------------------
def fuzzy_weights(current_state, reference_states):
    """mpc_control_fuzzy.py:90-119 (rule-based q/r weights, clipped to [1, 3.5])."""
    psi = float(current_state[3])
    v = float(current_state[5])
    reference_states = np.asarray(reference_states)
    ref_v = float(reference_states[5, 0]) if reference_states.size > 0 else 0.0
    hitch_norm = min(abs(psi) / 0.35, 1.0)
    reversing = (ref_v < -0.1) or (v < -0.1)
    q = np.ones(NX)
    r = np.ones(NU)
    hitch_gain = 1.0 + 2.0 * hitch_norm
    steer_gain = 1.0 + 1.2 * hitch_norm
    steer_rate_gain = 1.0 + 1.5 * hitch_norm
    if reversing:
        hitch_gain *= 1.1
        steer_gain *= 1.1
        steer_rate_gain *= 1.2
    q[2] = max(1.0, steer_gain)
    q[3] = max(1.0, hitch_gain)
    q[4] = max(1.0, steer_gain)
    r[1] = max(1.0, steer_rate_gain)
    return np.clip(q, 1.0, 3.5), np.clip(r, 1.0, 3.5)


def do_interpolation(state_traj, input_traj, dt_1, dt_2):
    """simulation.py:201-218 (linear states, zero-order-hold inputs)."""
    N = input_traj.shape[1]
    n = math.floor(dt_1 / dt_2)
    S = np.zeros((state_traj.shape[0], n * N + 1))
    U = np.zeros((input_traj.shape[0], n * N))
    for k in range(N):
        for mm in range(n):
            t = mm / n
            S[:, k * n + mm] = (1 - t) * state_traj[:, k] + t * state_traj[:, k + 1]
            U[:, k * n + mm] = input_traj[:, k]
    S[:, -1] = state_traj[:, -1]
    return S, U


def reference_window(ref_states, ref_inputs, k, horizon):
    """Reference windowing with end padding, simulation.py:485-499."""
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


# ----------------------------------------------------------------------------------------------
# closed-loop simulation pieces
# ----------------------------------------------------------------------------------------------
# simulation.py:26-32
DISTURBANCE_PARAMS = {"friction_coeff": 0.9, "slippage_coeff": 0.9, "process_noise_std": 0.02,
                      "lateral_slip_gain": 0.01, "slip_angle_max": 0.0}


def plant_update(q, u, p, dist=None, state_noise=None):
    """update(q, u, params, disturbance_params) of simulation.py:167-199, vectorised over leading axes:
    apply_disturbances (50-87: u scaled by friction / slippage; its noise draw is discarded),
    f_dyn (34-48), apply_slippage_to_dynamics (89-115), Euler step, apply_lateral_slip (117-149).
    state_noise: the NMPC / fuzzy drivers' update (simulation_nmpc.py:94-105, simulation_fuzzy.py:94-105), which
    keeps apply_disturbances' draw and adds state_noise * dt right after the Euler step."""
    q = np.asarray(q, dtype=np.float64)
    u = np.array(u, dtype=np.float64)
    if dist is not None:
        u[..., 0] = u[..., 0] * dist.get("friction_coeff", 1.0)
        u[..., 1] = u[..., 1] * dist.get("slippage_coeff", 1.0)
    qd = f(q, u, p)
    if dist is not None and "slip_angle_max" in dist:
        slip = 1.0 - np.minimum(np.abs(q[..., 4]) * np.abs(q[..., 5]) * dist["slip_angle_max"], 0.3)
        qd[..., 2] = qd[..., 2] * slip
        qd[..., 3] = qd[..., 3] * slip
    nq = q + qd * p["dt"]
    if state_noise is not None:
        nq = nq + np.asarray(state_noise, dtype=np.float64) * p["dt"]
    if dist is not None and "lateral_slip_gain" in dist:
        mag = dist["lateral_slip_gain"] * np.abs(q[..., 5]) * np.abs(q[..., 4])
        nq[..., 0] = nq[..., 0] + mag * np.cos(q[..., 2] + np.pi / 2) * p["dt"]
        nq[..., 1] = nq[..., 1] + mag * np.sin(q[..., 2] + np.pi / 2) * p["dt"]
    return nq


def step_indices(T_sim, dt):
    """simulation.py:484-531 loop counter: t = 0; while t <= T_sim: k = floor(t/dt); ...; t += dt."""
    ks, t = [], 0.0
    while t <= T_sim:
        ks.append(math.floor(t / dt))
        t += dt
    return ks


def closed_loop(solve, x_init, plan_x, plan_u, horizon, T_sim, p, dist=None, noise=None, zero_on_fail=False,
                policy=None, fuzzy=False, plant_noise=None):
    """The reference loop for B instances sharing one plan (plan_x (6,Np+1), plan_u (2,Np)).
    solve(x_meas (B,6), Xr (B,N+1,6), Ur (B,N,2)[, w (B,8)]) -> (X (B,N+1,6), U (B,N,2), status (B,)).
    noise: (steps, B, 6) measurement noise (simulation.py:509-513) or None.
    plant_noise: (steps, B, 6) process noise inside the plant (simulation_nmpc.py:94-105) or None.
    policy: what follows a failed solve (status > 1) -- "track" (simulation.py:519-527: the returned
    inputs), "nmpc" (simulation_nmpc.py:206-216: zero control, stop after 20 consecutive failures),
    "fuzzy" (simulation_fuzzy.py:207-221: last successful control, zero after 15, stop after 30).  A
    stopped instance (the reference's `break`) keeps its state and applies nothing.  fuzzy=True: the solve
    gets the per-instance fuzzy weights and failed instances are re-solved once with unit weights
    (mpc_control_fuzzy.py:132-161).
    Returns states (steps+1,B,6), applied controls (steps,B,2), status (steps,B), and when policy or fuzzy is
    given also dict(failures, consecutive_failures, running)."""
    legacy = policy is None and not fuzzy
    if policy is None:
        policy = "nmpc" if zero_on_fail else "track"
    x = np.array(x_init, dtype=np.float64).reshape(-1, 6)
    B = x.shape[0]
    ks = step_indices(T_sim, p["dt"])
    S, Ua, St = [x.copy()], [], []
    u_last = np.zeros((B, 2))
    consec = np.zeros(B, dtype=np.int64)
    fails = np.zeros(B, dtype=np.int64)
    active = np.ones(B, dtype=bool)
    for j, k in enumerate(ks):
        Xr, Ur = reference_window(plan_x, plan_u, k, horizon)
        Xr = np.broadcast_to(Xr.T, (B, horizon + 1, NX)).copy()
        Ur = np.broadcast_to(Ur.T, (B, horizon, NU)).copy()
        xm = x + noise[j] if noise is not None else x
        if fuzzy:
            w = np.stack([np.concatenate(fuzzy_weights(xm[b], Xr[b].T)) for b in range(B)])
            X, U, st = solve(xm, Xr, Ur, w)
            st = np.asarray(st).copy()
            bad = np.where((st > 1) & active)[0]
            if bad.size:
                _, U2, st2 = solve(xm[bad], Xr[bad], Ur[bad], np.ones((bad.size, 8)))
                U = U.copy()
                U[bad], st[bad] = U2, st2
        else:
            _, U, st = solve(xm, Xr, Ur)
            st = np.asarray(st)
        u0 = np.zeros((B, 2))
        for b in range(B):
            if not active[b]:
                continue
            if st[b] <= 1:
                u0[b] = U[b, 0]
                u_last[b] = u0[b]
                consec[b] = 0
                continue
            fails[b] += 1
            consec[b] += 1
            if policy == "nmpc":
                u_last[b] = 0.0
                if consec[b] > 20:
                    active[b] = False
            elif policy == "fuzzy":
                u0[b] = u_last[b]
                if consec[b] > 15:
                    u0[b] = 0.0
                if consec[b] > 30:
                    active[b] = False
                    u0[b] = 0.0
            else:
                u0[b] = U[b, 0]
        xn = plant_update(x, u0, p, dist, None if plant_noise is None else plant_noise[j])
        x = np.where(active[:, None], xn, x)
        S.append(x.copy())
        Ua.append(u0)
        St.append(st.copy())
    out = np.array(S), np.array(Ua), np.array(St)
    if legacy:
        return out
    return out + ({"failures": fails, "consecutive_failures": consec, "running": active},)


def lqr_riccati(p, Q, R, x_goal):
    """LQR_cost.py:7-34 with the reference's own DARE solver (scipy.linalg.solve_discrete_are); the
    CasADi Jacobian of the Euler map is the analytic jac_f (sympy-verified)."""
    from scipy.linalg import solve_discrete_are
    A = np.eye(NX) + p["dt"] * jac_f(np.asarray(x_goal, dtype=np.float64), p)
    B = p["dt"] * B_F
    P = solve_discrete_are(A, B, np.asarray(Q, dtype=np.float64), np.asarray(R, dtype=np.float64))
    return 0.5 * (P + P.T)


def lqr_distance(x_current, x_goal, p, Q, R):
    """LQR_cost.py:37-41."""
    P = lqr_riccati(p, Q, R, x_goal)
    dx = np.asarray(x_current, dtype=np.float64) - np.asarray(x_goal, dtype=np.float64)
    return float(dx @ P @ dx)
