"""GPU suite: batched LQR terminal score (csrc/tt_lqr.hip, doubling algorithm) against the reference's
algorithm (LQR_cost.py: scipy.linalg.solve_discrete_are on the Euler linearisation at the goal).
Tolerance: the GPU P satisfies the DARE to a relative residual <= 1e-12, and agrees with scipy's P (and
score) to max(1e-9, 1e6 x scipy's own relative residual): at near-stationary goals (|v| ~ 0.01, P ~ 1e7)
the DARE is ill-conditioned and scipy's Schur solution carries residuals ~1e-11 while the doubling
iteration reaches ~1e-14, so the two differ at the 1e-7 level there."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

P6 = {"M": 0.15, "L1": 7.05, "L2": 12.45, "W1": 3.05, "W2": 2.95, "dt": 0.05}


def test_lqr_scores_match_scipy_dare(golden_ref):
    from oracle import ttmpc_oracle as to
    from ttmpc import lqr
    rng = np.random.default_rng(9)
    B = 96
    xg = golden_ref["interp_states"].T[rng.integers(0, 400, B)].copy()
    xg[:, 5] = rng.uniform(-3, 3, B)          # goals with motion (well conditioned) ...
    xg[:8, 5] = rng.uniform(-0.05, 0.05, 8)   # ... and near-stationary ones (P up to ~1e7)
    xg[-1] = golden_ref["interp_states"][:, -1]   # the plan's own final state, as simulation.py:563 scores it
    xc = xg + rng.normal(scale=0.2, size=(B, 6))
    Q, R = np.eye(6), 10 * np.eye(2)
    s, P, it = lqr.lqr_scores(xc, xg, P6, Q, R)
    s, P, it = s.cpu().numpy(), P.cpu().numpy(), it.cpu().numpy()
    assert np.all(it > 0)
    def resid(Pm, x):
        A = np.eye(6) + P6["dt"] * to.jac_f(x, P6)
        Bm = P6["dt"] * to.B_F
        K = np.linalg.solve(R + Bm.T @ Pm @ Bm, Bm.T @ Pm @ A)
        return np.abs(A.T @ Pm @ A - Pm - A.T @ Pm @ Bm @ K + Q).max() / np.abs(Pm).max()
    for b in range(B):
        Pr = to.lqr_riccati(P6, Q, R, xg[b])
        assert resid(P[b], xg[b]) <= 1e-12, b
        rs = resid(Pr, xg[b])
        assert resid(P[b], xg[b]) <= max(1e-13, rs), b          # at least as accurate as scipy
        tol = max(1e-9, 1e6 * rs)                                 # forward error <= cond x residual
        assert np.max(np.abs(P[b] - Pr)) <= tol * np.max(np.abs(Pr)), b
        sr = float((xc[b] - xg[b]) @ Pr @ (xc[b] - xg[b]))
        assert abs(s[b] - sr) <= tol * abs(sr), b


def test_lqr_reference_signatures():
    from oracle import ttmpc_oracle as to
    from ttmpc import lqr
    xg = np.array([10.0, 5.0, 0.3, 0.1, 0.05, 1.5])
    xc = xg + 0.1
    d = lqr.lqr_distance(xc, xg, P6, None, np.eye(6), 10 * np.eye(2), np.zeros(2))
    assert d == pytest.approx(to.lqr_distance(xc, xg, P6, np.eye(6), 10 * np.eye(2)), rel=1e-9)
    P = lqr.lqr_riccati(P6, None, np.eye(6), 10 * np.eye(2), xg, np.zeros(2))
    assert np.allclose(P, P.T) and np.all(np.linalg.eigvalsh(P) > 0)
