"""GPU suite: batched LQR terminal score (csrc/tt_lqr.hip, doubling algorithm) against the reference's
algorithm (LQR_cost.py: scipy.linalg.solve_discrete_are on the Euler linearisation at the goal).
Tolerance: |P - P_scipy| <= 1e-8 |P_scipy|_max, score relative 1e-8 (FP64; both solvers are backward
stable, the DARE condition at slow goals reaches ~1e7)."""
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
    for b in range(B):
        Pr = to.lqr_riccati(P6, Q, R, xg[b])
        assert np.max(np.abs(P[b] - Pr)) <= 1e-8 * np.max(np.abs(Pr)), b
        sr = float((xc[b] - xg[b]) @ Pr @ (xc[b] - xg[b]))
        assert abs(s[b] - sr) <= 1e-8 * abs(sr), b


def test_lqr_reference_signatures():
    from oracle import ttmpc_oracle as to
    from ttmpc import lqr
    xg = np.array([10.0, 5.0, 0.3, 0.1, 0.05, 1.5])
    xc = xg + 0.1
    d = lqr.lqr_distance(xc, xg, P6, None, np.eye(6), 10 * np.eye(2), np.zeros(2))
    assert d == pytest.approx(to.lqr_distance(xc, xg, P6, np.eye(6), 10 * np.eye(2)), rel=1e-9)
    P = lqr.lqr_riccati(P6, None, np.eye(6), 10 * np.eye(2), xg, np.zeros(2))
    assert np.allclose(P, P.T) and np.all(np.linalg.eigvalsh(P) > 0)
