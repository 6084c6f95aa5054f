"""CPU suite: the oracle against the reference's own outputs and the committed golden optima."""
import math

import numpy as np
import pytest

from conftest import fixture_instance
from oracle import c_oracle as co
from oracle import ttmpc_oracle as to

P = dict(to.DEFAULT_PARAMS)


def test_model_matches_reference_f_dyn(golden_ref):
    # simulation.py:34-48 executed by the reference itself (tests/golden/make_golden.py)
    f = to.f(golden_ref["q"], golden_ref["u"], P)
    assert np.max(np.abs(f - golden_ref["fdyn"])) <= 1e-13


def test_euler_matches_reference_update(golden_ref):
    # simulation.py:167-199 with disturbance_params=None is exactly x + dt f (truck_trailer_model.py:26-29)
    nxt = to.step(golden_ref["q"], golden_ref["u"], P)
    assert np.max(np.abs(nxt - golden_ref["upd_nom"])) <= 1e-13


def test_committed_obca_solution_satisfies_restated_dynamics(golden_ref):
    # data/state_traj.txt + input_traj.txt: an IPOPT OBCA solution, N=200, dt=0.1
    S, U = golden_ref["state_traj"], golden_ref["input_traj"]
    p = dict(P, dt=0.1)
    res = S[:, 1:].T - to.step(S[:, :-1].T, U.T, p)
    assert np.max(np.abs(res)) < 1e-11
    # OBCA bounds (trajectory_animation.py:77-80) hold up to IPOPT's bound relaxation
    assert np.all(np.abs(S[3]) <= np.pi / 3 + 1e-7) and np.all(np.abs(S[4]) <= np.pi / 4 + 1e-7)
    assert np.all(np.abs(U[0]) <= 5 + 1e-7) and np.all(np.abs(U[1]) <= np.pi / 2 + 1e-7)


def test_do_interpolation_matches_reference(golden_ref):
    S2, U2 = to.do_interpolation(golden_ref["state_traj"], golden_ref["input_traj"], 0.1, 0.05)
    assert np.array_equal(S2, golden_ref["interp_states"])
    assert np.array_equal(U2, golden_ref["interp_inputs"])


def test_jacobian_matches_finite_differences():
    rng = np.random.default_rng(0)
    for _ in range(20):
        q = rng.uniform([-5, -5, -3, -1, -0.7, -5], [5, 5, 3, 1, 0.7, 5])
        J = to.jac_f(q, P)
        for j in range(6):
            e = np.zeros(6)
            e[j] = 1e-6
            fd = (to.f(q + e, np.zeros(2), P) - to.f(q - e, np.zeros(2), P)) / 2e-6
            assert np.allclose(J[:, j], fd, atol=1e-7)
        w = rng.normal(size=6)
        H = to.hess_f_contract(q, w, P)
        for j in range(6):
            e = np.zeros(6)
            e[j] = 1e-5
            fd = (w @ to.jac_f(q + e, P) - w @ to.jac_f(q - e, P)) / 2e-5
            assert np.allclose(H[j], fd, atol=1e-6)


def test_golden_optima_are_kkt_points(golden_opt):
    for i in range(len(golden_opt["tag"])):
        tag, N, x0, xr, ur, wq, wr, z = fixture_instance(golden_opt, i)
        nlp = to.TrackingNLP(N)
        k = nlp.kkt_residual(z, x0, xr.T, ur.T, wq, wr)
        assert k["prim"] <= 1e-10 and k["stat"] <= 1e-6 and k["bviol"] <= 1e-7, (tag, k)


def _oracle_problem(N):
    nlp = to.TrackingNLP(N)
    return nlp, co.make_problem(N, P, nlp.Q, nlp.R, nlp.xlb, nlp.xub, nlp.ulb, nlp.uub)


def test_c_oracle_reproduces_golden_optima(golden_opt):
    """The C interior-point oracle against the scipy (trust-constr + SLSQP) optima: 1e-6 abs."""
    for i in range(len(golden_opt["tag"])):
        tag, N, x0, xr, ur, wq, wr, z = fixture_instance(golden_opt, i)
        _, Pp = _oracle_problem(N)
        zc, st, it, kk = co.solve_batch(Pp, x0[None], xr[None], ur[None], wq=wq[None], wr=wr[None])
        assert st[0] == 0, (tag, st, kk)
        scale = np.maximum(1.0, np.abs(z))
        assert np.max(np.abs(zc[0] - z) / scale) <= 1e-6, tag


def test_c_oracle_infeasible_initial_state():
    nlp, Pp = _oracle_problem(10)
    from ttmpc.scenarios import synthetic_batch
    x0, xr, ur = synthetic_batch(2, 10, seed=3)
    x0[0, 3] = 1.2  # hitch angle beyond pi/3: x_0 = x_init violates the box
    z, st, _, _ = co.solve_batch(Pp, x0, xr, ur)
    assert st[0] == 3 and st[1] == 0


def test_fuzzy_weights_rules():
    # mpc_control_fuzzy.py:90-119 evaluated by hand
    Xr = np.zeros((6, 5))
    q, r = to.fuzzy_weights(np.zeros(6), Xr)
    assert np.all(q == 1) and np.all(r == 1)
    q, r = to.fuzzy_weights(np.array([0, 0, 0, 0.175, 0, 1.0]), Xr)  # h = 0.5, forward
    assert np.allclose(q, [1, 1, 1.6, 2.0, 1.6, 1]) and np.allclose(r, [1, 1.75])
    Xr[5, 0] = -1.0  # reversing, h = 1
    q, r = to.fuzzy_weights(np.array([0, 0, 0, -0.5, 0, 0]), Xr)
    assert np.allclose(q, [1, 1, 2.2 * 1.1, 3.3, 2.2 * 1.1, 1]) and np.allclose(r, [1, 2.5 * 1.2])


def test_shift_solution_reproduces_reference_slicing():
    N = 4
    nlp = to.TrackingNLP(N)
    z = np.arange(8 * N + 6, dtype=float)
    s = nlp.shift_solution(z)
    assert s.size == z.size
    assert np.array_equal(s[: 8 * (N - 1)], z[8: 8 * N])
    # last_state = z[-8:-2] = [u_{N-1}, x_N[0:4]], last_input = z[-2:] = x_N[4:6]
    assert np.array_equal(s[8 * (N - 1): 8 * (N - 1) + 6], z[-8:-2])
    assert np.array_equal(s[8 * (N - 1) + 6: 8 * N], z[-2:])
    assert np.array_equal(s[8 * N:], z[-8:-2])


def test_product_layout_helpers_match_oracle():
    from ttmpc import layout
    N = 5
    nlp = to.TrackingNLP(N)
    z = np.random.default_rng(1).normal(size=(3, 8 * N + 6))
    X, U = layout.unpack(z, N)
    for b in range(3):
        Xo, Uo = nlp.unpack(z[b])
        assert np.array_equal(X[b], Xo) and np.array_equal(U[b], Uo)
        assert np.array_equal(layout.shift(z[b:b + 1], N)[0], nlp.shift_solution(z[b]))
    assert np.array_equal(layout.pack(X, U), z)


def test_product_fuzzy_weights_match_oracle():
    from ttmpc.mpc_control_fuzzy import fuzzy_weights
    rng = np.random.default_rng(5)
    for _ in range(50):
        x = rng.normal(size=6) * [1, 1, 1, 0.4, 0.3, 2]
        Xr = rng.normal(size=(6, 4))
        a, b = fuzzy_weights(x, Xr), to.fuzzy_weights(x, Xr)
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_synthetic_generator_is_feasible_and_deterministic():
    from ttmpc.scenarios import synthetic_batch
    a = synthetic_batch(64, 20, seed=9)
    b = synthetic_batch(64, 20, seed=9)
    for u, v in zip(a, b):
        assert np.array_equal(u, v)
    x0, xr, ur = a
    res = xr[:, 1:] - to.step(xr[:, :-1], ur, P)
    assert np.max(np.abs(res)) < 1e-12
    assert np.all(np.abs(xr[..., 3]) <= math.pi / 3) and np.all(np.abs(x0[:, 3]) <= math.pi / 3)


@pytest.mark.parametrize("N", [1, 3, 40])
def test_c_oracle_batch_converges(N):
    from ttmpc.scenarios import synthetic_batch
    nlp, Pp = _oracle_problem(N)
    x0, xr, ur = synthetic_batch(16, N, seed=N)
    z, st, it, kk = co.solve_batch(Pp, x0, xr, ur)
    assert np.all(st == 0) and np.all(kk <= 1e-8)
    for b in range(0, 16, 5):
        k = nlp.kkt_residual(z[b], x0[b], xr[b].T, ur[b].T)
        assert k["prim"] <= 1e-9 and k["stat"] <= 1e-6
