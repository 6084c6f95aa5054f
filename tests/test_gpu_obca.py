"""GPU parity for the OBCA path (TrajectoryOptimization / MPCTrackingControlObs) through the C ABI.

The GPU (car-trailer-mpc_amd/csrc/tt_obca.hip) and the CPU oracle (oracle/c/tt_obca.c) run the same
restated IPOPT (reference duals, least-squares multipliers, soft restoration, restoration phase), but not
bit-identical arithmetic (device sin/cos/tan/log, reciprocal refinement, FMA contraction, structured vs
dense block algebra).  On easy instances the iterates coincide (the MPC+OBCA windows agree to 1e-14); on
harder ones -- hundreds to thousands of iterations through several restoration phases -- the filter line
search can branch differently on rounding-level differences, so those tests compare statuses on most
instances, the primal solution where both converge (same local optimum to <= 1e-6 on most; the OBCA
duals mu/lam are not unique) and check properties:
feasibility, collision-free plans, bitwise-deterministic reruns.  Independent optimality: the finite-difference KKT certificate of
oracle/obca_nlp.py (numpy restatement of the reference NLP) on the GPU's output.
"""
import numpy as np
import pytest

from conftest import GOLDEN

from test_obca_oracle import P6, toy_plan

pytestmark = pytest.mark.gpu


def _solver(N, obs, variant=None, params=P6, bounds=None, **kw):
    import ttmpc
    from ttmpc import scenarios as sc
    b = bounds or (sc.OBCA_XLB, sc.OBCA_XUB, sc.OBCA_ULB, sc.OBCA_UUB)
    v = ttmpc.TT_VARIANT_OBCA_PLAN if variant is None else variant
    return ttmpc.ObcaSolver(N, params, sc.OBCA_Q, sc.OBCA_R, *b, obs, variant=v, **kw)


def _oracle(N, obs, mode=0, params=P6, bounds=None, **kw):
    from oracle import c_oracle as co
    from ttmpc import scenarios as sc
    b = bounds or (sc.OBCA_XLB, sc.OBCA_XUB, sc.OBCA_ULB, sc.OBCA_UUB)
    return co.make_obca_problem(N, params, sc.OBCA_Q, sc.OBCA_R, *b, obs, mode=mode, **kw)


def _ipopt_check_at_gpu_points(P, x0, I, st, kk, **inputs):
    """Independent check of the GPU's own end points: for every instance the kernel reports optimal
    (status 0), the ORACLE evaluates IPOPT's optimality error at the GPU's returned primal-dual iterate (the diagnostic
    export tt_obca_solve_batch_iterate; oracle/c/tt_obca.c tto_obca_eval_iterate): the point must be interior and pass
    IPOPT's full convergence test there -- scaled E_0 <= tol AND the unscaled dual infeasibility <= dual_inf_tol (1),
    complementarity <= compl_inf_tol (1e-4) -- and the oracle's E_0 must agree with the one the kernel reported."""
    from oracle import c_oracle as co
    opt = np.flatnonzero(st == 0)
    if opt.size == 0:
        return None
    r = co.obca_eval_iterate(P, x0[opt], I[opt], **{k: None if v is None else v[opt] for k, v in inputs.items()})
    assert r["interior"].all(), opt[~r["interior"]]
    assert r["converged"].all(), [(int(b), float(e), float(d), float(c), float(sd)) for b, e, d, c, sd, ok in
                                  zip(opt, r["E0"], r["dinf"], r["compl"], r["sd"], r["converged"]) if not ok]
    assert np.all(np.abs(r["E0"] - kk[opt]) <= 1e-9), np.abs(r["E0"] - kk[opt]).max()
    return r


def test_toy_plan_matches_oracle_and_is_kkt():
    from oracle import c_oracle as co
    from oracle.obca_nlp import ObcaNLP
    from ttmpc import collision
    from ttmpc import scenarios as sc
    N, M, obs, x0, xg, zg = toy_plan()
    X, U, Z, st, it, kk, I = _solver(N, obs).solve(x0, xg, z_guess=zg, iterate=True)
    zc, stc, itc, kkc = co.obca_solve_batch(_oracle(N, obs), x0, xg, z_guess=zg)
    assert np.array_equal(st, stc) and np.all(st == 0)
    _ipopt_check_at_gpu_points(_oracle(N, obs), x0, I, st, kk, x_goal=xg)
    nlp = ObcaNLP(N, M, P6, sc.OBCA_Q, sc.OBCA_R, sc.OBCA_XLB, sc.OBCA_XUB, sc.OBCA_ULB, sc.OBCA_UUB, obs)
    for b in range(len(x0)):  # same local optimum (primal; the OBCA duals are not unique)
        (Xg, Ug, _, _), (Xo, Uo, _, _) = nlp.split(Z[b]), nlp.split(zc[b])
        assert np.max(np.abs(Xg - Xo)) <= 1e-6 and np.max(np.abs(Ug - Uo)) <= 1e-6
    r = nlp.kkt_check(Z[1], x0[1], xg[1])
    assert r["stat_rel"] < 1e-6 and r["prim"] < 1e-7 and r["bviol"] < 1e-7, r
    assert collision.sat_gap(X[1], P6, obs).min() > 0.0
    # outputs are the split of z (trajectory_optimization.py:277-309)
    Xs, Us, _, _ = nlp.split(Z[0])
    assert np.array_equal(X[0], Xs) and np.array_equal(U[0], Us)


def test_mpc_obca_windows_match_oracle():
    """MPC+OBCA (mpc_control_obs.py, simulation.py:417-424 setup: N=50, dt=0.05, all 11 obstacles) on all 16
    windows of the reference's interpolated plan, from the reference's own start (x = Xref, u = Uref,
    mu = 100, lam pattern; mpc_control_obs.py:216-239) with max_iter 5000 and IPOPT's restoration phase.
    Windows whose perturbed start overlaps an obstacle (SAT gap < 0) are infeasible NLPs (x_0 = x_init is a
    constraint) and cannot converge on either side."""
    from oracle import c_oracle as co
    from ttmpc import collision
    from ttmpc import scenarios as sc
    import ttmpc
    g = np.load(GOLDEN / "reference_numpy.npz")
    obs = g["obstacles"]
    x0, xr, ur = sc.mpc_obs_batch(g["state_traj"], g["input_traj"], 16, 50, seed=0)
    p = dict(P6, dt=0.05)
    bnd = (sc.XLB, sc.XUB, sc.ULB, sc.UUB)
    X, U, Z, st, it, kk, I = _solver(50, obs, ttmpc.TT_VARIANT_TRACK_OBCA, p, bnd).solve(x0, xref=xr, uref=ur,
                                                                                       iterate=True)
    zc, stc, itc, kkc = co.obca_solve_batch(_oracle(50, obs, co.OBCA_TRACK, p, bnd), x0, xref=xr, uref=ur, nthreads=16)
    _ipopt_check_at_gpu_points(_oracle(50, obs, co.OBCA_TRACK, p, bnd), x0, I, st, kk, xref=xr, uref=ur)
    sens = _sensitive("windows")
    # identical statuses on every window whose oracle outcome is not rounding-sensitive (measured: all 16)
    assert np.array_equal(st[~sens], stc[~sens]), (st, stc, np.flatnonzero(sens))
    both = (st <= 1) & (stc <= 1)
    assert both.sum() >= 9, (st, stc)
    Xc = co.obca_split(zc, 50, 11)[0]
    # the same optimum: to 1e-8 wherever both runs stop at the tol-1e-8 optimum (to round-off where they take the
    # same path); a run that stops at an acceptable point (acceptable_tol 1e-6 on the scaled KKT error, 15 times)
    # is compared within that tolerance's reach
    opt = both & (st == 0) & (stc == 0) & ~sens
    assert np.max(np.abs(X[opt] - Xc[opt])) <= 1e-8, np.abs(X - Xc).max(axis=(1, 2))
    assert np.max(np.abs(X[both & ~sens] - Xc[both & ~sens])) <= 1e-6, np.abs(X - Xc).max(axis=(1, 2))
    gap = collision.sat_gap(x0[:, :4], p, obs).min(axis=(-1, -2))
    assert np.all(st[gap < 0.0] > 1) and np.all(stc[gap < 0.0] > 1)
    assert np.all(st[:4] == 0)                          # the open-road windows


def _sensitive(name):
    """Instances of a small parity batch whose oracle outcome (status, or converged end point) changes under a one-ulp
    perturbation of the oracle's input: tests/golden/obca_sensitivity.json (make_obca_sensitivity.py).  The GPU must match
    the oracle on every other instance; on these the kernel's last-bit differences may legitimately decide otherwise."""
    import json
    return np.asarray(json.loads((GOLDEN / "obca_sensitivity.json").read_text())[name]["rounding_sensitive"], dtype=bool)


def _c4_cases(B, seed=0):
    import json
    from ttmpc import scenarios as sc
    cases = json.loads((GOLDEN / "test_cases.json").read_text())["cases"]
    obs = sc.obstacles_array(sc.load_obstacles(GOLDEN / "obstacles.json"))[:6]
    x0, xg, zg = sc.obca_case_batch(cases, B, 200, 6, seed=seed)
    return obs, x0, xg, zg


def test_c4_test_cases_vs_oracle():
    """BASELINE C4 workload: the reference's test_cases.json cases with their 2-waypoint
    initialize.json guess (apply_case.py:16-34, trajectory_optimization.py:227-274), reference duals,
    N=200, M=6 (obstacles.json[0:6]), max_iter 5000.  Cases 0, 5, 6 put the start or the goal pose inside an
    obstacle of that set (SAT, the reference's own collision test): those NLPs are infeasible."""
    from oracle import c_oracle as co
    from ttmpc import collision
    from ttmpc import scenarios as sc
    obs, x0, xg, zg = _c4_cases(14)
    X, U, Z, st, it, kk, I = _solver(200, obs).solve(x0, xg, z_guess=zg, iterate=True)
    zc, stc, itc, kkc = co.obca_solve_batch(_oracle(200, obs), x0, xg, z_guess=zg, nthreads=16)
    # every GPU-optimal end point -- in particular where the two runs end at different points or only the GPU
    # converges -- passes IPOPT's full convergence test as the oracle evaluates it at the GPU's primal-dual point
    _ipopt_check_at_gpu_points(_oracle(200, obs), x0, I, st, kk, x_goal=xg)
    sens = _sensitive("c4_cases")
    # identical statuses wherever the oracle's own outcome is not rounding-sensitive (sensitive: cases 2, 9, 11)
    assert np.array_equal(st[~sens], stc[~sens]), (st, stc, np.flatnonzero(sens))
    gs = collision.sat_gap(x0[:, :4], P6, obs).min(axis=(-1, -2))
    gg = collision.sat_gap(xg[:, :4], P6, obs).min(axis=(-1, -2))
    blocked = (gs < 0.0) | (gg < 0.0)
    # infeasible by construction: IPOPT's restoration failure (status 3) on both sides, not max_iter
    assert blocked.sum() == 6 and np.all(st[blocked] == 3) and np.all(stc[blocked] == 3), (st, stc)
    assert (st[~blocked] <= 1).sum() >= 6 and (stc[~blocked] <= 1).sum() >= 6, (st, stc)
    both = (st <= 1) & (stc <= 1)
    assert both.sum() >= 6, (st, stc)
    Xc, Uc, _, _ = co.obca_split(zc, 200, 6)
    same = np.abs(X - Xc).max(axis=(1, 2)) <= 1e-6       # same local optimum (OBCA is nonconvex)
    # Every both-converged pair ends at the same point unless the instance is rounding-sensitive.  The two runs compute
    # the same iterates while they stay in lockstep (test_obca_lockstep_with_oracle); these runs last 1,000-5,000
    # iterations, and on a sensitive instance (case 9: the oracle itself ends elsewhere under a one-ulp perturbation)
    # rounding decides the basin of the nonconvex NLP.  Both ends are then KKT points: IPOPT's full convergence test
    # holds at the GPU's own primal-dual point (_ipopt_check_at_gpu_points above).
    assert same[both & ~sens].all(), np.abs(X - Xc).max(axis=(1, 2))
    ok = st <= 1
    assert np.abs(X[ok, -1] - xg[ok]).max() <= 1e-2 + 1e-7
    assert np.all(collision.sat_gap(X[ok], P6, obs).min(axis=(-1, -2, -3)) > 0.0)


def test_helper_workgroups_are_bitwise_neutral():
    """The block passes (factor_block / nres_block chunks of the flat block index) run on helper workgroups once CUs are
    idle -- here from the start, the batches being smaller than the CU count.  A chunk's arithmetic does not depend on
    which workgroup runs it, so the outputs with helpers (the default) equal those without (every instance running its
    own chunks) bit for bit: the 14 C4 test cases and the 16 MPC+OBCA windows, stopped at max_iter 400."""
    import ttmpc
    from ttmpc import scenarios as sc
    g = np.load(GOLDEN / "reference_numpy.npz")
    obs, x0, xg, zg = _c4_cases(14)
    x0w, xr, ur = sc.mpc_obs_batch(g["state_traj"], g["input_traj"], 16, 50, seed=0)
    runs = []
    for nh in (-1, 0):
        s = _solver(200, obs, max_iter=400)
        s.set_helpers(nh)
        sw = _solver(50, g["obstacles"], ttmpc.TT_VARIANT_TRACK_OBCA, dict(P6, dt=0.05), (sc.XLB, sc.XUB, sc.ULB, sc.UUB),
                     max_iter=400)
        sw.set_helpers(nh)
        runs.append((s.solve(x0, xg, z_guess=zg), sw.solve(x0w, xref=xr, uref=ur)))
    for a, b in zip(runs[0], runs[1]):
        for u, v in zip(a, b):
            assert np.array_equal(u, v)


def test_helper_handoff_timeout_is_reported_and_isolated():
    """A hand-off that never completes (advisor r5): with ttx_obca_set_handoff_debug one instance
    leaves all its chunks to the helpers and waits for a done count that never comes, under a 2 ms spin limit.  It must
    end with its own status TT_HANDOFF_TIMEOUT (6) -- not TT_NONFINITE -- and a RuntimeWarning, and every other instance
    of the launch must be bit for bit what it is without the debug switch (the 16 MPC+OBCA windows, max_iter 400)."""
    import ttmpc
    from ttmpc import scenarios as sc
    g = np.load(GOLDEN / "reference_numpy.npz")
    x0w, xr, ur = sc.mpc_obs_batch(g["state_traj"], g["input_traj"], 16, 50, seed=0)
    mk = lambda: _solver(50, g["obstacles"], ttmpc.TT_VARIANT_TRACK_OBCA, dict(P6, dt=0.05),  # noqa: E731
                         (sc.XLB, sc.XUB, sc.ULB, sc.UUB), max_iter=400)
    ref = mk().solve(x0w, xref=xr, uref=ur)
    s = mk()
    s.set_handoff_debug(spin_us=2000, fail_b=5)
    with pytest.warns(RuntimeWarning, match="hand-off timed out"):
        out = s.solve(x0w, xref=xr, uref=ur)
    st = out[3]
    assert st[5] == ttmpc.TT_HANDOFF_TIMEOUT, st
    keep = np.arange(16) != 5
    for u, v in zip(out, ref):
        assert np.array_equal(u[keep], v[keep])
    # the switch is per handle: back to the defaults, the same handle reproduces the reference run bit for bit
    s.set_handoff_debug()
    for u, v in zip(s.solve(x0w, xref=xr, uref=ur), ref):
        assert np.array_equal(u, v)


def test_helpers_long_horizon_many_chunks():
    """Advisor r5 (high): a pass of N = 2100 at M = 16 has ceil(2 M (N + 1) / 256) = 263 chunks, more than the 8-bit
    chunk field of round 5's claim word could hold, so helpers dropped chunks and the instance timed out.  With the
    20-bit field (kClaimChunkShift) a small batch with helpers from the start runs bitwise as without helpers."""
    from ttmpc import scenarios as sc
    N, M = 2100, 16
    obs = np.array([[20.0 * i, 40.0, 4.0, 2.0] for i in range(M)])
    x0 = np.array([[0.0, 0.0, 0.0, 0.0, 0.0, 2.0], [0.0, 1.0, 0.05, 0.0, 0.0, 2.0]])
    xg = np.array([[300.0, 0.0, 0.0, 0.0, 0.0, 0.0], [300.0, 2.0, 0.0, 0.0, 0.0, 0.0]])
    zg = np.stack([sc.obca_guess(np.array([a[:2], b[:2]]), np.array([a[2], b[2]]), np.zeros(2), N, M, complete=True)
                   for a, b in zip(x0, xg)])
    runs = []
    for nh in (-1, 0):
        s = _solver(N, obs, max_iter=3)
        s.set_helpers(nh)
        runs.append(s.solve(x0, xg, z_guess=zg))
    assert np.all(runs[0][3] <= 2), runs[0][3]        # no hand-off timeout, nothing non-finite
    for u, v in zip(runs[0], runs[1]):
        assert np.array_equal(u, v)


def test_obca_lockstep_with_oracle():
    """Step-level parity: every instance of the three parity workloads (16 MPC+OBCA windows, the 14 C4 test cases, 16
    re-plans), GPU and oracle both stopped at max_iter K.  Both run the same restated IPOPT on the same inputs, so
    their iterates agree to round-off while no decision (filter, inertia, barrier update, restoration) has flipped
    on a last-bit difference: after 25 iterations every instance agrees to <= 1e-9 (measured <= 9e-11), after 50
    all but a few (measured 43 / 46; DESIGN.md 5 records where the paths separate)."""
    from oracle import c_oracle as co
    from ttmpc import scenarios as sc
    import json
    import ttmpc
    g = np.load(GOLDEN / "reference_numpy.npz")
    obs6 = sc.obstacles_array(sc.load_obstacles(GOLDEN / "obstacles.json"))[:6]
    cases = json.loads((GOLDEN / "test_cases.json").read_text())["cases"]
    p50 = dict(P6, dt=0.05)
    bnd50 = (sc.XLB, sc.XUB, sc.ULB, sc.UUB)
    x0w, xr, ur = sc.mpc_obs_batch(g["state_traj"], g["input_traj"], 16, 50, seed=0)
    plans = [sc.obca_case_batch(cases, 14, 200, 6, seed=0), sc.obca_replan_batch(g["state_traj"], 16, 200, 6, seed=0)]
    for K, need in ((25, 46), (50, 40)):
        d = []
        X, *_ = _solver(50, g["obstacles"], ttmpc.TT_VARIANT_TRACK_OBCA, p50, bnd50, max_iter=K).solve(x0w, xref=xr, uref=ur)
        zc, *_ = co.obca_solve_batch(_oracle(50, g["obstacles"], co.OBCA_TRACK, p50, bnd50, max_iter=K), x0w, xref=xr,
                                     uref=ur, nthreads=16)
        d.append(np.abs(X - co.obca_split(zc, 50, 11)[0]).max(axis=(1, 2)))
        for x0, xg, zg in plans:
            X, *_ = _solver(200, obs6, max_iter=K).solve(x0, xg, z_guess=zg)
            zc, *_ = co.obca_solve_batch(_oracle(200, obs6, max_iter=K), x0, xg, z_guess=zg, nthreads=16)
            d.append(np.abs(X - co.obca_split(zc, 200, 6)[0]).max(axis=(1, 2)))
        d = np.concatenate(d)
        assert (d <= 1e-9).sum() >= need, (K, d)


def test_hbm_source_sweeps_lockstep():
    """N = 230: the serial sweeps' stage records no longer fit the dynamic LDS (kObcaLdsMax), so the Riccati, forward,
    soft and correction sweeps read their operands straight from the HBM workspace (the GSrc / SoftG / VecG / SoftFG
    sources) -- a path no other test reaches.  Lockstep with the oracle at max_iter 25, as the census above."""
    from oracle import c_oracle as co
    from ttmpc import scenarios as sc
    import json
    obs6 = sc.obstacles_array(sc.load_obstacles(GOLDEN / "obstacles.json"))[:6]
    cases = json.loads((GOLDEN / "test_cases.json").read_text())["cases"]
    N, B = 230, 8
    x0, xg, zg = sc.obca_case_batch(cases, B, N, 6, seed=3, obstacles=obs6)
    X, U, Z, st, it, kk = _solver(N, obs6, max_iter=25).solve(x0, xg, z_guess=zg)
    zc, stc, itc, kkc = co.obca_solve_batch(_oracle(N, obs6, max_iter=25), x0, xg, z_guess=zg, nthreads=16)
    d = np.abs(X - co.obca_split(zc, N, 6)[0]).max(axis=(1, 2))
    assert np.all(np.isfinite(X)) and (d <= 1e-9).sum() >= B - 1, d


def test_c4_replan_subset_vs_oracle():
    """Re-plans around the reference's committed plan (8 Hybrid-A*-style waypoints), reference duals."""
    from oracle import c_oracle as co
    from oracle.obca_nlp import ObcaNLP
    from ttmpc import collision
    from ttmpc import scenarios as sc
    g = np.load(GOLDEN / "reference_numpy.npz")
    obs = sc.obstacles_array(sc.load_obstacles(GOLDEN / "obstacles.json"))[:6]
    x0, xg, zg = sc.obca_replan_batch(g["state_traj"], 16, 200, 6, seed=0)
    X, U, Z, st, it, kk, I = _solver(200, obs).solve(x0, xg, z_guess=zg, iterate=True)
    zc, stc, itc, kkc = co.obca_solve_batch(_oracle(200, obs), x0, xg, z_guess=zg, nthreads=16)
    _ipopt_check_at_gpu_points(_oracle(200, obs), x0, I, st, kk, x_goal=xg)
    ok = st <= 1
    assert ok.sum() >= 15 and (stc <= 1).sum() >= 15, (st, stc)
    both = ok & (stc <= 1)
    assert both.sum() >= 14, (st, stc)
    Xc = co.obca_split(zc, 200, 6)[0]
    same = np.abs(X - Xc).max(axis=(1, 2)) <= 1e-6
    sens = _sensitive("replans")
    # the same local optimum wherever both stop, except on rounding-sensitive re-plans
    assert same[both & ~sens].all(), np.abs(X - Xc).max(axis=(1, 2))[both]
    nlp = ObcaNLP(200, 6, P6, sc.OBCA_Q, sc.OBCA_R, sc.OBCA_XLB, sc.OBCA_XUB, sc.OBCA_ULB, sc.OBCA_UUB, obs)
    for b in np.flatnonzero(ok):
        gv, lbg, ubg = nlp.g(Z[b], x0[b], xg[b])
        assert np.all(gv >= lbg - 1e-6) and np.all(gv <= ubg + 1e-6)
        assert collision.sat_gap(X[b], P6, obs).min() > 0.0


def c4_census_compare(st, X, cen, Xc):
    """Per-instance comparison of a GPU C4 batch with the oracle census of the same batch (tests/golden/c4_census.json,
    tests/golden/make_c4_census.py).  Returns the table: status agreement, shared / kernel-only / oracle-only failures,
    both-converged pairs at the same end point, and which disagreements fall on rounding-sensitive instances (the oracle's
    own status or end point changes when its guess is perturbed by one ulp)."""
    stc = np.asarray(cen["status"])
    sens = np.asarray(cen["rounding_sensitive"], dtype=bool)
    ok, okc = st <= 1, stc <= 1
    both = ok & okc
    d = np.abs(X - Xc).max(axis=(1, 2))
    far = both & (d > 1e-6)
    return {"equal_status": int((st == stc).sum()), "instances": int(st.size),
            "shared_failures": np.flatnonzero(~ok & ~okc).tolist(),
            "kernel_only_failures": np.flatnonzero(~ok & okc).tolist(),
            "oracle_only_failures": np.flatnonzero(ok & ~okc).tolist(),
            "both_converged": int(both.sum()), "both_converged_same_point": int((both & ~far).sum()),
            "both_converged_other_point": np.flatnonzero(far).tolist(),
            "status_mismatch_not_sensitive": np.flatnonzero((st != stc) & ~sens).tolist(),
            "other_point_not_sensitive": np.flatnonzero(far & ~sens).tolist(),
            "rounding_sensitive": int(sens.sum())}


def _objective(X, U, xg):
    """The plan-mode objective (trajectory_optimization.py:170-190; Q = I, R = 10 I, 100 Q terminal): the same formula as
    tests/golden/make_c4_census.py plan_objective, per instance."""
    from ttmpc import scenarios as sc
    Q, R = np.asarray(sc.OBCA_Q, float), np.asarray(sc.OBCA_R, float)
    E = X - xg[:, None, :]
    return (np.einsum("bki,ij,bkj->b", U, R, U) + np.einsum("bki,ij,bkj->b", E[:, :-1], Q, E[:, :-1])
            + 100.0 * np.einsum("bi,ij,bj->b", E[:, -1], Q, E[:, -1]))


def c4_objective_compare(st, X, U, xg, cen):
    """For every instance where the GPU and the oracle both converge but to different points (a rounding-sensitive
    instance of the nonconvex NLP), the GPU objective against the oracle's, and against the spread of the oracle's own
    objectives over its one-ulp-perturbed runs (the perturbed runs that converged).  Returns the per-instance table and the
    signed relative differences."""
    Jg = _objective(X, U, xg)
    Jo = np.asarray(cen["objective"])
    stc = np.asarray(cen["status"])
    rows = []
    for b in np.flatnonzero((st <= 1) & (stc <= 1)):
        pert = [p["objective"][b] for p in cen["perturbed"] if p["status"][b] <= 1]
        rows.append({"instance": int(b), "gpu": float(Jg[b]), "oracle": float(Jo[b]),
                     "rel": float((Jg[b] - Jo[b]) / Jo[b]),
                     "oracle_perturbed_rel": [float((v - Jo[b]) / Jo[b]) for v in pert]})
    return rows


def test_c4_full_batch_properties_and_determinism():
    """BASELINE config C4 at full size: B=256 test_cases.json scenarios, N=200, M=6, max_iter 5000, compared instance by
    instance with the oracle's census of the same batch.  Where the GPU's status differs from the
    oracle's, or both converge to different points, the instance must be rounding-sensitive in the oracle itself: its
    outcome changed when the oracle's guess was perturbed by one ulp (tests/golden/make_c4_census.py), i.e. it is decided
    by last-bit differences, which is what separates the kernel's arithmetic from the oracle's."""
    import json
    from ttmpc import collision
    obs, x0, xg, zg = _c4_cases(256, seed=1)
    s = _solver(200, obs)
    X, U, Z, st, it, kk, I = s.solve(x0, xg, z_guess=zg, iterate=True)
    X2, U2, Z2, st2, it2, kk2 = s.solve(x0, xg, z_guess=zg)
    assert np.array_equal(Z, Z2) and np.array_equal(st, st2)   # bitwise-deterministic
    _ipopt_check_at_gpu_points(_oracle(200, obs), x0, I, st, kk, x_goal=xg)
    ok = st <= 1
    gs = collision.sat_gap(x0[:, :4], P6, obs).min(axis=(-1, -2))
    gg = collision.sat_gap(xg[:, :4], P6, obs).min(axis=(-1, -2))
    blocked = (gs < 0.0) | (gg < 0.0)
    cen = json.loads((GOLDEN / "c4_census.json").read_text())["test"]
    Xc = np.load(GOLDEN / "c4_census_test_x.npz")["X"]
    assert np.array_equal(np.asarray(cen["blocked"], dtype=bool), blocked)
    sens = np.asarray(cen["rounding_sensitive"], dtype=bool)
    # infeasible by construction: they never converge, and they end as IPOPT's restoration failure (status 3) instead of
    # running to max_iter -- except where the oracle itself flips between the two under a one-ulp perturbation (blocked
    # instance 61: max_iter unperturbed, status 3 in both perturbed runs; tests/golden/c4_census.json)
    assert np.all(st[blocked] > 1), np.bincount(st[blocked])
    assert np.all((st[blocked] == 3) | sens[blocked]), np.flatnonzero(blocked & (st != 3))
    tab = c4_census_compare(st, X, cen, Xc)
    print("C4 census comparison:", json.dumps(tab))
    # every disagreement with the oracle -- a different status, or a different optimum -- is on an instance whose
    # outcome the oracle itself changes under a one-ulp perturbation of its guess
    assert not tab["status_mismatch_not_sensitive"], tab
    assert not tab["other_point_not_sensitive"], tab
    dyn = X[:, 1:] - (X[:, :-1] + 0.1 * _f(X[:, :-1], U))
    assert np.abs(dyn[ok]).max() <= 1e-8
    assert np.abs(X[ok, 0] - x0[ok]).max() <= 1e-8
    assert np.abs(X[ok, -1] - xg[ok]).max() <= 1e-2 + 1e-7               # final box
    assert np.all(collision.sat_gap(X[ok], P6, obs).min(axis=(-1, -2, -3)) > 0.0)
    _assert_other_optima_unbiased(st, X, U, xg, cen, Xc)


def _oracle_perturbation_spread(cen):
    """The relative objective changes the oracle itself shows between two legitimate runs: for every instance and
    perturbed census run where both the unperturbed and the perturbed oracle runs converge but end more than 1e-6 apart,
    (J_perturbed - J) / J."""
    st = np.asarray(cen["status"])
    J = np.asarray(cen["objective"])
    out = []
    for p in cen["perturbed"]:
        sp, dx, Jp = np.asarray(p["status"]), np.asarray(p["dx_max"]), np.asarray(p["objective"])
        m = (st <= 1) & (sp <= 1) & (dx > 1e-6)
        out.extend(((Jp[m] - J[m]) / J[m]).tolist())
    return np.asarray(out)


def _assert_other_optima_unbiased(st, X, U, xg, cen, Xc):
    """on the both-converged pairs that end at different local optima, the GPU's optima must not be
    systematically worse than the oracle's.  The yardstick is the oracle itself: its one-ulp-perturbed runs of the same
    batch end at other optima too, with objectives from -50 % to +100 % of the unperturbed run's on this nonconvex NLP.
    The GPU's signed relative differences must not lean against the GPU (mean <= +5 %, median <= +1 %), and its largest
    increase must stay within the largest increase the oracle's own perturbed runs show on the batch (+5 %).  Measured:
    bench batch 37 pairs, GPU lower on 23, mean -5.2 %, median -0.3 %, max +12 %; test batch 17 pairs, GPU lower on 10,
    mean -2.6 %, median -0.6 %, max +27 % (#79) against the oracle's own +26 % (#58 under one perturbation)."""
    import json
    rows = c4_objective_compare(st, X, U, xg, cen)
    d = np.abs(X - Xc).max(axis=(1, 2))
    far = [r for r in rows if d[r["instance"]] > 1e-6]
    same = [r for r in rows if d[r["instance"]] <= 1e-6]
    print("C4 other-optimum objectives:", json.dumps(far))
    assert all(abs(r["rel"]) <= 1e-7 for r in same), same     # the same end point: the same objective
    if not far:
        return
    rel = np.array([r["rel"] for r in far])
    spread = _oracle_perturbation_spread(cen)
    print(f"GPU vs oracle on {rel.size} other-optimum pairs: mean {rel.mean():+.4f} median {np.median(rel):+.4f} "
          f"max {rel.max():+.4f}; the oracle's own perturbed runs: {spread.size} pairs, max {spread.max():+.4f}")
    assert rel.mean() <= 0.05 and np.median(rel) <= 0.01, rel
    assert rel.max() <= spread.max() + 0.05, (rel.max(), spread.max())


def _kernel_sensitive(s, x0, xg, zg, st, X):
    """The kernel's own rounding sensitivity (tools/obca_gpu_sensitivity.py): the batch re-solved with the guess scaled
    by the census factors; an instance is kernel-sensitive when a perturbed run changes its status, or moves a converged
    end point by more than 1e-6 -- the experiment of tests/golden/make_c4_census.py, on the GPU."""
    import sys
    sys.path.insert(0, str(GOLDEN))
    from make_c4_census import PERTURB
    sens = np.zeros(len(st), dtype=bool)
    for f in PERTURB:
        Xp, Up, Zp, stp, itp, kkp = s.solve(x0, xg, z_guess=zg * f)
        sens |= (stp != st) | ((st <= 1) & (np.abs(Xp - X).max(axis=(1, 2)) > 1e-6))
    return sens


def test_c4_bench_batch_against_census():
    """The bench's own C4 batch (bench.py --config c4: B = 256, seed 7, the collision-free cases) instance by instance
    against the oracle census of that batch with THREE one-ulp-class perturbations (tests/golden/make_c4_census.py,
    VERDICT r5 item 1): equal status and the same end point on every instance whose oracle outcome is not
    rounding-sensitive; every GPU-optimal end point passes IPOPT's convergence test at the oracle's evaluation; the
    other-optimum pairs are not biased against the GPU."""
    import json
    from ttmpc import collision
    from ttmpc import scenarios as sc
    cases = json.loads((GOLDEN / "test_cases.json").read_text())["cases"]
    obs = sc.obstacles_array(sc.load_obstacles(GOLDEN / "obstacles.json"))[:6]
    x0, xg, zg = sc.obca_case_batch(cases, 256, 200, 6, seed=7, obstacles=obs, params=sc.OBCA_PARAMS)
    s = _solver(200, obs)
    X, U, Z, st, it, kk, I = s.solve(x0, xg, z_guess=zg, iterate=True)
    _ipopt_check_at_gpu_points(_oracle(200, obs), x0, I, st, kk, x_goal=xg)
    cen = json.loads((GOLDEN / "c4_census.json").read_text())["bench"]
    Xc = np.load(GOLDEN / "c4_census_bench_x.npz")["X"]
    assert len(cen["perturbed"]) == 3 and not np.any(cen["blocked"])
    tab = c4_census_compare(st, X, cen, Xc)
    print("C4 bench-batch census comparison:", json.dumps(tab))
    # Two instances (28: the kernel at max_iter, 168: acceptable instead of optimal) disagree although the oracle's outcome
    # is robust under its three perturbations.  Both are rounding-decided on the kernel's side: the kernel's OWN perturbed
    # runs converge on 28 (1,723-1,971 iterations) and reach the optimum on 168, and the
    # oracle built with FMA contraction (make -C oracle fma) needs 1,824 iterations on 28 instead of 983.  So a disagreement
    # must be rounding-sensitive on one side or the other.
    ksens = _kernel_sensitive(s, x0, xg, zg, st, X)
    print("kernel-sensitive:", np.flatnonzero(ksens).tolist())
    assert set(tab["status_mismatch_not_sensitive"]) <= set(np.flatnonzero(ksens).tolist()), tab
    assert set(tab["other_point_not_sensitive"]) <= set(np.flatnonzero(ksens).tolist()), tab
    ok = st <= 1
    assert np.all(collision.sat_gap(X[ok], P6, obs).min(axis=(-1, -2, -3)) > 0.0)
    _assert_other_optima_unbiased(st, X, U, xg, cen, Xc)


def test_default_plan_matches_oracle():
    """The reference's own default OBCA call (trajectory_animation.py:43-52, 77-83, 109): N = 200, dt = 0.1, all 11
    obstacles of obstacles.json, the Hybrid-A*-shaped 8-waypoint guess of tests/golden/make_golden_default_plan.py,
    max_iter 5000.  The kernel reaches the oracle's optimum (the committed fixture): same status, the same primal
    solution to 1e-6, cost 64,914, collision-free with d_min active."""
    from oracle import c_oracle as co
    from ttmpc import collision
    g = np.load(GOLDEN / "oracle_default_plan.npz")
    ob = np.load(GOLDEN / "reference_numpy.npz")["obstacles"].reshape(-1, 4)
    N, M = 200, ob.shape[0]
    X, U, Z, st, it, kk, I = _solver(N, ob).solve(g["x_init"], g["x_goal"], z_guess=g["z_guess"], iterate=True)
    assert st[0] == int(g["status"][0]) == 0, (st, it, kk)
    _ipopt_check_at_gpu_points(_oracle(N, ob), g["x_init"], I, st, kk, x_goal=g["x_goal"])
    Xc, Uc, _, _ = co.obca_split(g["z"], N, M)
    assert np.abs(X - Xc).max() <= 1e-6 and np.abs(U - Uc).max() <= 1e-6
    d = X[0] - g["x_goal"][0]
    cost = float((d[:-1] ** 2).sum() + 100.0 * (d[-1] ** 2).sum() + 10.0 * (U[0] ** 2).sum())
    assert abs(cost - float(g["cost"])) <= 1e-6 * float(g["cost"])
    gap = collision.sat_gap(X[0], P6, ob).min()
    assert 0.199 < gap <= 0.2 + 1e-6


def _f(X, U):
    L1, L2, M = P6["L1"], P6["L2"], P6["M"]
    th, psi, phi, v = X[..., 2], X[..., 3], X[..., 4], X[..., 5]
    return np.stack([v * np.cos(th), v * np.sin(th), v * np.tan(phi) / L1,
                     -v * np.tan(phi) / L1 * (1 + M / L2 * np.cos(psi)) - v * np.sin(psi) / L2,
                     U[..., 1], U[..., 0]], axis=-1)


def test_reference_call_surface_obca(capsys, tmp_path, monkeypatch):
    """TrajectoryOptimization.plan / .optimize and MPCTrackingControlObs.solve mirror the reference
    signatures; plan() builds its guess from initialize.json as trajectory_optimization.py:232,312 does."""
    import json
    import ttmpc
    from ttmpc import scenarios as sc
    model = ttmpc.TruckTrailerModel(dict(P6, horizon=60))
    obstacle_list = [{"center": (10.5, 2.6), "width": 3.0, "height": 2.0}]
    ini = tmp_path / "initialize.json"   # start / goal headings in the initialize.json convention (-pi/2)
    ini.write_text(json.dumps({"Positions": [[0.0, 0.0], [26.0, -0.2]], "Headings": [0.02 - np.pi / 2, -np.pi / 2],
                               "HitchAngles": [0.0, 0.0]}))
    args = (model, dict(P6, horizon=60), sc.OBCA_Q, sc.OBCA_R, {"lb": sc.OBCA_XLB, "ub": sc.OBCA_XUB},
            {"lb": sc.OBCA_ULB, "ub": sc.OBCA_UUB}, obstacle_list)
    planner = ttmpc.TrajectoryOptimization(*args, initialize_path=str(ini))
    states, inputs = planner.plan(np.array([0.0, 0.0, 0.02, 0.0, 0.0, 0.0]), np.array([26.0, -0.2, 0, 0, 0, 0]))
    assert states.shape == (6, 61) and inputs.shape == (2, 60)
    assert planner.last_status[0] == 0
    states2, inputs2 = planner.optimize(np.array([0.0, 0.0, 0.02, 0.0, 0.0, 0.0]), np.array([26.0, -0.2, 0, 0, 0, 0]))
    assert np.array_equal(states, states2) and np.array_equal(inputs, inputs2)
    # without initialize.json the reference's open() fails; so does the mirror
    monkeypatch.chdir(tmp_path / "..")
    monkeypatch.delenv("TTMPC_INITIALIZE", raising=False)
    if not (tmp_path / ".." / "initialize.json").exists() and not (tmp_path / ".." / ".." / "initialize.json").exists():
        with pytest.raises(FileNotFoundError):
            ttmpc.TrajectoryOptimization(*args).plan(np.zeros(6), np.zeros(6))
    g = np.load(GOLDEN / "reference_numpy.npz")
    p = dict(P6, dt=0.05, horizon=50)
    ctrl = ttmpc.MPCTrackingControlObs(model, p, sc.OBCA_Q, sc.OBCA_R, {"lb": sc.XLB, "ub": sc.XUB},
                                       {"lb": sc.ULB, "ub": sc.UUB},
                                       obstacle_list=[{"center": (o[0], o[1]), "width": o[2], "height": o[3]}
                                                      for o in g["obstacles"]])
    x0, xr, ur = sc.mpc_obs_batch(g["state_traj"], g["input_traj"], 1, 50, seed=0)
    st_, in_ = ctrl.solve(x0[0], xr[0].T, ur[0].T)
    assert st_.shape == (6, 51) and in_.shape == (2, 50)
    assert "Cannot find a solution!" not in capsys.readouterr().out
    with pytest.raises(ValueError):
        ttmpc.TrajectoryOptimization(model, dict(P6, horizon=60), sc.OBCA_Q, sc.OBCA_R,
                                     {"lb": sc.OBCA_XLB, "ub": sc.OBCA_XUB}, {"lb": sc.OBCA_ULB, "ub": sc.OBCA_UUB}, [])


def test_obca_abi_errors():
    import ctypes as C
    import ttmpc
    from ttmpc import _lib
    L = ttmpc.lib()
    cfg = _lib.TTConfig()
    cfg.nx, cfg.nu, cfg.N, cfg.M = 6, 2, 20, 0
    cfg.dt, cfg.L1, cfg.L2, cfg.Mh, cfg.W1, cfg.W2 = 0.1, 7.05, 12.45, 0.15, 3.05, 2.95
    cfg.variant = ttmpc.TT_VARIANT_OBCA_PLAN
    z6, z2 = np.zeros(36), np.zeros(4)
    lb, ub = np.full(6, -1e20), np.full(6, 1e20)
    h = C.c_void_p()
    p = _lib._ptr
    assert L.tt_create(C.byref(cfg), p(z6), p(z2), p(lb), p(ub), p(lb[:2].copy()), p(ub[:2].copy()), None, 0,
                       C.byref(h)) == -22  # M = 0 obstacles
    assert L.tt_obca_n(200, 6) == 200 * (8 + 96) + 6 + 96
