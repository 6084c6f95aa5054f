"""GPU suite: the closed-loop simulation kernels (tt_sim.hip through the C ABI) against the reference's
own outputs (tests/golden/reference_numpy.npz) and the oracle, and a batched closed loop against the
oracle's restatement of the simulation.py loop.

Tolerances: window / shift / record / interpolation / collision flags are bit-exact (pure data movement,
contraction-free arithmetic); the plant update matches the reference's numpy to 1e-13 (device libm
sin/cos/tan vs glibc); closed-loop trajectories match the oracle loop to 1e-6 (per-step solves agree to
1e-7).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

P = {"M": 0.15, "L1": 7.05, "L2": 12.45, "W1": 3.05, "W2": 2.95, "dt": 0.05}


def _t(a, dtype=torch.float64):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dtype).cuda()


@pytest.fixture(scope="module")
def plan(golden_ref):
    from oracle import ttmpc_oracle as to
    return to.do_interpolation(golden_ref["state_traj"], golden_ref["input_traj"], 0.1, 0.05)


def test_interpolation_kernel_is_bit_exact(golden_ref):
    from ttmpc import simulation as sim
    S, U = sim.interpolate(_t(golden_ref["state_traj"].T[None]), _t(golden_ref["input_traj"].T[None]), 0.1, 0.05)
    torch.cuda.synchronize()
    assert np.array_equal(S.cpu().numpy()[0].T, golden_ref["interp_states"])
    assert np.array_equal(U.cpu().numpy()[0].T, golden_ref["interp_inputs"])


@pytest.mark.parametrize("N", [20, 50])
def test_window_kernel_matches_reference_padding(plan, N):
    from oracle import ttmpc_oracle as to
    from ttmpc import simulation as sim
    S, U = plan
    Np = U.shape[1]
    px, pu = _t(S.T[None]), _t(U.T[None])
    rng = np.random.default_rng(N)
    B = 5
    state = rng.normal(size=(B, 6))
    noise = rng.normal(scale=0.02, size=(B, 6))
    for k in (0, 17, Np - N, Np - N + 3, Np - 1, Np, Np + 9):
        xm, xr, ur = sim.window(px, pu, k, N, _t(state), _t(noise))
        torch.cuda.synchronize()
        Xr, Ur = to.reference_window(S, U, k, N)
        assert np.array_equal(xr.cpu().numpy(), np.broadcast_to(Xr.T, (B, N + 1, 6))), k
        assert np.array_equal(ur.cpu().numpy(), np.broadcast_to(Ur.T, (B, N, 2))), k
        assert np.array_equal(xm.cpu().numpy(), state + noise)


def test_window_kernel_per_instance_plans(plan):
    from oracle import ttmpc_oracle as to
    from ttmpc import simulation as sim
    S, U = plan
    B, N = 3, 20
    shift = np.arange(B)[:, None, None] * 1.5
    px, pu = S.T[None] + shift, U.T[None] * (1 + shift[:, :, :2])
    _, xr, ur = sim.window(_t(px), _t(pu), 390, N, _t(np.zeros((B, 6))))
    torch.cuda.synchronize()
    for b in range(B):
        Xr, Ur = to.reference_window(px[b].T, pu[b].T, 390, N)
        assert np.array_equal(xr.cpu().numpy()[b], Xr.T) and np.array_equal(ur.cpu().numpy()[b], Ur.T)


def test_collision_kernel_reproduces_reference_outputs(golden_ref):
    """simulation.check_state_collision executed by the reference on 256 poses (make_golden.py)."""
    from ttmpc import simulation as sim
    poses = np.concatenate([golden_ref["poses"], np.zeros((256, 2))], axis=1)[:, None, :]
    flag = sim.collision_flags(_t(poses), _t(golden_ref["obstacles"]), P)
    torch.cuda.synchronize()
    assert np.array_equal(flag.cpu().numpy().astype(bool), golden_ref["collide"].astype(bool))


def test_collision_kernel_on_trajectories_matches_host_checker(golden_ref):
    from ttmpc import collision
    from ttmpc import simulation as sim
    rng = np.random.default_rng(5)
    B, K = 300, 51
    base = golden_ref["state_traj"].T[rng.integers(0, 150, B)]
    traj = base[:, None, :] + np.cumsum(rng.normal(scale=[0.3, 0.3, 0.03, 0.03, 0, 0], size=(B, K, 6)), axis=1)
    flag = sim.collision_flags(_t(traj), _t(golden_ref["obstacles"]), P).cpu().numpy().astype(bool)
    ref = np.array([collision.check_trajectory_collision(traj[b].T, P, golden_ref["obstacles"]) for b in range(B)])
    assert np.array_equal(flag, ref) and 0 < ref.sum() < B
    # the reference's committed OBCA plan never collides
    f0 = sim.collision_flags(_t(golden_ref["state_traj"].T[None]), _t(golden_ref["obstacles"]), P)
    assert int(f0.cpu()[0]) == 0


def test_plant_kernel_matches_reference_update(golden_ref):
    from oracle import ttmpc_oracle as to
    from ttmpc import simulation as sim
    for dist, key in ((None, "upd_nom"), (sim.DISTURBANCE_PARAMS, "upd_dist")):
        s = _t(golden_ref["q"])
        ua = torch.empty((64, 2), dtype=torch.float64, device="cuda")
        sim.plant_update(s, _t(golden_ref["u"]), P, dist, u_applied=ua)
        torch.cuda.synchronize()
        assert np.max(np.abs(s.cpu().numpy() - golden_ref[key])) <= 1e-13, key
        assert np.array_equal(ua.cpu().numpy(), golden_ref["u"])
    # slip_angle_max > 0 exercises apply_slippage_to_dynamics
    d = dict(sim.DISTURBANCE_PARAMS, slip_angle_max=0.2)
    s = _t(golden_ref["q"])
    sim.plant_update(s, _t(golden_ref["u"]), P, d)
    assert np.max(np.abs(s.cpu().numpy() - to.plant_update(golden_ref["q"], golden_ref["u"], P, d))) <= 1e-13


def test_plant_kernel_with_in_plant_noise_matches_nmpc_update():
    """tt_plant_update_noise_device against the NMPC / fuzzy drivers' update executed by the reference
    (tests/golden/nmpc_plant.npz: simulation_nmpc.py / simulation_fuzzy.py:94-105 with recorded noise draws)."""
    from conftest import GOLDEN
    from ttmpc import simulation as sim
    g = np.load(GOLDEN / "nmpc_plant.npz")
    keys = ("friction_coeff", "slippage_coeff", "process_noise_std", "lateral_slip_gain", "slip_angle_max")
    for tag in ("nmpc", "fuzzy"):
        for which in ("own", "full"):
            dist = {k: float(g[f"{which}_{k}"]) for k in keys}
            s = _t(g["q"])
            sim.plant_update(s, _t(g["u"]), P, dist, state_noise=_t(g[f"{tag}_{which}_noise"]))
            torch.cuda.synchronize()
            assert np.max(np.abs(s.cpu().numpy() - g[f"{tag}_{which}_next"])) <= 1e-13, (tag, which)
    # host convenience with the reference signature + explicit draw
    q1 = sim.update(g["q"][3], g["u"][3], P, {k: float(g[f"full_{k}"]) for k in keys},
                    state_noise=g["nmpc_full_noise"][3])
    assert np.max(np.abs(q1 - g["nmpc_full_next"][3])) <= 1e-13


def test_plant_kernel_applies_first_input_and_zero_on_failure(golden_ref):
    from oracle import ttmpc_oracle as to
    from ttmpc import simulation as sim
    rng = np.random.default_rng(2)
    B, N = 64, 20
    U = rng.normal(size=(B, N, 2))
    st = np.where(np.arange(B) % 3 == 0, 2, 0).astype(np.int32)
    s = _t(golden_ref["q"])
    sim.plant_update(s, _t(U), P, None, status=_t(st, torch.int32), zero_on_fail=True)
    u0 = U[:, 0].copy()
    u0[st > 1] = 0.0
    assert np.max(np.abs(s.cpu().numpy() - to.plant_update(golden_ref["q"], u0, P))) <= 1e-13


@pytest.mark.parametrize("bug_compatible", [True, False])
def test_warm_start_and_record_kernels_match_shift(bug_compatible):
    from ttmpc import layout, lib
    import ctypes as C
    rng = np.random.default_rng(3)
    B, N = 7, 20
    X, U = rng.normal(size=(B, N + 1, 6)), rng.normal(size=(B, N, 2))
    xr, ur = rng.normal(size=(B, N + 1, 6)), rng.normal(size=(B, N, 2))
    st = np.array([0, 1, 2, 0, 4, 0, 3], dtype=np.int32)
    dX, dU, dst = _t(X), _t(U), _t(st, torch.int32)
    last = torch.zeros((B, 8 * N + 6), dtype=torch.float64, device="cuda")
    have = torch.zeros(B, dtype=torch.int32, device="cuda")
    zg = torch.empty_like(last)
    L = lib()
    s0 = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert L.tt_record_solution_device(B, N, dX.data_ptr(), dU.data_ptr(), dst.data_ptr(), last.data_ptr(),
                                       have.data_ptr(), s0) == 0
    assert L.tt_warm_start_device(B, N, last.data_ptr(), have.data_ptr(), _t(xr).data_ptr(), _t(ur).data_ptr(),
                                  int(bug_compatible), zg.data_ptr(), s0) == 0
    torch.cuda.synchronize()
    ok = st <= 1
    assert np.array_equal(have.cpu().numpy().astype(bool), ok)
    z = layout.pack(X, U)
    exp = np.where(ok[:, None], layout.shift(z, N, bug_compatible), layout.pack(xr, ur))
    assert np.array_equal(zg.cpu().numpy(), exp)
    assert np.array_equal(last.cpu().numpy()[ok], z[ok]) and not last.cpu().numpy()[~ok].any()


def _oracle_solver(N):
    from oracle import c_oracle as co
    from oracle import ttmpc_oracle as to
    from ttmpc import layout
    nlp = to.TrackingNLP(N)
    Pp = co.make_problem(N, P, nlp.Q, nlp.R, nlp.xlb, nlp.xub, nlp.ulb, nlp.uub)

    def solve(x, Xr, Ur):
        z, st, _, _ = co.solve_batch(Pp, x, Xr, Ur)
        X, Uo = layout.unpack(z, N)
        return X, Uo, st
    return solve


@pytest.mark.parametrize("disturbed", [False, True])
def test_closed_loop_matches_oracle_loop(plan, golden_ref, disturbed):
    """simulation.py's loop for B=6 perturbed starts, 1.5 s, N=20, with the same measurement noise."""
    import ttmpc
    from oracle import ttmpc_oracle as to
    from ttmpc import simulation as sim
    S, U = plan
    N, B, T = 20, 6, 1.5
    rng = np.random.default_rng(11)
    x0 = S[:, 0][None] + rng.normal(scale=[0.3, 0.3, 0.02, 0.02, 0.0, 0.0], size=(B, 6))
    K = len(to.step_indices(T, 0.05))
    dist = sim.DISTURBANCE_PARAMS if disturbed else None
    noise = rng.normal(scale=0.002, size=(K, B, 6)) if disturbed else None
    solver = ttmpc.BatchSolver(N, P, to.DEFAULT_Q, to.DEFAULT_R, to.MPC_XLB, to.MPC_XUB, to.MPC_ULB, to.MPC_UUB)
    cl = sim.ClosedLoop(solver, S, U, P, dist, obstacles=golden_ref["obstacles"])
    out = cl.run(x0, T, noise=noise)
    ref_states, ref_u, ref_st = to.closed_loop(_oracle_solver(N), x0, S, U, N, T, P, dist, noise)
    assert np.array_equal(out["status"], ref_st)
    assert np.max(np.abs(out["states"] - ref_states)) <= 1e-6
    assert np.max(np.abs(out["controls"] - ref_u)) <= 1e-6
    # the collision check of every step ran on the previous prediction / the first window
    assert out["collide"].shape == (K, B)


def test_nmpc_closed_loop_warm_start(plan):
    """TruckTrailerNMPC loop (simulation_nmpc.py): shifted warm start on the device, tol 1e-3.  As with
    IPOPT (no warm_start_init_point: duals and mu restart), the shifted primal does not save iterations;
    the closed loop must land on the same trajectories as the cold-started one."""
    import ttmpc
    from oracle import ttmpc_oracle as to
    from ttmpc import simulation as sim
    S, U = plan
    N, B = 20, 16
    rng = np.random.default_rng(4)
    x0 = S[:, 0][None] + rng.normal(scale=[0.2, 0.2, 0.01, 0.01, 0, 0], size=(B, 6))
    mk = lambda: ttmpc.BatchSolver(N, P, to.DEFAULT_Q, to.DEFAULT_R, to.MPC_XLB, to.MPC_XUB, to.MPC_ULB,  # noqa: E731
                                   to.MPC_UUB, variant=ttmpc.TT_VARIANT_NMPC)
    warm = sim.ClosedLoop(mk(), S, U, P, None, warm_start=True, zero_on_fail=True).run(x0, 2.0)
    cold = sim.ClosedLoop(mk(), S, U, P, None, warm_start=False, zero_on_fail=True).run(x0, 2.0)
    assert warm["success"].all() and cold["success"].all()
    assert np.array_equal(warm["iters"][0], cold["iters"][0])          # step 0: no previous solution yet
    assert not np.array_equal(warm["iters"][1:], cold["iters"][1:])    # later steps start from the shift
    assert np.max(np.abs(warm["states"] - cold["states"])) < 0.05   # tol 1e-3 solves of the same NLPs


def test_switch_mode_routes_colliding_instances_to_obca(plan, golden_ref):
    """USE_SWITCH_MPC: instances whose first window collides are solved by MPCTrackingControlObs."""
    import ttmpc
    from oracle import ttmpc_oracle as to
    from ttmpc import collision
    from ttmpc import simulation as sim
    S, U = plan
    N, B = 20, 4
    # an extra obstacle next to the course ahead of the start
    obs = np.concatenate([golden_ref["obstacles"], [[S[0, 10], S[1, 10] + 4.0, 2.0, 2.0]]])
    x0 = np.repeat(S[:, 0][None], B, 0)
    solver = ttmpc.BatchSolver(N, P, to.DEFAULT_Q, to.DEFAULT_R, to.MPC_XLB, to.MPC_XUB, to.MPC_ULB, to.MPC_UUB)
    obca = ttmpc.ObcaSolver(N, P, to.DEFAULT_Q, to.DEFAULT_R, to.MPC_XLB, to.MPC_XUB, to.MPC_ULB, to.MPC_UUB, obs,
                            variant=ttmpc.TT_VARIANT_TRACK_OBCA, max_iter=300)
    cl = sim.ClosedLoop(solver, S, U, P, None, obstacles=obs, switch_solver=obca)
    out = cl.run(x0, 0.1)
    Xr, _ = to.reference_window(S, U, 0, N)
    assert bool(out["collide"][0, 0]) == collision.check_trajectory_collision(Xr, P, obs)
    assert np.isfinite(out["states"]).all()


def test_obca_plans_feed_tracking_batch_on_device(golden_ref):
    """§8(f) row 2: B device-resident OBCA-style plans -> do_interpolation on the GPU -> per-instance
    ClosedLoop references, equal to the reference's host resampling of each plan."""
    from oracle import ttmpc_oracle as to
    from ttmpc import handoff
    S, U = golden_ref["state_traj"], golden_ref["input_traj"]
    B = 4
    X = np.stack([S.T + 0.5 * b for b in range(B)])
    Uu = np.stack([U.T * (1 + 0.1 * b) for b in range(B)])
    Xr, Ur = handoff.plan_batch_to_references(_t(X), _t(Uu))
    torch.cuda.synchronize()
    for b in range(B):
        S2, U2 = to.do_interpolation(X[b].T, Uu[b].T, 0.1, 0.05)
        assert np.array_equal(Xr.cpu().numpy()[b], S2.T) and np.array_equal(Ur.cpu().numpy()[b], U2.T)


@pytest.mark.parametrize("warm", [False, True])
def test_graph_replay_equals_eager_loop(plan, golden_ref, warm):
    """run_graph (one captured step replayed through a hipGraph, step index on the device) reproduces the
    eager run() bit for bit, disturbances, noise, collision checks and the NMPC warm start included (the NMPC
    policy puts the noise into the plant, simulation_nmpc.py:94-105: the device-selected draw of the step)."""
    import ttmpc
    from oracle import ttmpc_oracle as to
    from ttmpc import simulation as sim
    S, U = plan
    N, B, T = 20, 32, 1.0
    rng = np.random.default_rng(12)
    x0 = S[:, 0][None] + rng.normal(scale=[0.3, 0.3, 0.02, 0.02, 0.0, 0.0], size=(B, 6))
    K = len(to.step_indices(T, 0.05))
    noise = rng.normal(scale=0.002, size=(K, B, 6))
    variant = ttmpc.TT_VARIANT_NMPC if warm else ttmpc.TT_VARIANT_TRACK
    mk = lambda: ttmpc.BatchSolver(N, P, to.DEFAULT_Q, to.DEFAULT_R, to.MPC_XLB, to.MPC_XUB, to.MPC_ULB,  # noqa: E731
                                   to.MPC_UUB, variant=variant)
    kw = dict(obstacles=golden_ref["obstacles"], warm_start=warm, zero_on_fail=warm)
    eager = sim.ClosedLoop(mk(), S, U, P, sim.DISTURBANCE_PARAMS, **kw).run(x0, T, noise=noise)
    graph = sim.ClosedLoop(mk(), S, U, P, sim.DISTURBANCE_PARAMS, **kw).run_graph(x0, T, noise=noise)
    for key in ("states", "controls", "status", "iters", "collide"):
        assert np.array_equal(eager[key], graph[key]), key


def _oracle_solver_cfg(N, tol, acc_tol, max_iter, acc_iter):
    """Oracle solve with the NMPC / fuzzy IPOPT options and optional per-instance weights w (B,8)."""
    from oracle import c_oracle as co
    from oracle import ttmpc_oracle as to
    from ttmpc import layout
    nlp = to.TrackingNLP(N)
    Pp = co.make_problem(N, P, nlp.Q, nlp.R, nlp.xlb, nlp.xub, nlp.ulb, nlp.uub, tol=tol, acc_tol=acc_tol,
                         max_iter=max_iter, acc_iter=acc_iter)

    def solve(x, Xr, Ur, w=None):
        z, st, _, _ = co.solve_batch(Pp, x, Xr, Ur, wq=None if w is None else w[:, :6], wr=None if w is None else w[:, 6:])
        X, Uo = layout.unpack(z, N)
        return X, Uo, st
    return solve


@pytest.mark.parametrize("policy, variant", [("nmpc", "NMPC"), ("fuzzy", "FUZZY")])
def test_disturbed_nmpc_fuzzy_loops_match_oracle_loop(plan, policy, variant):
    """simulation_nmpc.py / simulation_fuzzy.py with ENABLE_DISTURBANCES: the solver sees the exact state and the
    process noise enters the plant (q_ += noise * dt, 94-105; tt_policy_plant_noise_device), against the oracle
    loop with the same draws.  The modules' own IPOPT options (tol 1e-3, acceptable 1e-2 x 5, max_iter 2000)."""
    import ttmpc
    from oracle import ttmpc_oracle as to
    from ttmpc import simulation as sim
    S, U = plan
    N, B, T = 20, 6, 1.5
    rng = np.random.default_rng(31)
    x0 = S[:, 0][None] + rng.normal(scale=[0.3, 0.3, 0.02, 0.02, 0.0, 0.0], size=(B, 6))
    K = len(to.step_indices(T, 0.05))
    dist = {"friction_coeff": 1, "slippage_coeff": 1, "process_noise_std": 0.02, "lateral_slip_gain": 0.0,
            "slip_angle_max": 0.0}                  # simulation_nmpc.py:20-26 / simulation_fuzzy.py:20-26
    noise = rng.normal(scale=dist["process_noise_std"], size=(K, B, 6))
    tol, acc, mi, ai = 1e-3, 1e-2, 2000, 5
    solver = ttmpc.BatchSolver(N, P, to.DEFAULT_Q, to.DEFAULT_R, to.MPC_XLB, to.MPC_XUB, to.MPC_ULB, to.MPC_UUB,
                               variant=getattr(ttmpc, f"TT_VARIANT_{variant}"), tol=tol, acc_tol=acc, max_iter=mi,
                               acc_iter=ai)
    cl = sim.ClosedLoop(solver, S, U, P, dist, policy=policy)
    assert cl.noise_in_plant and not cl.measurement_noise
    out = cl.run(x0, T, noise=noise)
    ref_S, ref_u, ref_st, pol = to.closed_loop(_oracle_solver_cfg(N, tol, acc, mi, ai), x0, S, U, N, T, P, dist,
                                               policy=policy, fuzzy=variant == "FUZZY", plant_noise=noise)
    assert np.array_equal(out["status"], ref_st)
    assert np.max(np.abs(out["controls"] - ref_u)) <= 1e-6
    assert np.max(np.abs(out["states"] - ref_S)) <= 1e-6
    # the plant noise moved the states: the noise-free loop ends elsewhere
    calm = to.closed_loop(_oracle_solver_cfg(N, tol, acc, mi, ai), x0, S, U, N, T, P, dist, policy=policy,
                          fuzzy=variant == "FUZZY")[0]
    assert np.max(np.abs(calm[-1] - ref_S[-1])) > 1e-4


@pytest.mark.parametrize("policy, variant", [("nmpc", "NMPC"), ("fuzzy", "FUZZY")])
def test_failure_policies_match_oracle_loop(plan, policy, variant):
    """simulation_nmpc.py / simulation_fuzzy.py failure handling on the device (tt_policy_plant_device,
    tt_fuzzy_weights_device + the unit-weight retry) against the oracle loop.  max_iter is cut to 3 so that
    most solves fail and every branch runs: zero / last control, the 15-failure zero-control switch and the
    20 / 30 consecutive-failure stop."""
    import ttmpc
    from oracle import ttmpc_oracle as to
    from ttmpc import simulation as sim
    S, U = plan
    N, B, T = 20, 8, 2.0
    rng = np.random.default_rng(21)
    x0 = S[:, 0][None] + rng.normal(scale=[0.4, 0.4, 0.05, 0.05, 0.0, 0.0], size=(B, 6))
    tol, acc, mi, ai = 1e-3, 1e-2, 3, 5
    solver = ttmpc.BatchSolver(N, P, to.DEFAULT_Q, to.DEFAULT_R, to.MPC_XLB, to.MPC_XUB, to.MPC_ULB, to.MPC_UUB,
                               variant=getattr(ttmpc, f"TT_VARIANT_{variant}"), tol=tol, acc_tol=acc, max_iter=mi,
                               acc_iter=ai)
    cl = sim.ClosedLoop(solver, S, U, P, None, policy=policy)
    out = cl.run(x0, T)
    ref_S, ref_u, ref_st, pol = to.closed_loop(_oracle_solver_cfg(N, tol, acc, mi, ai), x0, S, U, N, T, P,
                                               policy=policy, fuzzy=variant == "FUZZY")
    assert np.array_equal(out["status"], ref_st)
    assert np.array_equal(out["failures"], pol["failures"])
    assert np.array_equal(out["running"], pol["running"])
    assert np.max(np.abs(out["controls"] - ref_u)) <= 1e-6
    assert np.max(np.abs(out["states"] - ref_S)) <= 1e-6
    assert out["failures"].max() > 20            # the failure branches ran
    if policy == "nmpc":
        assert not out["running"].all()          # some instance hit the 20-failure stop
