"""GPU suite: the HIP path (through the C ABI) against the oracle and the golden optima.

Tolerances (FP64 throughout):
  * vs golden optima (scipy trust-constr/SLSQP agreement): |dz| <= 1e-6 * max(1, |z|)
  * vs the C oracle on identical inputs (same NLP, same IPM constants, different linear algebra):
    |dz| <= 1e-7 * max(1, |z|), identical status
  * full-size property checks: every instance converged, reported optimality error <= tol,
    dynamics residual <= 1e-9, bounds hold to IPOPT's relaxation, bitwise-deterministic reruns.
"""
import numpy as np
import pytest

from conftest import fixture_instance

pytestmark = pytest.mark.gpu

P = {"M": 0.15, "L1": 7.05, "L2": 12.45, "W1": 3.05, "W2": 2.95, "dt": 0.05}


def _gpu_solver(N, **kw):
    import ttmpc
    from oracle import ttmpc_oracle as to
    return ttmpc.BatchSolver(N, P, to.DEFAULT_Q, to.DEFAULT_R, to.MPC_XLB, to.MPC_XUB, to.MPC_ULB, to.MPC_UUB, **kw)


def _oracle(N, x0, xr, ur, wq=None, wr=None, zg=None):
    from oracle import c_oracle as co
    from oracle import ttmpc_oracle as to
    nlp = to.TrackingNLP(N)
    Pp = co.make_problem(N, P, nlp.Q, nlp.R, nlp.xlb, nlp.xub, nlp.ulb, nlp.uub)
    return co.solve_batch(Pp, x0, xr, ur, wq=wq, wr=wr, z_guess=zg)


def _z(X, U):
    from ttmpc import layout
    return layout.pack(X, U)


def test_golden_optima(golden_opt):
    for i in range(len(golden_opt["tag"])):
        tag, N, x0, xr, ur, wq, wr, z = fixture_instance(golden_opt, i)
        s = _gpu_solver(N)
        w = np.concatenate([wq, wr])[None]
        X, U, st, it, kk = s.solve(x0[None], xr[None], ur[None], wq_wr=w)
        assert st[0] == 0, (tag, st, kk)
        zg = _z(X, U)[0]
        assert np.max(np.abs(zg - z) / np.maximum(1.0, np.abs(z))) <= 1e-6, tag


@pytest.mark.parametrize("N,psi,B", [(20, 0.3, 256), (30, 0.5, 256), (40, 0.9, 256), (50, 0.5, 128), (1, 0.3, 64),
                                     (63, 0.3, 64), (64, 0.3, 64), (70, 0.5, 32)])
def test_matches_c_oracle(N, psi, B):
    from ttmpc.scenarios import synthetic_batch
    x0, xr, ur = synthetic_batch(B, N, seed=1000 + N, psi_range=psi)
    X, U, st, it, kk = _gpu_solver(N).solve(x0, xr, ur)
    zc, stc, itc, kkc = _oracle(N, x0, xr, ur)
    assert np.array_equal(st, stc)
    assert np.all(st == 0)
    zg = _z(X, U)
    assert np.max(np.abs(zg - zc) / np.maximum(1.0, np.abs(zc))) <= 1e-7


def test_kkt_of_gpu_solutions_independent_checker():
    from oracle import ttmpc_oracle as to
    from ttmpc.scenarios import synthetic_batch
    N = 40
    x0, xr, ur = synthetic_batch(32, N, seed=77, psi_range=0.9)
    X, U, st, it, kk = _gpu_solver(N).solve(x0, xr, ur)
    nlp = to.TrackingNLP(N)
    zg = _z(X, U)
    for b in range(0, 32, 4):
        k = nlp.kkt_residual(zg[b], x0[b], xr[b].T, ur[b].T)
        assert k["prim"] <= 1e-9 and k["stat"] <= 1e-6 and k["bviol"] <= 1e-7


def test_c1_initialize_json_case(golden_ref, golden_opt):
    """C1: x0 from initialize.json, reference = first window of do_interpolation(state_traj)."""
    i = list(golden_opt["tag"]).index("c1")
    tag, N, x0, xr, ur, wq, wr, z = fixture_instance(golden_opt, i)
    assert np.allclose(xr.T, golden_ref["interp_states"][:, :21])
    X, U, st, it, kk = _gpu_solver(N).solve(x0[None], xr[None], ur[None])
    assert st[0] == 0
    assert np.max(np.abs(_z(X, U)[0] - z) / np.maximum(1, np.abs(z))) <= 1e-6


def test_fuzzy_weights_and_warm_shift():
    from oracle import ttmpc_oracle as to
    from ttmpc import layout
    from ttmpc.scenarios import synthetic_batch
    N = 30
    x0, xr, ur = synthetic_batch(64, N, seed=5, psi_range=0.6)
    w = np.empty((64, 8))
    for b in range(64):
        q, r = to.fuzzy_weights(x0[b], xr[b].T)
        w[b, :6], w[b, 6:] = q, r
    X, U, st, _, _ = _gpu_solver(N).solve(x0, xr, ur, wq_wr=w)
    zc, stc, _, _ = _oracle(N, x0, xr, ur, wq=w[:, :6], wr=w[:, 6:])
    assert np.all(st == 0) and np.array_equal(st, stc)
    assert np.max(np.abs(_z(X, U) - zc) / np.maximum(1, np.abs(zc))) <= 1e-7
    # NMPC warm start: bug-compatible shift of the previous optimum (mpc_control_nmpc.py:69-88)
    zg = layout.shift(zc, N)
    X2, U2, st2, _, _ = _gpu_solver(N).solve(x0, xr, ur, wq_wr=w, z_guess=zg)
    zc2, stc2, _, _ = _oracle(N, x0, xr, ur, wq=w[:, :6], wr=w[:, 6:], zg=zg)
    assert np.array_equal(st2, stc2)
    ok = st2 == 0
    assert ok.mean() > 0.9
    # converged from a different guess -> the same local optimum as the cold start
    assert np.max(np.abs(_z(X2, U2)[ok] - zc[ok]) / np.maximum(1, np.abs(zc[ok]))) <= 1e-6


def test_relaxed_tolerance_variant_status_and_accuracy():
    import ttmpc
    from ttmpc.scenarios import synthetic_batch
    N = 30
    x0, xr, ur = synthetic_batch(128, N, seed=6)
    Xt, Ut, _, _, _ = _gpu_solver(N).solve(x0, xr, ur)
    X, U, st, it, kk = _gpu_solver(N, variant=ttmpc.TT_VARIANT_NMPC, tol=1e-3, acc_tol=1e-2, max_iter=2000,
                                   acc_iter=5).solve(x0, xr, ur)
    assert np.all(st <= 1) and np.all(kk <= 1e-2)
    assert np.max(np.abs(X - Xt)) <= 1e-2  # tol 1e-3 solutions: comparable to ~1e-2 only


def test_infeasible_and_edge_batches():
    from ttmpc.scenarios import synthetic_batch
    N = 12
    x0, xr, ur = synthetic_batch(5, N, seed=8)
    x0[1, 3] = 1.3            # hitch angle beyond pi/3
    x0[3, 2] = 4.0            # heading beyond pi
    s = _gpu_solver(N)
    X, U, st, _, _ = s.solve(x0, xr, ur)
    assert list(st) == [0, 3, 0, 3, 0]
    Xb, Ub, stb, _, _ = s.solve(x0[:1], xr[:1], ur[:1])  # B = 1
    assert stb[0] == 0 and np.array_equal(Xb[0], X[0])
    # B = 0 is a no-op
    import ctypes
    assert s._L.tt_solve_batch(s._h, 0, None, None, None, None, None, None, None, None, None, None) == 0


def test_rejects_bad_arguments():
    import ttmpc
    with pytest.raises(ttmpc.TTError):
        _gpu_solver(0)
    with pytest.raises(ttmpc.TTError):
        _gpu_solver(10_000)  # does not fit in LDS
    from oracle import ttmpc_oracle as to
    with pytest.raises(ttmpc.TTError):
        ttmpc.BatchSolver(10, P, to.DEFAULT_Q, to.DEFAULT_R, to.MPC_XUB, to.MPC_XLB, to.MPC_ULB, to.MPC_UUB)


@pytest.mark.parametrize("N,B,psi", [(20, 1024, 0.3), (40, 8192, 0.9), (30, 8192, 0.5), (50, 1024, 0.5)])
def test_full_size_properties(N, B, psi):
    """BASELINE configs C2 / C3 at full size, and the stage-unrolled builds of the drivers' other horizons (N = 30
    two-wave, N = 50): size-independent properties, and a random subsample against the oracle."""
    from oracle import ttmpc_oracle as to
    from ttmpc.scenarios import synthetic_batch
    x0, xr, ur = synthetic_batch(B, N, seed=2024 + N, psi_range=psi)
    s = _gpu_solver(N)
    X, U, st, it, kk = s.solve(x0, xr, ur)
    assert np.all(st == 0) and np.all(kk <= 1e-8)
    res = X[:, 1:] - to.step(X[:, :-1], U, P)
    assert np.max(np.abs(res)) <= 1e-9
    assert np.max(np.abs(X[:, 0] - x0)) <= 1e-9
    lb = np.array([-np.inf, -np.inf, -np.pi, -np.pi / 3, -np.pi / 4, -10]) - 1e-7
    assert np.all(X >= lb) and np.all(X <= -lb)
    assert np.all(np.abs(U[..., 0]) <= 5 + 1e-7) and np.all(np.abs(U[..., 1]) <= np.pi / 2 + 1e-7)
    X2, U2, st2, it2, kk2 = s.solve(x0, xr, ur)
    assert np.array_equal(X, X2) and np.array_equal(U, U2) and np.array_equal(it, it2)
    # a random subsample against the oracle
    idx = np.random.default_rng(0).choice(B, 24, replace=False)
    zc, stc, _, _ = _oracle(N, x0[idx], xr[idx], ur[idx])
    assert np.max(np.abs(_z(X[idx], U[idx]) - zc) / np.maximum(1, np.abs(zc))) <= 1e-7


def test_device_pointer_entry_point_with_torch():
    import torch
    from ttmpc.scenarios import synthetic_batch
    N, B = 20, 300
    x0, xr, ur = synthetic_batch(B, N, seed=31)
    s = _gpu_solver(N)
    Xh, Uh, sth, _, _ = s.solve(x0, xr, ur)
    dev = torch.device("cuda", s.device)
    tx0, txr, tur = (torch.from_numpy(a).to(dev) for a in (x0, xr, ur))
    X = torch.empty((B, N + 1, 6), dtype=torch.float64, device=dev)
    U = torch.empty((B, N, 2), dtype=torch.float64, device=dev)
    st = torch.empty(B, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    s.solve_device(B, tx0.data_ptr(), txr.data_ptr(), tur.data_ptr(), X.data_ptr(), U.data_ptr(), st.data_ptr(),
                   stream=stream.cuda_stream)
    torch.cuda.synchronize(dev)
    assert np.array_equal(X.cpu().numpy(), Xh) and np.array_equal(U.cpu().numpy(), Uh)
    assert np.array_equal(st.cpu().numpy(), sth)


def test_small_host_batches_zero_copy_match_the_device_path():
    """Host calls with B <= 64 at N < 64 run zero-copy (the kernel reads and writes the coherent pinned staging block,
    tt_api.hip zero_copy_max); B = 65 and N = 64 go through the staged copies.  Every size must give bitwise the
    device-buffer results, and back-to-back calls on one handle must each see their own inputs (no stale pages)."""
    import torch
    from ttmpc.scenarios import synthetic_batch
    for N in (20, 64):
        x0, xr, ur = synthetic_batch(70, N, seed=47)
        s = _gpu_solver(N)
        dev = torch.device("cuda", s.device)
        tx0, txr, tur = (torch.from_numpy(a).to(dev) for a in (x0, xr, ur))
        X = torch.empty((70, N + 1, 6), dtype=torch.float64, device=dev)
        U = torch.empty((70, N, 2), dtype=torch.float64, device=dev)
        st = torch.empty(70, dtype=torch.int32, device=dev)
        s.solve_device(70, tx0.data_ptr(), txr.data_ptr(), tur.data_ptr(), X.data_ptr(), U.data_ptr(), st.data_ptr(),
                       stream=torch.cuda.current_stream(dev).cuda_stream)
        torch.cuda.synchronize(dev)
        Xd, Ud, std = X.cpu().numpy(), U.cpu().numpy(), st.cpu().numpy()
        for lo, B in ((0, 1), (1, 1), (0, 1), (3, 5), (0, 64), (2, 64), (0, 65), (5, 1)):
            Xh, Uh, sth, _, _ = s.solve(x0[lo:lo + B], xr[lo:lo + B], ur[lo:lo + B])
            assert np.array_equal(Xh, Xd[lo:lo + B]) and np.array_equal(Uh, Ud[lo:lo + B]), (N, lo, B)
            assert np.array_equal(sth, std[lo:lo + B]), (N, lo, B)
    # the optional inputs travel in the same staging block: a warm-start guess (B = 1 and 64) and fuzzy weights
    import ttmpc
    from ttmpc import layout
    N = 20
    x0, xr, ur = synthetic_batch(64, N, seed=48)
    zg = layout.pack(xr + 0.01, ur)
    wq = 1.0 + 0.5 * np.random.default_rng(3).random((64, 8))
    for variant, kw in ((ttmpc.TT_VARIANT_TRACK, {"z_guess": zg}), (ttmpc.TT_VARIANT_FUZZY, {"wq_wr": wq})):
        s = _gpu_solver(N, variant=variant)
        dev = torch.device("cuda", s.device)
        td = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev)
              for k, v in (("x0", x0), ("xr", xr), ("ur", ur), ("zg", zg), ("wq", wq))}
        X = torch.empty((64, N + 1, 6), dtype=torch.float64, device=dev)
        U = torch.empty((64, N, 2), dtype=torch.float64, device=dev)
        st = torch.empty(64, dtype=torch.int32, device=dev)
        s.solve_device(64, td["x0"].data_ptr(), td["xr"].data_ptr(), td["ur"].data_ptr(), X.data_ptr(), U.data_ptr(),
                       st.data_ptr(), wq_wr=td["wq"].data_ptr() if "wq_wr" in kw else 0,
                       z_guess=td["zg"].data_ptr() if "z_guess" in kw else 0,
                       stream=torch.cuda.current_stream(dev).cuda_stream)
        torch.cuda.synchronize(dev)
        Xd, Ud = X.cpu().numpy(), U.cpu().numpy()
        for lo, B in ((0, 1), (7, 1), (0, 64)):
            sub = {k: v[lo:lo + B] for k, v in kw.items()}
            Xh, Uh, _, _, _ = s.solve(x0[lo:lo + B], xr[lo:lo + B], ur[lo:lo + B], **sub)
            assert np.array_equal(Xh, Xd[lo:lo + B]) and np.array_equal(Uh, Ud[lo:lo + B]), (variant, lo, B)


def test_reference_call_surface():
    """MPCTrackingControl / TruckTrailerNMPC / MPCTrackingControlFuzzy as the reference drivers use them."""
    import ttmpc
    from oracle import ttmpc_oracle as to
    params = dict(P, horizon=20)
    model = ttmpc.TruckTrailerModel(params)
    sb = {"lb": to.MPC_XLB, "ub": to.MPC_XUB}
    ib = {"lb": to.MPC_ULB, "ub": to.MPC_UUB}
    S = np.loadtxt if False else None  # noqa: F841
    from ttmpc.scenarios import synthetic_batch
    x0, xr, ur = synthetic_batch(1, 20, seed=3)
    Xr, Ur = xr[0].T, ur[0].T
    c = ttmpc.MPCTrackingControl(model, params, to.DEFAULT_Q, to.DEFAULT_R, sb, ib)
    states, inputs = c.solve(x0[0], Xr, Ur)
    assert states.shape == (6, 21) and inputs.shape == (2, 20)
    zc, _, _, _ = _oracle(20, x0, xr, ur)
    Xo, Uo = to.TrackingNLP(20).split(zc[0])
    assert np.allclose(states, Xo, atol=1e-7) and np.allclose(inputs, Uo, atol=1e-7)
    n = ttmpc.TruckTrailerNMPC(model, params, to.DEFAULT_Q, to.DEFAULT_R, sb, ib)
    s1, i1 = n.solve(x0[0], Xr, Ur)
    s2, i2 = n.solve(s1[:, 1], Xr, Ur)  # second call uses the (bug-compatible) shift warm start
    assert s1 is not None and s2 is not None
    bad = x0[0].copy()
    bad[3] = 1.4
    assert n.solve(bad, Xr, Ur) == (None, None)
    f = ttmpc.MPCTrackingControlFuzzy(model, params, to.DEFAULT_Q, to.DEFAULT_R, sb, ib)
    sf, uf = f.solve(x0[0], Xr, Ur)
    assert sf.shape == (6, 21)
    assert f.solve(bad, Xr, Ur) == (None, None)


def test_max_horizon_matches_oracle():
    """The largest horizon whose instance fits one CU's LDS (tt_max_horizon: 118-double stage records)."""
    import ttmpc
    from ttmpc.scenarios import synthetic_batch
    N = ttmpc.lib().tt_max_horizon()
    assert N >= 170
    x0, xr, ur = synthetic_batch(32, N, seed=77)
    X, U, st, it, kk = _gpu_solver(N).solve(x0, xr, ur)
    zc, stc, itc, kkc = _oracle(N, x0, xr, ur)
    assert np.array_equal(st, stc) and np.all(st <= 1)
    assert np.max(np.abs(_z(X, U) - zc) / np.maximum(1.0, np.abs(zc))) <= 1e-7


def test_non_finite_reference_is_reported_not_propagated():
    """A NaN in one instance's reference ends that instance with TT_NONFINITE; its neighbours are untouched."""
    import ttmpc
    from ttmpc.scenarios import synthetic_batch
    N = 20
    x0, xr, ur = synthetic_batch(6, N, seed=21)
    X0, U0, st0, _, _ = _gpu_solver(N).solve(x0, xr, ur)
    xr[2, 7, 1] = np.nan
    ur[4, 3, 0] = np.inf
    X, U, st, it, kk = _gpu_solver(N).solve(x0, xr, ur)
    assert st[2] == ttmpc.TT_NONFINITE and st[4] == ttmpc.TT_NONFINITE
    ok = [0, 1, 3, 5]
    assert np.array_equal(st[ok], st0[ok]) and np.array_equal(X[ok], X0[ok]) and np.array_equal(U[ok], U0[ok])


def test_non_diagonal_weights_match_oracle():
    """Dense (non-diagonal) Q and R take the general weight path of the kernel (the reference's diagonal
    Q = I, R = 10 I take the specialised one); both must agree with the oracle."""
    import ttmpc
    from oracle import c_oracle as co
    from oracle import ttmpc_oracle as to
    from ttmpc.scenarios import synthetic_batch
    N = 20
    rng = np.random.default_rng(5)
    A = rng.normal(size=(6, 6))
    Q = np.eye(6) + 0.1 * (A @ A.T)
    R = np.array([[10.0, 1.5], [1.5, 8.0]])
    x0, xr, ur = synthetic_batch(64, N, seed=55)
    s = ttmpc.BatchSolver(N, P, Q, R, to.MPC_XLB, to.MPC_XUB, to.MPC_ULB, to.MPC_UUB)
    X, U, st, it, kk = s.solve(x0, xr, ur)
    nlp = to.TrackingNLP(N)
    Pp = co.make_problem(N, P, Q, R, nlp.xlb, nlp.xub, nlp.ulb, nlp.uub)
    zc, stc, itc, kkc = co.solve_batch(Pp, x0, xr, ur)
    assert np.array_equal(st, stc) and np.all(st <= 1)
    assert np.max(np.abs(_z(X, U) - zc) / np.maximum(1.0, np.abs(zc))) <= 1e-7


def test_c5_full_batch_through_the_sharded_path():
    """BASELINE config C5 at full size (one global batch of 65,536 test_cases.json scenarios) through
    ttmpc.sharded on one rank (scatter/gather degenerate to device copies): every instance converges,
    x_0 = x_init, the dynamics hold, results come back in instance order and reruns are bitwise equal."""
    import torch

    import bench
    import ttmpc
    from oracle import ttmpc_oracle as to
    from ttmpc.sharded import ShardedBatch, gpu_shard_solver
    B, N = 65536, 20
    x0, xr, ur = bench.workload("c5", B, N, seed=3)
    dev = torch.device("cuda", 0)
    solver = ttmpc.BatchSolver(N, P, to.DEFAULT_Q, to.DEFAULT_R, to.MPC_XLB, to.MPC_XUB, to.MPC_ULB, to.MPC_UUB)
    sb = ShardedBatch(B, N, gpu_shard_solver(solver), device=dev)
    sb.pack_inputs(x0, xr, ur)
    stats = ShardedBatch.stats(*sb.step())
    X, U, st, it, kk = sb.results()
    assert stats["instances"] == B and stats["converged"] == B and np.all(st <= 1)
    assert np.max(np.abs(X[:, 0] - x0)) <= 1e-9
    for b in np.arange(0, B, 997):   # dynamics residual on a spread sample (forward Euler, float64)
        res = X[b, 1:] - np.array([to.step(X[b, k], U[b, k], P) for k in range(N)])
        assert np.max(np.abs(res)) <= 1e-9
    sb.step()
    X2, U2, st2, _, _ = sb.results()
    assert np.array_equal(X, X2) and np.array_equal(U, U2) and np.array_equal(st, st2)


@pytest.mark.parametrize("N", [20, 30])
def test_occupancy_build_is_bitwise_the_latency_build(N):
    """Large batches (B > 2048, reference box, diagonal weights, N = 20 or the NMPC driver's N = 30) launch the
    two-waves-per-SIMD build of the stage-unrolled kernel, small ones its one-wave build: the same code under a
    different register budget, so every instance's result is bitwise independent of the batch size (and of the sharded
    path's chunk size).  Two seeds, 4608 instances each, against 1152-instance batches."""
    from ttmpc.scenarios import synthetic_batch
    B = 4608
    s = _gpu_solver(N)
    for seed in (77, 78):
        x0, xr, ur = synthetic_batch(B, N, seed=seed, psi_range=0.6)
        big = s.solve(x0, xr, ur)
        for lo in range(0, B, 1152):
            small = s.solve(x0[lo:lo + 1152], xr[lo:lo + 1152], ur[lo:lo + 1152])
            for a, b in zip(big, small):
                assert np.array_equal(a[lo:lo + 1152], b), seed
    # the NMPC driver's warm-started relaxed-tolerance solves (its own load path: a guess instead of the reference copy)
    import ttmpc
    from ttmpc import layout
    sn = _gpu_solver(N, variant=ttmpc.TT_VARIANT_NMPC, tol=1e-3, acc_tol=1e-2, max_iter=2000, acc_iter=5)
    x0, xr, ur = synthetic_batch(B, N, seed=79, psi_range=0.6)
    zg = layout.shift(layout.pack(xr, ur), N)
    big = sn.solve(x0, xr, ur, z_guess=zg)
    for lo in range(0, B, 1152):
        small = sn.solve(x0[lo:lo + 1152], xr[lo:lo + 1152], ur[lo:lo + 1152], z_guess=zg[lo:lo + 1152])
        for a, b in zip(big, small):
            assert np.array_equal(a[lo:lo + 1152], b), "nmpc"


def test_occupancy_build_boundary_n31_n32():
    """launch_track's occupancy switch: B = 4097 at N = 31 still fits 5 waves' LDS per CU (two-waves build),
    at N = 32 it does not (one-wave build).  Both must equal the same instances solved in small batches
    (one-wave build)."""
    from ttmpc.scenarios import synthetic_batch
    B = 4097
    for N in (31, 32):
        x0, xr, ur = synthetic_batch(B, N, seed=5 + N)
        s = _gpu_solver(N)
        big = s.solve(x0, xr, ur)
        for lo in (0, 2048, 4096):
            hi = min(B, lo + 1024)
            small = s.solve(x0[lo:hi], xr[lo:hi], ur[lo:hi])
            for a, b in zip(big, small):
                assert np.array_equal(a[lo:hi], b), N


def test_n50_hbm_band_build_is_bitwise_the_lds_build():
    """N = 50 (simulation.py's horizon): above three instances per CU the launch takes the build that keeps the Riccati
    factor band of the stage record in HBM (four instances per CU), below it the all-LDS build.  Same arithmetic: the
    instances of a 1,024 batch equal the same instances solved 256 at a time, and the HBM workspace survives a batch
    that grows from one call to the next."""
    from ttmpc.scenarios import synthetic_batch
    N = 50
    s = _gpu_solver(N)
    x0, xr, ur = synthetic_batch(1024, N, seed=91, psi_range=0.5)
    small = [s.solve(x0[lo:lo + 256], xr[lo:lo + 256], ur[lo:lo + 256]) for lo in range(0, 1024, 256)]
    big = s.solve(x0[:800], xr[:800], ur[:800])       # first HBM-band launch: the workspace is allocated
    bigger = s.solve(x0, xr, ur)                      # a larger batch: the workspace grows
    for lo, sm in zip(range(0, 1024, 256), small):
        for a, b in zip(bigger, sm):
            assert np.array_equal(a[lo:lo + 256], b), lo
    for a, b in zip(big, bigger):
        assert np.array_equal(a, b[:800])
