"""CPU checks of the committed C4 census fixtures and of the measurement sources bench.py quotes (no GPU).

tests/golden/c4_census.json is the oracle's census of the two full-size C4 batches (tests/golden/make_c4_census.py):
its objectives must be the plan-mode objective of the NLP as oracle/obca_nlp.py states it, its sensitivity masks must
follow from its own perturbed runs, and the end points committed beside it must be the ones the statuses describe.
bench.py's roofline.traffic for every config must come from committed rocprofv3 passes that exist.
"""
import json
import sys

import numpy as np

from conftest import GOLDEN, REPO

sys.path.insert(0, str(GOLDEN))


def _census():
    return json.loads((GOLDEN / "c4_census.json").read_text())


def test_census_objective_is_the_nlp_objective():
    """plan_objective (make_c4_census.py) against ObcaNLP.cost (oracle/obca_nlp.py: trajectory_optimization.py:170-190)
    on random primal points."""
    from make_c4_census import plan_objective
    from oracle.obca_nlp import ObcaNLP
    from ttmpc import scenarios as sc
    N, M = 200, 6
    obs = sc.obstacles_array(sc.load_obstacles(GOLDEN / "obstacles.json"))[:M]
    nlp = ObcaNLP(N, M, sc.OBCA_PARAMS, sc.OBCA_Q, sc.OBCA_R, sc.OBCA_XLB, sc.OBCA_XUB, sc.OBCA_ULB, sc.OBCA_UUB, obs)
    rng = np.random.default_rng(3)
    n = N * (8 + 16 * M) + 6 + 16 * M
    for _ in range(3):
        z = rng.normal(size=n)
        xg = rng.normal(size=6)
        X, U, _, _ = nlp.split(z)
        J = plan_objective(X[None], U[None], xg[None])[0]
        assert abs(J - nlp.cost(z, xg)) <= 1e-10 * abs(J)


def test_census_sensitivity_masks_follow_from_the_perturbed_runs():
    for name in ("test", "bench"):
        cen = _census()[name]
        st = np.asarray(cen["status"])
        assert len(cen["perturbed"]) == 3
        sens = np.zeros(st.size, dtype=bool)
        for p in cen["perturbed"]:
            sens |= (np.asarray(p["status"]) != st) | ((st <= 1) & (np.asarray(p["dx_max"]) > 1e-6))
        assert np.array_equal(sens, np.asarray(cen["rounding_sensitive"], dtype=bool)), name
    assert int(np.sum(_census()["bench"]["rounding_sensitive"])) == 77
    assert int(np.sum(_census()["test"]["rounding_sensitive"])) == 43


def test_census_end_points_match_the_statuses():
    for name in ("test", "bench"):
        cen = _census()[name]
        z = np.load(GOLDEN / f"c4_census_{name}_x.npz")
        assert np.array_equal(z["status"], np.asarray(cen["status"]))
        X = z["X"]
        assert X.shape == (256, 201, 6) and np.all(np.isfinite(X[np.asarray(cen["status"]) <= 1]))
        if "objective" in z.files:
            assert np.array_equal(z["objective"], np.asarray(cen["objective"]))


def test_bench_traffic_sources_are_committed_full_launch_passes():
    """Every roofline.traffic bench.py quotes is a committed pass; the OBCA ones are full launches whose instance-
    iterations match the configs' deterministic launches (traffic_estimated false)."""
    sys.path.insert(0, str(REPO))
    import bench
    for cfg, d in bench.TRACK_PMC.items():
        for pas in ("fetch", "write"):
            assert (REPO / d / pas / f"{pas}_counter_collection.csv").exists(), (cfg, d)
        assert bench.read_traffic([REPO / d / "fetch" / "fetch_counter_collection.csv",
                                   REPO / d / "write" / "write_counter_collection.csv"]) > 0
    for cfg, d in bench.OBCA_PMC.items():
        rec = json.loads((REPO / d / "fetch.bench.json").read_text())["solver"]
        iters = rec["iters_mean"] * rec["instances"]
        traffic, src, est = bench.obca_traffic(cfg, iters)
        assert traffic > 0 and est is False and "full obca_kernel launch" in src, (cfg, src)
        # a launch with other iterations is scaled, and flagged as an estimate
        assert bench.obca_traffic(cfg, 2 * iters)[2] is True
