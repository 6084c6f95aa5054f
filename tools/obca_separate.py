"""Where one C4 instance's GPU and oracle runs separate (development tool).

    python tools/obca_separate.py oracle SEED IDX OUT.npz K1,K2,...     # CPU: the oracle stopped at each max_iter K
    python tools/obca_separate.py gpu SEED IDX OUT.npz K1,K2,...        # GPU box: the kernel, the same K
    python tools/obca_separate.py compare ORACLE.npz GPU.npz

Instance IDX of the bench's C4 batch (bench.py --config c4: collision-free cases, SEED 7 on rank 0) is solved alone at
max_iter K for every K (an instance's iterates do not depend on the rest of its batch: no shared state, and the helper
workgroups are bitwise neutral), with the final primal-dual iterate exported; `compare` prints, per K, the status,
iterations, E0, the barrier parameter mu and max |dX| / max |d(mu, lam)| between the two runs, so the first K where they
part is the iteration whose decision (filter, inertia, barrier update, restoration) fell the other way.
"""
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "car-trailer-mpc_amd")]
import numpy as np  # noqa: E402

N, M = 200, 6


def batch(seed, idx):
    from ttmpc import scenarios as sc
    G = REPO / "tests" / "golden"
    obs = sc.obstacles_array(sc.load_obstacles(G / "obstacles.json"))[:M]
    cases = json.loads((G / "test_cases.json").read_text())["cases"]
    x0, xg, zg = sc.obca_case_batch(cases, 256, N, M, seed=seed, obstacles=obs, params=sc.OBCA_PARAMS)
    return obs, x0[idx:idx + 1], xg[idx:idx + 1], zg[idx:idx + 1]


def run(side, seed, idx, out, Ks):
    from ttmpc import scenarios as sc
    obs, x0, xg, zg = batch(seed, idx)
    res = {"K": np.array(Ks)}
    rows = {k: [] for k in ("X", "st", "it", "kk", "I")}
    for K in Ks:
        if side == "oracle":
            from oracle import c_oracle as co
            P = co.make_obca_problem(N, sc.OBCA_PARAMS, sc.OBCA_Q, sc.OBCA_R, sc.OBCA_XLB, sc.OBCA_XUB, sc.OBCA_ULB,
                                     sc.OBCA_UUB, obs, max_iter=K)
            z, st, it, kk, I = co.obca_solve_batch(P, x0, xg, z_guess=zg, nthreads=1, iterate=True)
            X = co.obca_split(z, N, M)[0]
        else:
            import ttmpc
            s = ttmpc.ObcaSolver(N, sc.OBCA_PARAMS, sc.OBCA_Q, sc.OBCA_R, sc.OBCA_XLB, sc.OBCA_XUB, sc.OBCA_ULB,
                                 sc.OBCA_UUB, obs, max_iter=K)
            X, U, Z, st, it, kk, I = s.solve(x0, xg, z_guess=zg, iterate=True)
        for k, v in zip(("X", "st", "it", "kk", "I"), (X[0], st[0], it[0], kk[0], I[0])):
            rows[k].append(v)
        print(side, K, int(st[0]), int(it[0]), float(kk[0]), flush=True)
    res.update({k: np.asarray(v) for k, v in rows.items()})
    np.savez_compressed(out, **res)


def compare(a, b):
    A, B = np.load(a), np.load(b)
    print(f"{'K':>6s} {'st o/g':>7s} {'it o/g':>11s} {'E0 oracle':>10s} {'E0 gpu':>10s} {'max|dX|':>9s} {'max|dI|':>9s}")
    for j, K in enumerate(A["K"]):
        dX = np.abs(A["X"][j] - B["X"][j]).max()
        dI = np.abs(A["I"][j] - B["I"][j]).max()
        print(f"{int(K):6d} {int(A['st'][j])}/{int(B['st'][j]):<5d} {int(A['it'][j]):5d}/{int(B['it'][j]):<5d} "
              f"{A['kk'][j]:10.3e} {B['kk'][j]:10.3e} {dX:9.2e} {dI:9.2e}")


if __name__ == "__main__":
    if sys.argv[1] == "compare":
        compare(sys.argv[2], sys.argv[3])
    else:
        run(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], [int(k) for a in sys.argv[5:] for k in a.split(",")])
