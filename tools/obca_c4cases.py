"""The 14 C4 test-case instances of tests/test_gpu_obca.py::test_c4_test_cases_vs_oracle, GPU against oracle, with IPOPT's
optimality error re-evaluated by the oracle at BOTH end points (the GPU's exported primal-dual iterate and the oracle's own;
tto_obca_eval_iterate).  VERDICT r4 item 1: where the two runs end at different points, or only one converges, this is
the independent evidence of what each end point is.   python tools/obca_c4cases.py [seed] [B]"""
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "car-trailer-mpc_amd"), str(REPO / "tests")]
import numpy as np  # noqa: E402

import ttmpc  # noqa: E402
from oracle import c_oracle as co  # noqa: E402
from ttmpc import collision  # noqa: E402
from ttmpc import scenarios as sc  # noqa: E402

seed = int(sys.argv[1]) if len(sys.argv) > 1 else 0
B = int(sys.argv[2]) if len(sys.argv) > 2 else 14
G = REPO / "tests" / "golden"
cases = json.loads((G / "test_cases.json").read_text())["cases"]
obs = sc.obstacles_array(sc.load_obstacles(G / "obstacles.json"))[:6]
x0, xg, zg = sc.obca_case_batch(cases, B, 200, 6, seed=seed)
bnd = (sc.OBCA_XLB, sc.OBCA_XUB, sc.OBCA_ULB, sc.OBCA_UUB)
s = ttmpc.ObcaSolver(200, sc.OBCA_PARAMS, sc.OBCA_Q, sc.OBCA_R, *bnd, obs)
X, U, Z, st, it, kk, I = s.solve(x0, xg, z_guess=zg, iterate=True)
P = co.make_obca_problem(200, sc.OBCA_PARAMS, sc.OBCA_Q, sc.OBCA_R, *bnd, obs)
zc, stc, itc, kkc, Ic = co.obca_solve_batch(P, x0, xg, z_guess=zg, nthreads=16, iterate=True)
Xc = co.obca_split(zc, 200, 6)[0]
eg = co.obca_eval_iterate(P, x0, I, x_goal=xg)
eo = co.obca_eval_iterate(P, x0, Ic, x_goal=xg)
blocked = sc.blocked_poses(x0, obs, sc.OBCA_PARAMS) | sc.blocked_poses(xg, obs, sc.OBCA_PARAMS)
d = np.abs(X - Xc).max(axis=(1, 2))
print(f"C4 test cases (seed {seed}, B {B}): GPU status {np.bincount(st, minlength=6).tolist()}, oracle "
      f"{np.bincount(stc, minlength=6).tolist()}, equal statuses {int((st == stc).sum())}/{B}")
print(" #  blk | GPU st  iters  E0(oracle eval)   dinf     compl     s_d    conv | ORC st  iters  E0        dinf"
      "      s_d     | max|dX|   cost GPU      cost oracle")
for b in range(B):
    def cost(Xb, Ub):
        dd = Xb - xg[b]
        return float((dd[:-1] ** 2).sum() + 100.0 * (dd[-1] ** 2).sum() + 10.0 * (Ub ** 2).sum())
    cg = cost(X[b], U[b]) if st[b] <= 1 else float("nan")
    Uc = co.obca_split(zc, 200, 6)[1]
    cc = cost(Xc[b], Uc[b]) if stc[b] <= 1 else float("nan")
    print(f"{b:2d}  {int(blocked[b])}   |   {st[b]}  {it[b]:5d}  {eg['E0'][b]:9.2e}  {eg['dinf'][b]:9.2e} {eg['compl'][b]:9.2e} "
          f"{eg['sd'][b]:8.2e}  {int(eg['converged'][b])}   |   {stc[b]}  {itc[b]:5d}  {eo['E0'][b]:9.2e} {eo['dinf'][b]:9.2e} "
          f"{eo['sd'][b]:8.2e} | {d[b]:9.2e}  {cg:12.3f}  {cc:12.3f}")
gap = collision.sat_gap(X[st <= 1], sc.OBCA_PARAMS, obs).min(axis=(-1, -2, -3)) if (st <= 1).any() else np.array([])
print("GPU-optimal end points passing IPOPT's convergence test at the oracle's evaluation:",
      int(eg["converged"][st == 0].sum()), "/", int((st == 0).sum()), "; min SAT gap of GPU plans", gap.min() if gap.size else None)
