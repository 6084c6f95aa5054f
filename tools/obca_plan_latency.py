"""Latency of one OBCA plan (B = 1): the reference's default call (trajectory_animation.py:43-52, 77-83, 109; N = 200,
all 11 obstacles, tests/golden/oracle_default_plan.npz's guess) and one C4 test case, with and without the helper
workgroups (with B = 1 every other CU can help), against the oracle's solve of the same problem on one CPU core.

    python tools/obca_plan_latency.py [repeats]
"""
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "car-trailer-mpc_amd")]
import numpy as np  # noqa: E402

import ttmpc  # noqa: E402
from oracle import c_oracle as co  # noqa: E402
from ttmpc import scenarios as sc  # noqa: E402

G = REPO / "tests" / "golden"
R = int(sys.argv[1]) if len(sys.argv) > 1 else 3
g = np.load(G / "oracle_default_plan.npz")
ob = np.load(G / "reference_numpy.npz")["obstacles"].reshape(-1, 4)
cases = json.loads((G / "test_cases.json").read_text())["cases"]
obs6 = sc.obstacles_array(sc.load_obstacles(G / "obstacles.json"))[:6]
x0c, xgc, zgc = sc.obca_case_batch(cases, 14, 200, 6, seed=0)
probs = {"default_plan": (ob, g["x_init"], g["x_goal"], g["z_guess"]),
         "c4_case_1": (obs6, x0c[1:2], xgc[1:2], zgc[1:2])}
bnd = (sc.OBCA_XLB, sc.OBCA_XUB, sc.OBCA_ULB, sc.OBCA_UUB)
for name, (obs, x0, xg, zg) in probs.items():
    row = {}
    for nh, label in ((0, "no_helpers"), (-1, "helpers")):
        s = ttmpc.ObcaSolver(200, sc.OBCA_PARAMS, sc.OBCA_Q, sc.OBCA_R, *bnd, obs)
        s.set_helpers(nh)
        s.solve(x0, xg, z_guess=zg)  # warm-up
        ts = []
        for _ in range(R):
            t = time.perf_counter()
            X, U, Z, st, it, kk = s.solve(x0, xg, z_guess=zg)
            ts.append(time.perf_counter() - t)
        row[label] = {"s": round(float(np.median(ts)), 4), "status": int(st[0]), "iters": int(it[0])}
    if name == "default_plan":  # (the C4 case runs ~1,000 oracle iterations: minutes on one core)
        P = co.make_obca_problem(200, sc.OBCA_PARAMS, sc.OBCA_Q, sc.OBCA_R, *bnd, obs)
        t = time.perf_counter()
        z, st, it, kk = co.obca_solve_batch(P, x0, xg, z_guess=zg, nthreads=1)
        row["oracle_1core"] = {"s": round(time.perf_counter() - t, 3), "status": int(st[0]), "iters": int(it[0])}
    print(name, json.dumps(row), flush=True)
