"""The C4 bench instances the kernel and the oracle disagree on, re-solved by the oracle built with FMA contraction
(make -C oracle fma: build/libttoracle_fma.so), i.e. the same restated IPOPT in another rounding (diagnostic, CPU).

    TTO_ORACLE_LIB=oracle/build/libttoracle_fma.so python tools/obca_fma_check.py 28,168,37,113,121,189
"""
import json, sys, numpy as np
from pathlib import Path
REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "car-trailer-mpc_amd")]
from oracle import c_oracle as co
from ttmpc import scenarios as sc
G = str(REPO / "tests" / "golden") + "/"
obs = sc.obstacles_array(sc.load_obstacles(G + "obstacles.json"))[:6]
cases = json.loads(open(G + "test_cases.json").read())["cases"]
x0, xg, zg = sc.obca_case_batch(cases, 256, 200, 6, seed=7, obstacles=obs, params=sc.OBCA_PARAMS)
idx = [int(a) for a in sys.argv[1].split(",")]
P = co.make_obca_problem(200, sc.OBCA_PARAMS, sc.OBCA_Q, sc.OBCA_R, sc.OBCA_XLB, sc.OBCA_XUB, sc.OBCA_ULB, sc.OBCA_UUB, obs)
z, st, it, kk = co.obca_solve_batch(P, x0[idx], xg[idx], z_guess=zg[idx], nthreads=len(idx))
X = co.obca_split(z, 200, 6)[0]
ref = np.load(G + "c4_census_bench_x.npz")["X"][idx]
for j, b in enumerate(idx):
    print(b, "status", int(st[j]), "iters", int(it[j]), "kkt %.3g" % kk[j], "max|dX| vs census %.3g" % np.abs(X[j] - ref[j]).max(), flush=True)
