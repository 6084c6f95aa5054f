"""Oracle refinement corrections per iteration on given instances of the bench's C4 batch (seed 7), one core each:
    python tools/obca_corrections_census.py 13,28,37 4000 > corr4000.log   (and again with 5000)
The TTO_CENSUS line of each solve (stderr) carries the refined step solves and corrections; differencing the max_iter 4000
and 5000 runs gives iterations 4,000-5,000 (profiles/r05/corrections/)."""
import os, sys, json
from pathlib import Path
os.environ["TTO_CENSUS"] = "1"
REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "car-trailer-mpc_amd")]
import numpy as np
from oracle import c_oracle as co
from ttmpc import scenarios as sc
G = str(REPO / "tests" / "golden") + "/"
obs = sc.obstacles_array(sc.load_obstacles(G + "obstacles.json"))[:6]
cases = json.loads(open(G + "test_cases.json").read())["cases"]
x0, xg, zg = sc.obca_case_batch(cases, 256, 200, 6, seed=7, obstacles=obs, params=sc.OBCA_PARAMS)
idx = [int(a) for a in sys.argv[1].split(",")]
K = int(sys.argv[2])
P = co.make_obca_problem(200, sc.OBCA_PARAMS, sc.OBCA_Q, sc.OBCA_R, sc.OBCA_XLB, sc.OBCA_XUB, sc.OBCA_ULB, sc.OBCA_UUB,
                         obs, max_iter=K)
for b in idx:
    z, st, it, kk = co.obca_solve_batch(P, x0[b:b+1], xg[b:b+1], z_guess=zg[b:b+1], nthreads=1)
    print("INST", b, "K", K, "status", int(st[0]), "iters", int(it[0]), flush=True)
