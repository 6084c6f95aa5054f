"""The C4 full batch of tests/test_gpu_obca.py (seed 1, B = 256) on the GPU, compared instance by instance with the oracle
census (tests/golden/c4_census.json, make_c4_census.py): the table VERDICT r4 item 2 asks for -- shared failures (the
restated IPOPT's behaviour), kernel-only and oracle-only failures, and which disagreements fall on rounding-sensitive
instances.   python tools/obca_census_compare.py"""
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "car-trailer-mpc_amd"), str(REPO / "tests")]
import numpy as np  # noqa: E402

import ttmpc  # noqa: E402
from ttmpc import scenarios as sc  # noqa: E402
from test_gpu_obca import c4_census_compare  # noqa: E402

G = REPO / "tests" / "golden"
cases = json.loads((G / "test_cases.json").read_text())["cases"]
obs = sc.obstacles_array(sc.load_obstacles(G / "obstacles.json"))[:6]
x0, xg, zg = sc.obca_case_batch(cases, 256, 200, 6, seed=1)
s = ttmpc.ObcaSolver(200, sc.OBCA_PARAMS, sc.OBCA_Q, sc.OBCA_R, sc.OBCA_XLB, sc.OBCA_XUB, sc.OBCA_ULB, sc.OBCA_UUB, obs)
X, U, Z, st, it, kk = s.solve(x0, xg, z_guess=zg)
cen = json.loads((G / "c4_census.json").read_text())["test"]
Xc = np.load(G / "c4_census_test_x.npz")["X"]
stc = np.asarray(cen["status"])
blocked = np.asarray(cen["blocked"], dtype=bool)
sens = np.asarray(cen["rounding_sensitive"], dtype=bool)
tab = c4_census_compare(st, X, cen, Xc)
print("C4 full batch (seed 1, B 256): GPU status counts", np.bincount(st, minlength=6).tolist(), " oracle",
      np.bincount(stc, minlength=6).tolist())
print(f"  blocked (infeasible NLP: start or goal inside an obstacle): {int(blocked.sum())}; GPU statuses there "
      f"{np.bincount(st[blocked], minlength=6).tolist()}, oracle {np.bincount(stc[blocked], minlength=6).tolist()}")
print(f"  equal statuses {tab['equal_status']} / {tab['instances']}; rounding-sensitive in the oracle {tab['rounding_sensitive']}")
for key in ("shared_failures", "kernel_only_failures", "oracle_only_failures", "both_converged_other_point"):
    ids = tab[key]
    print(f"  {key:28s} {len(ids):3d}  (not blocked: {sum(1 for i in ids if not blocked[i])}; rounding-sensitive: "
          f"{sum(1 for i in ids if sens[i])})  {ids}")
print(f"  both converged {tab['both_converged']}, at the same point {tab['both_converged_same_point']}")
print("  status mismatches on non-sensitive instances:", tab["status_mismatch_not_sensitive"])
print("  other optima on non-sensitive instances:", tab["other_point_not_sensitive"])
for i in tab["kernel_only_failures"] + tab["oracle_only_failures"]:
    print(f"    #{i:3d} case {i % 7} blocked {int(blocked[i])} GPU {st[i]} ({it[i]} it)  oracle {stc[i]} ({cen['iters'][i]} it)"
          f"  perturbed oracle {[p['status'][i] for p in cen['perturbed']]}  sensitive {int(sens[i])}")
