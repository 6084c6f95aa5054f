"""KKT certificate of the reference's committed OBCA plan (CPU, ~1 min).

    python tools/obca_certify_reference.py

1. certify data/state_traj.txt + input_traj.txt against the restated NLP (oracle/obca_certificate.py,
   every multiplier and x_goal free) and print where the residual sits;
2. solve the same problem with the oracle (x_init = the plan's first state, x_goal = its end pose with zero
   steering and speed, 11 obstacles) from two starts -- the committed plan itself and the reference's
   8-waypoint guess -- and compare the optima with the committed plan (cost, distance), then certify the
   oracle's optimum the same way.
Numbers are quoted in DESIGN.md section 1 ("KKT certificate of the committed plan")."""
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "car-trailer-mpc_amd")]
import numpy as np  # noqa: E402

from oracle import c_oracle as co  # noqa: E402
from oracle.obca_certificate import certify_plan  # noqa: E402
from ttmpc import scenarios as sc  # noqa: E402

g = np.load(REPO / "tests" / "golden" / "reference_numpy.npz")
S, U, ob = g["state_traj"], g["input_traj"], g["obstacles"].reshape(-1, 4)
N, M = U.shape[1], ob.shape[0]
box = (sc.OBCA_XLB, sc.OBCA_XUB, sc.OBCA_ULB, sc.OBCA_UUB)


def report(tag, X, Uk, bounded):
    t = time.time()
    r = certify_plan(X, Uk, ob, sc.OBCA_PARAMS, sc.OBCA_Q, sc.OBCA_R, *box, act_tol=1e-6 if not bounded else 1e-4,
                     bounded=bounded)
    res, nx, nu = r["residual"], r["nrow_x"], r["nrow_u"]
    ru = np.abs(res[nx:nx + nu]).reshape(-1, 2).max(1)
    print(f"{tag}: stat_rel {r['stat_rel']:.3e} (abs {r['stat']:.3e}, gradient scale {r['grad_scale']:.1f}), "
          f"{r['n_active']} active blocks, min distance {r['min_dist']:.6f}, {time.time() - t:.1f}s")
    print(f"  largest input-row residuals (stage, value): "
          f"{[(int(i), round(float(ru[i]), 3)) for i in np.argsort(-ru)[:6]]}")


report("committed plan (free multipliers)", S.T, U.T, bounded=False)
x0 = S[:, 0][None].repeat(2, 0)
xg = np.r_[S[:4, -1], 0.0, 0.0][None].repeat(2, 0)
_, _, zw = sc.obca_replan_batch(S, 1, N, M, seed=7)
st_ = 8 + 16 * M
zp = zw[0].copy()
for k in range(N):
    zp[k * st_:k * st_ + 6], zp[k * st_ + 6:k * st_ + 8] = S[:, k], U[:, k]
zp[N * st_:N * st_ + 6] = S[:, N]
P = co.make_obca_problem(N, sc.OBCA_PARAMS, sc.OBCA_Q, sc.OBCA_R, *box, ob)
t = time.time()
z, st, it, kk = co.obca_solve_batch(P, x0, xg, z_guess=np.stack([zp, zw[0]]), nthreads=2)
X, Uo, _, _ = co.obca_split(z, N, M)
print(f"oracle from (committed plan, 8-waypoint guess): status {st.tolist()} iterations {it.tolist()} "
      f"{time.time() - t:.1f}s")


def cost(X, Uk):
    d = X - xg[0]
    return float((d[:-1] ** 2).sum() + 100.0 * (d[-1] ** 2).sum() + 10.0 * (Uk ** 2).sum())


print(f"cost: committed {cost(S.T, U.T):.2f}, oracle {[round(cost(X[b], Uo[b]), 2) for b in range(2)]}; "
      f"oracle optima agree to {np.abs(X[0] - X[1]).max():.1e}; max |X_oracle - X_committed| per state "
      f"{np.abs(X[1] - S.T).max(0).round(3).tolist()}")
report("oracle optimum (bounded multipliers)", X[1], Uo[1], bounded=True)
