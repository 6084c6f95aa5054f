"""Generate tests/golden/oracle_default_plan.npz: the C ORACLE's solution (not an output of the reference, which cannot
run here: CasADi/IPOPT are absent) of the reference's own default OBCA call (run HERE; ~1 min on one core).

The reference's default plan (trajectory_animation.py:43-52, 77-83, 109) is N = 200, dt = 0.1, the OBCA bounds and
all 11 obstacles of obstacles.json, with plan()'s guess built from a Hybrid-A* initialize.json
(trajectory_optimization.py:227-274).  The initialize.json behind the committed data/state_traj.txt is not in the
repository, so the guess is the Hybrid-A*-shaped one rebuilt from that plan: 8 waypoints subsampled from it
(scenarios.obca_replan_batch instance 0, unperturbed), x_init = its first state, x_goal = its end pose with zero
steering and speed (get_initial_goal_states.py + trajectory_animation.py:83-92).  The oracle (oracle/c/tt_obca.c,
the restated IPOPT) converges there to a collision-free optimum of cost 64,914; the
committed plan itself is not a stationary point of the restated NLP (its KKT certificate).

Writes x_init, x_goal, z_guess, the oracle's z, status, iterations and KKT error, and the cost.
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REPO = HERE.parents[1]
sys.path[:0] = [str(REPO), str(REPO / "car-trailer-mpc_amd")]

from oracle import c_oracle as co  # noqa: E402
from ttmpc import scenarios as sc  # noqa: E402


def problem():
    g = np.load(HERE / "reference_numpy.npz")
    S, U, ob = g["state_traj"], g["input_traj"], g["obstacles"].reshape(-1, 4)
    N, M = U.shape[1], ob.shape[0]
    x0 = S[:, 0][None]
    xg = np.r_[S[:4, -1], 0.0, 0.0][None]
    _, _, zg = sc.obca_replan_batch(S, 1, N, M, seed=7)
    return N, M, ob, x0, xg, zg


def plan_cost(X, U, xg):
    d = X - xg
    return float((d[:-1] ** 2).sum() + 100.0 * (d[-1] ** 2).sum() + 10.0 * (U ** 2).sum())  # Q = I, R = 10 I


def main():
    N, M, ob, x0, xg, zg = problem()
    P = co.make_obca_problem(N, sc.OBCA_PARAMS, sc.OBCA_Q, sc.OBCA_R, sc.OBCA_XLB, sc.OBCA_XUB, sc.OBCA_ULB,
                             sc.OBCA_UUB, ob)
    z, st, it, kk = co.obca_solve_batch(P, x0, xg, z_guess=zg, nthreads=1)
    X, Uo, _, _ = co.obca_split(z, N, M)
    c = plan_cost(X[0], Uo[0], xg[0])
    prov = ("C oracle (oracle/c/tt_obca.c, restated IPOPT incl. its perturbation handler and, since round 5, its full "
            "convergence test) optimum of the reference's "
            "default OBCA problem; not produced by the reference (CasADi/IPOPT absent). OBCA optimality parity with "
            "IPOPT itself is unpinned beyond dynamics, bounds and collision (DESIGN.md section 5).")
    np.savez_compressed(HERE / "oracle_default_plan.npz", x_init=x0, x_goal=xg, z_guess=zg, z=z, status=st,
                        iters=it, kkt=kk, cost=c, provenance=np.array(prov))
    print(f"oracle_default_plan.npz: status {st.tolist()} iterations {it.tolist()} kkt {kk.tolist()} cost {c:.3f}")


if __name__ == "__main__":
    main()
