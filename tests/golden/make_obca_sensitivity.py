"""Rounding sensitivity of the three small OBCA parity batches of tests/test_gpu_obca.py (the 16 MPC+OBCA windows, the 14
C4 test cases, the 16 re-plans): the oracle (oracle/c/tt_obca.c) solves each batch as the tests do and twice more with
the guess perturbed by one unit in the last place (z * (1 + 2^-52), z * (1 - 2^-53); the windows have no guess, so their
initial state x_init is perturbed instead).  An instance whose status changes, or whose converged end point moves (max |dX| >
1e-6), under that perturbation is rounding-sensitive: its outcome is decided by last-bit differences, which is what separates the
kernel's arithmetic from the oracle's.  The GPU tests require the kernel to match the oracle's status and end point on
every instance that is NOT rounding-sensitive.

Writes tests/golden/obca_sensitivity.json.  Test infrastructure only.   python tests/golden/make_obca_sensitivity.py
"""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REPO = HERE.parents[1]
sys.path[:0] = [str(REPO), str(REPO / "car-trailer-mpc_amd")]

from oracle import c_oracle as co  # noqa: E402
from ttmpc import scenarios as sc  # noqa: E402

F_UP, F_DN = 1.0 + 2.0 ** -52, 1.0 - 2.0 ** -53


def batches():
    """The batches and oracle problems exactly as tests/test_gpu_obca.py builds them (P6 = OBCA_PARAMS)."""
    g = np.load(HERE / "reference_numpy.npz")
    cases = json.loads((HERE / "test_cases.json").read_text())["cases"]
    obs6 = sc.obstacles_array(sc.load_obstacles(HERE / "obstacles.json"))[:6]
    obca_b = (sc.OBCA_XLB, sc.OBCA_XUB, sc.OBCA_ULB, sc.OBCA_UUB)
    p50 = dict(sc.OBCA_PARAMS, dt=0.05)
    x0w, xr, ur = sc.mpc_obs_batch(g["state_traj"], g["input_traj"], 16, 50, seed=0)
    Pw = co.make_obca_problem(50, p50, sc.OBCA_Q, sc.OBCA_R, sc.XLB, sc.XUB, sc.ULB, sc.UUB, g["obstacles"],
                              mode=co.OBCA_TRACK)
    P200 = co.make_obca_problem(200, sc.OBCA_PARAMS, sc.OBCA_Q, sc.OBCA_R, *obca_b, obs6)
    c4 = sc.obca_case_batch(cases, 14, 200, 6, seed=0)
    rp = sc.obca_replan_batch(g["state_traj"], 16, 200, 6, seed=0)
    return {"windows": (Pw, 50, 11, dict(x0=x0w, xref=xr, uref=ur), "x0"),
            "c4_cases": (P200, 200, 6, dict(x0=c4[0], x_goal=c4[1], z_guess=c4[2]), "z_guess"),
            "replans": (P200, 200, 6, dict(x0=rp[0], x_goal=rp[1], z_guess=rp[2]), "z_guess")}


def main():
    out = {"provenance": "tests/golden/make_obca_sensitivity.py: oracle/c/tt_obca.c (round 5) under one-ulp perturbations"}
    for name, (P, N, M, data, key) in batches().items():
        t = time.time()
        z, st, it, _ = co.obca_solve_batch(P, **data, nthreads=8)
        X = co.obca_split(z, N, M)[0]
        sens = np.zeros(len(st), dtype=bool)
        runs = []
        for f in (F_UP, F_DN):
            d = dict(data)
            d[key] = data[key] * f
            zp, stp, itp, _ = co.obca_solve_batch(P, **d, nthreads=8)
            dx = np.abs(co.obca_split(zp, N, M)[0] - X).max(axis=(1, 2))
            sens |= (stp != st) | ((st <= 1) & (dx > 1e-6))
            runs.append({"factor": f, "status": stp.tolist(), "iters": itp.tolist(), "dx_max": [float(v) for v in dx]})
        out[name] = {"status": st.tolist(), "iters": it.tolist(), "perturbed": runs,
                     "rounding_sensitive": sens.astype(int).tolist(), "perturbed_input": key}
        print(name, "status", st.tolist(), "sensitive", np.flatnonzero(sens).tolist(), f"{time.time() - t:.0f}s",
              flush=True)
    (HERE / "obca_sensitivity.json").write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main()
