"""The kernel's own rounding sensitivity on the bench's C4 batch (diagnostic, GPU box).

    python tools/obca_gpu_sensitivity.py OUT.npz [seed]

tests/golden/make_c4_census.py classifies an instance as rounding-sensitive when the ORACLE's outcome changes under a
one-ulp-class perturbation of its guess.  This is the same experiment on the kernel: the batch (bench.py --config c4,
seed 7) solved as given and with the guess scaled by the census factors; per instance the statuses, iterations, end
points and plan objectives of all four runs.  An instance the oracle solves robustly but the kernel does not is rounding-
decided on the kernel's side when the kernel's own perturbed runs do converge.
"""
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "car-trailer-mpc_amd"), str(REPO / "tests"), str(REPO / "tests" / "golden")]
import numpy as np  # noqa: E402

from make_c4_census import PERTURB, plan_objective  # noqa: E402


def main():
    import ttmpc
    from ttmpc import scenarios as sc
    out = sys.argv[1]
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 7
    G = REPO / "tests" / "golden"
    obs = sc.obstacles_array(sc.load_obstacles(G / "obstacles.json"))[:6]
    cases = json.loads((G / "test_cases.json").read_text())["cases"]
    x0, xg, zg = sc.obca_case_batch(cases, 256, 200, 6, seed=seed, obstacles=obs, params=sc.OBCA_PARAMS)
    s = ttmpc.ObcaSolver(200, sc.OBCA_PARAMS, sc.OBCA_Q, sc.OBCA_R, sc.OBCA_XLB, sc.OBCA_XUB, sc.OBCA_ULB, sc.OBCA_UUB,
                         obs)
    res = {}
    for j, f in enumerate((1.0,) + tuple(PERTURB)):
        X, U, Z, st, it, kk = s.solve(x0, xg, z_guess=zg * f)
        res.update({f"X{j}": X, f"st{j}": st, f"it{j}": it, f"obj{j}": plan_objective(X, U, xg)})
        print(json.dumps({"factor": f, "status_counts": np.bincount(st, minlength=7).tolist(),
                          "iters_mean": float(it.mean())}), flush=True)
    np.savez_compressed(out, factors=np.array((1.0,) + tuple(PERTURB)), **res)


if __name__ == "__main__":
    main()
