"""Generate tests/golden/nmpc_plant.npz (run HERE, in the survey container): the plant of the NMPC and fuzzy
drivers, ``update`` of python-files/simulation_nmpc.py:94-105 and simulation_fuzzy.py:94-105, imported from the
reference behind a never-called ``casadi`` stub (as make_golden.py does).

That update differs from simulation.py's (167-199) by the process noise apply_disturbances draws
(np.random.normal(0, process_noise_std, 6)), added as q_ += state_noise * dt right after the Euler step.  Each
vector re-seeds np.random, draws the noise the reference will draw, re-seeds and calls the reference, so the
recorded noise is exactly the one its update used.  Two disturbance sets: the modules' own DISTURBANCE_PARAMS
(friction and slippage 1, noise 0.02, no slip) and a set that switches every disturbance on.

Only data arrays are written; no reference source is copied.
"""
from __future__ import annotations

import sys
import types
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REF = Path("/root/reference/python-files")


def main():
    sys.dont_write_bytecode = True
    sys.modules.setdefault("casadi", types.ModuleType("casadi"))  # never called by update
    sys.path.insert(0, str(REF))
    import simulation_fuzzy as sf  # noqa: E402
    import simulation_nmpc as sn  # noqa: E402

    rng = np.random.default_rng(4321)
    p = {"M": 0.15, "L1": 7.05, "L2": 12.45, "W1": 3.05, "W2": 2.95, "dt": 0.05}
    B = 64
    Q = np.column_stack([rng.uniform(0, 60, B), rng.uniform(0, 60, B), rng.uniform(-np.pi, np.pi, B),
                         rng.uniform(-1, 1, B), rng.uniform(-0.7, 0.7, B), rng.uniform(-8, 8, B)])
    U = np.column_stack([rng.uniform(-5, 5, B), rng.uniform(-1.5, 1.5, B)])
    full = {"friction_coeff": 0.9, "slippage_coeff": 0.85, "process_noise_std": 0.05, "lateral_slip_gain": 0.02,
            "slip_angle_max": 0.1}
    out = {"q": Q, "u": U, "dt": p["dt"]}
    for tag, mod in (("nmpc", sn), ("fuzzy", sf)):
        for dname, dist in (("own", mod.DISTURBANCE_PARAMS), ("full", full)):
            noise = np.empty((B, 6))
            qn = np.empty((B, 6))
            for i in range(B):
                np.random.seed(9000 + i)
                noise[i] = np.random.normal(0, dist["process_noise_std"], 6)
                np.random.seed(9000 + i)
                qn[i] = mod.update(Q[i], U[i], p, disturbance_params=dist)
            out[f"{tag}_{dname}_noise"] = noise
            out[f"{tag}_{dname}_next"] = qn
        out[f"{tag}_nominal_next"] = np.array([mod.update(Q[i], U[i], p) for i in range(B)])
    for k, v in full.items():
        out["full_" + k] = v
    for k, v in sn.DISTURBANCE_PARAMS.items():
        out["own_" + k] = v
    np.savez_compressed(HERE / "nmpc_plant.npz", **out)
    print("nmpc_plant.npz:", sorted(out))


if __name__ == "__main__":
    main()
