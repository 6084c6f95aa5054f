"""Dump the OBCA kernel's outputs on fixed batches (development check: bitwise A/B of two builds).

    TTMPC_LIB=<build> python tools/obca_dump.py OUT.npz [B] [max_iter]
    python tools/obca_dump.py --compare A.npz B.npz
Solves the seed-0 cobs windows (B) and c4 plans (B/4) of the bench workloads and saves X, U, status, iters.
OBCA_HELPERS=n sets the helper workgroups (0: none)."""
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "car-trailer-mpc_amd"), str(REPO / "tools")]
import numpy as np  # noqa: E402


def dump(out, B, max_iter):
    import ttmpc
    from obca_diag import workload
    from ttmpc import scenarios as sc
    res = {}
    for cfg, b in (("cobs", B), ("c4", max(1, B // 4))):
        P, data = workload(cfg, B=max(b, 8))
        data = {k: v[:b] for k, v in data.items()}
        variant = ttmpc.TT_VARIANT_TRACK_OBCA if cfg == "cobs" else ttmpc.TT_VARIANT_OBCA_PLAN
        s = ttmpc.ObcaSolver(P["N"], P["params"], sc.OBCA_Q, sc.OBCA_R, *P["bnd"], P["obs"], variant=variant,
                             max_iter=max_iter)
        if os.environ.get("OBCA_HELPERS"):  # helper workgroups: -1 one per CU (default), 0 none
            s.set_helpers(int(os.environ["OBCA_HELPERS"]))
        if cfg == "cobs":
            X, U, Z, st, it, kk = s.solve(data["x0"], xref=data["xref"], uref=data["uref"])
        else:
            X, U, Z, st, it, kk = s.solve(data["x0"], data["x_goal"], z_guess=data["z_guess"])
        res.update({f"{cfg}_X": X, f"{cfg}_U": U, f"{cfg}_st": st, f"{cfg}_it": it})
        print(cfg, "status", np.bincount(st, minlength=6).tolist(), "iters mean", float(it.mean()))
    np.savez(out, **res)


def compare(a, b):
    A, Bz = np.load(a), np.load(b)
    for k in A.files:
        same = np.array_equal(A[k], Bz[k])
        d = np.abs(A[k].astype(float) - Bz[k].astype(float)).max()
        print(f"{k:10s} bitwise {same}  max|diff| {d:.3e}")


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        compare(sys.argv[2], sys.argv[3])
    else:
        dump(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 64, int(sys.argv[3]) if len(sys.argv) > 3 else 400)
