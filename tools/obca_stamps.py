"""Per-phase cycle breakdown of the OBCA kernel (diagnostic hook ttx_obca_set_stamps).

    python tools/obca_stamps.py [B] [c4|replan|cobs] [max_iter]
Phase clocks are thread 0's shader cycles between phase boundaries (clock64), summed per instance."""
import ctypes as C
import json
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "car-trailer-mpc_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ttmpc  # noqa: E402
from ttmpc import scenarios as sc  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
wl = sys.argv[2] if len(sys.argv) > 2 else "c4"
mi = int(sys.argv[3]) if len(sys.argv) > 3 else 5000
G = REPO / "tests" / "golden"
g = np.load(G / "reference_numpy.npz")
obs_all = sc.obstacles_array(sc.load_obstacles(G / "obstacles.json"))
L = ttmpc.lib()
L.ttx_obca_set_stamps.argtypes = [C.c_void_p, C.c_void_p]
L.ttx_obca_set_stamps.restype = C.c_int
nph = L.ttx_obca_set_stamps(None, None)
d = torch.zeros((B, nph), dtype=torch.int64, device="cuda")
if wl == "cobs":
    x0, xr, ur = sc.mpc_obs_batch(g["state_traj"], g["input_traj"], B, 50, seed=0)
    s = ttmpc.ObcaSolver(50, dict(sc.OBCA_PARAMS, dt=0.05), sc.OBCA_Q, sc.OBCA_R, sc.XLB, sc.XUB, sc.ULB, sc.UUB,
                         obs_all, variant=ttmpc.TT_VARIANT_TRACK_OBCA, max_iter=mi)
    run = lambda: s.solve(x0, xref=xr, uref=ur)  # noqa: E731
else:
    if wl == "c4":
        cases = json.loads((G / "test_cases.json").read_text())["cases"]
        x0, xg, zg = sc.obca_case_batch(cases, B, 200, 6, seed=0, obstacles=obs_all[:6], params=sc.OBCA_PARAMS)
    else:
        x0, xg, zg = sc.obca_replan_batch(g["state_traj"], B, 200, 6, seed=7)
    s = ttmpc.ObcaSolver(200, sc.OBCA_PARAMS, sc.OBCA_Q, sc.OBCA_R, sc.OBCA_XLB, sc.OBCA_XUB, sc.OBCA_ULB,
                         sc.OBCA_UUB, obs_all[:6], max_iter=mi)
    run = lambda: s.solve(x0, xg, z_guess=zg)  # noqa: E731
if os.environ.get("OBCA_HELPERS"):  # helper workgroups: -1 one per CU (default), 0 none
    s.set_helpers(int(os.environ["OBCA_HELPERS"]))
run()  # warm-up
L.ttx_obca_set_stamps(s._h, d.data_ptr())
X, U, Z, st, it, kk = run()
torch.cuda.synchronize()
L.ttx_obca_set_stamps(s._h, None)
cyc = d.cpu().numpy().astype(np.float64)
names = ["lin", "compl", "factor", "riccati", "forward", "recover(+resid)", "trial", "update/other", "riccati_soft",
         "forward_soft", "ref_sweeps", "ref_recover_resid", "ref_staging", "TOTAL"]
counters = ["factorisations", "resto_iters", "soft_resto", "corrections", "soc", "pretend_singular", "trial_points"]
per_it = cyc / np.maximum(it, 1)[:, None]
print(f"{wl} B={B} iters mean {it.mean():.1f} max {it.max()}  status {np.bincount(st, minlength=6).tolist()}")
for i, n in enumerate(names):
    print(f"  {n:13s} {per_it[:, i].mean():12.0f} cycles/iter  ({100 * cyc[:, i].sum() / cyc[:, len(names) - 1].sum():5.1f}%)")
for i, n in enumerate(counters[:max(0, nph - len(names))]):  # (an older build has fewer slots)
    print(f"  {n:17s} {per_it[:, len(names) + i].mean():8.3f} per iteration")
