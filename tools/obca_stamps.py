"""Per-phase cycle breakdown of the OBCA kernel (diagnostic hook ttx_obca_set_stamps) on the C4 workload."""
import ctypes as C
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "car-trailer-mpc_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ttmpc  # noqa: E402
from ttmpc import scenarios as sc  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
g = np.load(REPO / "tests" / "golden" / "reference_numpy.npz")
obs = sc.obstacles_array(sc.load_obstacles(REPO / "tests" / "golden" / "obstacles.json"))[:6]
x0, xg, zg = sc.obca_replan_batch(g["state_traj"], B, 200, 6, seed=7)
L = ttmpc.lib()
L.ttx_obca_set_stamps.argtypes = [C.c_void_p]
L.ttx_obca_set_stamps.restype = C.c_int
nph = L.ttx_obca_set_stamps(None)
d = torch.zeros((B, nph), dtype=torch.int64, device="cuda")
L.ttx_obca_set_stamps(d.data_ptr())
s = ttmpc.ObcaSolver(200, sc.OBCA_PARAMS, sc.OBCA_Q, sc.OBCA_R, sc.OBCA_XLB, sc.OBCA_XUB, sc.OBCA_ULB, sc.OBCA_UUB, obs,
                     max_iter=1000)
X, U, Z, st, it, kk = s.solve(x0, xg, z_guess=zg)
torch.cuda.synchronize()
L.ttx_obca_set_stamps(None)
cyc = d.cpu().numpy().astype(np.float64)
names = ["lin", "compl", "factor", "riccati", "forward", "recover", "trial", "update/other", "TOTAL"]
per_it = cyc / np.maximum(it, 1)[:, None]
print(f"B={B} iters mean {it.mean():.1f}  status {np.bincount(st).tolist()}")
for i, n in enumerate(names):
    print(f"  {n:13s} {per_it[:, i].mean():12.0f} cycles/iter  ({100 * cyc[:, i].sum() / cyc[:, -1].sum():5.1f}%)")
