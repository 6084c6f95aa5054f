"""Diagnostic: per-phase cycle shares of the tracking kernel (TT_STAMPS build, never shipped).

    python tools/phase_stamps.py [B] [N]
Reads s_memtime sums per phase per instance; prints mean cycles per instance and per IPM iteration.
Shares only -- the stamped build's absolute time is not the real kernel's (MI355X guide §7)."""
import ctypes as C
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "car-trailer-mpc_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from ttmpc import _lib  # noqa: E402
from ttmpc.scenarios import synthetic_batch  # noqa: E402
from oracle import ttmpc_oracle as to  # noqa: E402

PH = ["load", "linearize", "mu+barrier", "riccati", "forward", "step", "merit", "soc", "update", "#riccati",
      "#trials", "sub0", "sub1", "sub2", "sub3", "sub4", "sub5", "sub6", "sub7", "total"]
B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
N = int(sys.argv[2]) if len(sys.argv) > 2 else 20
psi = 0.9 if N >= 40 else 0.3
L = C.CDLL(str(REPO / "car-trailer-mpc_amd" / "ttmpc" / "libttmpc_stamps.so"))
L.tt_create.argtypes = [C.POINTER(_lib.TTConfig)] + [C.POINTER(C.c_double)] * 7 + [C.c_int, C.POINTER(C.c_void_p)]
L.ttx_solve_stamped.argtypes = [C.c_void_p, C.c_int] + [C.c_void_p] * 8 + [C.c_void_p]
cfg = _lib.TTConfig()
cfg.nx, cfg.nu, cfg.N, cfg.M = 6, 2, N, 0
p = to.DEFAULT_PARAMS
cfg.dt, cfg.L1, cfg.L2, cfg.Mh = p["dt"], p["L1"], p["L2"], p["M"]
cfg.variant = 0
arr = [np.ascontiguousarray(a, dtype=np.float64) for a in (to.DEFAULT_Q, to.DEFAULT_R, to.MPC_XLB, to.MPC_XUB,
                                                            to.MPC_ULB, to.MPC_UUB)]
arr = [np.where(np.isinf(a), np.sign(a) * 1e300, a) for a in arr]
h = C.c_void_p()
dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))  # noqa: E731
assert L.tt_create(C.byref(cfg), *[dp(a) for a in arr], None, 0, C.byref(h)) == 0
x0, xr, ur = synthetic_batch(B, N, seed=7, psi_range=psi)
d = torch.device("cuda", 0)
tx, txr, tur = (torch.from_numpy(a).to(d) for a in (x0, xr, ur))
X = torch.empty((B, N + 1, 6), dtype=torch.float64, device=d)
U = torch.empty((B, N, 2), dtype=torch.float64, device=d)
st = torch.empty(B, dtype=torch.int32, device=d)
it = torch.empty(B, dtype=torch.int32, device=d)
stamps = torch.zeros((B, len(PH)), dtype=torch.int64, device=d)
s = torch.cuda.Stream(d)
for rep in range(2):
    rc = L.ttx_solve_stamped(h, B, tx.data_ptr(), txr.data_ptr(), tur.data_ptr(), X.data_ptr(), U.data_ptr(),
                             st.data_ptr(), it.data_ptr(), stamps.data_ptr(), s.cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
S = stamps.cpu().numpy().astype(np.float64)
iters = it.cpu().numpy()
print(f"B={B} N={N} iters mean {iters.mean():.2f}  status {np.bincount(st.cpu().numpy(), minlength=5)}")
tot = S[:, -1].mean()
for i, name in enumerate(PH):
    m = S[:, i].mean()
    if name.startswith("#"):
        print(f"{name:12s} {m:12.2f} per instance  {m / max(iters.mean(), 1):10.2f} per iter")
        continue
    print(f"{name:12s} {m:12.0f} cyc/instance  {m / max(iters.mean(), 1):10.0f} cyc/iter  {100 * m / tot:6.1f}%")
nric = S[:, PH.index("#riccati")].mean()
print(f"riccati cycles per attempt {S[:, PH.index('riccati')].mean() / max(nric, 1):.0f}; "
      f"merit cycles per trial {S[:, PH.index('merit')].mean() / max(S[:, PH.index('#trials')].mean(), 1):.0f}")
