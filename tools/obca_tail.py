"""Where an iteration of the C4 max_iter tail goes (diagnostic, GPU box).

    python tools/obca_tail.py [B] [K1] [K2] [out.npz] [seed]
Runs the bench's C4 batch (B instances, bench.py's seed, the 4 collision-free test cases) twice with the phase clocks and event
counters on (ttx_obca_set_stamps), stopped at max_iter K1 and K2.  For the instances that run to max_iter in both, the
difference of the two runs is exactly their iterations K1..K2: per phase the shader cycles per iteration, and per
iteration the factorisations (inertia attempts), restoration iterations, soft-restoration steps, refinement
corrections, second-order corrections and trial points.  The launch wall times give the effective shader clock
(cycles of the slowest instance / launch time) and the wall time per tail iteration."""
import ctypes as C
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "car-trailer-mpc_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ttmpc  # noqa: E402
from ttmpc import scenarios as sc  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
K1 = int(sys.argv[2]) if len(sys.argv) > 2 else 4000
K2 = int(sys.argv[3]) if len(sys.argv) > 3 else 5000
G = REPO / "tests" / "golden"
obs = sc.obstacles_array(sc.load_obstacles(G / "obstacles.json"))[:6]
cases = json.loads((G / "test_cases.json").read_text())["cases"]
SEED = int(sys.argv[5]) if len(sys.argv) > 5 else 7  # 7 = bench.py's rank-0 seed (rank_seed(0)): the bench's C4 batch
x0, xg, zg = sc.obca_case_batch(cases, B, 200, 6, seed=SEED, obstacles=obs, params=sc.OBCA_PARAMS)
L = ttmpc.lib()
L.ttx_obca_set_stamps.argtypes = [C.c_void_p, C.c_void_p]
L.ttx_obca_set_stamps.restype = C.c_int
nph = L.ttx_obca_set_stamps(None, None)
names = ["lin", "compl", "factor", "riccati", "forward", "recover(+resid)", "trial", "update/other", "riccati_soft",
         "forward_soft", "ref_sweeps", "ref_recover_resid", "ref_staging"]
counters = ["factorisations", "resto_iters", "soft_resto", "corrections", "soc", "pretend_singular", "trial_points"]
TOT = len(names)


def run(K):
    s = ttmpc.ObcaSolver(200, sc.OBCA_PARAMS, sc.OBCA_Q, sc.OBCA_R, sc.OBCA_XLB, sc.OBCA_XUB, sc.OBCA_ULB,
                         sc.OBCA_UUB, obs, max_iter=K)
    s.solve(x0[:1], xg[:1], z_guess=zg[:1])  # warm-up (module load)
    d = torch.zeros((B, nph), dtype=torch.int64, device="cuda")
    L.ttx_obca_set_stamps(s._h, d.data_ptr())
    torch.cuda.synchronize()
    t = time.perf_counter()
    X, U, Z, st, it, kk = s.solve(x0, xg, z_guess=zg)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t
    L.ttx_obca_set_stamps(s._h, None)
    return d.cpu().numpy().astype(np.float64), st, it, wall


c1, st1, it1, w1 = run(K1)
c2, st2, it2, w2 = run(K2)
if len(sys.argv) > 4:
    np.savez(sys.argv[4], c1=c1, st1=st1, it1=it1, w1=w1, c2=c2, st2=st2, it2=it2, w2=w2)
tail = (it1 == K1) & (it2 == K2)
print(f"C4 B={B}: max_iter {K1}: {w1:.2f} s, status {np.bincount(st1, minlength=6).tolist()};  max_iter {K2}: {w2:.2f} s, "
      f"status {np.bincount(st2, minlength=6).tolist()};  {int(tail.sum())} instances at max_iter in both")
for K, c, w in ((K1, c1, w1), (K2, c2, w2)):
    print(f"  max_iter {K}: slowest instance {c[:, TOT].max():.4e} cycles in a {w:.3f} s launch (host wall, incl. "
          f"launch + copies) -> effective shader clock {c[:, TOT].max() / w / 1e9:.3f} GHz")
if tail.any():
    dc = (c2 - c1)[tail] / float(K2 - K1)
    dt_it = (w2 - w1) / float(K2 - K1)
    tot = dc[:, TOT].mean()
    print(f"iterations {K1}..{K2} of the {int(tail.sum())} tail instances: {tot:.0f} cycles per iteration "
          f"(max over them {dc[:, TOT].max():.0f}); launch-time difference per iteration {dt_it * 1e3:.3f} ms "
          f"= {dc[:, TOT].max() / dt_it / 1e9:.3f} GHz effective at the slowest")
    ssum = 0.0
    for i, n in enumerate(names):
        v = dc[:, i].mean()
        ssum += v
        print(f"  {n:18s} {v:12.0f} cycles/iter  ({100 * v / tot:5.1f}%)")
    print(f"  {'sum of phases':18s} {ssum:12.0f}  (TOTAL {tot:.0f})")
    for i, n in enumerate(counters):
        print(f"  {n:18s} {dc[:, TOT + 1 + i].mean():8.3f} per iteration")
    print("  per instance (cycles/iter, factorisations/iter, resto iters/iter):")
    for b in np.flatnonzero(tail):
        r = (c2[b] - c1[b]) / float(K2 - K1)
        print(f"    #{b:3d}: {r[TOT]:10.0f}  {r[TOT + 1]:6.3f}  {r[TOT + 2]:6.3f}")

# the instances that set the K2 launch time: their whole run, per phase (the phases sum to the instance's clock, and the
# slowest instance's clock / the effective shader clock is the launch time)
print(f"slowest instances of the max_iter {K2} launch (whole run):")
order = np.argsort(-c2[:, TOT])[:5]
for b in order:
    r = c2[b]
    print(f"  #{b:3d}: status {st2[b]} iters {it2[b]:5d}  {r[TOT]:.4e} cycles = {r[TOT] / (c2[:, TOT].max() / w2):.2f} s "
          f"({r[TOT] / max(it2[b], 1) / 1e6:.2f} M cycles/iter; factorisations/iter {r[TOT + 1] / max(it2[b], 1):.2f}, "
          f"resto iters {r[TOT + 2]:.0f}, corrections/iter {r[TOT + 4] / max(it2[b], 1):.2f}, "
          f"trial points/iter {r[TOT + 7] / max(it2[b], 1):.2f})")
b = order[0]
print(f"  phases of #{b} (cycles per iteration over its {it2[b]} iterations):")
for i, n in enumerate(names):
    print(f"    {n:18s} {c2[b, i] / max(it2[b], 1):12.0f}  ({100 * c2[b, i] / c2[b, TOT]:5.1f}%)")
