"""OBCA GPU-vs-oracle parity census on the workloads of tests/test_gpu_obca.py (development tool).

The oracle side is deterministic for a given build of oracle/build/libttoracle.so, so it is computed once (here, on
the CPU) and cached; a GPU call then only runs the kernel, once per library build, and the comparison evaluates the
assertions of tests/test_gpu_obca.py for every build.

    python tools/obca_parity.py oracle OUT.npz                 # CPU: oracle results of every workload
    python tools/obca_parity.py gpu OUT.npz [SO]                # GPU box: kernel results (SO: TTMPC_LIB build)
    python tools/obca_parity.py compare ORACLE.npz GPU.npz...   # the test assertions, per GPU build
    python tools/obca_parity.py lock-oracle OUT.npz / lock-gpu OUT.npz [SO] / lock-compare ORACLE.npz GPU.npz
        # lockstep census: every workload stopped at max_iter K (25 ... 1600); the iterates after K iterations agree
        # to round-off exactly while the two runs still take the same path
"""
LOCK_K = (25, 50, 100, 200, 400, 800, 1600)
import json
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "car-trailer-mpc_amd"), str(REPO / "tests")]
import numpy as np  # noqa: E402

G = REPO / "tests" / "golden"


def workloads():
    from ttmpc import scenarios as sc
    ref = np.load(G / "reference_numpy.npz")
    obs11 = ref["obstacles"]
    obs6 = sc.obstacles_array(sc.load_obstacles(G / "obstacles.json"))[:6]
    cases = json.loads((G / "test_cases.json").read_text())["cases"]
    out = {}
    x0, xr, ur = sc.mpc_obs_batch(ref["state_traj"], ref["input_traj"], 16, 50, seed=0)
    out["cobs"] = dict(kind="track", N=50, obs=obs11, x0=x0, xr=xr, ur=ur)
    x0, xg, zg = sc.obca_case_batch(cases, 14, 200, 6, seed=0)
    out["c4"] = dict(kind="plan", N=200, obs=obs6, x0=x0, xg=xg, zg=zg)
    x0, xg, zg = sc.obca_replan_batch(ref["state_traj"], 16, 200, 6, seed=0)
    out["replan"] = dict(kind="plan", N=200, obs=obs6, x0=x0, xg=xg, zg=zg)
    if os.environ.get("OBCA_PARITY_FULL"):
        x0, xg, zg = sc.obca_case_batch(cases, 256, 200, 6, seed=1)
        out["c4full"] = dict(kind="plan", N=200, obs=obs6, x0=x0, xg=xg, zg=zg)
    return out


def _params(w):
    from test_obca_oracle import P6
    from ttmpc import scenarios as sc
    if w["kind"] == "track":
        return dict(P6, dt=0.05), (sc.XLB, sc.XUB, sc.ULB, sc.UUB)
    return P6, (sc.OBCA_XLB, sc.OBCA_XUB, sc.OBCA_ULB, sc.OBCA_UUB)


def run_oracle(path, ks=(None,)):
    from oracle import c_oracle as co
    from ttmpc import scenarios as sc
    res = {}
    for name0, w, K in ((n + ("" if K is None else f"_{K}"), w, K) for K in ks for n, w in workloads().items()):
        name = name0
        p, b = _params(w)
        mode = co.OBCA_TRACK if w["kind"] == "track" else co.OBCA_PLAN
        P = co.make_obca_problem(w["N"], p, sc.OBCA_Q, sc.OBCA_R, *b, w["obs"], mode=mode, max_iter=K or 5000)
        t = time.time()
        if w["kind"] == "track":
            z, st, it, kk = co.obca_solve_batch(P, w["x0"], xref=w["xr"], uref=w["ur"], nthreads=os.cpu_count())
        else:
            z, st, it, kk = co.obca_solve_batch(P, w["x0"], w["xg"], z_guess=w["zg"], nthreads=os.cpu_count())
        X = co.obca_split(z, w["N"], w["obs"].shape[0])[0]
        print(f"oracle {name}: {time.time() - t:.1f}s status {st.tolist()} iters {it.tolist()}", flush=True)
        res[name + "_X"], res[name + "_st"], res[name + "_it"] = X, st, it
    np.savez_compressed(path, **res)


def run_gpu(path, ks=(None,)):
    import ttmpc
    from ttmpc import scenarios as sc
    res = {}
    for name, w, K in ((n + ("" if K is None else f"_{K}"), w, K) for K in ks for n, w in workloads().items()):
        p, b = _params(w)
        v = ttmpc.TT_VARIANT_TRACK_OBCA if w["kind"] == "track" else ttmpc.TT_VARIANT_OBCA_PLAN
        s = ttmpc.ObcaSolver(w["N"], p, sc.OBCA_Q, sc.OBCA_R, *b, w["obs"], variant=v, max_iter=K or 5000)
        t = time.time()
        if w["kind"] == "track":
            X, U, Z, st, it, kk = s.solve(w["x0"], xref=w["xr"], uref=w["ur"])
        else:
            X, U, Z, st, it, kk = s.solve(w["x0"], w["xg"], z_guess=w["zg"])
        print(f"gpu {name}: {time.time() - t:.1f}s status {st.tolist()} iters {it.tolist()}", flush=True)
        res[name + "_X"], res[name + "_st"], res[name + "_it"] = X, st, it
    np.savez_compressed(path, **res)


def compare(opath, gpath):
    from test_obca_oracle import P6
    from ttmpc import collision
    o, g, w = np.load(opath), np.load(gpath), workloads()
    fails = []

    def chk(cond, what):
        if not cond:
            fails.append(what)

    st, stc = g["cobs_st"], o["cobs_st"]
    both = (st <= 1) & (stc <= 1)
    d = np.abs(g["cobs_X"] - o["cobs_X"]).max(axis=(1, 2))
    same_it = g["cobs_it"] == o["cobs_it"]
    print(f"  cobs: status agree {(st == stc).sum()}/16, both {both.sum()}, same iters {same_it.sum()}, "
          f"max|dX| both {d[both].max() if both.any() else 0:.1e}, same-path {d[both & same_it].max() if (both & same_it).any() else 0:.1e}")
    chk((st == stc).all(), "cobs statuses 16/16")
    chk(both.sum() >= 9, "cobs both >= 9")
    chk(d[both].max() <= 1e-8, "cobs windows <= 1e-8")
    x0 = w["cobs"]["x0"]
    gap = collision.sat_gap(x0[:, :4], dict(P6, dt=0.05), w["cobs"]["obs"]).min(axis=(-1, -2))
    chk(np.all(st[gap < 0] > 1) and np.all(stc[gap < 0] > 1), "cobs blocked never converge")

    st, stc = g["c4_st"], o["c4_st"]
    wc = w["c4"]
    gs = collision.sat_gap(wc["x0"][:, :4], P6, wc["obs"]).min(axis=(-1, -2))
    gg = collision.sat_gap(wc["xg"][:, :4], P6, wc["obs"]).min(axis=(-1, -2))
    blocked = (gs < 0) | (gg < 0)
    both = (st <= 1) & (stc <= 1)
    d = np.abs(g["c4_X"] - o["c4_X"]).max(axis=(1, 2))
    same = d <= 1e-6
    print(f"  c4: status agree {(st == stc).sum()}/14, both {both.sum()}, gpu conv {(st[~blocked] <= 1).sum()}, "
          f"cpu conv {(stc[~blocked] <= 1).sum()}, same[both] {same[both].sum()}; gpu {st.tolist()} cpu {stc.tolist()}")
    chk((st == stc).sum() >= 12, "c4 status agree >= 12")
    chk(blocked.sum() == 6 and np.all(st[blocked] == 3) and np.all(stc[blocked] == 3), "c4 blocked status 3")
    chk((st[~blocked] <= 1).sum() >= 6 and (stc[~blocked] <= 1).sum() >= 6, "c4 each side >= 6")
    chk(both.sum() >= 6, "c4 both >= 6")
    chk(same[both & (st == 0) & (stc == 0)].all(), "c4 optimal pairs same")
    chk(same[both].sum() >= both.sum() - 1, "c4 same[both] >= both-1")

    st, stc = g["replan_st"], o["replan_st"]
    both = (st <= 1) & (stc <= 1)
    d = np.abs(g["replan_X"] - o["replan_X"]).max(axis=(1, 2))
    print(f"  replan: gpu conv {(st <= 1).sum()} cpu conv {(stc <= 1).sum()} both {both.sum()} "
          f"max|dX| both {np.array2string(d[both], precision=1)}")
    chk((st <= 1).sum() >= 15 and (stc <= 1).sum() >= 15, "replan each side >= 15")
    chk(both.sum() >= 14, "replan both >= 14")
    chk((d[both] <= 1e-6).all(), "replan same[both].all()")
    if "c4full_st" in g:
        os.environ["OBCA_PARITY_FULL"] = "1"
        wf = workloads()["c4full"]
        st = g["c4full_st"]
        gs = collision.sat_gap(wf["x0"][:, :4], P6, wf["obs"]).min(axis=(-1, -2))
        gg = collision.sat_gap(wf["xg"][:, :4], P6, wf["obs"]).min(axis=(-1, -2))
        blocked = (gs < 0) | (gg < 0)
        print(f"  c4full: blocked {np.bincount(st[blocked], minlength=6).tolist()} "
              f"feasible {np.bincount(st[~blocked], minlength=6).tolist()} max iters {g['c4full_it'].max()}")
        chk(np.all(st[blocked] == 3), "c4full blocked all status 3")
        chk((st[~blocked] <= 1).mean() >= 0.85, "c4full feasible >= 85%")
    print("  FAILS: " + ("; ".join(fails) if fails else "none"))
    return not fails


def lock_compare(opath, gpath):
    o, g = np.load(opath), np.load(gpath)
    names = [n for n in workloads() if n != "c4full"]
    print("max |X_gpu - X_oracle| per instance after K iterations (runs stopped at max_iter K)")
    for n in names:
        print(f"  {n}:")
        for K in LOCK_K:
            d = np.abs(g[f"{n}_{K}_X"] - o[f"{n}_{K}_X"]).max(axis=(1, 2))
            lock = int((d <= 1e-9).sum())
            print(f"    K={K:5d}  lockstep (<= 1e-9) {lock:2d}/{len(d)}  max {d.max():.1e}  " + " ".join(f"{v:.0e}" for v in d))


if __name__ == "__main__":
    cmd = sys.argv[1]
    if cmd in ("gpu", "lock-gpu") and len(sys.argv) > 3 and sys.argv[3]:
        os.environ["TTMPC_LIB"] = sys.argv[3]
    if cmd == "oracle":
        run_oracle(sys.argv[2])
    elif cmd == "gpu":
        run_gpu(sys.argv[2])
    elif cmd == "lock-oracle":
        os.environ.pop("OBCA_PARITY_FULL", None)
        run_oracle(sys.argv[2], LOCK_K)
    elif cmd == "lock-gpu":
        os.environ.pop("OBCA_PARITY_FULL", None)
        run_gpu(sys.argv[2], LOCK_K)
    elif cmd == "lock-compare":
        lock_compare(sys.argv[2], sys.argv[3])
    else:
        ok = True
        for gp in sys.argv[3:]:
            print(gp)
            ok &= compare(sys.argv[2], gp)
        sys.exit(0 if ok else 1)
