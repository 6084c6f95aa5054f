"""HBM traffic of the C4 max_iter tail alone (diagnostic, GPU box).

    rocprofv3 --pmc FETCH_SIZE --kernel-trace -d OUT/fetch -o fetch --output-format csv -- python3 tools/obca_tail_traffic.py run 4000 5000
    (the same with WRITE_SIZE, and with any other counter group, each pass in its own run)
    python tools/obca_tail_traffic.py report OUT
    (run K1 K2 0: the same without helper workgroups, ttx_obca_set_helpers)

`run` solves the bench's C4 batch (bench.py's seed 7, B = 256) twice, stopped at max_iter K1 and K2 (plain solves: no
stamps), and writes the per-instance iterations of both to OUT-independent stdout as one JSON line.  The difference of the
two obca_kernel dispatches' counters is the traffic of the instance-iterations K1..K2, i.e. of the tail alone, where a
handful of instances run on an otherwise idle GPU (the launch's busy phase, 256 instances at once, is in both dispatches
and cancels).  `report` prints counter differences per tail instance-iteration for every pass found under OUT.
"""
import csv
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "car-trailer-mpc_amd")]


def run(K1, K2, nhelp=-1):
    import numpy as np
    import ttmpc
    from ttmpc import scenarios as sc
    G = REPO / "tests" / "golden"
    obs = sc.obstacles_array(sc.load_obstacles(G / "obstacles.json"))[:6]
    cases = json.loads((G / "test_cases.json").read_text())["cases"]
    x0, xg, zg = sc.obca_case_batch(cases, 256, 200, 6, seed=7, obstacles=obs, params=sc.OBCA_PARAMS)
    its = []
    for K in (K1, K2):
        s = ttmpc.ObcaSolver(200, sc.OBCA_PARAMS, sc.OBCA_Q, sc.OBCA_R, sc.OBCA_XLB, sc.OBCA_XUB, sc.OBCA_ULB,
                             sc.OBCA_UUB, obs, max_iter=K)
        s.set_helpers(nhelp)
        X, U, Z, st, it, kk = s.solve(x0, xg, z_guess=zg)
        its.append(it.astype(np.int64))
    d = its[1] - its[0]
    print(json.dumps({"K1": K1, "K2": K2, "helpers": nhelp, "iters_K1": int(its[0].sum()), "iters_K2": int(its[1].sum()),
                      "tail_instance_iterations": int(d.sum()), "tail_instances": int((d > 0).sum())}))


def report(out):
    out = Path(out)
    for csvf in sorted(out.rglob("*counter_collection.csv")):
        vals = {}
        with open(csvf) as fh:
            for row in csv.DictReader(fh):
                if "obca_kernel" in row["Kernel_Name"]:
                    vals.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
        meta = next((p for p in (csvf.parent.with_suffix(".json"), csvf.parent / "run.json") if p.exists()), None)
        info = json.loads(meta.read_text()) if meta else None
        for name, v in vals.items():
            if len(v) != 2:
                print(f"{csvf}: {name}: {len(v)} obca_kernel dispatches (expected 2)")
                continue
            line = f"{csvf.parent.name:10s} {name:24s} K1 {v[0]:.4g}  K2 {v[1]:.4g}  tail {v[1] - v[0]:.4g}"
            if info:
                line += f"  per tail instance-iteration {(v[1] - v[0]) / info['tail_instance_iterations']:.4g}"
            print(line)


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]) if len(sys.argv) > 4 else -1)
    else:
        report(sys.argv[2])
