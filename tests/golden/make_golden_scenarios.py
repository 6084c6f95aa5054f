"""Generate tests/golden/scenario_io.json: outputs of the reference's own scenario-file helpers
(run HERE, in the survey container; pure-json modules, no casadi involved):

  * make_parking_obstacles.build_obstacles(open_spot, depth)   make_parking_obstacles.py:6-51
  * apply_case.write_initialize(case, path)                    apply_case.py:16-34
    for every case of the committed test_cases.json

Only the produced data is written (no reference source is copied).
"""
from __future__ import annotations

import json
import sys
import tempfile
from pathlib import Path

HERE = Path(__file__).resolve().parent
REF = Path("/root/reference/python-files")


def main():
    sys.dont_write_bytecode = True
    sys.path.insert(0, str(REF))
    import apply_case
    import make_parking_obstacles
    out = {"parking": {}, "initialize": {}}
    for spot in range(1, 11):
        for depth in (20.0, 12.5):
            out["parking"][f"{spot}_{depth}"] = make_parking_obstacles.build_obstacles(spot, depth)
    cases = json.loads((HERE / "test_cases.json").read_text())["cases"]
    with tempfile.TemporaryDirectory() as td:
        for c in cases:
            p = Path(td) / "init.json"
            apply_case.write_initialize(c, p)
            out["initialize"][c["name"]] = json.loads(p.read_text())
    (HERE / "scenario_io.json").write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
