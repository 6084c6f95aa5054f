import sys
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parents[1]
PKG = REPO / "car-trailer-mpc_amd"
GOLDEN = Path(__file__).resolve().parent / "golden"
for p in (str(REPO), str(PKG)):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) GPU and the built libttmpc.so")


@pytest.fixture(scope="session")
def golden_ref():
    return dict(np.load(GOLDEN / "reference_numpy.npz"))


@pytest.fixture(scope="session")
def golden_opt():
    return dict(np.load(GOLDEN / "nlp_optima.npz"))


def fixture_instance(g, i):
    """Unpad one nlp_optima row -> (tag, N, x0, xref (N+1,6), uref (N,2), wq, wr, z)."""
    N = int(g["N"][i])
    return (str(g["tag"][i]), N, g["x0"][i], g["xref"][i][: N + 1], g["uref"][i][:N], g["wq"][i], g["wr"][i],
            g["z"][i][: 8 * N + 6])
