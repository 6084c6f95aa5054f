"""The straight-line FP64 sin / cos / tan of csrc/tt_trig.hpp against the device library (advisor r5): the kernels use the
restatement wherever every lane's argument is finite and below 2^30, and their bitwise trail -- the lockstep parity of
the OBCA tests, the bitwise-neutral build A/Bs -- assumes it IS the library's result.  tools/trig_check.hip (built in-tree
by the package Makefile as tools/bin/trig_check) draws 2^22 arguments over its five families (angles, magnitudes up
to 2^30, neighbours of k pi/4, tiny and subnormal values) and counts bitwise mismatches; the round-5 run covered 2^28."""
import re
import subprocess

import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu


def test_straight_line_trig_is_bitwise_the_library():
    exe = REPO / "tools" / "bin" / "trig_check"
    if not exe.exists():
        raise FileNotFoundError(f"{exe} is not built (make -C car-trailer-mpc_amd)")
    out = subprocess.run([str(exe), str(1 << 22)], capture_output=True, text=True, timeout=120, check=True).stdout
    counts = [(int(a), int(b)) for a, b in re.findall(r"(\d+) arguments, (\d+) bitwise mismatches", out)]
    assert len(counts) == 2, out
    assert all(n == 1 << 22 and bad == 0 for n, bad in counts), out
