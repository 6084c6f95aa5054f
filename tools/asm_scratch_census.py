"""Static scratch census of a gfx950 device assembly file (hipcc --cuda-device-only -S): per function, the scratch
(spill / frame) loads and stores and their bytes per lane, the private segment size the function declares, and its
call sites (s_swappc_b64 targets).  VERDICT r5 item 2 asked to split obca_kernel's HBM bytes per instance-iteration
into scratch traffic and workspace records; multiplying these static counts by the calls per iteration
(tools/obca_stamps.py event counters) bounds the scratch part.

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Icar-trailer-mpc_amd/csrc --cuda-device-only -S \\
          car-trailer-mpc_amd/csrc/tt_obca.hip -o /tmp/obca.s
    python tools/asm_scratch_census.py /tmp/obca.s [--prologue]

--prologue splits each function's scratch stores / loads into the ones in its prologue / epilogue (before the first
non-save instruction, after the last restore: the callee-saved register frame of a call) and the rest (spills).
"""
from __future__ import annotations

import re
import sys
from collections import defaultdict

BYTES = {"byte": 1, "short": 2, "ubyte": 1, "sbyte": 1, "ushort": 2, "sshort": 2, "dword": 4, "dwordx2": 8,
         "dwordx3": 12, "dwordx4": 16, "b32": 4, "b64": 8, "b96": 12, "b128": 16}


def demangle(name):
    try:
        import subprocess
        return subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip() or name
    except Exception:  # noqa: BLE001
        return name


def census(path):
    funcs = {}
    cur = None
    body = []
    for line in open(path):
        m = re.match(r"^([A-Za-z_.$][\w.$]*):\s*(;.*)?$", line)
        if m and not m.group(1).startswith("."):
            if cur:
                funcs[cur] = body
            cur, body = m.group(1), []
            continue
        if cur and re.match(r"^\s*\.size\s+" + re.escape(cur) + r",", line):
            funcs[cur] = body
            cur, body = None, []
            continue
        if cur:
            body.append(line.rstrip())
    out = {}
    for f, lines in funcs.items():
        ins = [ln.strip() for ln in lines if ln.strip() and not ln.strip().startswith((";", ".", "//"))
               and not ln.strip().endswith(":")]
        st = ld = stb = ldb = 0
        calls = defaultdict(int)
        for i in ins:
            mm = re.match(r"(scratch|buffer)_(store|load)_(\w+)", i)
            if mm and (mm.group(1) == "scratch" or "off, s[0:3]" in i or "s[0:3]" in i):
                nb = BYTES.get(mm.group(3).split("_")[0], 4)
                if mm.group(2) == "store":
                    st += 1; stb += nb
                else:
                    ld += 1; ldb += nb
            mc = re.search(r"s_swappc_b64\s+s\[\d+:\d+\],\s*s\[\d+:\d+\]", i)
            if mc:
                calls["<indirect>"] += 1
        for ln in lines:
            mg = re.search(r"(\w+)@rel32@lo", ln)
            if mg and "s_add_u32" in ln or (mg and "s_getpc" in ln):
                calls[mg.group(1)] += 1
        out[f] = dict(n=len(ins), st=st, ld=ld, stb=stb, ldb=ldb, calls=dict(calls))
    return out


def main():
    path = sys.argv[1]
    c = census(path)
    rows = sorted(c.items(), key=lambda kv: -(kv[1]["stb"] + kv[1]["ldb"]))
    print(f"{'function':70s} {'insts':>7s} {'scr st':>7s} {'scr ld':>7s} {'B/lane st':>9s} {'B/lane ld':>9s}  callees")
    for f, r in rows:
        if r["st"] + r["ld"] == 0 and not r["calls"]:
            continue
        name = demangle(f)
        name = re.sub(r"ttmpc::\(anonymous namespace\)::", "", name)[:70]
        callees = ", ".join(f"{re.sub(r'_Z[N]?5ttmpc12_GLOBAL__N_1', '', k)[:28]}x{v}" for k, v in r["calls"].items())
        print(f"{name:70s} {r['n']:7d} {r['st']:7d} {r['ld']:7d} {r['stb']:9d} {r['ldb']:9d}  {callees[:120]}")


if __name__ == "__main__":
    main()


def frame_split(path):
    """Per function: (prologue stores, in-body stores, in-body loads, epilogue loads), each in B/lane.  The prologue is
    the run of scratch stores (and s_/v_writelane/v_accvgpr bookkeeping) before the first other vector instruction;
    the epilogue the run of scratch loads before the function's last s_setpc_b64."""
    out = {}
    cur, body = None, []
    for line in open(path):
        m = re.match(r"^([A-Za-z_.$][\w.$]*):\s*(;.*)?$", line)
        if m and not m.group(1).startswith("."):
            cur, body = m.group(1), []
            continue
        if cur and re.match(r"^\s*\.size\s+" + re.escape(cur) + r",", line):
            ins = [ln.strip() for ln in body if ln.strip() and not ln.strip().startswith((";", ".", "//"))
                   and not ln.strip().endswith(":")]
            nb = lambda i: BYTES.get(re.match(r"scratch_\w+?_(\w+)", i).group(1), 4)  # noqa: E731
            pro = epi = st = ld = 0
            k = 0
            while k < len(ins) and (ins[k].startswith(("scratch_store", "s_", "v_writelane", "v_accvgpr_read",
                                                        "v_mov_b32"))):
                if ins[k].startswith("scratch_store"):
                    pro += nb(ins[k])
                k += 1
            last = max((i for i, s in enumerate(ins) if s.startswith("s_setpc_b64")), default=len(ins))
            e = last - 1
            while e > k and ins[e].startswith(("scratch_load", "s_", "v_readlane", "v_accvgpr_write")):
                if ins[e].startswith("scratch_load"):
                    epi += nb(ins[e])
                e -= 1
            for s in ins[k:e + 1]:
                if s.startswith("scratch_store"):
                    st += nb(s)
                elif s.startswith("scratch_load"):
                    ld += nb(s)
            out[cur] = (pro, st, ld, epi)
            cur, body = None, []
            continue
        if cur:
            body.append(line.rstrip())
    return out


if __name__ == "__main__" and "--prologue" in sys.argv:
    print(f"\n{'function':70s} {'prologue st':>11s} {'body st':>8s} {'body ld':>8s} {'epilogue ld':>11s}  (B/lane)")
    for f, (pro, st, ld, epi) in sorted(frame_split(sys.argv[1]).items(), key=lambda kv: -sum(kv[1])):
        if pro + st + ld + epi:
            name = re.sub(r"ttmpc::\(anonymous namespace\)::", "", demangle(f))[:70]
            print(f"{name:70s} {pro:11d} {st:8d} {ld:8d} {epi:11d}")
