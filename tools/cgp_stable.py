#!/usr/bin/env python3
"""Smaller v_bitop3 networks for the LifeStable fragments, exact wherever the
kernels' inputs can actually be.

The fragments (bitslicing/stable_count.hpp, stable_signal.hpp,
stable_vulnerable.hpp) are functions of neighbourhood-count bits and option
planes.  Counts come from NeighbourCount (NeighbourCount.hpp:40-70, the
inclusive 3x3 count) of planes of the same LifeStable, so for ANY plane
contents only some input rows occur -- e.g. UpdateOptions' on-count
(state) and off-count (~unknown & ~state) count disjoint cells of one 3x3
block, and a centre that is on is counted in the on-count.  Rows that cannot
occur are don't-cares: the kernels never evaluate them, whatever the caller's
planes hold, so a network exact on the reachable rows computes exactly what
the reference's fragment computes on every input the kernels see.

  python tools/cgp_stable.py problem NAME       -> build/cgp/NAME.{bin,seed.txt}
      NAME in count, signal, vulnerable; the seed is the committed network
      (lifeapi_amd/csrc/stable_NAME_circuit.inc), exact on every row.
  ./build/cgp_circuit build/cgp/NAME.bin SEED OUT SECONDS RNG SPARE
      (tools/cgp_circuit.c) shrinks it, exact on the reachable rows.
  python tools/cgp_stable.py emit NAME OUT     -> the .inc, re-checked here on
      every reachable row against the reference-generated truth table
      (tests/golden/stable_NAME_tt.npz).

reachable_rows(NAME) is the care set; tests/test_oracle.py checks every
committed network against the table on it, and the GPU parity tests run the
kernels against the reference on arbitrary planes."""
from __future__ import annotations

import os
import re
import struct
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "lifeapi_amd", "csrc")
GOLD = os.path.join(ROOT, "tests", "golden")
OUT = os.path.join(ROOT, "build", "cgp")


def _bits(v: int, n: int):
    return [(v >> (n - 1 - k)) & 1 for k in range(n)]  # msb first (x[i] order: bit2, bit1, bit0)


def _row(xs) -> int:
    """the table's row index of input values x[0], x[1], ...: x[i] is bit i"""
    return sum(int(v) << i for i, v in enumerate(xs))


def reachable_rows(name: str) -> np.ndarray:
    """Input rows (as integers, input x[i] = bit i: the npz tables' row
    order) that NeighbourCount-derived inputs can take
    for any planes.  Each of the 8 neighbours and the centre is one cell;
    counts are inclusive."""
    rows = set()
    if name == "count":
        # x: on2 on1 on0 (state count mod 8), off3..off0 (count of ~unknown &
        # ~state), known_on = state, known_off = ~unknown & ~state (centre).
        # A cell is on (state), off, or neither (unknown & ~state); on and
        # off are disjoint.
        for centre in ("on", "off", "neither"):
            for a in range(9):          # neighbours on
                for b in range(9 - a):  # neighbours off
                    on = a + (centre == "on")
                    off = b + (centre == "off")
                    r = _bits(on % 8, 3) + _bits(off, 4) + [int(centre == "on"), int(centre == "off")]
                    rows.add(_row(r))
    elif name == "signal":
        # x: 8 option planes (any), s2 s1 s0 (state count mod 8), m3..m0
        # (count of state | unknown), stateon, stateunk (centre).  A cell is
        # in state (unknown anything), unknown only, or neither.
        cnt = set()
        for cs in (0, 1):
            for cu in (0, 1):
                for a in range(9):          # neighbours in state
                    for b in range(9 - a):  # neighbours unknown, not in state
                        s = a + cs
                        m = a + b + (cs | cu)
                        cnt.add(tuple(_bits(s % 8, 3) + _bits(m, 4) + [cs, cu]))
        for opt in range(256):
            ob = _bits(opt, 8)
            for c in cnt:
                rows.add(_row(ob + list(c)))
    elif name == "vulnerable":
        # x: 8 option planes, s2 s1 s0 (state count mod 8), unk3..unk0
        # (unknown count): state and unknown may overlap, so the two counts
        # are independent 0..9
        for opt in range(256):
            for s in range(10):
                for u in range(10):
                    rows.add(_row(_bits(opt, 8) + _bits(s % 8, 3) + _bits(u, 4)))
    else:
        raise SystemExit(f"unknown fragment {name}")
    return np.array(sorted(rows), dtype=np.int64)


def table(name: str):
    d = np.load(os.path.join(GOLD, f"stable_{name}_tt.npz"))
    return d["tt"].astype(np.uint8), [str(s) for s in d["inputs"]], [str(s) for s in d["outputs"]]


def inc_path(name: str) -> str:
    return os.path.join(CSRC, f"stable_{name}_circuit.inc")


_GATE = re.compile(r"const T t(\d+) = lut3<0x([0-9A-Fa-f]+)>\(([^,]+), ([^,]+), ([^)]+)\);")
_OUTL = re.compile(r"^\s*(\w+) = (~?)(t\d+|x\[\d+\]);")


def parse_inc(path: str, nin: int, out_names):
    """(gates [(fn, a, b, c)] with sources 0..nin-1 inputs, nin + k gate k;
    outputs [(node, inv)] in out_names order)"""
    gates, idx, outs = [], {}, {}

    def src(s):
        s = s.strip()
        if s.startswith("x["):
            return int(s[2:-1])
        return nin + idx[int(s[1:])]
    for ln in open(path):
        m = _GATE.search(ln)
        if m:
            idx[int(m.group(1))] = len(gates)
            gates.append((int(m.group(2), 16), src(m.group(3)), src(m.group(4)), src(m.group(5))))
            continue
        m = _OUTL.match(ln)
        if m and m.group(1) not in ("const",):
            outs[m.group(1)] = (src(m.group(3)), int(m.group(2) == "~"))
    return gates, [outs[n] for n in out_names]


def simulate(gates, outs, nin: int, rows: np.ndarray) -> np.ndarray:
    """outputs (nout, len(rows)) of the network on the given input rows"""
    x = [((rows >> i) & 1).astype(np.uint8) for i in range(nin)]
    vals = list(x)
    for fn, a, b, c in gates:
        k = (vals[a].astype(np.int64) << 2) | (vals[b].astype(np.int64) << 1) | vals[c].astype(np.int64)
        vals.append(((fn >> k) & 1).astype(np.uint8))
    return np.stack([vals[n] ^ inv for n, inv in outs])


def _pack(bits: np.ndarray, words: int) -> np.ndarray:
    pad = np.zeros(words * 64, np.uint8)
    pad[: len(bits)] = bits
    pad[len(bits):] = bits[0]  # padding rows repeat row 0 (exact there too)
    return np.packbits(pad.reshape(-1, 8)[:, ::-1], axis=1).reshape(-1).view(np.uint64)


def problem(name: str):
    tt, ins, outs_names = table(name)
    nin = len(ins)
    rows = reachable_rows(name)
    gates, outs = parse_inc(inc_path(name), nin, outs_names)
    got = simulate(gates, outs, nin, np.arange(1 << nin))
    assert (got == tt).all(), "the committed network is not the table"
    words = (len(rows) + 63) // 64
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, f"{name}.bin"), "wb") as f:
        f.write(struct.pack("<3i", nin, len(outs_names), words))
        for i in range(nin):
            f.write(_pack(((rows >> i) & 1).astype(np.uint8), words).tobytes())
        for o in range(len(outs_names)):
            f.write(_pack(tt[o][rows], words).tobytes())
    with open(os.path.join(OUT, f"{name}.seed.txt"), "w") as f:
        f.write(f"{len(gates)} {len(outs)}\n")
        for g in gates:
            f.write("%d %d %d %d\n" % g)
        for n, inv in outs:
            f.write(f"{n} {inv}\n")
    print(f"{name}: {nin} inputs, {len(outs_names)} outputs, {len(rows)} reachable rows of {1 << nin}, "
          f"seed {len(gates)} gates")


def load_result(path: str):
    with open(path) as f:
        g, no = map(int, f.readline().split())
        gates = [tuple(map(int, f.readline().split())) for _ in range(g)]
        outs = [tuple(map(int, f.readline().split())) for _ in range(no)]
    return gates, outs


def emit(name: str, result: str):
    tt, ins, outs_names = table(name)
    nin = len(ins)
    rows = reachable_rows(name)
    gates, outs = load_result(result)
    got = simulate(gates, outs, nin, rows)
    assert (got == tt[:, rows]).all(), "result is not exact on the reachable rows"
    lines = [f"// GENERATED by tools/cgp_stable.py + tools/cgp_circuit.c from stable_{name}_tt.npz -- do not edit.",
             f"// {len(gates)} v_bitop3_b32 per 32-bit half; exact on the {len(rows)} input rows of 2^{nin} that",
             "// NeighbourCount-derived inputs can take for any planes (cgp_stable.reachable_rows).",
             "// inputs x[i]: " + ", ".join(f"{i}={n}" for i, n in enumerate(ins))]

    def ref(s):
        return f"x[{s}]" if s < nin else f"t{s - nin}"
    for k, (fn, a, b, c) in enumerate(gates):
        lines.append(f"  const T t{k} = lut3<0x{fn:02X}>({ref(a)}, {ref(b)}, {ref(c)});")
    for nm, (n, inv) in zip(outs_names, outs):
        lines.append(f"  {nm} = {'~' if inv else ''}{ref(n)};")
    with open(inc_path(name), "w") as f:
        f.write("\n".join(lines) + "\n")
    print(f"{name}: {len(gates)} gates written to {os.path.relpath(inc_path(name), ROOT)}")


if __name__ == "__main__":
    if sys.argv[1] == "problem":
        problem(sys.argv[2])
    elif sys.argv[1] == "emit":
        emit(sys.argv[2], sys.argv[3])
    else:
        raise SystemExit(__doc__)
