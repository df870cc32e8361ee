#!/usr/bin/env python3
"""Synthesises a v_bitop3_b32 circuit for a multi-output Boolean function
given as a full truth table (measurement/codegen tool, run at build time).

Method: a shared, reduced, ordered BDD with complement edges.  Every BDD node
ITE(v, hi, lo) -- with either child possibly complemented -- is ONE
v_bitop3_b32 (a 3-input LUT), and a node that is just a literal costs
nothing.  The variable order is searched by sifting from several random
starts, minimising the number of non-literal nodes (= instructions).  The
emitted circuit is re-simulated on all 2^n input combinations before it is
written, so it is exactly the tabled function (don't-cares included).

Used for config 5: the truth table of bitslicing/unknown_step_refined.hpp
(16 inputs, 3 outputs) extracted from the reference build
(tests/golden/make_golden.py -> tests/golden/unknown_step_refined_tt.npz).
"""
from __future__ import annotations

import argparse
import random
import sys

import numpy as np

TA, TB, TC = 0xF0, 0xCC, 0xAA


def level_tables(tt: np.ndarray, order: list[int]) -> list[np.ndarray]:
    """tt: (outputs, 2^n) bool, index bit i = variable i.  Returns, per level
    k, the (outputs*2^k, 2^(n-k)) matrix of sub-tables below the first k
    variables of `order` (order[0] = top)."""
    nvar = tt.shape[1].bit_length() - 1
    nout = tt.shape[0]
    # axis j of reshape([2]*n) is variable n-1-j
    cube = tt.reshape([nout] + [2] * nvar)
    axes = [0] + [1 + (nvar - 1 - v) for v in order]
    t = np.ascontiguousarray(cube.transpose(axes))
    return [t.reshape(nout * (1 << k), 1 << (nvar - k)) for k in range(nvar + 1)]


def _norm(rows: np.ndarray):
    flip = rows[:, 0].copy()
    return rows ^ flip[:, None], flip


def count_nodes(tt: np.ndarray, order: list[int]) -> int:
    """Non-literal BDD nodes (complement edges) for this order."""
    nvar = len(order)
    total = 0
    for k, m in enumerate(level_tables(tt, order)[:nvar]):
        rows, _ = _norm(m)
        half = rows.shape[1] // 2
        dep = (rows[:, :half] != rows[:, half:]).any(axis=1)
        rows = rows[dep]
        if rows.size == 0:
            continue
        packed = np.packbits(rows, axis=1)
        uniq = np.unique(packed.view(np.dtype((np.void, packed.shape[1]))))
        # a literal node: lo = const 0 and hi = const 1 (after normalisation)
        u = np.unpackbits(uniq.view(np.uint8).reshape(len(uniq), -1), axis=1)[:, :rows.shape[1]]
        lit = (~u[:, :half].any(axis=1)) & u[:, half:].all(axis=1)
        total += int(len(uniq) - lit.sum())
    return total


def sift(tt, order, rounds=2, log=None):
    best = count_nodes(tt, order)
    for _ in range(rounds):
        improved = False
        for v in list(order):
            cur = [x for x in order if x != v]
            cands = []
            for pos in range(len(order)):
                o = cur[:pos] + [v] + cur[pos:]
                cands.append((count_nodes(tt, o), o))
            c, o = min(cands, key=lambda z: z[0])
            if c < best:
                best, order, improved = c, o, True
        if log:
            log(f"  sift pass: {best}")
        if not improved:
            break
    return best, order


class Circuit:
    """Builds the BDD for a fixed order and emits bitop3 instructions."""

    def __init__(self, tt, order, names):
        self.tt, self.order, self.names = tt, order, names
        self.nvar = len(order)
        self.nodes = {}       # key -> node id
        self.ops = []         # (id, var, hi(id,neg), lo(id,neg))
        self.literal = {}     # node id -> var (pure literal nodes)
        self.next_id = 1      # 0 = constant FALSE

    def build(self):
        outs = []
        for o in range(self.tt.shape[0]):
            perm = level_tables(self.tt[o:o + 1], self.order)[0][0]
            outs.append(self._node(perm, 0))
        return outs

    def _node(self, table: np.ndarray, level: int):
        """table: bool sub-table over variables order[level:] (top first)."""
        neg = bool(table[0])
        t = table ^ neg
        if not t.any():
            return (0, neg)
        while True:
            half = t.size // 2
            lo, hi = t[:half], t[half:]
            if (lo == hi).all():
                t, level = lo, level + 1
                continue
            break
        key = (level, t.tobytes())
        if key in self.nodes:
            return (self.nodes[key], neg)
        v = self.order[level]
        hi_ref = self._node(hi, level + 1)
        lo_ref = self._node(lo, level + 1)
        nid = self.next_id
        self.next_id += 1
        self.nodes[key] = nid
        if hi_ref == (0, True) and lo_ref == (0, False):
            self.literal[nid] = v
        else:
            self.ops.append((nid, v, hi_ref, lo_ref))
        return (nid, neg)

    def emit(self, outs, out_names, fn_name="refined_circuit"):
        """C++ body: inputs x[0..n) (W), returns outputs via references."""
        def ref(r):
            nid, neg = r
            if nid == 0:
                return None, neg
            if nid in self.literal:
                return f"x[{self.literal[nid]}]", neg
            return f"t{nid}", neg

        lines = []
        for nid, v, hi, lo in self.ops:  # children were appended first: topological
            a = f"x[{v}]"
            (hn, hneg), (ln, lneg) = ref(hi), ref(lo)
            # f = ITE(a, hi, lo) on the 3 bitop3 inputs (a, h, l)
            B = (TB ^ 0xFF) if hneg else TB
            C = (TC ^ 0xFF) if lneg else TC
            if hn is None:
                B = 0xFF if hneg else 0x00
                hn = a
            if ln is None:
                C = 0xFF if lneg else 0x00
                ln = a
            table = ((TA & B) | (~TA & C)) & 0xFF
            lines.append(f"  const T t{nid} = lut3<0x{table:02X}>({a}, {hn}, {ln});")
        for name, r in zip(out_names, outs):
            n, neg = ref(r)
            if n is None:
                lines.append(f"  {name} = {'~T(0)' if neg else 'T(0)'};")
            elif neg:
                lines.append(f"  {name} = ~{n};")
            else:
                lines.append(f"  {name} = {n};")
        return lines

    def simulate(self, outs) -> np.ndarray:
        """Evaluate the emitted circuit on all 2^n inputs."""
        n = 1 << self.nvar
        idx = np.arange(n, dtype=np.uint32)
        x = [((idx >> i) & 1).astype(bool) for i in range(self.nvar)]
        val = {}

        def get(r):
            nid, neg = r
            if nid == 0:
                v = np.zeros(n, bool)
            elif nid in self.literal:
                v = x[self.literal[nid]]
            else:
                v = val[nid]
            return ~v if neg else v

        for nid, v, hi, lo in self.ops:
            val[nid] = np.where(x[v], get(hi), get(lo))
        return np.stack([get(r) for r in outs])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tt", help=".npz with 'tt' (outputs, 2^n) uint8/bool and 'inputs', 'outputs'")
    ap.add_argument("out", help="generated .inc path")
    ap.add_argument("--restarts", type=int, default=6)
    ap.add_argument("--seed", type=int, default=1)
    args = ap.parse_args()
    d = np.load(args.tt)
    tt = d["tt"].astype(bool)
    names = [str(s) for s in d["inputs"]]
    out_names = [str(s) for s in d["outputs"]]
    nvar = tt.shape[1].bit_length() - 1
    rng = random.Random(args.seed)
    log = lambda *a: print(*a, file=sys.stderr)  # noqa: E731
    best = (count_nodes(tt, list(range(nvar))), list(range(nvar)))
    log(f"identity order: {best[0]}")
    for r in range(args.restarts):
        o = list(range(nvar))
        if r:
            rng.shuffle(o)
        c, o = sift(tt, o, rounds=3, log=log)
        log(f"restart {r}: {c}")
        if c < best[0]:
            best = (c, o)
    cnt, order = best
    circ = Circuit(tt, order, names)
    outs = circ.build()
    sim = circ.simulate(outs)
    assert (sim == tt).all(), "synthesised circuit differs from the truth table"
    assert len(circ.ops) == cnt, (len(circ.ops), cnt)
    lines = circ.emit(outs, out_names)
    hdr = [
        "// GENERATED by tools/synth_bitop3.py from " + args.tt.split("/")[-1] + " -- do not edit.",
        f"// {len(circ.ops)} v_bitop3_b32 per 32-bit half; variable order (top first): "
        + ", ".join(names[v] for v in order),
        "// inputs x[i]: " + ", ".join(f"{i}={n}" for i, n in enumerate(names)),
        "// verified against the full 2^16-entry truth table before writing.",
    ]
    with open(args.out, "w") as f:
        f.write("\n".join(hdr + lines) + "\n")
    log(f"wrote {args.out}: {len(circ.ops)} ops")


if __name__ == "__main__":
    main()
