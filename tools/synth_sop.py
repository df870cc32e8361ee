#!/usr/bin/env python3
"""Two-level (sum-of-products) synthesis of a multi-output Boolean function
into a v_bitop3_b32 network -- the alternative to tools/synth_bitop3.py's
BDD mapping (codegen tool, run at build time).

1. Cover: for each output choose a phase (cover the ON-set, or the OFF-set
   and complement at the end, which is free in a 3-input LUT).  Cover all
   outputs jointly with cubes grown greedily from uncovered minterms:
   literals are dropped one at a time, each time the one whose removal
   covers the most still-uncovered (output, minterm) pairs while the cube
   stays inside the chosen set of every output it serves; a cube may serve
   several outputs (shared products).  Redundant cubes are then removed.
   Several randomised restarts; the cheapest network wins.
2. Factor: literal pairs/triples that occur in many cubes become one AND
   node each (one bitop3), substituted back into the cubes.
3. Map: each cube's AND is folded 3 operands per bitop3 down to <= 2
   operands, and each output's OR absorbs one pending 2-operand product per
   bitop3 (x | (a & b)), so most cubes cost ceil(k/2) instructions.
The network is re-simulated on all 2^n input combinations before it is
written, so it computes exactly the tabled function (don't-cares included).
"""
from __future__ import annotations

import argparse
import itertools
import random
import sys

import numpy as np

TA, TB, TC = 0xF0, 0xCC, 0xAA


class Cover:
    def __init__(self, tt: np.ndarray, phases, rng):
        self.n = tt.shape[1].bit_length() - 1
        self.idx = np.arange(tt.shape[1], dtype=np.uint32)
        self.sets = [tt[o] if not ph else ~tt[o] for o, ph in enumerate(phases)]
        self.rng = rng

    def mask(self, care, val):
        return (self.idx & care) == val

    def expand(self, care, val, S, uncovered):
        cur = self.mask(care, val)
        while True:
            best = None
            for v in range(self.n):
                if not (care >> v) & 1:
                    continue
                m = cur | self.mask(care, val ^ (1 << v))
                if any((m & ~self.sets[o]).any() for o in S):
                    continue
                gain = sum(int((m & uncovered[o]).sum()) for o in S)
                key = (gain, self.rng.random())
                if best is None or key > best[0]:
                    best = (key, care & ~(1 << v), val & ~(1 << v), m)
            if best is None:
                return care, val, cur
            _, care, val, cur = best

    def run(self):
        nout = len(self.sets)
        unc = [s.copy() for s in self.sets]
        cubes = []
        full = (1 << self.n) - 1
        while any(u.any() for u in unc):
            o = max(range(nout), key=lambda k: int(unc[k].sum()))
            cand = np.flatnonzero(unc[o])
            m = int(cand[self.rng.randrange(len(cand))])
            others = [k for k in range(nout) if k != o and self.sets[k][m]]
            best = None
            for r in range(len(others) + 1):
                for extra in itertools.combinations(others, r):
                    S = (o,) + extra
                    care, val, cm = self.expand(full, m, S, unc)
                    gain = sum(int((cm & unc[k]).sum()) for k in S)
                    lits = bin(care).count("1")
                    cost = max(1, (lits + 1) // 2) + len(S) - 1
                    key = (gain / cost, gain)
                    if best is None or key > best[0]:
                        best = (key, care, val, S, cm)
            _, care, val, S, cm = best
            cubes.append([care, val, set(S)])
            for k in S:
                unc[k] &= ~cm
        # irredundant: drop (cube, output) uses that other cubes fully cover
        cnt = [np.zeros(len(self.idx), np.int32) for _ in range(nout)]
        ms = [self.mask(c, v) for c, v, _ in cubes]
        for (c, v, S), m in zip(cubes, ms):
            for k in S:
                cnt[k] += m
        order = sorted(range(len(cubes)), key=lambda i: bin(cubes[i][0]).count("1"), reverse=True)
        for i in order:
            m = ms[i]
            for k in sorted(cubes[i][2]):
                if (cnt[k][m] >= 2).all():
                    cnt[k] -= m
                    cubes[i][2].discard(k)
        return [(c, v, S) for c, v, S in cubes if S]


class Net:
    """bitop3 network builder with operands (signal, negated)."""

    def __init__(self, nvar):
        self.nvar = nvar
        self.ops = []  # (name, table, a, b, c) ; a/b/c are signal names
        self.k = 0

    def new(self, table, a, b, c):
        name = f"t{self.k}"
        self.k += 1
        self.ops.append((name, table & 0xFF, a, b, c))
        return name

    @staticmethod
    def _lit(base, neg):
        return (base ^ 0xFF) if neg else base

    def and_(self, opers):
        """AND of 2 or 3 operands -> (signal, False)."""
        if len(opers) == 2:
            (a, na), (b, nb) = opers
            t = self._lit(TA, na) & self._lit(TB, nb)
            return (self.new(t, a, b, a), False)
        (a, na), (b, nb), (c, nc) = opers
        t = self._lit(TA, na) & self._lit(TB, nb) & self._lit(TC, nc)
        return (self.new(t, a, b, c), False)

    def or3(self, opers):
        (a, na), (b, nb), *rest = opers
        if rest:
            (c, nc), = rest
            t = self._lit(TA, na) | self._lit(TB, nb) | self._lit(TC, nc)
            return (self.new(t, a, b, c), False)
        t = self._lit(TA, na) | self._lit(TB, nb)
        return (self.new(t, a, b, a), False)

    def or_pair(self, x, pair):
        (s, ns), ((a, na), (b, nb)) = x, pair
        t = self._lit(TA, ns) | (self._lit(TB, na) & self._lit(TC, nb))
        return (self.new(t, s, a, b), False)

    def reduce_and(self, opers):
        """Fold to <= 2 operands, 3 at a time."""
        opers = list(opers)
        while len(opers) > 2:
            take = opers[:3] if len(opers) != 4 else opers[:3]
            opers = [self.and_(take)] + opers[3:]
        return opers


def factor(cubes, nvar, min_uses=3):
    """Greedy extraction of shared literal pairs/triples; returns (cubes as
    operand lists, extracted definitions)."""
    lists = []
    for care, val, S in cubes:
        lits = [(f"x[{v}]", not ((val >> v) & 1)) for v in range(nvar) if (care >> v) & 1]
        lists.append([set(lits), S])
    defs = []
    while True:
        best = None
        for size in (3, 2):
            cnt = {}
            for L, _ in lists:
                if len(L) < size:
                    continue
                for comb in itertools.combinations(sorted(L), size):
                    cnt[comb] = cnt.get(comb, 0) + 1
            for comb, f in cnt.items():
                saving = f * (size - 1) / 2.0 - 1.0
                if f >= min_uses and (best is None or saving > best[0]):
                    best = (saving, comb)
        if best is None or best[0] <= 0:
            break
        comb = best[1]
        name = f"f{len(defs)}"
        defs.append((name, list(comb)))
        for L, _ in lists:
            if set(comb) <= L:
                L.difference_update(comb)
                L.add((name, False))
    return lists, defs


def build(cubes, phases, nvar, nout, do_factor=True):
    net = Net(nvar)
    lists, defs = factor(cubes, nvar) if do_factor else factor(cubes, nvar, min_uses=10 ** 9)
    sig = {}
    for name, comb in defs:  # definitions may reference earlier factors
        ops = [(sig.get(s, s), n) for s, n in comb]
        r = net.and_(ops) if len(ops) >= 2 else ops[0]
        sig[name] = r[0]
    # Accumulate each product into its outputs as soon as it exists, so only
    # a running OR (plus at most two pending singles) per output stays live:
    # this keeps the network's register footprint small.
    acc = [None] * nout                   # running OR per output (single operand)
    pend = [[] for _ in range(nout)]      # pending single operands per output

    def push_single(k, s):
        pend[k].append(s)
        if acc[k] is not None and len(pend[k]) == 2:
            acc[k] = net.or3([acc[k]] + pend[k])
            pend[k].clear()
        elif acc[k] is None and len(pend[k]) == 3:
            acc[k] = net.or3(pend[k])
            pend[k].clear()

    for L, S in lists:
        opers = sorted((sig.get(s, s), n) for s, n in L)
        red = net.reduce_and(opers)
        if len(S) > 1 or len(red) == 1:
            single = red[0] if len(red) == 1 else net.and_(red)
            for k in sorted(S):
                push_single(k, single)
        else:
            (k,) = tuple(S)
            if acc[k] is None and pend[k]:
                acc[k], pend[k] = pend[k][0], pend[k][1:]
            if acc[k] is None:
                acc[k] = net.and_(red)
            else:
                acc[k] = net.or_pair(acc[k], tuple(red))
    outs = []
    for k in range(nout):
        items = ([acc[k]] if acc[k] is not None else []) + pend[k]
        while len(items) > 1:
            items = [net.or3(items[:3])] + items[3:]
        if not items:
            outs.append(("0", phases[k]))
        else:
            s, neg = items[0]
            outs.append((s, neg ^ bool(phases[k])))
    return net, outs


def simulate(net, outs, nvar):
    n = 1 << nvar
    idx = np.arange(n, dtype=np.uint32)
    val = {f"x[{i}]": ((idx >> i) & 1).astype(bool) for i in range(nvar)}
    val["0"] = np.zeros(n, bool)
    for name, tab, a, b, c in net.ops:
        va, vb, vc = val[a], val[b], val[c]
        out = np.zeros(n, bool)
        for bit in range(8):
            if (tab >> bit) & 1:
                out |= (va == bool((TA >> bit) & 1)) & (vb == bool((TB >> bit) & 1)) & \
                       (vc == bool((TC >> bit) & 1))
        val[name] = out
    return np.stack([~val[s] if neg else val[s] for s, neg in outs])


def emit(net, outs, out_names, header):
    lines = list(header)
    for name, tab, a, b, c in net.ops:
        lines.append(f"  const T {name} = lut3<0x{tab:02X}>({a}, {b}, {c});")
    for nm, (s, neg) in zip(out_names, outs):
        src = "T(0)" if s == "0" else s
        lines.append(f"  {nm} = {'~' if neg else ''}{src};")
    return lines


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tt")
    ap.add_argument("out")
    ap.add_argument("--restarts", type=int, default=3)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--phases", default="", help="e.g. 111: only this output-phase combination")
    args = ap.parse_args()
    d = np.load(args.tt)
    tt = d["tt"].astype(bool)
    names = [str(s) for s in d["inputs"]]
    out_names = [str(s) for s in d["outputs"]]
    nvar, nout = tt.shape[1].bit_length() - 1, tt.shape[0]
    rng = random.Random(args.seed)
    log = lambda *a: print(*a, file=sys.stderr, flush=True)  # noqa: E731
    best = None
    combos = ([tuple(int(c) for c in args.phases)] if args.phases
              else list(itertools.product((0, 1), repeat=nout)))
    for phases in combos:
        for r in range(args.restarts):
            cubes = Cover(tt, phases, rng).run()
            for fac in (True, False):
                net, outs = build(cubes, phases, nvar, nout, fac)
                log(f"phases {phases} restart {r} factor {fac}: {len(cubes)} cubes, {len(net.ops)} ops")
                if best is None or len(net.ops) < len(best[0].ops):
                    best = (net, outs, phases, len(cubes))
    net, outs, phases, ncubes = best
    sim = simulate(net, outs, nvar)
    assert (sim == tt).all(), "SOP network differs from the truth table"
    hdr = [
        "// GENERATED by tools/synth_sop.py from " + args.tt.split("/")[-1] + " -- do not edit.",
        f"// {len(net.ops)} v_bitop3_b32 per 32-bit half: {ncubes} cubes, output phases {phases}",
        "// inputs x[i]: " + ", ".join(f"{i}={n}" for i, n in enumerate(names)),
        f"// verified against the full 2^{nvar}-entry truth table before writing.",
    ]
    with open(args.out, "w") as f:
        f.write("\n".join(emit(net, outs, out_names, hdr)) + "\n")
    log(f"wrote {args.out}: {len(net.ops)} ops, {ncubes} cubes, phases {phases}")


if __name__ == "__main__":
    main()
