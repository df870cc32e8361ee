#!/usr/bin/env python3
"""Generates the golden fixtures in tests/golden/ FROM THE REFERENCE ITSELF.

Run in the build container (needs oracle/_ref, i.e. /root/reference at build
time):  make -C oracle ref && python tests/golden/make_golden.py

Every expected output below is produced by the reference's own code
(LifeState::Step / StepAlt / NeighbourCount / Parse / RandomState / GetPop /
Contains, compiled from /root/reference by oracle/Makefile).  Inputs come from
the build-defined splitmix64 generator (oracle_fill), from the reference's
own RandomState(), or are hand-placed seam cases.  The fixtures are data only
(inputs + expected outputs).  Digest fixtures use the build-defined hash
(oracle_universe_hash / oracle_batch_digest), applied to reference outputs.
"""
from __future__ import annotations

import glob
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle.oracle import Port, Ref  # noqa: E402

P, R = Port(), Ref()

import ctypes  # noqa: E402

_u64p = ctypes.POINTER(ctypes.c_uint64)
R.lib.ref_unknown_step_refined.argtypes = [_u64p, _u64p]
R.lib.ref_refined_step_batch.argtypes = [_u64p, _u64p, ctypes.c_size_t]

# the fragment's input variables, in bitslicing/unknown_step_refined.py:105-113
# order with the live-count encoding the fragment was generated from
REFINED_INPUTS = ["l2", "l3", "d0", "d1", "d2", "d4", "d5", "d6", "current_unknown",
                  "current_on", "s2", "s1", "s0", "on2", "on1", "on0"]
REFINED_OUTPUTS = ["next_on", "next_unknown", "next_unknown_stable"]


def _p64(a):
    return a.ctypes.data_as(_u64p)


def fragment_truth_table(fn, nin: int, nout: int) -> np.ndarray:
    """(nout, 2^nin) uint8: output bits of a reference fragment wrapper `fn`
    (in words -> out words) for every input combination c (bit i of c = input
    i), evaluated 64 combinations per call."""
    rows = 1 << nin
    c = np.arange(rows, dtype=np.uint64).reshape(rows // 64, 64)
    shifts = np.arange(64, dtype=np.uint64)
    words = np.stack([(((c >> np.uint64(i)) & np.uint64(1)) << shifts).sum(axis=1, dtype=np.uint64)
                      for i in range(nin)])  # (nin, rows/64)
    out = np.zeros((nout, rows // 64), np.uint64)
    for w in range(rows // 64):
        a = np.ascontiguousarray(words[:, w])
        o = np.zeros(nout, np.uint64)
        fn(_p64(a), _p64(o))
        out[:, w] = o
    return np.unpackbits(out.view(np.uint8), bitorder="little").reshape(nout, rows)


def refined_truth_table() -> np.ndarray:
    return fragment_truth_table(R.lib.ref_unknown_step_refined, 16, 3)


STABLE_COUNT_INPUTS = ["on2", "on1", "on0", "off3", "off2", "off1", "off0", "known_on", "known_off"]
STABLE_COUNT_OUTPUTS = ["l2", "l3", "d0", "d1", "d2", "d4", "d5", "d6", "abort"]
STABLE_SIGNAL_INPUTS = ["l2", "l3", "d0", "d1", "d2", "d4", "d5", "d6", "s2", "s1", "s0",
                        "m3", "m2", "m1", "m0", "stateon", "stateunk"]
STABLE_SIGNAL_OUTPUTS = ["signaloff", "signalon", "centeroff", "centeron"]
STABLE_VULNERABLE_INPUTS = ["l2", "l3", "d0", "d1", "d2", "d4", "d5", "d6", "s2", "s1", "s0",
                            "unk3", "unk2", "unk1", "unk0"]
STABLE_VULNERABLE_OUTPUTS = ["vulnerable_on", "vulnerable_off", "vulnerable_center_on",
                             "vulnerable_center_off"]


def moved(s, dx, dy):
    """LifeState::Move on the torus (columns x+dx, rows y+dy)."""
    s = np.roll(np.asarray(s, np.uint64), dx)
    k = dy % 64
    return np.array([((int(w) << k) | (int(w) >> (64 - k))) & (2**64 - 1) if k else int(w)
                     for w in s], dtype=np.uint64)


def rect(x0, y0, w, h):
    col = ((1 << h) - 1) << y0
    s = np.zeros(64, np.uint64)
    s[x0:x0 + w] = np.uint64(col & (2**64 - 1))
    return s


def stable_inputs(n: int, seed: int = 8080) -> np.ndarray:
    """Seeded LifeStable planes {state, unknown, live2, live3, dead0, dead1,
    dead2, dead4, dead5, dead6}: still lifes around an unknown window with
    fresh options, sparse random soups around a window, and random planes."""
    rng = np.random.default_rng(seed)
    lifes = [R.parse(r) for r in ("2o$2o!", "b2o$o2bo$b2o!", "2o$obo$bo!", "2b2o$bobo$bo$2o!",
                                   "b2o$o2bo$bobo$2bo!", "bo$obo$bo!")]
    out = np.zeros((n, 10, 64), np.uint64)
    for u in range(n):
        kind = u % 3
        w, h = int(rng.integers(6, 24)), int(rng.integers(6, 24))
        x0, y0 = int(rng.integers(0, 64 - w)), int(rng.integers(0, 64 - h))
        unk = rect(x0, y0, w, h)
        if kind == 0:
            st = np.zeros(64, np.uint64)
            for _ in range(int(rng.integers(4, 12))):
                st |= moved(lifes[int(rng.integers(len(lifes)))], int(rng.integers(64)), int(rng.integers(64)))
            out[u, 0] = st & ~unk
            out[u, 1] = unk
        elif kind == 1:
            f = P.fill(2, seed=int(rng.integers(1 << 30)))
            out[u, 0] = f[0] & f[1] & ~unk
            out[u, 1] = unk
        else:
            f = P.fill(10, seed=int(rng.integers(1 << 30)))
            g = P.fill(10, seed=int(rng.integers(1 << 30)))
            h2 = P.fill(10, seed=int(rng.integers(1 << 30)))
            out[u, 0] = f[0]
            out[u, 1] = g[1] & unk
            out[u, 2:] = f[2:] & g[2:] & h2[2:]
    return out.reshape(n, 640)


def pop_words(s):
    return int(sum(bin(int(w)).count("1") for w in s))


def edge_cases():
    names, out = [], []

    def add(name, s):
        names.append(name)
        out.append(np.asarray(s, dtype=np.uint64).reshape(64))

    add("empty", np.zeros(64))
    add("all_on", np.full(64, 2**64 - 1, dtype=np.uint64))
    add("checkerboard", [0xAAAAAAAAAAAAAAAA if x % 2 == 0 else 0x5555555555555555 for x in range(64)])
    g = R.parse("bo$2bo$3o!")
    add("glider", g)
    add("glider_col_seam", np.roll(g, 62))
    add("glider_row_seam", [((int(w) << 62) | (int(w) >> 2)) & (2**64 - 1) for w in g])
    add("glider_corner", [((int(w) << 62) | (int(w) >> 2)) & (2**64 - 1) for w in np.roll(g, 62)])
    s = np.zeros(64, np.uint64)
    s[63] = s[0] = s[1] = np.uint64(1 << 63)          # blinker across column seam on row 63
    add("blinker_both_seams", s)
    s = np.zeros(64, np.uint64)
    s[0] = np.uint64((1 << 63) | 1)
    s[63] = np.uint64((1 << 63) | 1)                  # block split over all four corners
    add("block_corners", s)
    s = np.zeros(64, np.uint64)
    s[0] = s[63] = np.uint64(0xFFFFFFFFFFFFFFFF)      # two full columns on the seam
    add("full_seam_columns", s)
    s = np.zeros(64, np.uint64)
    for x in range(64):
        s[x] = np.uint64(1 << 0) | np.uint64(1 << 63)  # full rows 0 and 63
    add("full_seam_rows", s)
    add("single_cell_corner", [1 if x == 0 else 0 for x in range(64)])
    add("rpentomino", R.parse("b2o$2o$bo!"))
    add("eater_pair", (R.parse("2b2o$bobo$bo$2o!") | np.roll(R.parse("2b2o$bobo$bo$2o!"), 5)))
    add("randomstate_like", P.fill(1, 77, 0, 1)[0])
    add("dense_random", P.fill(1, 78)[0] | P.fill(1, 79)[0])
    return names, np.stack(out)


def batch_digests() -> dict:
    """6. batch digests (checksum of checksums over reference outputs) for
    the bench workloads and the shard layouts bench.py checks per rank."""
    dig = {}
    for name, n, seed, g in (("config2", 1 << 20, 2, 1), ("config3", 1 << 16, 3, 1024)):
        xin = P.fill(n, seed=seed)
        out = R.step_batch(xin, g, nthreads=8)
        dig[name] = {"universes": n, "seed": seed, "generations": g,
                     "input_digest": f"{P.digest(P.hashes(xin)):016x}",
                     "output_digest": f"{P.digest(P.hashes(out)):016x}",
                     "output_pop_total": int(P.pop(out).astype(np.uint64).sum())}
    # config 3 as the search loop (LifeTarget.hpp:44-51): Step() then
    # Contains() after every generation, a 2 x 2 block with its empty ring
    # as the target; batch_digest over the first-hit generations
    xin = P.fill(1 << 16, seed=3)
    wanted, unwanted = np.zeros(64, np.uint64), np.zeros(64, np.uint64)
    wanted[10] = wanted[11] = np.uint64(3 << 40)
    for c in (9, 10, 11, 12):
        unwanted[c] = np.uint64(15 << 39)
    unwanted &= ~wanted
    first, out = R.step_contains_batch(xin, wanted, unwanted, 1024, nthreads=8)
    dig["config3_contains"] = {
        "universes": 1 << 16, "seed": 3, "generations": 1024,
        "wanted": [f"{int(v):016x}" for v in wanted], "unwanted": [f"{int(v):016x}" for v in unwanted],
        "first_digest": f"{P.digest(first.astype(np.uint64)):016x}", "hits": int((first > 0).sum()),
        "output_digest": f"{P.digest(P.hashes(out)):016x}"}
    # config 4: 16M universes, 8 shards of 2M; additive digests per shard
    shard, total, totin = [], 0, 0
    for k in range(8):
        xin = P.fill(1 << 21, seed=4, first_universe=k << 21)
        out = R.step_batch(xin, 1, nthreads=8)
        di = P.digest(P.hashes(xin), k << 21)
        do = P.digest(P.hashes(out), k << 21)
        shard.append(f"{do:016x}")
        total = (total + do) % 2**64
        totin = (totin + di) % 2**64
    dig["config4"] = {"universes": 1 << 24, "seed": 4, "generations": 1, "shards": 8,
                      "input_digest": f"{totin:016x}", "output_digest": f"{total:016x}",
                      "shard_output_digests": shard}
    # bench.py weak scaling: rank r owns [r*2^20, (r+1)*2^20) of the seed-2 array;
    # Step^1 output digest of each rank's shard (rank 0 == config 2)
    weak = []
    for k in range(8):
        xin = P.fill(1 << 20, seed=2, first_universe=k << 20)
        weak.append(f"{P.digest(P.hashes(R.step_batch(xin, 1, nthreads=8)), k << 20):016x}")
    dig["weak_shards_seed2"] = {"universes_per_rank": 1 << 20, "seed": 2, "generations": 1,
                                "shard_output_digests": weak}
    # the same shard layouts at test sizes (tests/test_bench_ranks.py runs
    # bench.py's rank path on them): config 4 as 16K universes in 8 chunks of
    # 2K, config 2's weak shards as 2K universes per rank
    shard, total = [], 0
    for k in range(8):
        xin = P.fill(1 << 11, seed=4, first_universe=k << 11)
        do = P.digest(P.hashes(R.step_batch(xin, 1)), k << 11)
        shard.append(f"{do:016x}")
        total = (total + do) % 2**64
    dig["config4_small"] = {"universes": 1 << 14, "seed": 4, "generations": 1, "shards": 8,
                            "output_digest": f"{total:016x}", "shard_output_digests": shard}
    weak = []
    for k in range(8):
        xin = P.fill(1 << 11, seed=2, first_universe=k << 11)
        weak.append(f"{P.digest(P.hashes(R.step_batch(xin, 1)), k << 11):016x}")
    dig["weak_shards_seed2_small"] = {"universes_per_rank": 1 << 11, "seed": 2, "generations": 1,
                                      "shard_output_digests": weak}
    return dig


def filter_targets():
    """The search-filter targets of bench.py's secondary.filter: the config-3
    block + ring (care columns 9-12) and a whole-board one (row 10 of every
    third column must be dead: a care window of 62 columns, K = 64 at g = 1)"""
    bw, bu = np.zeros(64, np.uint64), np.zeros(64, np.uint64)
    bw[10] = bw[11] = np.uint64(3 << 40)
    for c in (9, 10, 11, 12):
        bu[c] = np.uint64(15 << 39)
    bu &= ~bw
    ww, wu = np.zeros(64, np.uint64), np.zeros(64, np.uint64)
    wu[0::3] = np.uint64(1 << 10)
    return {"block": (bw, bu), "whole_board": (ww, wu)}


def filter_digests() -> dict:
    """The 1- and 2-generation search filter and batched Contains on the config-2
    input (1M universes, seed 2): the reference's own Step() + Contains and
    Contains (ref_shim.cpp), as digests of the per-universe answers"""
    x = P.fill(1 << 20, seed=2)
    out = {"universes": 1 << 20, "seed": 2, "generations": 1, "targets": {}}
    for name, (w, u) in filter_targets().items():
        first, _ = R.step_contains_batch(x, w, u, 1, nthreads=8)
        first2, _ = R.step_contains_batch(x, w, u, 2, nthreads=8)
        cont = R.contains_batch(x, w, u)
        out["targets"][name] = {
            "wanted": [f"{int(v):016x}" for v in w], "unwanted": [f"{int(v):016x}" for v in u],
            "first_digest": f"{P.digest(first.astype(np.uint64)):016x}", "hits": int((first > 0).sum()),
            "first_digest_2gen": f"{P.digest(first2.astype(np.uint64)):016x}", "hits_2gen": int((first2 > 0).sum()),
            "contains_digest": f"{P.digest(cont.astype(np.uint64)):016x}", "contained": int(cont.sum())}
    return out


def full_height_target():
    """A whole-board target whose care cells sit in every fourth row, one per
    row at column 3y mod 64, all required dead: no column window, no row
    window (its care rows leave no run of 4 empty rows), so the iterated
    filter runs the full board in the split layout; 16 dead cells are
    found in about 0.3 % of stepped random universes, so the answers carry
    first hits at every generation count"""
    w, u = np.zeros(64, np.uint64), np.zeros(64, np.uint64)
    for y in range(0, 64, 4):
        u[(3 * y) % 64] |= np.uint64(1 << y)
    return w, u


FILTER_ITER_GENS = {"block": (5, 8, 13), "whole_board": (5, 8), "full_height": (1, 2, 3, 5, 8)}


def filter_iter_digests() -> dict:
    """The iterated search filter (first hits only, 3-13 generations) on the
    config-2 input (1M universes, seed 2): the reference's own loop of Step()
    then Contains(LifeTarget) after every generation (ref_shim.cpp
    ref_step_contains_batch), as digests of the per-universe first-hit
    generations -- bench.py secondary_filter_iter's check"""
    x = P.fill(1 << 20, seed=2)
    tg = dict(filter_targets())
    tg["full_height"] = full_height_target()
    out = {"universes": 1 << 20, "seed": 2, "targets": {}}
    for name, (w, u) in tg.items():
        row = {"wanted": [f"{int(v):016x}" for v in w], "unwanted": [f"{int(v):016x}" for v in u], "gens": {}}
        for g in FILTER_ITER_GENS[name]:
            first, _ = R.step_contains_batch(x, w, u, g, nthreads=8)
            row["gens"][str(g)] = {"first_digest": f"{P.digest(first.astype(np.uint64)):016x}",
                                   "hits": int((first > 0).sum())}
        out["targets"][name] = row
    return out


def config5_digest() -> dict:
    """Config 5 at bench size: 256K universes of 11 planes (the seed-6
    splitmix64 fill of 256K x 11 universes, bench.py secondary_config5)
    through the reference's unknown_step_refined.hpp fragment in the
    harness (ref_shim.cpp); batch digest of the 3 output planes taken as
    3 x 256K consecutive 64-word blocks"""
    n = 1 << 18
    xin = P.fill(n * 11, seed=6).reshape(n, 11 * 64)
    out = R.refined_step(xin)
    return {"universes": n, "seed": 6, "planes_in": 11, "planes_out": 3,
            "output_digest": f"{P.digest(P.hashes(out.reshape(n * 3, 64))):016x}"}


def main():
    if "--only-config5" in sys.argv:  # add / refresh digests.config5 alone
        path = os.path.join(HERE, "golden.json")
        with open(path) as f:
            meta = json.load(f)
        meta["digests"]["config5"] = config5_digest()
        with open(path, "w") as f:
            json.dump(meta, f, indent=1)
        print(json.dumps(meta["digests"]["config5"], indent=1))
        return
    if "--only-filter-iter" in sys.argv:  # add / refresh digests.config2_filter_iter alone
        path = os.path.join(HERE, "golden.json")
        with open(path) as f:
            meta = json.load(f)
        meta["digests"]["config2_filter_iter"] = filter_iter_digests()
        with open(path, "w") as f:
            json.dump(meta, f, indent=1)
        print(json.dumps(meta["digests"]["config2_filter_iter"]["targets"], indent=1))
        return
    if "--only-filter" in sys.argv:  # add / refresh digests.config2_filter alone
        path = os.path.join(HERE, "golden.json")
        with open(path) as f:
            meta = json.load(f)
        meta["digests"]["config2_filter"] = filter_digests()
        with open(path, "w") as f:
            json.dump(meta, f, indent=1)
        print(json.dumps(meta["digests"]["config2_filter"]["targets"], indent=1))
        return
    meta = {"generator": "tests/golden/make_golden.py", "reference_lib": os.path.basename(R.path),
            "reference": "scorbiclife/LifeAPI snapshot 2025-02-22 (/root/reference)"}

    # 1. R-pentomino known answer, LifeAPI.hpp:1196 Step(), population trace 0..1103
    r = R.parse("b2o$2o$bo!")
    trace, s = [pop_words(r)], r.copy()
    for _ in range(1103):
        s = R.step_batch(s[None], 1)[0]
        trace.append(pop_words(s))
    np.savez(os.path.join(HERE, "rpentomino.npz"), initial=r, final=s,
             pop_trace=np.array(trace, dtype=np.uint16))
    meta["rpentomino"] = {"rle": "b2o$2o$bo!", "generations": 1103, "final_pop": trace[-1],
                          "pop_at": {g: trace[g] for g in (0, 1, 2, 10, 100, 500, 1000, 1103)}}

    # 2. seeded uniform random universes: Step^1, Step^1024
    x = P.fill(256, seed=12345)
    np.savez(os.path.join(HERE, "random_step.npz"), input=x, step1=R.step_batch(x, 1),
             step1024=R.step_batch(x, 1024))
    meta["random_step"] = {"n": 256, "seed": 12345, "mode": "uniform", "gens": [1, 1024]}

    # 3. seam / edge cases: Step^g for g in 1, 2, 3, 4, 64, 256
    names, e = edge_cases()
    gens = [1, 2, 3, 4, 64, 256]
    np.savez(os.path.join(HERE, "edge_cases.npz"), input=e, gens=np.array(gens),
             **{f"step{g}": R.step_batch(e, g) for g in gens})
    meta["edge_cases"] = {"names": names, "gens": gens}

    # 4. the reference's own RandomState() distribution (StepAltTest.cpp:5-13):
    #    Step, StepAlt and the NeighbourCount rule all from the reference
    #    (RandomState is random_device seeded: keep the committed draws unless
    #    --refresh-randomstate, and re-check them against the reference)
    kat = os.path.join(HERE, "randomstate_kat.npz")
    if os.path.exists(kat) and "--refresh-randomstate" not in sys.argv:
        rs = np.load(kat)["input"]
    else:
        rs = np.stack([R.random_state() for _ in range(256)])
    st = R.step_batch(rs, 1)
    assert (R.step_alt(rs) == st).all() and (R.step_nc(rs) == st).all()
    nc = np.stack([R.neighbour_count(rs[u]) for u in range(32)])
    np.savez(kat, input=rs, step=st, neighbour_count=nc)
    meta["randomstate_kat"] = {"n": 256, "source": "LifeState::RandomState() (random_device seeded)",
                               "neighbour_count_for_first": 32, "planes": "bit3,bit2,bit1,bit0"}

    # 5. Contains(LifeTarget) (LifeTarget.hpp:44-51) on stepped random states
    w = R.parse("2o$2o!")
    wanted = np.roll(w, 20)
    unwanted = np.zeros(64, np.uint64)
    unwanted[19] = unwanted[22] = np.uint64(0xF)
    unwanted[20] |= np.uint64(0x4)
    unwanted[21] |= np.uint64(0x4)
    y = P.fill(64, seed=31337)
    y[:16] = 0
    y[:8, 20] = y[:8, 21] = np.uint64(3)
    y[8:12, 20] = y[8:12, 21] = np.uint64(3)
    y[8:12, 19] = np.uint64(1)   # neighbouring cell -> unwanted violated
    cont = np.array([R.contains(y[u], wanted, unwanted) for u in range(64)], dtype=np.uint8)
    np.savez(os.path.join(HERE, "contains.npz"), states=y, wanted=wanted, unwanted=unwanted,
             contains=cont)
    meta["contains"] = {"n": 64, "true": int(cont.sum())}

    # 5a. neighbourhood counters: NeighbourCount planes and
    #     InteractionCountsAndNext planes, from the reference, on edge cases +
    #     32 seeded universes
    cin = np.concatenate([e, P.fill(32, seed=4242)])
    ncs = np.stack([R.neighbour_count(cin[u]) for u in range(len(cin))])
    ics = np.stack([R.interaction_counts(cin[u]) for u in range(len(cin))])
    np.savez(os.path.join(HERE, "counts.npz"), input=cin, neighbour_count=ncs,
             interaction_counts=ics)
    meta["counts"] = {"n": int(len(cin)), "neighbour_count_planes": "bit3,bit2,bit1,bit0",
                      "interaction_planes": "out1,out2,outMore,next"}

    # 5c. LifeWeld::Step (LifeWeld.hpp:169-186): the RequiredTest welds of
    #     tests/LifeWeldTest.cpp:19-33 built by the reference's FromRequired
    #     (must be invariant), plus seeded random welds stepped 1 and 7 times
    R.lib.ref_weld_from_required.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int,
                                             ctypes.c_int, _u64p]
    req = [("2b2o$bobo$bo$2o!", "2b2o$b3o$b4o$5o$4o$4o!"),
           ("2o$o2bob2o$b3obobo$5bobo$b5ob3o$bo4bo3bo$4bobo2b2o$4b2o!",
            "4o$5o2bo$4o$5o4bo$b5ob5o$b12o$b12o$b12o$4b9o$4b4o!"),
           ("4b2ob2o$3bobobobo$b3o3bobo$o4bobob3o$b3ob2obo3bo$3bo4bo2b2o$5b3o$4b2o!",
            "4b2o$3b2o2bo2b2o$b4o6bo$6obob5o$15o$15o$b14o$3b12o$4b6o$4b4o!")]
    req_welds = np.zeros((len(req), 256), np.uint64)
    for i, (srle, rrle) in enumerate(req):
        R.lib.ref_weld_from_required(srle.encode(), rrle.encode(), -1, -1, _p64(req_welds[i]))
    rw = P.fill(64 * 4, seed=6060).reshape(64, 256)
    rw[:, 64:] &= P.fill(64 * 3, seed=6061).reshape(64, 192) & P.fill(64 * 3, seed=6062).reshape(64, 192)
    wel = np.concatenate([req_welds, rw])
    np.savez(os.path.join(HERE, "weld.npz"), input=wel, step1=R.weld_step(wel, 1),
             step7=R.weld_step(wel, 7), n_required=len(req))
    meta["weld"] = {"n": int(len(wel)), "required_examples": len(req),
                    "layout": "state,frozen2,frozen1,frozen0"}

    stable_fixture(meta)

    # 5b. config 5: bitslicing/unknown_step_refined.hpp (the reference's espresso
    #     fragment) as a complete truth table over its 16 inputs, plus seeded
    #     11-plane universes through the build-defined harness (ref_shim.cpp)
    tt = refined_truth_table()
    np.savez_compressed(os.path.join(HERE, "unknown_step_refined_tt.npz"), tt=tt,
                        inputs=np.array(REFINED_INPUTS), outputs=np.array(REFINED_OUTPUTS))
    xin = P.fill(64 * 11, seed=5).reshape(64, 11 * 64)
    rout = np.zeros((64, 3 * 64), np.uint64)
    R.lib.ref_refined_step_batch(_p64(xin), _p64(rout), 64)
    np.savez(os.path.join(HERE, "refined_step.npz"), input=xin, output=rout)
    meta["unknown_step_refined"] = {"inputs": REFINED_INPUTS, "outputs": REFINED_OUTPUTS,
                                    "ones_per_output": [int(v) for v in tt.sum(axis=1)],
                                    "harness_universes": 64, "harness_seed": 5,
                                    "planes_in": ["stable.state", "current.state", "current.unknown",
                                                  "live2", "live3", "dead0", "dead1", "dead2",
                                                  "dead4", "dead5", "dead6"]}

    meta["digests"] = batch_digests()
    meta["digests"]["config2_filter"] = filter_digests()
    meta["digests"]["config2_filter_iter"] = filter_iter_digests()
    meta["digests"]["config5"] = config5_digest()
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(json.dumps(meta["digests"], indent=1))


def stable_fixture(meta):
    # 5d. LifeStable passes: the two espresso fragments as
    #     complete truth tables, and seeded 10-plane LifeStables through the
    #     reference's SynchroniseStateKnown / UpdateOptions / SignalNeighbours /
    #     PropagateStep / Propagate
    R.lib.ref_stable_count_frag.argtypes = [_u64p, _u64p]
    R.lib.ref_stable_signal_frag.argtypes = [_u64p, _u64p]
    R.lib.ref_stable_pass.argtypes = [_u64p, ctypes.c_int]
    sc = fragment_truth_table(R.lib.ref_stable_count_frag, 9, 9)
    np.savez_compressed(os.path.join(HERE, "stable_count_tt.npz"), tt=sc,
                        inputs=np.array(STABLE_COUNT_INPUTS), outputs=np.array(STABLE_COUNT_OUTPUTS))
    ss = fragment_truth_table(R.lib.ref_stable_signal_frag, 17, 4)
    np.savez_compressed(os.path.join(HERE, "stable_signal_tt.npz"), tt=ss,
                        inputs=np.array(STABLE_SIGNAL_INPUTS), outputs=np.array(STABLE_SIGNAL_OUTPUTS))
    st_in = stable_inputs(48)
    res = {}
    for which, name in enumerate(["sync", "options", "signal", "step", "propagate", "stabilise"]):
        planes = st_in.copy()
        flags = np.array([R.lib.ref_stable_pass(_p64(planes[u]), which) for u in range(len(planes))],
                         dtype=np.uint8)
        res[name] = planes
        res[name + "_flags"] = flags
    # LifeStable::Vulnerable (LifeStable.hpp:366-412): its fragment's table and
    # the reference's result on every input
    R.lib.ref_stable_vulnerable_frag.argtypes = [_u64p, _u64p]
    R.lib.ref_stable_vulnerable.argtypes = [_u64p, _u64p]
    sv = fragment_truth_table(R.lib.ref_stable_vulnerable_frag, 15, 4)
    np.savez_compressed(os.path.join(HERE, "stable_vulnerable_tt.npz"), tt=sv,
                        inputs=np.array(STABLE_VULNERABLE_INPUTS), outputs=np.array(STABLE_VULNERABLE_OUTPUTS))
    vul = np.zeros((len(st_in), 64), np.uint64)
    for u in range(len(st_in)):
        R.lib.ref_stable_vulnerable(_p64(st_in[u]), _p64(vul[u]))
    res["vulnerable"] = vul
    np.savez_compressed(os.path.join(HERE, "stable.npz"), input=st_in, **res)
    meta["stable"] = {"n": int(len(st_in)), "passes": ["sync", "options", "signal", "step", "propagate", "stabilise"],
                      "flags": "bit0 consistent, bit1 changed",
                      "step_consistent": int((res["step_flags"] & 1).sum()),
                      "propagate_consistent": int((res["propagate_flags"] & 1).sum()),
                      "stable_count_ones": [int(v) for v in sc.sum(axis=1)],
                      "stable_signal_ones": [int(v) for v in ss.sum(axis=1)],
                      "stable_vulnerable_ones": [int(v) for v in sv.sum(axis=1)],
                      "vulnerable_nonempty": int((vul != 0).any(axis=1).sum())}


# RLE batch I/O (Parsing.hpp:143-204): tricky inputs for LifeState::Parse
# (all cells on the board, so the reference's behaviour is defined) and
# states for LifeState::RLE().  Strings are stored as one uint8 text blob +
# n+1 offsets, as the C ABI takes them.
PARSE_CASES = [
    "b2o$2o$bo!", "bo$2bo$3o!", "x = 3, y = 3, rule = B3/S23\nbo$2bo$3o!",
    "x = 0, y = 0\r\nb2o$\r\n2o$\r\nbo!\r\n", "#N name\nbo$2bo$3o!", "1 2o$o!", "1\n2b2o$o!",
    "64o!", "b63o$64b$63bo!", "o129$o!", "o3$o59$o!", "2o!3o", "3o", "", "!", "$$$o!",
    "10$10$10$10$10$10$3o!", "obo$A.*$3o!", "o\n\nx skipped line\n2o!", "xo$oo!", "5bo\n$2o!",
    "o0$o!", "00o$0o!", "2b3o5$o2bo$obo!", "o$" * 63 + "o!",
]


def rle_fixture():
    rng = np.random.default_rng(4242)
    states = []
    for d in (0.0, 1.0, 0.5, 0.02, 0.1, 0.3, 0.7, 0.95):
        for _ in range(8):
            bits = rng.random((64, 64)) < d
            states.append(np.array([sum(1 << y for y in range(64) if bits[x, y]) for x in range(64)],
                                   dtype=np.uint64))
    chk = np.array([0x5555555555555555 if x % 2 else 0xAAAAAAAAAAAAAAAA for x in range(64)], np.uint64)
    states += [chk, R.parse("bo$2bo$3o!"), moved(R.parse("bo$2bo$3o!"), 62, 62),
               moved(R.parse("bo$2bo$3o!"), 30, 31), rect(31, 31, 2, 2), rect(0, 0, 64, 1)]
    for x, y in ((0, 0), (31, 31), (32, 32), (63, 63), (32, 0), (0, 32), (33, 31)):
        st = np.zeros(64, np.uint64)
        st[x] = np.uint64(1 << y)
        states.append(st)
    states = np.stack(states)
    rles = [R.rle(st).encode() for st in states]
    cases = [c.encode() for c in PARSE_CASES]

    def blob(strs):
        off = np.zeros(len(strs) + 1, np.uint64)
        off[1:] = np.cumsum([len(x) for x in strs])
        return np.frombuffer(b"".join(strs), np.uint8).copy(), off

    rtext, roff = blob(rles)
    ptext, poff = blob(cases)
    parsed = np.stack([R.parse(c) for c in PARSE_CASES])
    np.savez_compressed(os.path.join(HERE, "rle.npz"), states=states, rle_text=rtext, rle_offsets=roff,
                        parse_text=ptext, parse_offsets=poff, parsed=parsed)


def stable_window_fixture():
    """stable_window.npz: LifeStables on which Propagate's window width
    matters -- found by tools/stable_window_mutant_search.py on the GPU (the
    shipped library against a build trusting only 1 row of the window;
    inputs kept in stable_window_inputs/) -- with the reference's own
    Propagate (LifeStable.hpp:718-729) planes and flags"""
    xs = [np.load(f) for f in sorted(glob.glob(os.path.join(HERE, "stable_window_inputs", "*.npy")))]
    x = np.concatenate(xs).reshape(-1, 640)
    out, flags = x.copy(), np.zeros(len(x), np.uint8)
    for u in range(len(x)):
        obj = np.ascontiguousarray(out[u])
        flags[u] = R.stable_pass(obj, 4)
        out[u] = obj
    np.savez_compressed(os.path.join(HERE, "stable_window.npz"), input=x, propagate=out, flags=flags)


if __name__ == "__main__":
    if "--only-stable-window" in sys.argv:
        stable_window_fixture()
    elif "--only-rle" in sys.argv:
        rle_fixture()
    elif "--only-digests" in sys.argv:  # refresh golden.json["digests"] only
        gj = os.path.join(HERE, "golden.json")
        with open(gj) as f:
            m = json.load(f)
        m["digests"] = batch_digests()
        with open(gj, "w") as f:
            json.dump(m, f, indent=1)
    elif "--only-stable" in sys.argv:  # refresh stable*.npz and golden.json["stable"]
        gj = os.path.join(HERE, "golden.json")
        with open(gj) as f:
            m = json.load(f)
        stable_fixture(m)
        with open(gj, "w") as f:
            json.dump(m, f, indent=1)
    else:
        main()
        rle_fixture()
