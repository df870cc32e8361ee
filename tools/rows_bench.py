"""Throughput and HBM roofline fraction of every SURVEY 8(f) kernel on
1M objects (--n) (one JSON line each).  Algorithmic bytes = what the entry point
must read and write per object; peak = 8 TB/s (MI355X_MICROARCH.md).  A timing is K launches back to back
between two events (per launch: / K), median over 7 timings; `scrubbed`: the
launch alone after a 768 MiB scrub of the Infinity Cache (bench.py Scrub),
events around the launch only, median of 10.

The LifeStable passes write back only the lines they change,
so their rows are priced on the bytes each pass really moves, measured by
PMC on the same inputs (profiles/r06/pmc_rows.json, tools/pmc_rows.py:
FETCH_SIZE x 2 + WRITE_SIZE per LifeStable), and carry the VALU side beside
it: SQ_INSTS_VALU per LifeStable / (1024 SIMDs x one wave64 instruction per
2 clocks at 2.4 GHz = 1.2288e12 per second).  `bound_frac` = max(bytes time,
VALU time) / measured time: how close the pass is to the larger of its two
bounds."""
import json
import os
import sys

import numpy as np
import torch

ROOT_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT_DIR)
import bench  # noqa: E402
import lifeapi_amd.hip as hip  # noqa: E402


class _RT:
    kind = "hip"

    def __init__(self):
        self.device = torch.device("cuda", 0)
        self.stream = torch.cuda.current_stream()

    @staticmethod
    def event():
        return torch.cuda.Event(enable_timing=True)


RT = None
SCRUB = None


def scrubbed(fn, prep=None):
    """median ms of fn() alone after a scrub (prep() before each, untimed)"""
    ms = []
    for k in range(13):
        if prep:
            prep()
        SCRUB()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        if k >= 3:
            ms.append(a.elapsed_time(b))
    return sorted(ms)[len(ms) // 2]

PEAK = 8000.0  # GB/s
VALU_PEAK = 1024 * 2.4e9 / 2  # wave64 VALU instructions per second (MI355X_MICROARCH.md: 2 clocks each)
PMC_ROWS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "r06",
                        "pmc_rows.json")  # (tools/gpu_r05_pmc.sh on round 6's kernels)


def pmc_row(name):
    """(bytes per object, VALU per object, source) measured for a LifeStable row, or None"""
    try:
        with open(PMC_ROWS) as f:
            r = json.load(f)["rows"].get(name)
    except (OSError, ValueError, KeyError):
        return None
    if not r:
        return None
    return r["hbm_bytes_per_object"], r["valu_per_object"], "profiles/r06/pmc_rows.json"


K = 10  # launches per timing, back to back (the bench's own way: launch gaps hidden by the queue)


def timed(fn, reps=7):
    fn()
    torch.cuda.synchronize()
    ms = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(K):
            fn()
        b.record()
        b.synchronize()
        ms.append(a.elapsed_time(b) / K)
    return sorted(ms)[len(ms) // 2]


def report(name, n, nbytes, ms, extra=None, scrub_ms=None, pmc=None):
    """pmc: (measured bytes per object, VALU per object, source) -- the row
    is then priced on the measured bytes, with its VALU fraction beside it"""
    d = {"kernel": name, "objects": n, "algorithmic_bytes_per_object": nbytes}
    if pmc:
        nbytes, valu, src = pmc
        d.update({"bytes_per_object": nbytes, "bytes_basis": f"measured: FETCH_SIZE x 2 + WRITE_SIZE ({src})"
                  if "pmc_rows" in src else f"max(algorithmic, FETCH_SIZE x 2 + 4) ({src})",
                  "valu_per_object": valu})
    gbs = n * nbytes / (ms / 1e3) / 1e9
    d.update({"ms": ms, "objects_per_s": n / ms * 1e3, "GBps": gbs, "hbm_frac": gbs / PEAK})
    if pmc:
        t_hbm = n * nbytes / (PEAK * 1e9) * 1e3
        t_valu = n * valu / VALU_PEAK * 1e3
        d.update({"valu_frac": t_valu / ms, "bound_ms": max(t_hbm, t_valu),
                  "bound": "hbm" if t_hbm >= t_valu else "valu", "bound_frac": max(t_hbm, t_valu) / ms})
    if scrub_ms:
        d.update({"scrubbed_ms": scrub_ms, "scrubbed_objects_per_s": n / scrub_ms * 1e3,
                  "scrubbed_GBps": n * nbytes / (scrub_ms / 1e3) / 1e9,
                  "scrubbed_hbm_frac": n * nbytes / (scrub_ms / 1e3) / 1e9 / PEAK})
    d.update(extra or {})
    print(json.dumps(d), flush=True)


def both(name, n, nbytes, fn, extra=None, pmc=None):
    report(name, n, nbytes, timed(fn), extra, scrubbed(fn), pmc=pmc)


# (LIFEAPI_PMC_FILTER: a table collected earlier in the same GPU call, tools/gpu_r06.sh)
PMC_FILTER = os.environ.get("LIFEAPI_PMC_FILTER") or os.path.join(
    os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "r06", "pmc_filter.json")


def pmc_filter_row(target, gens, algo_bytes):
    """(bytes per universe, VALU per universe, source) of the shipped filter
    on this target at this many generations (tools/filter_iter_probe.py pmc +
    summarize), or None.  The bytes are the algorithmic ones (the cone's lines
    + the answer) unless the measured fetch exceeds them."""
    try:
        with open(PMC_FILTER) as f:
            rows = json.load(f)["rows"]
    except (OSError, ValueError, KeyError):
        return None
    r = rows.get(f"{target} {gens}")
    if not r or "valu_per_universe" not in r:
        return None
    fetched = r.get("fetch_bytes_per_universe", 0.0) + 4
    return max(algo_bytes, fetched), r["valu_per_universe"], os.path.relpath(PMC_FILTER, ROOT_DIR)


def stable_inputs(n):
    """Block still lifes with an unknown window, tiled from 256 seeded cases
    (the test_gpu_parity generator), as (n, 640) int64 planes."""
    rng = np.random.default_rng(5)
    base = np.zeros((256, 10, 64), np.uint64)
    blk = np.zeros(64, np.uint64)
    blk[0] = blk[1] = np.uint64(3)
    for u in range(256):
        st = np.zeros(64, np.uint64)
        for _ in range(6):
            bx, by = int(rng.integers(4)) * 16, int(rng.integers(4)) * 16
            st |= np.roll(blk, bx) << np.uint64(by)
        w0, h0 = int(rng.integers(4, 20)), int(rng.integers(4, 20))
        x0, y0 = int(rng.integers(0, 64 - w0)), int(rng.integers(0, 64 - h0))
        unk = np.zeros(64, np.uint64)
        unk[x0:x0 + w0] = np.uint64(((1 << h0) - 1) << y0)
        base[u, 0], base[u, 1] = st & ~unk, unk
    x = np.tile(base.reshape(256, 640), (n // 256, 1))
    return torch.from_numpy(x.view(np.int64)).cuda()


def stable_next_node(still):
    """A search's next node: `still` (stable_inputs) propagated to its
    fixpoint, then one unknown cell (the lowest of the first unknown column)
    decided ON -- Propagate from here changes a few columns, and the passes
    write back only the lines holding them (stable_kernels.hpp)."""
    nxt = still.clone()
    hip.stable_pass(nxt, "propagate")
    unk = nxt[:, 64:128]
    c = (unk != 0).to(torch.int8).argmax(1)
    u = unk.gather(1, c[:, None])
    low = u & -u
    nxt[:, 64:128].scatter_(1, c[:, None], u & ~low)
    st0 = nxt[:, 0:64].gather(1, c[:, None])
    nxt[:, 0:64].scatter_(1, c[:, None], st0 | low)
    return nxt


def main():
    global RT, SCRUB
    RT = _RT()
    SCRUB = bench.Scrub(RT)
    n = int(sys.argv[sys.argv.index('--n') + 1]) if '--n' in sys.argv else 1 << 20
    x = hip.fill_random(n, seed=7)
    y = torch.empty_like(x)
    pp = [x, y]

    def step_pingpong():  # a Step() loop over the batch, as bench.py's timed region
        hip.step(pp[0], out=pp[1], generations=1)
        pp.reverse()

    both("k_step (1 gen)", n, 1024, step_pingpong)
    x = hip.fill_random(n, seed=7)  # (the loop overwrote it)
    both("k_pop", n, 516, lambda: hip.pop(x))
    both("k_hash", n, 520, lambda: hip.hashes(x))
    w = x[:1].clone()
    both("k_cone Contains, whole-board target", n, 513, lambda: hip.contains(x, w, w))
    both("k_cone 1 gen (first hit only), whole-board target", n, 516, lambda: hip.step_contains(x, w, w, 1))
    # bench.py's whole-board target (row 10 of every third column must be dead):
    # its care rows, widened by the light cone, fit 8 rows up to 3 generations
    # (16 to 7, 32 to 15), so the filter runs the packed row-window pass
    # (DESIGN.md 3.2), beyond 4 generations too
    rw, ru = torch.zeros_like(w), torch.zeros_like(w)
    ru[0, 0::3] = 1 << 10
    for gens in (1, 2):
        both(f"filter {gens} gen (first hit only), whole-board target of one care row", n, 516,
             lambda g=gens: hip.step_contains(x, rw, ru, g))
    # the iterated filter (3+ generations): VALU-bound, so priced on the
    # larger of its bytes and its measured VALU (PMC, tools/filter_iter_probe.py
    # summarize -> profiles/r06/pmc_filter.json), as the LifeStable rows
    fu = torch.zeros_like(w)  # bench.py's full-height target: 16 dead cells, one in every fourth row
    for yy in range(0, 64, 4):
        fu[0, (3 * yy) % 64] |= 1 << yy
    iters = [("one_row", "whole-board target of one care row", rw, ru, (3, 5, 8, 13)),
             ("full_height", "full-height target (16 cells, every fourth row)", torch.zeros_like(w), fu,
              (3, 5, 8, 13)),
             ("full", "whole-board target, every row (a random universe)", w, w, (3, 5, 8))]
    for key, label, tw_, tu_, gl in iters:
        for gens in gl:
            both(f"filter {gens} gen (first hit only), {label}", n, 516,
                 lambda g=gens, a=tw_, b=tu_: hip.step_contains(x, a, b, g),
                 pmc=pmc_filter_row(key, gens, 512 + 4))
    bw, bu = torch.zeros_like(w), torch.zeros_like(w)
    bw[0, 10] = bw[0, 11] = 3 << 40
    bu[0, 9:13] = 15 << 39
    bu &= ~bw
    # the light cone of this target (columns 9-12, +-1 for a generation) lies in
    # one 128-byte line of each universe: the bytes the kernel must move are
    # that line and the answer (PMC: FETCH_SIZE x 2 = 128 B per universe)
    both("k_cone Contains, 2x2 block + ring (4 columns)", n, 128 + 1, lambda: hip.contains(x, bw, bu),
         {"lines_128B_per_object": 1, "full_read_equivalent_bytes": 513})
    both("k_cone 1 gen (first hit only), 2x2 block + ring", n, 128 + 4, lambda: hip.step_contains(x, bw, bu, 1),
         {"lines_128B_per_object": 1, "full_read_equivalent_bytes": 516})
    for gens in (3, 5, 8, 13):  # the column and row window widen with the generations (cone_split.hpp)
        xs = (9 - gens) % 64
        lines = len({((xs + c) % 64) // 16 for c in range(4 + 2 * gens)})
        both(f"filter {gens} gen (first hit only), 2x2 block + ring", n, 128 * lines + 4,
             lambda g=gens: hip.step_contains(x, bw, bu, g), {"lines_128B_per_object": lines},
             pmc=pmc_filter_row("block", gens, 128 * lines + 4))
    fp = [x.clone(), y]

    def filter_pingpong():  # a loop stepping its batch with the filter: final states ping-ponged
        hip.step_contains(fp[0], w, w, 1, final=fp[1])
        fp.reverse()

    both("k_step_contains 1 gen + final states (ping-pong)", n, 1028, filter_pingpong)
    both("k_fill", n, 512, lambda: hip.fill_random(n, seed=9))
    both("k_counts NeighbourCount", n, 512 + 2048, lambda: hip.neighbour_count(x))
    both("k_counts InteractionCounts", n, 512 + 1536, lambda: hip.interaction_counts(x))
    both("k_counts InteractionCountsAndNext", n, 512 + 2048, lambda: hip.interaction_counts(x, with_next=True))
    welds = torch.cat([hip.fill_random(n, seed=s).view(n, 1, 64) for s in (11, 12, 13, 14)], 1).reshape(n, 256)
    welds[:, 64:] &= hip.fill_random(3 * n, seed=15).view(n, 192)
    both("k_weld (1 gen)", n, 2048 + 512, lambda: hip.weld_step(welds, 1))
    # iterated welds (k_weld_split, VALU-bound): weld-generations per second
    nw, gw = 1 << 18, 256
    ms = timed(lambda: hip.weld_step(welds[:nw], gw))
    print(json.dumps({"kernel": "k_weld_split (256 gens)", "objects": nw, "gens": gw, "ms": ms,
                      "weld_gen_per_s": nw * gw / ms * 1e3}), flush=True)
    st = stable_inputs(n)
    # the passes work in place: each timing runs KS passes back to back, each
    # on its own fresh copy of the input (copied before the timed region)
    ks = 4
    works = [st.clone() for _ in range(ks)]
    nxt = stable_next_node(st)
    for name in list(hip.STABLE_PASSES) + [hip.STABLE_PASSES[0], "propagate next node"]:  # sync again: warm-up check
        src = nxt if name.endswith("next node") else st
        name_run = name.split()[0]
        ms = []
        for _ in range(7):
            for wk in works:
                wk.copy_(src)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for wk in works:
                hip.stable_pass(wk, name_run)
            b.record()
            b.synchronize()
            ms.append(a.elapsed_time(b) / ks)
        sm = scrubbed(lambda: hip.stable_pass(works[0], name_run), prep=lambda: works[0].copy_(src))
        label = f"k_stable {name_run} ({'next' if name.endswith('next node') else 'still'})"
        report(f"k_stable {name}", n, 2 * 5120 + 1, sorted(ms)[len(ms) // 2], scrub_ms=sm,
               pmc=pmc_row(label) if n == 1 << 20 else None)
    for name in ("sync", "options", "signal", "step", "stabilise"):  # the single passes on the next node
        ms = []
        for _ in range(7):
            for wk in works:
                wk.copy_(nxt)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for wk in works:
                hip.stable_pass(wk, name)
            b.record()
            b.synchronize()
            ms.append(a.elapsed_time(b) / ks)
        report(f"k_stable {name} next node", n, 2 * 5120 + 1, sorted(ms)[len(ms) // 2],
               pmc=pmc_row(f"k_stable {name} (next)") if n == 1 << 20 else None)
    del works, nxt
    report("k_stable_vulnerable", n, 5120 + 512, timed(lambda: hip.stable_vulnerable(st)),
           scrub_ms=scrubbed(lambda: hip.stable_vulnerable(st)),
           pmc=pmc_row("k_stable_vulnerable (still)") if n == 1 << 20 else None)
    planes = hip.fill_random(11 * n, seed=21).view(n, 11 * 64)
    both("k_refined (config 5)", n, 7168, lambda: hip.refined_step(planes))
    n5 = 1 << 18
    p5 = planes[:n5].contiguous()
    both("k_refined (config 5, 256K)", n5, 7168, lambda: hip.refined_step(p5))


if __name__ == "__main__":
    main()
