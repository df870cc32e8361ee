#!/usr/bin/env python3
"""bench.py -- batched 64x64-torus LifeState::Step() on MI355X, 1..8 GPUs.

Workloads (BASELINE.json configs; the per-universe independence that lets them
shard with no collective is LifeAPI.hpp:1196-1216 -- Step() reads one object):

* config 2 (the N=1 default): 1M random-fill universes x 1 generation per step
  on each GPU ("weak": per-GPU work fixed; rank r owns universes
  [r*1M, (r+1)*1M) of the seed-2 array).
* config 4 (the N>1 default): ONE fixed problem of 16M universes x 1
  generation, split into N contiguous shards ("strong"; 8 GiB in + 8 GiB out
  over all ranks).  `--config 4 --gpus 1` runs the same 16M on one GPU, and
  the N=1 line carries that run as `secondary.config4`, so the 8-vs-1 ratio is
  the same problem.

A step is one launch of the HIP step kernel over the rank's whole shard
(device-resident ping-pong buffers, so the state keeps evolving).  With
`--gpus N` and no torch.distributed environment, this process starts N ranks
through `torch.distributed.run` as a child process (before touching the GPU)
and exits with its status; each rank drives one GPU.  The only collectives
are outside the timed region: the barrier/MAX of the timing contract, the
per-rank digest exchange of the first-launch check and the result
collection (an all-gather of per-universe 64-bit hashes over RCCL/xGMI),
timed and reported separately.

Prints ONE JSON line on rank 0 (contract: task brief).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from lifeapi_amd.digest import batch_digest, combine  # noqa: E402
from lifeapi_amd.shard import gather_hashes, strong_shard, weak_shard  # noqa: E402

METRIC = "64x64 universe-generations/sec (+ cell-updates/sec) at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md, chip table)
BYTES_PER_UNIVERSE_GEN = 1024  # 512 B read + 512 B write
OPS_PER_UNIVERSE_GEN = 2688    # reference's ~21 u64 ops/column = 42 int32 x 64
# Config 3's fixed algorithmic bound: 8 three-input LUTs per
# 32 cell-updates (the 2-LUT horizontal layer + the 6-LUT tail, the smallest
# network the exhaustive/CGP searches found) = 1024 lane-LUTs = 16 wave64
# VALU issue slots per universe-generation; peak = 1024 SIMDs x one wave64
# VALU op per 2 clk at 2.4 GHz.
C3_SLOTS_PER_UNIVERSE_GEN = 16
VALU_PEAK_SLOTS = 1024 * 2.4e9 / 2

CONFIGS = {
    2: {"name": "config2", "seed": 2, "universes": 1 << 20, "scaling": "weak",
        "golden": ("weak_shards_seed2", "weak_shards_seed2_small")},
    4: {"name": "config4", "seed": 4, "universes": 1 << 24, "scaling": "strong",
        "golden": ("config4", "config4_small")},
}

COLL_DEV = None  # device the collectives' tensors live on (set in main)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse_args(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--config", default="auto", choices=("auto", "2", "4"),
                   help="auto: config 2 at N=1, config 4 (16M strong-split) at N>1")
    p.add_argument("--universes", type=int, default=0,
                   help="override: per-rank universes (config 2) or the global total (config 4)")
    p.add_argument("--gens-per-step", type=int, default=1)
    p.add_argument("--seed", type=int, default=-1, help="override the config's seed")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=12.0,
                   help="wall budget of the config-2 CPU baseline (half at 1 thread, half on all host cores)")
    p.add_argument("--no-secondary", action="store_true", help="skip the config-3/4/5 side measurements")
    p.add_argument("--no-verify", action="store_true")
    return p.parse_args(argv)


# ----------------------------------------------------------------------------
# process launch: one rank per GPU
# ----------------------------------------------------------------------------
def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, argv: list[str]) -> int:
    """Start `n` ranks of the launching script (normally this one) under
    torch.distributed.run as a CHILD process (this process has not touched
    the GPU and never execs) and return its exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(sys.argv[0]), *argv]
    log("+ " + " ".join(cmd))
    return subprocess.call(cmd)


class HipRuntime:
    """Device, launch stream and timing events of one rank (one GPU)."""
    kind = "hip"

    def __init__(self, local_rank: int, world: int, backend: str):
        ndev = torch.cuda.device_count()
        if ndev == 0:
            raise RuntimeError("bench.py needs a GPU (no HIP device visible)")
        if world > ndev and backend == "nccl":
            raise RuntimeError(f"{world} ranks but only {ndev} visible GPUs")
        # the modulo only matters for a gloo rehearsal with more ranks than GPUs
        self.device = torch.device("cuda", local_rank % ndev)
        torch.cuda.set_device(self.device)
        self.stream = torch.cuda.current_stream(self.device)
        self.neutral, self.neutral_error, self.line_read = None, None, None
        try:  # the tuning build's streaming-step launcher (fixed order, explicit store policy)
            sys.path.insert(0, os.path.join(ROOT, "tools", "tune"))
            import tune_hip
            self.neutral = tune_hip.step_order
            self.line_read = tune_hip.line_read  # the light cone's access shape alone
        except (ImportError, OSError) as e:
            self.neutral_error = str(e)

    def sync(self):
        torch.cuda.synchronize(self.device)

    @staticmethod
    def event():
        return torch.cuda.Event(enable_timing=True)


def load_kernels(backend: str, local_rank: int, world: int):
    """The HIP library (lifeapi_amd.hip) and this rank's runtime.  There is
    no fallback: without a GPU or the built library this raises."""
    import lifeapi_amd.hip as hip
    return hip, HipRuntime(local_rank, world, backend)


# ----------------------------------------------------------------------------
# timing
# ----------------------------------------------------------------------------
def timed_launches(hip, rt, bufs, steps, gens):
    """`steps` back-to-back ping-pong launches on the rank's stream, bracketed
    by one pair of events on that same stream.  Returns ((start, end), index
    of the buffer holding the latest state)."""
    e0, e1 = rt.event(), rt.event()
    cur = 0
    e0.record(rt.stream)
    for _ in range(steps):
        hip.step(bufs[cur], out=bufs[1 - cur], generations=gens, stream=rt.stream)
        cur = 1 - cur
    e1.record(rt.stream)
    return (e0, e1), cur


def median_launch_ms(hip, rt, a, b, gens, reps=10):
    ms = []
    for _ in range(reps):
        e0, e1 = rt.event(), rt.event()
        e0.record(rt.stream)
        hip.step(a, out=b, generations=gens, stream=rt.stream)
        e1.record(rt.stream)
        e1.synchronize()
        ms.append(e0.elapsed_time(e1))
    return sorted(ms)[len(ms) // 2], ms


def pingpong_ms(rt, fn, a, b, reps=20, warm=5):
    """per-launch ms of fn(src, dst) ping-ponged between a and b: `warm`
    untimed launches, then `reps` launches each between a pair of events on
    the rank's stream.  Returns (median, min, all)."""
    bufs = [a, b]
    for k in range(warm):
        fn(bufs[k % 2], bufs[1 - k % 2])
    ms = []
    for k in range(reps):
        e0, e1 = rt.event(), rt.event()
        e0.record(rt.stream)
        fn(bufs[(warm + k) % 2], bufs[1 - (warm + k) % 2])
        e1.record(rt.stream)
        e1.synchronize()
        ms.append(e0.elapsed_time(e1))
    return float(np.median(ms)), float(min(ms)), ms


def back_to_back_ms(rt, fn, a, b, reps=20, warm=5, repeats=3):
    """per-launch ms of fn(src, dst) ping-ponged between a and b the way the
    timed region runs: `warm` untimed launches, then `reps` launches back to
    back between one pair of events on the rank's stream (the queue hides
    the launch gaps), / reps; the median of `repeats` such runs."""
    bufs = [a, b]
    k = 0
    for _ in range(warm):
        fn(bufs[k % 2], bufs[1 - k % 2])
        k += 1
    runs = []
    for _ in range(repeats):
        e0, e1 = rt.event(), rt.event()
        e0.record(rt.stream)
        for _ in range(reps):
            fn(bufs[k % 2], bufs[1 - k % 2])
            k += 1
        e1.record(rt.stream)
        e1.synchronize()
        runs.append(e0.elapsed_time(e1) / reps)
    return float(np.median(runs))


SCRUB_MIB = 768  # > 2 x the 256 MiB Infinity Cache (MI355X_MICROARCH.md, memory hierarchy)


class Scrub:
    """SCRUB_MIB of unrelated plain reads (one torch sum on the rank's stream):
    run before a timed launch, it leaves nothing that launch reads in the
    256 MiB memory-side Infinity Cache or the L2s, so the launch is timed
    from HBM alone.  Reads only (mode "read", the default): the lines it
    leaves cached are clean, so the timed launch pays no write-back of the
    scrub's own data; mode "rw" (one add_, plain reads and writes) leaves up
    to 256 MiB of dirty lines behind, kept for the comparison in
    tools/footprint_sweep.py."""

    def __init__(self, rt, mib=SCRUB_MIB, mode="read"):
        self.rt, self.mib, self.mode = rt, mib, mode
        self.buf = torch.ones(mib << 17, dtype=torch.int64, device=rt.device)
        self.sink = torch.empty((), dtype=torch.int64, device=rt.device)

    def __call__(self):
        with torch.cuda.stream(self.rt.stream):
            if self.mode == "rw":
                self.buf.add_(1)
            else:
                torch.sum(self.buf, 0, out=self.sink)


def scrubbed_ms(rt, fn, a, b, scrub, reps=10, warm=3):
    """per-launch ms of fn(src, dst) ping-ponged between a and b with a scrub
    before every launch: `warm` untimed launches, then `reps` launches each
    between a pair of events on the rank's stream that bracket the launch
    only (not the scrub).  Returns (median, all)."""
    bufs = [a, b]
    for k in range(warm):
        scrub()
        fn(bufs[k % 2], bufs[1 - k % 2])
    ms = []
    for k in range(reps):
        scrub()
        e0, e1 = rt.event(), rt.event()
        e0.record(rt.stream)
        fn(bufs[(warm + k) % 2], bufs[1 - (warm + k) % 2])
        e1.record(rt.stream)
        e1.synchronize()
        ms.append(e0.elapsed_time(e1))
    return float(np.median(ms)), ms


def interleaved_scrubbed_ms(rt, fns, a, scrub, reps=10, warm=3):
    """scrubbed_ms for several launches at once, interleaved launch by
    launch: per rep, each fn(a, a) in turn after its own scrub, timed alone;
    a clock or fabric state that drifts over a series then falls on all of
    them alike.  Returns [(median, all)] in the order of fns."""
    ms = [[] for _ in fns]
    for k in range(warm + reps):
        for i, fn in enumerate(fns):
            scrub()
            e0, e1 = rt.event(), rt.event()
            e0.record(rt.stream)
            fn(a, a)
            e1.record(rt.stream)
            e1.synchronize()
            if k >= warm:
                ms[i].append(e0.elapsed_time(e1))
    return [(float(np.median(v)), v) for v in ms]


def hbm_only_ms(rt, fn, a, b, scrub, reps=10, warm=3):
    """The launch's HBM-only time, deferred write-backs included
    (tools/writeback_ab.py's method): a launch timed alone
    after a scrub reads from HBM, but can leave up to 256 MiB of its writes
    dirty in the memory-side Infinity Cache, written back after its end
    event.  Per rep: scrub; a scrub timed after that scrub (nothing dirty:
    `clean`); the launch timed (`launch`); the next scrub timed (`after`: it
    evicts what the launch left dirty, so it pays those write-backs).
    inclusive = launch + after - clean.  Returns medians
    {"launch_ms", "inclusive_ms", "scrub_clean_ms", "scrub_after_ms"}."""
    bufs = [a, b]
    launch, after, clean = [], [], []

    def timed(f):
        e0, e1 = rt.event(), rt.event()
        e0.record(rt.stream)
        f()
        e1.record(rt.stream)
        return e0, e1

    for k in range(warm + reps):
        x, y = bufs[k % 2], bufs[1 - k % 2]
        scrub()
        s = timed(scrub)
        ln = timed(lambda: fn(x, y))
        af = timed(scrub)
        af[1].synchronize()
        if k >= warm:
            clean.append(s[0].elapsed_time(s[1]))
            launch.append(ln[0].elapsed_time(ln[1]))
            after.append(af[0].elapsed_time(af[1]))
    lm, am, cm = (float(np.median(v)) for v in (launch, after, clean))
    return {"launch_ms": lm, "inclusive_ms": lm + max(am - cm, 0.0), "scrub_clean_ms": cm, "scrub_after_ms": am}


HBM_ONLY_METHOD = ("HBM only, deferred write-backs included: per rep a 768 MiB read scrub, a timed scrub (clean), "
                   "the timed launch, a timed scrub (after); launch + after - clean, medians of 10")


def side_fn(rt, gens, neutral):
    """A side launch of the shipped streaming kernel's code through the
    tuning build (tools/tune step_order, kernel k_step_ab: the same code as
    the product's k_step under another name, so that a rocprofv3 trace of
    this bench tells side launches from the timed ones); None without the
    tuning build.
      neutral: the cache-neutral form -- ONE fixed group order, every store
               nontemporal, no plain-stored tail, so no launch can read what
               the one before it left in the 256 MB Infinity Cache;
      else:    the product's policy (step.hip): the order reversed on every
               launch of a ping-pong from 192K universes on (what the
               batch-keyed order does there), the last min(256 MiB, half)
               of each launch stored plain; above 4M universes one order,
               every store nontemporal, 8 universes per wave, at most 7
               blocks per CU and each XCD a contiguous eighth of the batch
               (both forms then use that launch, which reuses nothing from
               the cache).
    With gens = 0 the kernel is a copy of exactly that access shape."""
    if rt.neutral is None:
        return None
    flip = [False]

    def fn(src, dst):
        n = src.shape[0]
        big = n > (1 << 22)
        resident = 7 if big else 0
        if neutral or big:
            rt.neutral(src, dst, generations=gens, reverse=False, nts=True, resident=resident, upw=8 if big else 4,
                       plain_bytes=0, stream=rt.stream, xcd_chunk=big)
        else:
            rev = flip[0] and n >= 3 * (1 << 16)
            flip[0] = not flip[0]
            rt.neutral(src, dst, generations=gens, reverse=rev, nts=True, resident=resident, upw=4,
                       plain_bytes=min(256 << 20, n * 512 // 2), stream=rt.stream)
    return fn


def stream_figures(hip, rt, a, b, gens, reps=20):
    """Per-rank side measurements of the streaming launch on the rank's own
    buffers, after the timed region (side_fn): the cache-neutral step, and
    copy ceilings of the same access shape -- the kernel with 0 generations
    under the product's store/order policy and in the neutral form.  ms per
    launch, timed like the timed region: `reps` launches back to back after
    5 warm ones (back_to_back_ms)."""
    n = a.shape[0]
    out = {}
    for key, g, neu in (("neutral_ms", gens, True), ("copy_ms", 0, False), ("copy_neutral_ms", 0, True)):
        fn = side_fn(rt, g, neu)
        out[key] = back_to_back_ms(rt, fn, a, b, reps) if fn is not None else None
    # the shipped launch itself with a scrub before each launch, and the
    # write-backs it leaves behind: HBM only
    scrub = Scrub(rt) if rt.kind == "hip" else (lambda: None)
    h = hbm_only_ms(rt, lambda x, y: hip.step(x, out=y, generations=gens, stream=rt.stream), a, b, scrub)
    out["scrubbed_ms"], out["hbm_only_ms"] = h["launch_ms"], h["inclusive_ms"]
    del scrub
    out["bytes"] = n * BYTES_PER_UNIVERSE_GEN
    return out


def copy_ceiling(n: int):
    """Median GB/s of a plain copy with the step kernel's access shape,
    ping-ponged between two buffers of n universes as this bench does
    (tools/membw.hip `pingpong`, measured on MI355X and committed under
    profiles/): the streaming ceiling for this footprint, context for the
    roofline.  The nearest measured footprint is used, and the best of the
    occupancy settings, store policies and launch orders measured there
    (`membw snake`: the group order alternated between launches, as the
    step kernel runs batches of up to 2M universes)."""
    rows = []
    for name in ("membw_pingpong.jsonl", "membw_snake.jsonl"):
        path = os.path.join(ROOT, "profiles", "r02", name)
        try:
            with open(path) as f:
                for line in f:
                    try:
                        d = json.loads(line)
                    except ValueError:
                        continue
                    if "universes" in d and "GBps_median" in d:
                        rows.append((d, os.path.relpath(path, ROOT)))
        except OSError:
            continue
    if not rows:
        return None, None
    near = min(rows, key=lambda r: abs(np.log2(r[0]["universes"]) - np.log2(max(n, 1))))[0]["universes"]
    best, src = max((r for r in rows if r[0]["universes"] == near), key=lambda r: r[0]["GBps_median"])
    shape = ""
    if "snake" in best:
        shape = (f", {'nt' if best['mode'] & 2 else 'plain'} stores, "
                 f"{'alternating' if best['snake'] else 'one'} order")
    return best["GBps_median"], (f"{src} ({near} universes, "
                                 f"{best.get('resident_blocks', 0) or 'all'} blocks resident per CU{shape})")


def load_pmc_traffic(n: int):
    """HBM bytes per launch from the committed rocprofv3 PMC summary, if it matches."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        if d.get("universes") == n:
            return d.get("hbm_bytes_per_launch"), os.path.relpath(path, ROOT)
    except (OSError, ValueError):
        pass
    return None, None


# ----------------------------------------------------------------------------
# CPU baseline (the reference's own Step(), oracle/_ref; else the C port)
# ----------------------------------------------------------------------------
def host_cores():
    """Threads for the CPU baseline: every core in this process's affinity
    set, limited by a cgroup CPU quota when one is set (more threads than the
    quota would only be throttled).  Returns (threads, evidence)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            with open(path) as f:
                q, per = f.read().split()[:2]
            if q != "max":
                quota = int(q) / int(per)
        except (OSError, ValueError):
            pass
    if quota is None:
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                q = int(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                per = int(f.read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    threads = aff if quota is None else max(1, min(aff, int(quota)))
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), "")
    except OSError:
        pass
    return threads, {"affinity_cpus": aff, "cgroup_quota_cpus": quota, "os_cpu_count": os.cpu_count(),
                     "cpu_model": model}


def _cpu_stepper():
    from oracle.oracle import Port, Ref
    if Ref.available():
        return Ref(), "reference"
    return Port(), "port"


def cpu_baseline(x_host: np.ndarray, seconds: float):
    """The reference's Step() on the config-2 input (a bounded sample: at most
    the first 1M universes), 1 thread and all host cores."""
    o, kind = _cpu_stepper()
    threads, ev = host_cores()
    x = x_host[: 1 << 20]
    n = x.shape[0]
    out = {}
    for t in sorted({1, threads}):
        o.step_batch(x[: min(n, 4096)], 1, nthreads=t)  # warm
        passes, t0 = 0, time.perf_counter()
        while True:
            o.step_batch(x, 1, nthreads=t)
            passes += 1
            el = time.perf_counter() - t0
            if el >= seconds / 2:
                break
        out[t] = (n * passes / el, passes, el)
    v, passes, el = out[threads]
    return {
        "value": v, "unit": "universe-gen/s", "cores": threads, "kind": kind,
        "sample": f"config-2 input ({n} universes) x 1 gen, {passes} passes in {el:.2f}s, "
                  f"{threads} threads (contiguous slices); CPU: {ev['cpu_model']}",
        "value_1thread": out[1][0], "host": ev,
    }


def cpu_baseline_config3(x_host: np.ndarray, seconds: float):
    """The reference's Step(1024) on a bounded sample of the config-3
    universes, on all host cores (`seconds` of work)."""
    o, kind = _cpu_stepper()
    threads, ev = host_cores()
    sample = x_host[: 64 * threads]
    o.step_batch(sample[:threads], 1024, nthreads=threads)  # warm
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        o.step_batch(sample, 1024, nthreads=threads)
        done += sample.shape[0]
    el = time.perf_counter() - t0
    return {"value": done * 1024 / el, "unit": "universe-gen/s", "cores": threads, "kind": kind,
            "sample": f"{sample.shape[0]} of the config-3 universes x 1024 gens, {done // sample.shape[0]} "
                      f"passes in {el:.2f}s, {threads} threads"}


def cpu_baseline_config1():
    """Config 1 (BASELINE.json configs[0]): R-pentomino x 1103 single-universe
    Step() on the CPU, 1 thread -- the drop-in facade's Step()
    (include/lifeapi/LifeState.hpp) next to the reference's own, same
    compiler and flags, one binary (oracle/_ref/config1_bench, built from
    tests/cpp/config1_bench.cpp)."""
    exe = os.path.join(ROOT, "oracle", "_ref", "config1_bench")
    if not os.path.exists(exe):
        return None
    try:
        r = subprocess.run([exe, "200", "5"], capture_output=True, text=True, timeout=120)
        d = json.loads(r.stdout.strip().splitlines()[-1])
        d["exit_status"] = r.returncode
        return d
    except (OSError, ValueError, IndexError, subprocess.TimeoutExpired) as e:
        return {"error": str(e)}


# ----------------------------------------------------------------------------
# verification: first-launch digests vs the reference's (tests/golden/golden.json)
# ----------------------------------------------------------------------------
def expected_digests(cfg: int, seed: int, gens: int, world: int, n_rank: int, n_total: int, shards):
    """(per-rank expected digests or None, expected global digest or None, source)."""
    try:
        with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
            gold = json.load(f)["digests"]
    except (OSError, ValueError, KeyError):
        return [None] * world, None, None
    for key in CONFIGS[cfg]["golden"]:
        d = gold.get(key)
        if not d or d.get("seed") != seed or d.get("generations") != gens:
            continue
        if cfg == 2 and d["universes_per_rank"] == n_rank:
            ds = d["shard_output_digests"]
            per = [ds[r] if r < len(ds) else None for r in range(world)]
            glob = f"{combine(int(x, 16) for x in per):016x}" if None not in per else None
            return per, glob, key
        if cfg == 4 and d["universes"] == n_total:
            chunk = d["universes"] // d["shards"]
            chunks = [int(x, 16) for x in d["shard_output_digests"]]
            per = []
            for lo, cnt in shards:
                hi = lo + cnt
                per.append(f"{combine(chunks[lo // chunk: hi // chunk]):016x}"
                           if lo % chunk == 0 and hi % chunk == 0 else None)
            return per, d["output_digest"], key
    return [None] * world, None, None


def _golden(key: str, field: str):
    try:
        with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
            return json.load(f)["digests"][key][field]
    except (OSError, ValueError, KeyError):
        return None


def golden_digest(key: str):
    """the reference-generated output digest of a full-size config
    (tests/golden/golden.json, tests/golden/make_golden.py via oracle/_ref)"""
    return _golden(key, "output_digest")


def _i64(u: int) -> int:
    return u - (1 << 64) if u >= 1 << 63 else u


def all_gather_ints(vals, world):
    """All-gather a short list of int64 bit patterns from every rank (rank order)."""
    t = torch.tensor([_i64(v) for v in vals], dtype=torch.int64, device=COLL_DEV)
    if not dist.is_initialized():
        return [[int(x) % (1 << 64) for x in t.tolist()]]
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    return [[int(x) % (1 << 64) for x in p.tolist()] for p in parts]


def verify_first_launch(hip, rt, out, first, cfg, seed, gens, world, n_rank, n_total, shards):
    """Each rank digests its shard of the first launch's output; rank 0 gets
    every shard's digest and checks each one, and their sum, against the
    reference-generated digests (tests/golden/make_golden.py from oracle/_ref)."""
    got = batch_digest(hip.hashes(out, stream=rt.stream).cpu().numpy(), first)
    all_d = [v[0] for v in all_gather_ints([got], world)]
    per, glob, src = expected_digests(cfg, seed, gens, world, n_rank, n_total, shards)
    per_ok = [None if w is None else f"{g:016x}" == w for g, w in zip(all_d, per)]
    total = f"{combine(all_d):016x}"
    glob_ok = None if glob is None else total == glob
    known = [x for x in per_ok + [glob_ok] if x is not None]
    return {"ok": (all(known) if known else None), "per_rank_ok": per_ok, "global_ok": glob_ok,
            "rank_digests": [f"{g:016x}" for g in all_d], "global_digest": total, "expected_global": glob,
            "against": f"tests/golden/golden.json digests.{src} (reference Step() via oracle/_ref)"
            if src else "no golden digest for this size/seed"}


# ----------------------------------------------------------------------------
# side measurements at N=1
# ----------------------------------------------------------------------------
def secondary_config3(hip, rt, cpu_seconds=0.0):
    """Config 3: 64K universes x 1024 generations (state resident in VGPRs)."""
    n, gens = 1 << 16, 1024
    a = hip.fill_random(n, seed=3, device=rt.device, stream=rt.stream)
    b = torch.empty_like(a)
    for _ in range(20):  # warm: ~30 ms of back-to-back launches (clocks settle)
        hip.step(a, out=b, generations=gens, stream=rt.stream)
    med, ms = median_launch_ms(hip, rt, a, b, gens)
    t = med / 1e3
    gps = n * gens / t
    digest = f"{batch_digest(hip.hashes(b, stream=rt.stream).cpu().numpy()):016x}"
    cpu = None
    if cpu_seconds > 0:
        cpu = cpu_baseline_config3(a.cpu().numpy().view(np.uint64), cpu_seconds)
    achieved = gps * C3_SLOTS_PER_UNIVERSE_GEN
    want = golden_digest("config3")
    return {"workload": "config3: 64K universes x 1024 generations (one launch)",
            "value": gps, "unit": "universe-gen/s", "cell_updates_per_s": gps * 4096,
            "kernel_ms": med, "kernel_ms_min": min(ms), "kernel_ms_all": ms,
            "kernel": hip.step_kernel_name(gens),
            "output_digest": digest, "output_digest_expected": want,
            "verified": (digest == want) if want else None,
            "verified_against": "tests/golden/golden.json digests.config3 (reference Step(1024) via oracle/_ref)",
            "roofline": {"bound": "valu", "achieved": achieved / 1e12, "peak": VALU_PEAK_SLOTS / 1e12,
                         "unit": "T wave64-VALU slots/s", "frac": achieved / VALU_PEAK_SLOTS,
                         "algorithmic_slots_per_universe_gen": C3_SLOTS_PER_UNIVERSE_GEN,
                         "definition": "8 LUT3 per 32 cell-updates (2-LUT h-layer + 6-LUT tail) = 16 wave64 "
                                       "VALU slots per universe-gen; peak 1024 SIMDs x 1 op / 2 clk x 2.4 GHz "
                                       "(DESIGN.md 5.2)"},
            "reference_op_equivalent_Tops": OPS_PER_UNIVERSE_GEN * gps / 1e12,
            "search_loop": config3_search_loop(hip, rt, a, med),
            "cpu_baseline": cpu}


def config3_search_loop(hip, rt, a, step_ms):
    """Config 3 as callers consume Step (LifeTarget.hpp:44-51): the fused
    Step + Contains kernel pair on the same input, a 2 x 2 block with its
    empty ring as the target, final states written; first-hit generations and
    final states checked against the reference's own Step() + Contains() loop
    (tests/golden/golden.json digests.config3_contains, ref_shim.cpp)."""
    try:
        with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
            gold = json.load(f)["digests"]["config3_contains"]
    except (OSError, ValueError, KeyError):
        return None
    n, gens = a.shape[0], gold["generations"]
    tw, tu = (torch.from_numpy(np.array([[int(v, 16) for v in gold[k]]], dtype=np.uint64).view(np.int64))
              .to(a.device) for k in ("wanted", "unwanted"))
    fin = torch.empty_like(a)
    first, _ = hip.step_contains(a, tw, tu, gens, final=fin, stream=rt.stream)
    rt.sync()
    fd = f"{batch_digest(first.cpu().numpy().astype(np.uint64)):016x}"
    od = f"{batch_digest(hip.hashes(fin, stream=rt.stream).cpu().numpy()):016x}"
    hits = int((first > 0).sum().item())
    for _ in range(20):  # warm, as the plain step before it
        hip.step_contains(a, tw, tu, gens, final=fin, stream=rt.stream)
    ms = []
    for _ in range(20):
        e0, e1 = rt.event(), rt.event()
        e0.record(rt.stream)
        hip.step_contains(a, tw, tu, gens, final=fin, stream=rt.stream)
        e1.record(rt.stream)
        e1.synchronize()
        ms.append(e0.elapsed_time(e1))
    med = float(np.median(ms))
    return {"workload": f"config3 search loop: {n} universes x {gens} generations, Step + Contains(LifeTarget) "
                        "after every generation (one fused launch pair)",
            "kernel_ms": med, "kernel_ms_all": ms, "over_plain_step": med / step_ms,
            "hits": hits, "first_digest": fd, "output_digest": od,
            "verified": fd == gold["first_digest"] and hits == gold["hits"] and od == gold["output_digest"]}


def secondary_config4_1gpu(hip, rt, steps=20, warm=20):
    """Config 4's fixed 16M-universe problem on ONE GPU: the same-problem
    denominator of the 8-vs-1 strong-scaling ratio.  Warmed like config 3
    (`warm` back-to-back launches first, so the clock has settled), then
    `steps` ping-pong launches timed one by one; min and median, and the
    cache-neutral form (one fixed order, all stores nontemporal) and copy
    ceilings at the same size, so the ratio can be read both ways."""
    n = 1 << 24
    a = hip.fill_random(n, seed=4, device=rt.device, stream=rt.stream)
    b = torch.empty_like(a)
    hip.step(a, out=b, generations=1, stream=rt.stream)
    digest = f"{batch_digest(hip.hashes(b, stream=rt.stream).cpu().numpy()):016x}"
    step = lambda x, y: hip.step(x, out=y, generations=1, stream=rt.stream)  # noqa: E731
    med, mn, ms = pingpong_ms(rt, step, b, a, reps=steps, warm=warm)
    # the value is timed as the N > 1 lines' timed region is: launches back to back
    b2b = back_to_back_ms(rt, step, b, a, reps=steps, warm=0)
    figs = stream_figures(hip, rt, a, b, 1, reps=steps)
    del a, b
    torch.cuda.empty_cache()
    gb = lambda t: n * BYTES_PER_UNIVERSE_GEN / (t / 1e3) / 1e9 if t else None  # noqa: E731
    spread = (max(ms) - min(ms)) / med
    q = np.percentile(ms, [10, 90])
    spread_p = float((q[1] - q[0]) / med)  # robust to a single hiccup (a host interrupt between launches)
    return {"workload": "config4 on 1 GPU: 16777216 universes x 1 generation per launch",
            "value": n / (b2b / 1e3), "value_best": n / (mn / 1e3), "unit": "universe-gen/s",
            "kernel_ms": b2b,
            "kernel_ms_median": med, "kernel_ms_min": mn, "kernel_ms_all": ms,
            "kernel_ms_spread": spread, "flat_within_3pct": spread <= 0.03,
            "kernel_ms_spread_p10_p90": spread_p, "flat_within_3pct_p10_p90": spread_p <= 0.03,
            "timing": f"{warm} warm launches, then {steps} ping-pong launches each between events on the stream "
                      f"(kernel_ms_all: the series, flatness), then 3 runs of {steps} launches back to back between "
                      "one pair of events, median (kernel_ms, value, roofline: the timed region's method)",
            "output_digest": digest, "output_digest_expected": golden_digest("config4"),
            "verified": digest == golden_digest("config4"),
            "roofline": {"bound": "hbm", "achieved": gb(b2b), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": gb(b2b) / HBM_PEAK_GBS,
                         "hbm_only": {"achieved": gb(figs["hbm_only_ms"]),
                                      "frac": gb(figs["hbm_only_ms"]) / HBM_PEAK_GBS,
                                      "kernel_ms": figs["hbm_only_ms"], "launch_ms": figs["scrubbed_ms"],
                                      "method": HBM_ONLY_METHOD},
                         "fixed_order_nt_back_to_back": {"achieved": gb(figs["neutral_ms"]),
                                                         "kernel_ms": figs["neutral_ms"]},
                         "copy_same_shape_GBps": gb(figs["copy_ms"]),
                         "copy_note": "the step kernel's code with 0 generations in the same launch shape; at "
                                      "16M universes it runs below the step, so it is no ceiling here"},
            "kernel": hip.step_kernel_name(1, n)}


def _cone_columns(wanted: np.ndarray, unwanted: np.ndarray, gens: int):
    """(first column, columns) the light-cone kernels load for this target
    (cone_kernels.hpp cone_window: the smallest cyclic window of the care
    columns, widened by `gens` on each side; the whole board from column 0
    once that reaches 64)"""
    care = [bool(int(wanted[x]) | int(unwanted[x])) for x in range(64)]
    if not any(care):
        x0, w = 0, 1
    else:
        run, start = 0, 0
        for p in range(64):
            r = 0
            while r < 64 and not care[(p + r) % 64]:
                r += 1
            if r > run:
                run, start = r, p
        x0, w = (start + run) % 64, 64 - run
    k = w + 2 * gens
    return (0, 64) if k >= 64 else ((x0 - gens) % 64, k)


def _lines_touched(xs: int, k: int, line: int = 128) -> int:
    """128-byte lines of one 512-byte universe holding columns [xs, xs + k) mod 64"""
    return len({((xs + i) % 64) * 8 // line for i in range(k)})


def secondary_filter(hip, rt):
    """The search filter as loops consume Step (SURVEY 8(f) row 1,
    LifeTarget.hpp:44-51): 1M config-2 universes, Step() then
    Contains(target) at 1 and 2 generations, first hits only -- and batched
    Contains alone -- on the
    light-cone kernels (cone_kernels.hpp), which read only the columns within
    one generation of the target's care columns.  Each launch is timed alone
    after a 768 MiB scrub (the cone of a small target fits in the Infinity
    Cache, so back-to-back launches on one input would read it from there);
    results checked against the reference's own loop
    (tests/golden/golden.json digests.config2_filter, ref_shim.cpp)."""
    try:
        with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
            gold = json.load(f)["digests"]["config2_filter"]
    except (OSError, ValueError, KeyError):
        return None
    n = gold["universes"]
    x = hip.fill_random(n, seed=gold["seed"], device=rt.device, stream=rt.stream)
    scrub = Scrub(rt)
    out = {"workload": f"config2 input: {n} universes, Step() then Contains(target) at 1 and 2 generations "
                       "(first hits only), and Contains(target) alone",
           "timing": "3 warm, 10 timed launches, each after a 768 MiB scrub, events around the launch only, "
                     "median, the three operations interleaved launch by launch; b2b: 20 launches back to "
                     "back on the same input (Infinity Cache warm)",
           "targets": {}}
    for name, t in gold["targets"].items():
        w, u = (np.array([int(v, 16) for v in t[k]], dtype=np.uint64) for k in ("wanted", "unwanted"))
        tw, tu = (torch.from_numpy(v.view(np.int64)[None].copy()).to(rt.device) for v in (w, u))
        first, _ = hip.step_contains(x, tw, tu, 1, stream=rt.stream)
        first2, _ = hip.step_contains(x, tw, tu, 2, stream=rt.stream)
        cont = hip.contains(x, tw, tu, stream=rt.stream)
        rt.sync()
        fd = f"{batch_digest(first.cpu().numpy().astype(np.uint64)):016x}"
        fd2 = f"{batch_digest(first2.cpu().numpy().astype(np.uint64)):016x}"
        cd = f"{batch_digest(cont.cpu().numpy().astype(np.uint64)):016x}"
        hits, hits2 = int((first > 0).sum().item()), int((first2 > 0).sum().item())
        row = {"verified": fd == t["first_digest"] and hits == t["hits"] and cd == t["contains_digest"]
               and fd2 == t.get("first_digest_2gen") and hits2 == t.get("hits_2gen"),
               "hits": hits, "hits_2gen": hits2}
        ops = (("filter_1gen", 1, 4, lambda a, b: hip.step_contains(a, tw, tu, 1, stream=rt.stream)),
               ("filter_2gen", 2, 4, lambda a, b: hip.step_contains(a, tw, tu, 2, stream=rt.stream)),
               ("contains", 0, 1, lambda a, b: hip.contains(a, tw, tu, stream=rt.stream)))
        timed = interleaved_scrubbed_ms(rt, [op[3] for op in ops], x, scrub)
        for (op, gens, outb, fn), (ms, allms) in zip(ops, timed):
            xs, k = _cone_columns(w, u, gens)
            lines = _lines_touched(xs, k)
            b2b = back_to_back_ms(rt, fn, x, x)
            row[op] = {"objects_per_s": n / (ms / 1e3), "kernel_ms": ms, "kernel_ms_all": allms,
                       "kernel_ms_b2b": b2b, "objects_per_s_b2b": n / (b2b / 1e3),
                       "cone_columns": k, "cone_first_column": xs, "lines_128B_per_universe": lines,
                       "roofline": {"bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBS,
                                    "algorithmic_bytes_per_universe": lines * 128 + outb,
                                    "achieved": n * (lines * 128 + outb) / (ms / 1e3) / 1e9,
                                    "frac": n * (lines * 128 + outb) / (ms / 1e3) / 1e9 / HBM_PEAK_GBS,
                                    "definition": "the 128-byte lines of each universe that hold its light "
                                                  "cone (the fetch granularity) + the output, per launch"},
                       "full_read_equivalent_GBps": n * (512 + outb) / (ms / 1e3) / 1e9}
            if lines == 1 and rt.line_read is not None:
                # the same line of every universe read with as many lanes per
                # universe as the cone uses, nothing computed (tuning build
                # k_line_read): the ceiling of this access shape
                lpu = 4 if k <= 4 else 8 if k <= 8 else 16
                code = (xs // 16) + 4 * {16: 0, 4: 1, 8: 2}[lpu]
                pm, _ = scrubbed_ms(rt, lambda a, b: rt.line_read(a, code, stream=rt.stream), x, x, scrub)
                row[op]["access_shape"] = {"kernel": f"k_line_read<{lpu}> (tuning build)", "kernel_ms": pm,
                                           "frac_of_shape": pm / ms,
                                           "definition": "one 128-byte line of every universe read with the "
                                                         "cone's lanes per universe and one uint32 written, "
                                                         "nothing computed, timed as the kernel is"}
        out["targets"][name] = row
    del scrub, x
    torch.cuda.empty_cache()
    return out


def _cone_cells(wanted: np.ndarray, unwanted: np.ndarray, gens: int) -> int:
    """cell-updates the iterated filter cannot avoid per universe: at
    generation g (1..gens) the cells within Chebyshev distance gens - g of the
    target's care cells on the torus (the ones a later test reads)"""
    care = np.zeros((64, 64), bool)  # [column, row]
    for x in range(64):
        v = int(wanted[x]) | int(unwanted[x])
        care[x] = [(v >> y) & 1 for y in range(64)]
    total, cur = 0, care.copy()
    reach = [care.sum()]
    for _ in range(gens - 1):
        cur = cur | np.roll(cur, 1, 0) | np.roll(cur, -1, 0)
        cur = cur | np.roll(cur, 1, 1) | np.roll(cur, -1, 1)
        reach.append(cur.sum())
    for g in range(1, gens + 1):
        total += int(reach[gens - g])
    return total


def secondary_filter_iter(hip, rt):
    """The iterated search filter (LifeTarget.hpp:44-51,
    LifeAPI.hpp:877-881): 1M config-2 universes, Step() then Contains(target)
    after every generation up to 1-13 generations, first hits only, on three
    targets: bench's block + ring (a 4 x 4 care window) at 5 / 8 / 13, its
    one-row whole-board target at 5 / 8, and a full-height one (16 dead
    cells, one in every fourth row: no window of any kind) at 1 / 2 / 3 / 5
    / 8 generations.  Each call is timed alone after a 768
    MiB scrub (median of 10) and back to back; the answers of the first and
    the second call on each target (the first call has no launch report yet)
    are checked against the reference's own loop (tests/golden/golden.json
    digests.config2_filter_iter, make_golden.py).  Bounds per call: bytes =
    the 128-byte lines of each universe holding the light cone + the 4-byte
    answer at 8 TB/s; VALU = the cells each generation must update (those
    within gens - g of a care cell) at 16 wave64 issue slots per 4096 cells
    (config 3's fixed network bound) at 1.2288e12 slots/s."""
    gold = _golden("config2_filter_iter", "targets")
    if not gold:
        return None
    n = 1 << 20
    x = hip.fill_random(n, seed=2, device=rt.device, stream=rt.stream)
    scrub = Scrub(rt)
    out = {"workload": f"config2 input: {n} universes, the search loop Step() then Contains(target) up to "
                       "1-13 generations, first hits only",
           "timing": "alone: 3 warm, 10 timed calls each after a 768 MiB scrub, events around the call, "
                     "median; b2b: 20 calls back to back",
           "targets": {}}
    for name, t in gold.items():
        w, u = (np.array([int(v, 16) for v in t[k]], dtype=np.uint64) for k in ("wanted", "unwanted"))
        tw, tu = (torch.from_numpy(v.view(np.int64)[None].copy()).to(rt.device) for v in (w, u))
        rows = {}
        for gs, want in t["gens"].items():
            g = int(gs)
            ok = True
            for _ in range(2):  # the first call on a target, then the reported form
                first, _ = hip.step_contains(x, tw, tu, g, stream=rt.stream)
                rt.sync()
                d = f"{batch_digest(first.cpu().numpy().astype(np.uint64)):016x}"
                ok = ok and d == want["first_digest"] and int((first > 0).sum().item()) == want["hits"]
            fn = lambda a, b, g=g: hip.step_contains(a, tw, tu, g, stream=rt.stream)  # noqa: E731
            ms, allms = scrubbed_ms(rt, fn, x, x, scrub)
            b2b = back_to_back_ms(rt, fn, x, x)
            xs, k = _cone_columns(w, u, g)
            lines = _lines_touched(xs, k)
            bytes_ms = n * (lines * 128 + 4) / (HBM_PEAK_GBS * 1e9) * 1e3
            cells = _cone_cells(w, u, g)
            valu_ms = n * cells * C3_SLOTS_PER_UNIVERSE_GEN / 4096 / VALU_PEAK_SLOTS * 1e3
            board_ms = n * g * C3_SLOTS_PER_UNIVERSE_GEN / VALU_PEAK_SLOTS * 1e3
            bound = max(bytes_ms, valu_ms)
            rows[gs] = {"verified": ok, "hits": want["hits"], "kernel_ms": ms, "kernel_ms_all": allms,
                        "kernel_ms_b2b": b2b, "universes_per_s": n / (ms / 1e3),
                        "lines_128B_per_universe": lines, "cone_cells": cells,
                        "bound": {"bytes_ms": bytes_ms, "valu_ms": valu_ms,
                                  "bound": "hbm" if bytes_ms >= valu_ms else "valu", "bound_ms": bound,
                                  "bound_frac": bound / ms, "whole_board_valu_ms": board_ms,
                                  "whole_board_valu_frac": board_ms / ms}}
        out["targets"][name] = rows
    del scrub, x
    torch.cuda.empty_cache()
    return out


def secondary_config5(hip, rt):
    """Config 5: unknown_step_refined ternary step, 256K universes, one launch."""
    n = 1 << 18
    planes = hip.fill_random(n * 11, seed=6, device=rt.device, stream=rt.stream).reshape(n, 11 * 64)
    out = torch.empty((n, 3 * 64), dtype=torch.int64, device=rt.device)
    hip.refined_step(planes, out=out, stream=rt.stream)  # warm
    ms = []
    for _ in range(10):
        e0, e1 = rt.event(), rt.event()
        e0.record(rt.stream)
        hip.refined_step(planes, out=out, stream=rt.stream)
        e1.record(rt.stream)
        e1.synchronize()
        ms.append(e0.elapsed_time(e1))
    one = sorted(ms)[len(ms) // 2]
    fn = lambda a, b: hip.refined_step(planes, out=out, stream=rt.stream)  # noqa: E731
    # timed as the timed region is: launches back to back between one pair of events
    b2b = back_to_back_ms(rt, fn, planes, out)
    scrub = Scrub(rt)
    h = hbm_only_ms(rt, fn, planes, out, scrub)
    del scrub
    gb = lambda t: n * 7168 / (t / 1e3) / 1e9  # noqa: E731
    digest = f"{batch_digest(hip.hashes(out.reshape(n * 3, 64), stream=rt.stream).cpu().numpy()):016x}"
    want = _golden("config5", "output_digest")
    return {"workload": "config5: 256K universes, unknown_step_refined (11 planes in, 3 out)",
            "value": n / (b2b / 1e3), "unit": "universe-steps/s", "kernel_ms": b2b,
            "output_digest": digest, "output_digest_expected": want,
            "verified": (digest == want) if want else None,
            "verified_against": "tests/golden/golden.json digests.config5 (the reference's "
                                "unknown_step_refined.hpp fragment in its harness, via oracle/_ref)",
            "kernel_ms_single_launch_median": one, "kernel_ms_single_all": ms,
            "timing": "kernel_ms: 5 warm, then 3 runs of 20 launches back to back between one pair of events, "
                      "median (the timed region's method); single: one launch between events, median of 10",
            "roofline": {"bound": "hbm", "achieved": gb(b2b), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": gb(b2b) / HBM_PEAK_GBS,
                         "algorithmic_bytes_per_universe": 7168,
                         "single_launch_frac": gb(one) / HBM_PEAK_GBS,
                         "hbm_only": {"achieved": gb(h["inclusive_ms"]), "frac": gb(h["inclusive_ms"]) / HBM_PEAK_GBS,
                                      "kernel_ms": h["inclusive_ms"], "launch_ms": h["launch_ms"],
                                      "method": HBM_ONLY_METHOD}}}


# ----------------------------------------------------------------------------
# the printed line: compact, with a flat summary of the side measurements last
# ----------------------------------------------------------------------------
def compact_line(line: dict) -> dict:
    """The printed line: the full one (written to the detail file) without
    the per-launch series (lists longer than 8) and the long prose (strings
    longer than 160 characters) below the top level."""
    def walk(v, depth):
        if isinstance(v, dict):
            return {k: walk(x, depth + 1) for k, x in v.items()
                    if not (depth > 0 and ((isinstance(x, list) and len(x) > 8)
                                           or (isinstance(x, str) and len(x) > 160)))}
        if isinstance(v, list):
            return [walk(x, depth + 1) for x in v]
        return v
    return walk(line, 0)


def _get(d, *keys):
    for k in keys:
        if not isinstance(d, dict) or d.get(k) is None:
            return None
        d = d[k]
    return d


def _r(x, nd=4):
    return round(x, nd) if isinstance(x, float) else x


def secondary_summary(line: dict, sec: dict | None, cpu: dict | None) -> dict:
    """One flat dict of the figures a reader checks first: ms, roofline
    fraction and reference check of every config and of the search filter."""
    s = {"c2_kernel_ms": _r(line["kernel_ms_avg"]), "c2_frac": _r(_get(line, "roofline", "frac")),
         "c2_frac_hbm_only": _r(_get(line, "roofline", "hbm_only", "frac")),
         "c2_verified": _get(line, "verified", "ok")}
    c1 = _get(cpu, "config1")
    if c1:
        s.update(c1_facade_ns_per_gen=c1.get("facade_ns_per_gen"), c1_reference_ns_per_gen=c1.get("reference_ns_per_gen"),
                 c1_bit_exact=c1.get("bit_exact"), c1_pop_final=c1.get("pop_final"))
    if sec:
        c3, c4, c5, flt = (sec.get(k) for k in ("config3", "config4", "config5", "filter"))
        if c3:
            s.update(c3_kernel_ms=_r(c3["kernel_ms"]), c3_frac_valu=_r(_get(c3, "roofline", "frac")),
                     c3_verified=c3["verified"], c3_search_ms=_r(_get(c3, "search_loop", "kernel_ms")),
                     c3_search_verified=_get(c3, "search_loop", "verified"),
                     c3_cpu_universe_gen_per_s=_r(_get(c3, "cpu_baseline", "value"), 1))
        if c4:
            s.update(c4_1gpu_kernel_ms=_r(c4["kernel_ms"]), c4_1gpu_frac=_r(_get(c4, "roofline", "frac")),
                     c4_1gpu_frac_hbm_only=_r(_get(c4, "roofline", "hbm_only", "frac")),
                     c4_1gpu_verified=c4["verified"])
        if c5:
            s.update(c5_kernel_ms=_r(c5["kernel_ms"]), c5_frac=_r(_get(c5, "roofline", "frac")),
                     c5_frac_hbm_only=_r(_get(c5, "roofline", "hbm_only", "frac")), c5_verified=c5.get("verified"))
        for name, row in ((flt or {}).get("targets") or {}).items():
            for op in ("filter_1gen", "filter_2gen", "contains"):
                s[f"{op}_{name}_ms"] = _r(_get(row, op, "kernel_ms"), 5)
                s[f"{op}_{name}_frac"] = _r(_get(row, op, "roofline", "frac"))
            s[f"filter_{name}_verified"] = row.get("verified")
        for name, rows in ((sec.get("filter_iter") or {}).get("targets") or {}).items():
            for g, row in rows.items():
                s[f"iter_{name}_{g}gen_ms"] = _r(row.get("kernel_ms"), 5)
                s[f"iter_{name}_{g}gen_bound_frac"] = _r(_get(row, "bound", "bound_frac"))
                s[f"iter_{name}_{g}gen_verified"] = row.get("verified")
    return s


# ----------------------------------------------------------------------------
def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus, argv))  # before any GPU call in this process

    # stdout carries the one JSON line alone: everything else a rank prints to
    # fd 1 (RCCL's version banner, gloo's peer notes, ...) goes to stderr
    line_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; running {world} ranks")
    backend = os.environ.get("LIFEAPI_BENCH_BACKEND", "nccl")  # nccl == RCCL on ROCm
    hip, rt = load_kernels(backend, local, world)
    global COLL_DEV
    COLL_DEV = rt.device if backend == "nccl" else torch.device("cpu")
    # a process group whenever a launcher started this rank (torch.distributed.run
    # sets WORLD_SIZE and MASTER_PORT), so one rank under the launcher runs the
    # collective path of the N > 1 lines, RCCL included
    dist_on = world > 1 or ("WORLD_SIZE" in os.environ and "MASTER_PORT" in os.environ)
    if dist_on:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=rt.device)
        else:
            dist.init_process_group(backend)
        coll_world = dist.get_world_size()
    else:
        coll_world = 1

    cfg = (2 if world == 1 else 4) if args.config == "auto" else int(args.config)
    spec = CONFIGS[cfg]
    seed = spec["seed"] if args.seed < 0 else args.seed
    gens = args.gens_per_step
    if cfg == 2:
        n_rank = args.universes or spec["universes"]
        n_total = n_rank * world
        shards = [weak_shard(r, n_rank) for r in range(world)]
    else:
        n_total = args.universes or spec["universes"]
        shards = [strong_shard(r, world, n_total) for r in range(world)]
        n_rank = shards[rank][1]
    first, n = shards[rank]

    a = hip.fill_random(n, seed=seed, first_universe=first, device=rt.device, stream=rt.stream)
    b = torch.empty_like(a)
    want_cpu = rank == 0 and world == 1 and not args.no_cpu_baseline
    x_cpu = a[: 1 << 20].cpu().numpy().view(np.uint64).copy() if want_cpu else None
    bufs = [a, b]

    # warmup (untimed); the first launch's output is checked shard by shard
    hip.step(bufs[0], out=bufs[1], generations=gens, stream=rt.stream)
    verified = None
    if not args.no_verify:
        verified = verify_first_launch(hip, rt, bufs[1], first, cfg, seed, gens, world, n_rank, n_total,
                                       shards)
    _, cur = timed_launches(hip, rt, [bufs[1], bufs[0]], max(args.warmup - 1, 0), gens)
    bufs = [bufs[1], bufs[0]] if cur == 0 else [bufs[0], bufs[1]]
    rt.sync()

    # timed region: barrier + sync on both sides, max over ranks
    if dist_on:
        dist.barrier()
    rt.sync()
    t0 = time.perf_counter()
    evs, cur = timed_launches(hip, rt, bufs, args.steps, gens)
    rt.sync()
    if dist_on:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    span_ms = evs[0].elapsed_time(evs[1])   # GPU time of the K launches on their stream
    if dist_on:
        t = torch.tensor([elapsed], dtype=torch.float64, device=COLL_DEV)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        per = torch.tensor([span_ms / args.steps, float(n)], dtype=torch.float64, device=COLL_DEV)
        parts = [torch.empty_like(per) for _ in range(world)]
        dist.all_gather(parts, per)
        per_rank = [(float(p[0]), int(p[1])) for p in parts]
    else:
        per_rank = [(span_ms / args.steps, n)]
    final = bufs[cur]

    # result collection (not in the timed region): all-gather per-universe hashes
    h = hip.hashes(final, stream=rt.stream)
    rt.sync()
    # side figures on the rank's own buffers (after the hashes: they overwrite
    # both): cache-neutral step and live copy ceilings, gathered per rank
    figs = stream_figures(hip, rt, final, bufs[1 - cur], gens) if gens <= 2 else None
    fig_keys = ("scrubbed_ms", "copy_ms", "copy_neutral_ms", "neutral_ms", "hbm_only_ms")
    fv = [(-1.0 if figs is None or figs[k] is None else figs[k]) for k in fig_keys]
    if dist_on:
        ft = torch.tensor(fv, dtype=torch.float64, device=COLL_DEV)
        fparts = [torch.empty_like(ft) for _ in range(world)]
        dist.all_gather(fparts, ft)
        rank_figs = [[(None if x < 0 else float(x)) for x in fp.tolist()] for fp in fparts]
    else:
        rank_figs = [[(None if x < 0 else x) for x in fv]]
    collect = None
    if dist_on:
        dist.barrier()
        c0 = time.perf_counter()
        gathered = gather_hashes(h.to(COLL_DEV), world, [c for _, c in shards])
        rt.sync()
        cms = (time.perf_counter() - c0) * 1e3
        collect = {"op": f"all_gather(per-universe 64-bit hash, {'RCCL' if backend == 'nccl' else backend})",
                   "bytes_per_rank": n * 8, "ms": cms}
        if rank == 0:
            collect["final_digest"] = f"{batch_digest(gathered.cpu().numpy()):016x}"
            collect["universes_gathered"] = int(gathered.numel())

    secondary = None
    if rank == 0 and world == 1 and not args.no_secondary and rt.kind == "hip":
        csec = 0.0 if args.no_cpu_baseline else args.cpu_seconds / 3
        secondary = {"config3": secondary_config3(hip, rt, csec),
                     "config5": secondary_config5(hip, rt),
                     "filter": secondary_filter(hip, rt),
                     "filter_iter": secondary_filter_iter(hip, rt)}
        if cfg == 2:
            del a, b, bufs, final
            torch.cuda.empty_cache()
            secondary["config4"] = secondary_config4_1gpu(hip, rt)

    ceiling, ceiling_src = copy_ceiling(n)
    cpu = None
    if want_cpu:
        cpu = cpu_baseline(x_cpu, args.cpu_seconds)
        cpu["config1"] = cpu_baseline_config1()

    if dist_on:
        dist.barrier()
    if rank == 0:
        total = n_total * gens * args.steps
        value = total / elapsed
        avg_launch = per_rank[0][0]  # includes the ~1-2 us launch gaps: conservative
        bpl = n * gens * BYTES_PER_UNIVERSE_GEN
        achieved = bpl / (avg_launch / 1e3) / 1e9 if gens == 1 else None
        agg = sum(c * gens * BYTES_PER_UNIVERSE_GEN / (ms / 1e3) / 1e9 for ms, c in per_rank) if gens == 1 else None
        traffic, tsrc = load_pmc_traffic(n)

        def gbps(ms, c):
            return c * max(gens, 1) * BYTES_PER_UNIVERSE_GEN / (ms / 1e3) / 1e9 if ms else None

        def copy_gbps(ms, c):
            return c * BYTES_PER_UNIVERSE_GEN / (ms / 1e3) / 1e9 if ms else None

        def frac(gb, peak=HBM_PEAK_GBS):
            return gb / peak if gb else None

        after_scrub = [gbps(f[0], c) for f, (_, c) in zip(rank_figs, per_rank)]
        hbm = [gbps(f[4], c) for f, (_, c) in zip(rank_figs, per_rank)]
        cpy = [copy_gbps(f[1], c) for f, (_, c) in zip(rank_figs, per_rank)]
        cpy_neu = [copy_gbps(f[2], c) for f, (_, c) in zip(rank_figs, per_rank)]
        fixed = [gbps(f[3], c) for f, (_, c) in zip(rank_figs, per_rank)]
        agg_hbm = sum(hbm) if all(v is not None for v in hbm) else None
        val_hbm = (sum(c * gens / (f[4] / 1e3) for f, (_, c) in zip(rank_figs, per_rank))
                   if all(f[4] for f in rank_figs) else None)
        line = {
            "metric": METRIC, "value": value, "unit": "universe-gen/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True, "scaling": spec["scaling"], "vs_baseline": None, "dtype": "u64",
            "data": f"synthetic: splitmix64 uniform-fill universes (seed {seed}), generated on device",
            "config": {"workload": (f"{spec['name']}: {n_rank} random-fill 64x64 universes x {gens} generation "
                                    f"per step per GPU" if cfg == 2 else
                                    f"{spec['name']}: {n_total} random-fill 64x64 universes x {gens} generation "
                                    f"per step, split into {world} contiguous shards"),
                       "universes_per_gpu": n_rank, "global_universes": n_total, "gens_per_step": gens,
                       "parallelism": f"dp{world} (contiguous universe shards, no data-path collective)",
                       "kernel": hip.step_kernel_name(gens, n)},
            "cell_updates_per_s": value * 4096,
            "kernel_ms_avg": avg_launch,
            "kernel_timing": "HIP events on the launch stream around the K timed launches / K",
            "per_rank": [{"rank": r, "universes": c, "kernel_ms_avg": ms,
                          "GBps": c * gens * BYTES_PER_UNIVERSE_GEN / (ms / 1e3) / 1e9 if gens == 1 else None,
                          "kernel_ms_hbm_only": rank_figs[r][4], "GBps_hbm_only": hbm[r],
                          "GBps_launch_after_scrub": after_scrub[r],
                          "GBps_fixed_order_nt_back_to_back": fixed[r],
                          "copy_GBps": cpy[r], "copy_GBps_cache_neutral": cpy_neu[r]}
                         for r, (ms, c) in enumerate(per_rank)],
            "value_hbm_only": val_hbm,
            "value_hbm_only_note": ("universe-gen/s if every rank ran its shard at its HBM-only rate (the shipped "
                                    "launch after a 768 MiB scrub plus the write-backs it defers past its end event; "
                                    "per rank, after the timed region): the 8-vs-1 ratio without cache reuse"),
            "collective_world_size": coll_world,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": frac(achieved),
                         "frac_kind": ("effective: algorithmic bytes / launch time, back-to-back launches; part of "
                                       "each launch's reads is served by the 256 MB Infinity Cache (DESIGN.md 3.1)"
                                       if n <= (1 << 22) else
                                       "effective: algorithmic bytes / launch time, back-to-back launches; one "
                                       "order, every store nontemporal (no Infinity Cache reuse arranged)"),
                         "hbm_only": ({"achieved": hbm[0], "frac": frac(hbm[0]), "kernel_ms": rank_figs[0][4],
                                       "launch_ms": rank_figs[0][0], "method": HBM_ONLY_METHOD}
                                      if hbm[0] else None),
                         "launch_after_scrub": ({"achieved": after_scrub[0], "frac": frac(after_scrub[0]),
                                                 "kernel_ms": rank_figs[0][0],
                                                 "note": "reads from HBM alone, but up to 256 MiB of its writes "
                                                         "can still sit in the Infinity Cache at its end event"}
                                                if after_scrub[0] else None),
                         "fixed_order_nt_back_to_back": ({"achieved": fixed[0], "frac": frac(fixed[0]),
                                                          "kernel_ms": rank_figs[0][3]} if fixed[0] else None),
                         "cache_gain": (achieved / hbm[0] - 1) if (achieved and hbm[0]) else None,
                         "traffic": traffic, "traffic_source": tsrc,
                         "traffic_note": "FETCH_SIZE x 2 + WRITE_SIZE (MI355X_MICROARCH.md); L2-to-fabric bytes, "
                                         "so Infinity Cache hits count as HBM bytes",
                         "algorithmic_bytes_per_launch": bpl,
                         "aggregate_GBps": agg,
                         "aggregate_frac": (agg / (world * HBM_PEAK_GBS)) if agg else None,
                         "aggregate_GBps_hbm_only": agg_hbm,
                         "aggregate_frac_hbm_only": (agg_hbm / (world * HBM_PEAK_GBS)) if agg_hbm else None,
                         "read_only_GBps": achieved / 2 if achieved else None,
                         "copy_ceiling_GBps": cpy[0],
                         "copy_ceiling_source": "live, rank 0: the step kernel's code with 0 generations, same "
                                                "store policy and order (bench.py side_fn, k_step_ab)",
                         "frac_of_copy_ceiling": (achieved / cpy[0]) if (achieved and cpy[0]) else None,
                         "copy_ceiling_cache_neutral_GBps": cpy_neu[0],
                         "copy_ceiling_recorded_GBps": ceiling, "copy_ceiling_recorded_source": ceiling_src},
            "cpu_baseline": cpu,
            "verified": verified,
            "collect": collect,
            "secondary": secondary,
        }
        if rt.kind != "hip":
            line["kernel_backend"] = f"STUB {rt.kind} (CPU rank rehearsal, not a measurement)"
        detail = os.environ.get("LIFEAPI_BENCH_DETAIL", os.path.join(ROOT, "gpurun_out", "bench_detail.json"))
        try:
            os.makedirs(os.path.dirname(detail), exist_ok=True)
            with open(detail, "w") as f:
                json.dump(line, f, indent=1)
        except OSError as e:
            detail = f"not written: {e}"
        # the side measurements in full stay in the detail file; the flat
        # summary below carries their figures
        line = compact_line({k: v for k, v in line.items() if k != "secondary"})
        line["detail_file"] = os.path.relpath(detail, ROOT) if os.path.isabs(detail) else detail
        # last, so the driver's 2000-character tail of stdout holds it whole
        line["secondary_summary"] = secondary_summary(line, secondary, cpu)
        print(json.dumps(line), file=line_out, flush=True)
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
