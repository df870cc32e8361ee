#!/usr/bin/env python3
"""bench.py -- batched 64x64-torus LifeState::Step() on MI355X.

Headline workload (BASELINE.json configs[1], "config 2"): 1M random-fill
64x64 universes x 1 generation per step, per GPU.  A step is one launch of
the HIP step kernel over the rank's whole shard (device-resident, ping-pong
buffers, so the state keeps evolving).  With N GPUs (one process per GPU,
launched by torch.distributed.run) every rank steps its own contiguous shard
of the global universe array -- no collective on the data path ("weak"
scaling: per-GPU work fixed).  After the timed region the per-universe hashes
are all-gathered over RCCL (result collection, timed and reported separately).

Prints ONE JSON line on rank 0 (contract in the task brief / DESIGN.md).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from lifeapi_amd.digest import batch_digest  # noqa: E402
from lifeapi_amd.shard import gather_hashes, weak_shard  # noqa: E402

METRIC = "64x64 universe-generations/sec (+ cell-updates/sec) at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0       # MI355X HBM3E spec (MI355X_MICROARCH.md, chip table)
BYTES_PER_UNIVERSE_GEN = 1024  # 512 B read + 512 B write
OPS_PER_UNIVERSE_GEN = 2688    # reference's ~21 u64 ops/column = 42 int32 x 64


COLL_DEV = None  # device the collectives' tensors live on (set in main)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse_args():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--universes", type=int, default=1 << 20, help="universes per rank (config 2: 1M)")
    p.add_argument("--gens-per-step", type=int, default=1)
    p.add_argument("--seed", type=int, default=2)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=12.0,
                   help="wall budget of the CPU baseline (half at 1 thread, half at 16)")
    p.add_argument("--no-secondary", action="store_true", help="skip the config-3 side measurement")
    p.add_argument("--no-verify", action="store_true")
    return p.parse_args()


def timed_launches(hip, bufs, steps, gens, stream):
    """Run `steps` back-to-back ping-pong launches on `stream`, bracketed by one
    pair of HIP events on that same stream (no events between launches, so
    none of their cost lands between kernels).  Returns ((start, end), index
    of the buffer holding the latest state)."""
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    cur = 0
    e0.record(stream)
    for _ in range(steps):
        hip.step(bufs[cur], out=bufs[1 - cur], generations=gens, stream=stream)
        cur = 1 - cur
    e1.record(stream)
    return (e0, e1), cur


def copy_ceiling():
    """Best median GB/s of the same-shape HBM copy kernel (tools/membw.hip:
    dwordx2 lanes, 4 x 512 B in flight per wave, read + write) measured on
    MI355X and committed under profiles/; context for the roofline."""
    path = os.path.join(ROOT, "profiles", "r01", "membw.jsonl")
    best = None
    try:
        with open(path) as f:
            for line in f:
                try:
                    d = json.loads(line)
                except ValueError:
                    continue
                if d.get("mode") in (0, 1, 2, 3) and "GBps_median" in d:
                    best = max(best or 0.0, d["GBps_median"])
    except OSError:
        return None, None
    return best, os.path.relpath(path, ROOT)


def cpu_baseline(x_host: np.ndarray, seconds: float):
    """Reference CPU Step() (oracle/_ref, else the C port) on host cores."""
    from oracle.oracle import Port, Ref
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    threads = max(1, min(threads, 16))
    if Ref.available():
        o, kind = Ref(), "reference"
        run = lambda a, t: o.step_batch(a, 1, nthreads=t)  # noqa: E731
    else:
        o, kind = Port(), "port"
        run = lambda a, t: o.step_batch(a, 1, nthreads=t)  # noqa: E731
    n = x_host.shape[0]
    out = {}
    for t in sorted({1, threads}):
        run(x_host[: min(n, 4096)], t)  # warm
        passes, t0 = 0, time.perf_counter()
        while True:
            run(x_host, t)
            passes += 1
            el = time.perf_counter() - t0
            if el >= seconds / 2:
                break
        out[t] = (n * passes / el, passes, el)
    v, passes, el = out[threads]
    cpu = ""
    try:
        with open("/proc/cpuinfo") as f:
            cpu = next((l.split(":", 1)[1].strip() for l in f if l.startswith("model name")), "")
    except OSError:
        pass
    return {
        "value": v, "unit": "universe-gen/s", "cores": threads, "kind": kind,
        "sample": f"config-2 input ({n} universes) x 1 gen, {passes} passes in {el:.2f}s, "
                  f"{threads} threads, contiguous slices; CPU: {cpu}",
        "value_1thread": out[1][0],
    }


def cpu_baseline_config3(x_host: np.ndarray, seconds: float):
    """The reference's Step(gens) (oracle/_ref, else the C port) on the
    config-3 shape: a bounded sample of the same universes, 1024 generations
    each, on the host cores (`seconds` of work)."""
    from oracle.oracle import Port, Ref
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    threads = max(1, min(threads, 16))
    o, kind = (Ref(), "reference") if Ref.available() else (Port(), "port")
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


def secondary_config3(hip, device, stream, cpu_seconds=0.0):
    """Config 3: 64K universes x 1024 generations, state resident in VGPRs."""
    n, gens = 1 << 16, 1024
    a = hip.fill_random(n, seed=3, device=device, stream=stream)
    b = torch.empty_like(a)
    for _ in range(20):  # warm: ~30 ms of back-to-back launches (clocks settle)
        hip.step(a, out=b, generations=gens, stream=stream)
    reps, ms = 10, []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        hip.step(a, out=b, generations=gens, stream=stream)
        e1.record(stream)
        e1.synchronize()
        ms.append(e0.elapsed_time(e1))
    t = sorted(ms)[len(ms) // 2] / 1e3  # median launch
    gps = n * gens / t
    # VALU issue model of the default generation loop (rule 11, the
    # hand-allocated loop of split_asm.inc): per 4 universes
    # 64 v_bitop3 (one slot; the 6-LUT tail)
    # + 4 v_alignbit (two slots, tools/bank_probe2.hip) = 18 issue slots per
    # universe-gen; the exchange runs on the LDS pipe (ds_write_b128 x2,
    # ds_read_b128 x4).  peak: one wave64 VALU op per 2 clk per SIMD at
    # 2.4 GHz; the best rate measured for independent v_bitop3 is 0.978 ns
    # per instruction per SIMD (profiles/r01/bank_probe.jsonl), reported too.
    slots = 18
    peak_slots = 1024 * 2.4e9 / 2  # 1024 SIMDs
    measured_slots = 1024 / 0.978e-9
    cfg = hip.default_cfg(gens).as_dict()
    cpu = None
    if cpu_seconds > 0:
        cpu = cpu_baseline_config3(a.cpu().numpy().view(np.uint64), cpu_seconds)
    return {"workload": "config3: 64K universes x 1024 generations (one launch)",
            "value": gps, "unit": "universe-gen/s", "cell_updates_per_s": gps * 4096,
            "kernel_ms": t * 1e3, "kernel_ms_min": min(ms), "kernel_ms_all": ms, "launch_cfg": cfg,
            "roofline": {"bound": "valu", "achieved": gps * slots / 1e12, "peak": peak_slots / 1e12,
                         "unit": f"T VALU issue slots/s ({slots} per universe-gen)",
                         "frac": gps * slots / peak_slots,
                         "measured_issue_peak": measured_slots / 1e12,
                         "frac_of_measured_issue_peak": gps * slots / measured_slots},
            "reference_op_equivalent_Tops": OPS_PER_UNIVERSE_GEN * gps / 1e12,
            "cpu_baseline": cpu}


def verify_first_launch(hip, out, first, n, gens, seed, stream, world, device):
    """Digest of the first launch's output vs the reference's (golden.json)."""
    gold = os.path.join(ROOT, "tests", "golden", "golden.json")
    want = None
    try:
        with open(gold) as f:
            d = json.load(f)["digests"]["weak_shards_seed2"]
        k = first // n
        if (gens == 1 and seed == d["seed"] and n == d["universes_per_rank"]
                and k < len(d["shard_output_digests"])):
            want = d["shard_output_digests"][k]
    except (OSError, ValueError, KeyError):
        pass
    got = f"{batch_digest(hip.hashes(out, stream=stream).cpu().numpy(), first):016x}"
    ok = None if want is None else got == want
    if world > 1 and ok is not None:
        f = torch.tensor([0 if ok else 1], device=COLL_DEV)
        dist.all_reduce(f)
        ok = int(f.item()) == 0
    return {"ok": ok, "first_launch_digest_rank0": got, "expected": want,
            "against": "tests/golden/golden.json weak_shards_seed2 (reference Step(), all ranks)"}


def secondary_config5(hip, device, stream):
    """Config 5: unknown_step_refined ternary step, 256K universes, one launch."""
    n = 1 << 18
    planes = hip.fill_random(n * 11, seed=6, device=device, stream=stream).reshape(n, 11 * 64)
    out = torch.empty((n, 3 * 64), dtype=torch.int64, device=device)
    hip.refined_step(planes, out=out, stream=stream)  # warm
    ms = []
    for _ in range(10):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        hip.refined_step(planes, out=out, stream=stream)
        e1.record(stream)
        e1.synchronize()
        ms.append(e0.elapsed_time(e1))
    t = sorted(ms)[len(ms) // 2] / 1e3
    ups = n / t
    return {"workload": "config5: 256K universes, unknown_step_refined (11 planes in, 3 out)",
            "value": ups, "unit": "universe-steps/s", "kernel_ms_median": t * 1e3,
            "roofline": {"bound": "hbm", "achieved": n * 7168 / t / 1e9, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": n * 7168 / t / 1e9 / HBM_PEAK_GBS,
                         "algorithmic_bytes_per_universe": 7168}}


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


def main():
    args = parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; the modulo only matters for a rehearsal with more
    # ranks than GPUs (LIFEAPI_BENCH_BACKEND=gloo), never for the real run
    ndev = torch.cuda.device_count()
    device = torch.device("cuda", local % max(ndev, 1))
    torch.cuda.set_device(device)
    backend = os.environ.get("LIFEAPI_BENCH_BACKEND", "nccl")  # nccl == RCCL on ROCm
    global COLL_DEV
    COLL_DEV = device if backend == "nccl" else torch.device("cpu")
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)
    import lifeapi_amd.hip as hip

    n, gens = args.universes, args.gens_per_step
    first, _ = weak_shard(rank, n)           # contiguous shard of the global array
    stream = torch.cuda.current_stream(device)
    a = hip.fill_random(n, seed=args.seed, first_universe=first, device=device, stream=stream)
    b = torch.empty_like(a)
    want_cpu = rank == 0 and world == 1 and not args.no_cpu_baseline
    x_full = a.cpu().numpy().view(np.uint64).copy() if want_cpu else None
    bufs = [a, b]

    # warmup (untimed); the first launch's output is checked against the
    # reference-generated digest of this shard (tests/golden/golden.json)
    hip.step(bufs[0], out=bufs[1], generations=gens, stream=stream)
    verified = None
    if not args.no_verify:
        verified = verify_first_launch(hip, bufs[1], first, n, gens, args.seed, stream, world, device)
    _, cur = timed_launches(hip, [bufs[1], bufs[0]], max(args.warmup - 1, 0), gens, stream)
    bufs = [bufs[1], bufs[0]] if cur == 0 else [bufs[0], bufs[1]]
    torch.cuda.synchronize(device)

    # timed region: barrier + sync on both sides, max over ranks
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    evs, cur = timed_launches(hip, bufs, args.steps, gens, stream)
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=COLL_DEV)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    span_ms = evs[0].elapsed_time(evs[1])   # GPU time of the K launches on their stream
    final = bufs[cur]

    # result collection (not in the timed region): all-gather per-universe hashes
    h = hip.hashes(final, stream=stream)
    torch.cuda.synchronize(device)
    collect = None
    if world > 1:
        dist.barrier()
        c0 = time.perf_counter()
        gathered = gather_hashes(h.to(COLL_DEV), world)
        torch.cuda.synchronize(device)
        cms = (time.perf_counter() - c0) * 1e3
        collect = {"op": f"all_gather(per-universe hash, {'RCCL' if backend == 'nccl' else backend})",
                   "bytes_per_rank": n * 8,
                   "ms": cms}
        if rank == 0:
            collect["final_digest"] = f"{batch_digest(gathered.cpu().numpy()):016x}"

    secondary = None
    if rank == 0 and world == 1 and not args.no_secondary:
        secondary = {"config3": secondary_config3(hip, device, stream,
                                                  0.0 if args.no_cpu_baseline else args.cpu_seconds / 3),
                     "config5": secondary_config5(hip, device, stream)}

    ceiling, ceiling_src = copy_ceiling()

    cpu = None
    if want_cpu:
        cpu = cpu_baseline(x_full, args.cpu_seconds)

    if world > 1:
        dist.barrier()
    if rank == 0:
        total = n * world * gens * args.steps
        value = total / elapsed
        avg_launch = span_ms / args.steps  # includes the ~1-2 us launch gaps: conservative
        achieved = n * gens * BYTES_PER_UNIVERSE_GEN / (avg_launch / 1e3) / 1e9 if gens == 1 else None
        traffic, tsrc = load_pmc_traffic(n)
        cfg = hip.default_cfg(gens).as_dict()
        line = {
            "metric": METRIC, "value": value, "unit": "universe-gen/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64",
            "data": f"synthetic: splitmix64 uniform-fill universes (seed {args.seed}), generated on device",
            "config": {"workload": f"config2: {n} random-fill 64x64 universes x {gens} generation "
                                   f"per step per GPU", "universes_per_gpu": n,
                       "global_universes": n * world, "gens_per_step": gens,
                       "parallelism": f"dp{world} (contiguous universe shards, no collective)",
                       "launch_cfg": cfg},
            "cell_updates_per_s": value * 4096,
            "kernel_ms_avg": avg_launch,
            "kernel_timing": "HIP events on the launch stream around the K timed launches / K",
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
                         "traffic": traffic, "traffic_source": tsrc,
                         "algorithmic_bytes_per_launch": n * gens * BYTES_PER_UNIVERSE_GEN,
                         "read_only_GBps": achieved / 2 if achieved else None,
                         "copy_ceiling_GBps": ceiling, "copy_ceiling_source": ceiling_src,
                         "frac_of_copy_ceiling": (achieved / ceiling) if (achieved and ceiling) else None},
            "cpu_baseline": cpu,
            "verified": verified,
            "collect": collect,
            "secondary": secondary,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
