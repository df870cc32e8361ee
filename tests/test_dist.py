"""CPU, world_size 2 (gloo): the N>1 path -- contiguous universe shards, no
data-path collective, hash all-gather for result collection -- gives exactly
the single-process answer.  Compute here is the oracle (test infrastructure);
the GPU ranks run the same lifeapi_amd.shard logic around the HIP kernel."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, mode, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from lifeapi_amd.shard import gather_hashes, strong_shard, weak_shard
        from oracle.oracle import Port
        P = Port()
        if mode == "weak":
            first, cnt = weak_shard(rank, n)
            counts = [n] * world
        else:
            first, cnt = strong_shard(rank, world, n)
            counts = [strong_shard(r, world, n)[1] for r in range(world)]
        x = P.fill(cnt, seed=4, first_universe=first)
        out = P.step_batch(x, 3)
        h = torch.from_numpy(P.hashes(out).view(np.int64).copy())
        g = gather_hashes(h, world, counts)
        # shard digests are additive mod 2^64: gather them as int64 bit patterns
        d = P.digest(P.hashes(out), first)
        parts = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(parts, torch.tensor([d - (1 << 64) if d >= 1 << 63 else d]))
        if rank == 0:
            q.put((g.numpy().view(np.uint64).copy(), [int(p.item()) % (1 << 64) for p in parts]))
    finally:
        dist.destroy_process_group()


def _run(mode, n, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mode, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def _single(total, P):
    x = P.fill(total, seed=4)
    out = P.step_batch(x, 3)
    return P.hashes(out), P.digest(P.hashes(out))


def test_weak_shards_gather_equals_single_process():
    from oracle.oracle import Port
    P = Port()
    n = 1000
    gathered, shard_digests = _run("weak", n)
    h, d = _single(2 * n, P)
    assert (gathered == h).all()
    assert sum(shard_digests) % (1 << 64) == d


def test_strong_ragged_shards():
    from oracle.oracle import Port
    P = Port()
    n = 1001  # not divisible by world
    gathered, shard_digests = _run("strong", n)
    h, d = _single(n, P)
    assert (gathered == h).all()
    assert sum(shard_digests) % (1 << 64) == d
