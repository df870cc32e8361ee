"""GPU parity: the HIP path through the C ABI vs the CPU oracle.

Bit-exact on every word (integer work, no tolerance).  Oracle = the C
restatement (oracle/lifeapi_oracle.c) pinned against the reference's own
Step() (oracle/_ref, tests/test_oracle.py).  Mirrors tests/StepAltTest.cpp:5-13
(differential Step vs an independent formulation) on seeded inputs.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

def to_dev(a: np.ndarray) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int64).reshape(-1, 64).copy()).cuda()


def to_host(t: torch.Tensor) -> np.ndarray:
    torch.cuda.synchronize()
    return t.cpu().numpy().view(np.uint64).reshape(-1, 64)


def seam_cases(port):
    """Universes with cells on the torus seams (columns 0/63, rows 0/63)."""
    out = []
    s = np.zeros(64, np.uint64)
    s[0] = s[63] = s[1] = np.uint64(0x8000000000000003)
    out.append(s.copy())
    s = np.zeros(64, np.uint64)
    s[62] = s[63] = s[0] = np.uint64((1 << 63) | 1)       # blinker/block across both seams
    out.append(s.copy())
    out.append(np.full(64, np.uint64(2**64 - 1)))            # all on -> empty
    chk = np.array([0xAAAAAAAAAAAAAAAA if x % 2 == 0 else 0x5555555555555555 for x in range(64)],
                   dtype=np.uint64)
    out.append(chk)                                          # checkerboard -> empty
    g = port.parse("bo$2bo$3o!")                             # glider
    out.append(np.roll(g, 62))                               # glider straddling column seam
    out.append(np.array([(int(w) << 62 | int(w) >> 2) & (2**64 - 1) for w in g],
                        dtype=np.uint64))                    # glider straddling row seam
    out.append(np.zeros(64, np.uint64))
    return np.stack(out)


def test_single_runtime(hip):
    assert len(hip.loaded_hip_runtimes()) == 1, hip.loaded_hip_runtimes()


@pytest.mark.parametrize("n", [1, 2, 3, 5, 63, 64, 65, 4097])
def test_ragged_default(hip, port, n):
    x = port.fill(n, seed=n)
    for gens in (1, 3):
        got = to_host(hip.step(to_dev(x), generations=gens))
        assert (got == port.step_batch(x, gens)).all()


@pytest.mark.parametrize("n", [1, 3, 5, 4097, (1 << 21) - 1, (1 << 21) + 1])
def test_alternating_order_launches(hip, port, n):
    """The streaming step takes the groups in the reverse order on every
    other launch and stores the last min(256 MiB, half the batch) of each
    launch with plain stores (step.hip): four launches in a row, ping-pong
    and in place, each equal to the oracle whichever order it ran in, with
    the plain/nontemporal boundary inside the batch."""
    x = port.fill(n, seed=n + 11)
    want = [x]
    for _ in range(4):
        want.append(port.step_batch(want[-1], 1, nthreads=16))
    a, b = to_dev(x), torch.empty((n, 64), dtype=torch.int64, device="cuda")
    for k in range(1, 5):
        hip.step(a, out=b, generations=1)
        assert (to_host(b) == want[k]).all(), k
        a, b = b, a
    d = to_dev(x)
    for k in range(1, 3):
        hip.step(d, out=d, generations=1)
        assert (to_host(d) == want[k]).all(), k


def test_zero_gens_and_empty(hip, port):
    x = port.fill(17, seed=5)
    assert (to_host(hip.step(to_dev(x), generations=0)) == x).all()
    e = torch.empty((0, 64), dtype=torch.int64, device="cuda")
    hip.step(e, generations=1)


def test_inplace(hip, port):
    x = port.fill(3001, seed=77)
    d = to_dev(x)
    hip.step(d, out=d, generations=1)
    assert (to_host(d) == port.step_batch(x, 1)).all()
    hip.step(d, out=d, generations=9)
    assert (to_host(d) == port.step_batch(x, 10)).all()


def test_overlap_rejected(hip):
    d = torch.zeros((10, 64), dtype=torch.int64, device="cuda")
    with pytest.raises(hip.LifeApiError) as e:
        hip.step(d[:8], out=d[1:9], generations=1)
    assert e.value.code == -1


def test_iterated_randomstate_shaped(hip, port):
    """Config-3 shape at small n: RandomState()-shaped columns, many gens."""
    x = port.fill(1024, seed=3, mode=1)
    got = to_host(hip.step(to_dev(x), generations=300))
    assert (got == port.step_batch(x, 300, nthreads=8)).all()


def test_rpentomino_1103(hip, port):
    r = port.parse("b2o$2o$bo!")
    got = to_host(hip.step(to_dev(r[None]), generations=1103))[0]
    assert int(sum(bin(int(w)).count("1") for w in got)) == 113
    assert (got == port.step_batch(r[None], 1103)[0]).all()


def test_fill_matches_oracle(hip, port):
    for mode in (0, 1):
        got = to_host(hip.fill_random(1000, seed=42, first_universe=12345, mode=mode))
        assert (got == port.fill(1000, 42, 12345, mode)).all()


def test_pop_hash_digest(hip, port):
    x = port.fill(5000, seed=9)
    d = to_dev(x)
    assert (hip.pop(d).cpu().numpy().astype(np.uint32) == port.pop(x)).all()
    h = hip.hashes(d).cpu().numpy().view(np.uint64)
    assert (h == port.hashes(x)).all()


def test_contains(hip, port):
    x = port.fill(600, seed=11)
    block = port.parse("2o$2o!")
    x[:200] = 0
    x[:100, 10] |= np.uint64(3 << 20)
    x[:100, 11] |= np.uint64(3 << 20)
    wanted = np.roll(block, 10) << np.uint64(20)
    unwanted = np.zeros(64, np.uint64)
    for c in (9, 12):
        unwanted[c] = np.uint64(0xF << 19)
    unwanted[10] |= np.uint64(0x9 << 19)
    unwanted[11] |= np.uint64(0x9 << 19)
    got = hip.contains(to_dev(x), to_dev(wanted[None]), to_dev(unwanted[None])).cpu().numpy()
    want = np.array([port.contains(x[u], wanted, unwanted) for u in range(len(x))])
    assert (got.astype(bool) == want).all() and want[:100].all() and not want[100:200].any()


def _off8(a: np.ndarray) -> torch.Tensor:
    """a on the device at an address that is 8 mod 16 (8-byte aligned only)"""
    t = torch.zeros(a.size + 1, dtype=torch.int64, device="cuda")
    v = t[1:].view(a.shape)
    v.copy_(to_dev(a))
    assert v.data_ptr() % 16 == 8
    return v


@pytest.mark.parametrize("n", [1, 7, 4099])
def test_reductions_on_8_byte_aligned_batches(hip, port, n):
    """GetPop, Contains and the fill take 16-byte accesses on 16-byte
    aligned batches (reduce.hip) and fall back to 8-byte ones otherwise;
    both equal the oracle, ragged n included"""
    x = port.fill(n, seed=n + 900)
    w, u = x[0].copy(), np.zeros(64, np.uint64)
    u[5] = np.uint64(0xFF)
    u &= ~w
    want_c = np.array([port.contains(x[k], w, u) for k in range(n)])
    for d in (to_dev(x), _off8(x)):
        assert (hip.pop(d).cpu().numpy().astype(np.uint32) == port.pop(x)).all()
        got = hip.contains(d, to_dev(w[None]), to_dev(u[None])).cpu().numpy().astype(bool)
        assert (got == want_c).all() and got[0]
    out = _off8(np.zeros((n, 64), np.uint64))
    for mode in (0, 1):
        hip.fill_random(n, seed=3, first_universe=77, mode=mode, out=out)
        assert (to_host(out) == port.fill(n, 3, 77, mode)).all()


@pytest.mark.parametrize("gens", [1, 2, 3, 5, 8, 13])
def test_filter_on_8_byte_aligned_batches(hip, port, gens):
    """The search filter without final states takes LDS-DMA forms on 16-byte
    aligned batches (k_cone_adapt's DMA form at 1-2 generations, the merged
    split kernel's prefetch and the whole-board window pass's DMA chunks
    from 3) and 8-byte loads otherwise: a block + ring (column window, the
    shrinking pass), a one-row whole board (row window) and a full-height
    target (no window) on both alignments, ragged n, against the oracle"""
    n = 1001
    x = port.fill(n, seed=300 + gens) & port.fill(n, seed=400 + gens)
    bw, bu = np.zeros(64, np.uint64), np.zeros(64, np.uint64)
    bw[10] = bw[11] = np.uint64(3 << 40)
    bu[9:13] = np.uint64(15 << 39)
    bu &= ~bw
    ru = np.zeros(64, np.uint64)
    ru[0::3] = np.uint64(1 << 10)
    fu = np.zeros(64, np.uint64)
    for y in range(0, 64, 4):
        fu[(3 * y) % 64] |= np.uint64(1 << y)
    for w, u in ((bw, bu), (np.zeros(64, np.uint64), ru), (np.zeros(64, np.uint64), fu)):
        res, s = np.zeros(n, np.uint32), x.copy()
        for g in range(1, gens + 1):
            s = port.step_batch(s, 1, nthreads=8)
            hit = (((s ^ w) & (w | u)) == 0).all(axis=1)
            res[(res == 0) & hit] = g
        for d in (to_dev(x), _off8(x)):
            first, _ = hip.step_contains(d, to_dev(w[None]), to_dev(u[None]), gens)
            got = first.cpu().numpy().astype(np.uint32)
            assert (got == res).all(), (gens, d.data_ptr() % 16, int(np.count_nonzero(u)), int((got != res).sum()))


def test_step_contains(hip, port):
    # blinkers: contained every second generation
    b = np.zeros(64, np.uint64)
    b[30] = b[31] = b[32] = np.uint64(1 << 20)          # horizontal blinker
    vert = port.step_batch(b[None], 1)[0]
    x = np.stack([b, vert, port.fill(1, 5)[0]])
    wanted = vert
    unwanted = np.zeros(64, np.uint64)
    first, final = hip.step_contains(to_dev(x), to_dev(wanted[None]), to_dev(unwanted[None]), 6,
                                     final=torch.empty((3, 64), dtype=torch.int64, device="cuda"))
    f = first.cpu().numpy()
    exp = []
    for u in range(3):
        s, hit = x[u].copy(), 0
        for g in range(1, 7):
            s = port.step_batch(s[None], 1)[0]
            if hit == 0 and port.contains(s, wanted, unwanted):
                hit = g
        exp.append(hit)
    assert list(f) == exp and exp[0] == 1 and exp[1] == 2
    assert (to_host(final) == port.step_batch(x, 6)).all()


@pytest.mark.parametrize("gens", [1, 2, 3, 6, 37])
@pytest.mark.parametrize("with_final", [False, True])
def test_step_contains_batch(hip, port, gens, with_final):
    """First generation containing a block + its empty ring (LifeTarget.hpp:44-51)
    over ragged batches of sparse soups and planted blinkers/blocks, every layout
    the entry point picks (natural for gens <= 2, 8-way split above)."""
    n = 1003
    x = port.fill(n, seed=123) & port.fill(n, seed=124) & port.fill(n, seed=125)
    blk = np.zeros(64, np.uint64)
    blk[10] = blk[11] = np.uint64(0b11 << 40)
    ring = np.zeros(64, np.uint64)
    for c in (9, 10, 11, 12):
        ring[c] = np.uint64(0b1111 << 39)
    ring &= ~blk
    x[::7] &= ~ring & ~blk                               # clear the spot ...
    x[::14] |= blk                                       # ... and plant blocks in half of them
    wanted, unwanted = blk, ring
    fin = torch.empty((n, 64), dtype=torch.int64, device="cuda") if with_final else None
    first, final = hip.step_contains(to_dev(x), to_dev(wanted[None]), to_dev(unwanted[None]), gens, final=fin)
    got = first.cpu().numpy()
    exp = np.zeros(n, np.int64)
    s = x.copy()
    for g in range(1, gens + 1):
        s = port.step_batch(s, 1)
        hit = (((s ^ wanted) & (wanted | unwanted)) == 0).all(axis=1)
        exp[(exp == 0) & hit] = g
    assert (got == exp).all(), np.nonzero(got != exp)[0][:10]
    assert exp.any()
    if with_final:
        assert (to_host(final) == s).all()


def test_host_api(hip, port):
    x = port.fill(2500, seed=8)
    assert (hip.step_host(x, 4, device=0).reshape(-1, 64) == port.step_batch(x, 4)).all()
    assert (hip.step_host(x, 1, device=-1).reshape(-1, 64) == port.step_batch(x, 1)).all()
    assert (hip.pop_host(x) == port.pop(x)).all()


def test_host_api_many_chunks_pinned(hip, port):
    """More chunks than lanes (64 MiB chunks, two lanes: 300K universes is
    three chunks, the last ragged), in place and out of place, pageable and
    page-locked (lifeapi_host_register)."""
    n = 300_000
    x = port.fill(n, seed=9)
    want = port.step_batch(x, 2)
    out = np.zeros_like(x)
    assert (hip.step_host(x, 2, out=out).reshape(-1, 64) == want).all()
    # the call pinned the pageable arrays for its duration only (unpinned again)
    assert hip.lib.lifeapi_host_unregister(x.ctypes.data) != 0
    assert hip.lib.lifeapi_host_unregister(out.ctypes.data) != 0
    y = x.copy()
    with hip.host_pinned(y, out):  # the call must leave the caller's pins in place
        out[:] = 0
        assert (hip.step_host(y, 2, out=out).reshape(-1, 64) == want).all()
        hip.step_host(y, 2, out=y)  # in place, pinned
        assert (y == want).all()
    assert hip.lib.lifeapi_host_unregister(y.ctypes.data) != 0  # no longer registered


def test_host_api_concurrent_shared_input(hip, port):
    """Calls from several threads on one shared (pageable) input: each call
    pins it for its duration (a shared, counted pin), and none may unpin it
    under another's copies; afterwards it is no longer registered."""
    import threading
    n = 40_000  # 20 MiB: above the per-call pinning threshold
    x = port.fill(n, seed=21)
    want = port.step_batch(x, 3)
    outs = [np.zeros_like(x) for _ in range(4)]
    errs = []

    def run(o):
        try:
            for _ in range(3):
                o[:] = 0
                hip.step_host(x, 3, out=o)
                if not (o.reshape(-1, 64) == want).all():
                    errs.append("mismatch")
        except Exception as e:  # noqa: BLE001 - reported below
            errs.append(repr(e))

    ts = [threading.Thread(target=run, args=(o,)) for o in outs]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs
    assert hip.lib.lifeapi_host_unregister(x.ctypes.data) != 0


def test_host_api_small_and_partial_overlaps_of_a_pinned_range(hip, port):
    """While large calls pin a shared array per call, other threads make small
    calls (< 8 MiB, never pinned by themselves) inside it and large calls on
    ranges that only partly overlap it: every call takes a reference on each
    pin it touches (host.hip pin_acquire), so no copy of theirs can run from
    memory another call unpins.  All results must match the oracle, and the
    array ends unregistered."""
    import threading
    n = 48_000                                   # 24 MiB
    x = port.fill(n, seed=31)
    want = port.step_batch(x, 2)
    errs = []

    def big():
        o = np.zeros_like(x)
        for _ in range(3):
            hip.step_host(x, 2, out=o)
            if not (o == want).all():
                errs.append("big mismatch")

    def small(lo):
        for _ in range(6):
            got = hip.step_host(x[lo:lo + 1000], 2)        # 500 KiB inside the pinned range
            if not (got == want[lo:lo + 1000]).all():
                errs.append(f"small mismatch at {lo}")

    def partial(lo):
        for _ in range(3):
            got = hip.step_host(x[lo:lo + 30_000], 2)      # 15 MiB straddling other calls' ranges
            if not (got == want[lo:lo + 30_000]).all():
                errs.append(f"partial mismatch at {lo}")

    def guard(fn, *a):
        try:
            fn(*a)
        except Exception as e:  # noqa: BLE001 - reported below
            errs.append(repr(e))

    ts = [threading.Thread(target=guard, args=(big,)), threading.Thread(target=guard, args=(big,)),
          threading.Thread(target=guard, args=(small, 100)), threading.Thread(target=guard, args=(small, 40_000)),
          threading.Thread(target=guard, args=(partial, 0)), threading.Thread(target=guard, args=(partial, 18_000))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs
    assert hip.lib.lifeapi_host_unregister(x.ctypes.data) != 0


@pytest.mark.parametrize("gens", [2, 40])
def test_host_step_contains(hip, port, gens):
    """lifeapi_step_contains_batch on host arrays (natural layout for gens <= 2,
    the split layout above), in place and without final states, vs the oracle."""
    n = 2001
    x = port.fill(n, seed=51) & port.fill(n, seed=52) & port.fill(n, seed=53)
    blk = np.zeros(64, np.uint64)
    blk[20] = blk[21] = np.uint64(0b11 << 30)
    ring = np.zeros(64, np.uint64)
    for c in (19, 20, 21, 22):
        ring[c] = np.uint64(0b1111 << 29)
    ring &= ~blk
    x[::5] &= ~ring & ~blk
    x[::10] |= blk
    exp = np.zeros(n, np.uint32)
    s = x.copy()
    for g in range(1, gens + 1):
        s = port.step_batch(s, 1)
        hit = (((s ^ blk) & (blk | ring)) == 0).all(axis=1)
        exp[(exp == 0) & hit] = g
    assert exp.any()
    assert (hip.step_contains_host(x, blk, ring, gens) == exp).all()
    y = x.copy()
    assert (hip.step_contains_host(y, blk, ring, gens, final=y) == exp).all()
    assert (y == s).all()


def test_host_api_other_kernels(hip, port):
    """Host-pointer forms of the weld / stable / counts / refined / contains
    entry points (staged through device memory in chunks)."""
    L = hip.lib
    w = port.fill(300 * 4, seed=31).reshape(300, 256)
    w[:, 64:] &= port.fill(900, seed=32).reshape(300, 192)
    hw = w.copy()
    hip._check(L.lifeapi_weld_step_batch(hw.ctypes.data, 300, 3, 0))
    assert (hw == port.weld_step(w, 3)).all()
    x = port.fill(200, seed=33)
    nc = np.zeros((200, 4, 64), np.uint64)
    hip._check(L.lifeapi_neighbour_count_batch(x.ctypes.data, nc.ctypes.data, 200, 0))
    assert all((nc[u] == port.neighbour_count(x[u])).all() for u in range(200))
    ic = np.zeros((200, 3, 64), np.uint64)
    hip._check(L.lifeapi_interaction_counts_batch(x.ctypes.data, ic.ctypes.data, 200, 0, 0))
    assert all((ic[u] == port.interaction_counts(x[u])[:3]).all() for u in range(200))
    r = port.fill(50 * 11, seed=34).reshape(50, 704)
    ro = np.zeros((50, 192), np.uint64)
    hip._check(L.lifeapi_refined_step_batch(r.ctypes.data, ro.ctypes.data, 50, 0))
    assert (ro == port.refined_step(r)).all()
    want, unw = x[7].copy(), np.zeros(64, np.uint64)
    hit = np.zeros(200, np.uint8)
    hip._check(L.lifeapi_contains_batch(x.ctypes.data, want.ctypes.data, unw.ctypes.data,
                                        hit.ctypes.data, 200, 0))
    assert (hit.astype(bool) == [port.contains(x[u], want, unw) for u in range(200)]).all()
    import os
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "stable.npz"))
    sp = np.ascontiguousarray(g["input"]).copy()
    fl = np.zeros(len(sp), np.uint8)
    hip._check(L.lifeapi_stable_pass_batch(sp.ctypes.data, fl.ctypes.data, len(sp), 4, 0, 0))
    assert (sp == g["propagate"]).all() and (fl == g["propagate_flags"]).all()


def test_full_size_config2(hip, port):
    """Config 2 at full size (1M universes x 1 gen): every word vs the oracle."""
    n = 1 << 20
    d = hip.fill_random(n, seed=2)
    x = to_host(d)
    assert (x[:4096] == port.fill(4096, 2)).all()
    got = to_host(hip.step(d, generations=1))
    want = port.step_batch(x, 1, nthreads=16)
    assert (got == want).all()
    # checksum of checksums agrees too
    assert port.digest(hip.hashes(hip.step(d)).cpu().numpy().view(np.uint64)) == \
        port.digest(port.hashes(want))


def test_config4_all_shards_vs_reference_digests(hip):
    """Config 4 (16M universes x 1 gen, 8 shards of 2M): every shard's output
    digest equals the reference's (tests/golden/golden.json), one GPU doing
    the shards in turn -- the same contiguous shards the 8 ranks own."""
    import json
    import os

    from lifeapi_amd.digest import batch_digest, combine
    with open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")) as f:
        d = json.load(f)["digests"]["config4"]
    per = d["universes"] // d["shards"]
    a = torch.empty((per, 64), dtype=torch.int64, device="cuda")
    b = torch.empty_like(a)
    got = []
    for k in range(d["shards"]):
        hip.fill_random(per, seed=d["seed"], first_universe=k * per, out=a)
        hip.step(a, out=b, generations=1)
        got.append(batch_digest(hip.hashes(b).cpu().numpy(), k * per))
    assert [f"{g:016x}" for g in got] == d["shard_output_digests"]
    assert f"{combine(got):016x}" == d["output_digest"]


def test_config4_one_launch_vs_reference_digest(hip):
    """Config 4's 16M universes in ONE launch: the large-batch launch (above
    4M universes: one order, nontemporal, each XCD a contiguous eighth of the
    batch, step.hip shipped_step) against the reference's digest."""
    import json
    import os

    from lifeapi_amd.digest import batch_digest, combine
    with open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")) as f:
        d = json.load(f)["digests"]["config4"]
    n, per = d["universes"], d["universes"] // d["shards"]
    a = hip.fill_random(n, seed=d["seed"])
    b = hip.step(a, generations=1)
    h = hip.hashes(b).cpu().numpy()
    got = [batch_digest(h[k * per:(k + 1) * per], k * per) for k in range(d["shards"])]
    assert f"{combine(got):016x}" == d["output_digest"]
    del a, b
    torch.cuda.empty_cache()


@pytest.mark.parametrize("n", [(1 << 22) + 4099, (5 << 20) + 3])
def test_large_batch_launch_equals_small_batch_launches(hip, n):
    """Batches above 4M universes take the XCD-chunked launch, whose grid
    need not be a multiple of 8 blocks (ragged n here): ping-pong and in
    place, every universe equals the small-batch launches (checked against
    the reference above) stepping the same universes in pieces of <= 4M."""
    x = hip.fill_random(n, seed=31)
    want = torch.empty_like(x)
    half = n // 2
    hip.step(x[:half], out=want[:half], generations=1)
    hip.step(x[half:], out=want[half:], generations=1)
    got = hip.step(x, generations=1)
    assert torch.equal(got, want)
    y = x.clone()
    hip.step(y, out=y, generations=1)
    assert torch.equal(y, want)
    del x, want, got, y
    torch.cuda.empty_cache()


def test_config3_full_size_vs_reference_digest(hip):
    """Config 3 (64K x 1024 generations, one launch) vs the reference's digest."""
    import json
    import os

    from lifeapi_amd.digest import batch_digest
    with open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")) as f:
        d = json.load(f)["digests"]["config3"]
    x = hip.fill_random(d["universes"], seed=d["seed"])
    out = hip.step(x, generations=d["generations"])
    assert f"{batch_digest(hip.hashes(out).cpu().numpy()):016x}" == d["output_digest"]
    assert int(hip.pop(out).sum().item()) == d["output_pop_total"]


# ---- neighbourhood counters ----

def test_counts_golden_gpu(hip):
    import os
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "counts.npz"))
    d = to_dev(g["input"])
    nc = hip.neighbour_count(d)
    ic = hip.interaction_counts(d, with_next=True)
    ic3 = hip.interaction_counts(d, with_next=False)
    torch.cuda.synchronize()
    assert (nc.cpu().numpy().view(np.uint64) == g["neighbour_count"]).all()
    assert (ic.cpu().numpy().view(np.uint64) == g["interaction_counts"]).all()
    assert (ic3.cpu().numpy().view(np.uint64) == g["interaction_counts"][:, :3]).all()


def test_counts_vs_oracle_ragged(hip, port):
    x = np.concatenate([seam_cases(port), port.fill(2001, seed=8080)])
    d = to_dev(x)
    nc = hip.neighbour_count(d).cpu().numpy().view(np.uint64)
    ic = hip.interaction_counts(d, with_next=True).cpu().numpy().view(np.uint64)
    for u in range(0, len(x), 7):
        assert (nc[u] == port.neighbour_count(x[u])).all()
        assert (ic[u] == port.interaction_counts(x[u])).all()
    assert (ic[:, 3] == port.step_batch(x, 1)).all()


# ---- LifeWeld::Step ----

def test_weld_golden_gpu(hip):
    import os
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "weld.npz"))
    for gens, key in ((1, "step1"), (7, "step7")):
        d = to_dev(g["input"]).reshape(-1, 256)
        hip.weld_step(d, gens)
        torch.cuda.synchronize()
        assert (d.cpu().numpy().view(np.uint64) == g[key]).all()


@pytest.mark.parametrize("n,gens", [(3003, 1), (3003, 2), (3003, 4), (3003, 12), (3003, 31), (5, 33), (1, 13), (1026, 100)])
def test_weld_vs_oracle_ragged(hip, port, n, gens):
    """Natural layout (gens < 12) and the split-layout kernel (k_weld_split,
    4 welds per wave: ragged n; nontemporal below 32 gens) against the
    oracle's LifeWeld::Step."""
    w = port.fill(n * 4, seed=9191 + gens).reshape(n, 256)
    w[:, 64:] &= port.fill(n * 3, seed=9192 + gens).reshape(n, 192)
    d = to_dev(w).reshape(n, 256)
    hip.weld_step(d, gens)
    torch.cuda.synchronize()
    assert (d.cpu().numpy().view(np.uint64) == port.weld_step(w, gens)).all()


# ---- LifeStable passes ----

def test_stable_passes_golden_gpu(hip):
    import os
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "stable.npz"))
    for name in hip.STABLE_PASSES:
        d = to_dev(g["input"]).reshape(-1, 640)
        fl = hip.stable_pass(d, name)
        torch.cuda.synchronize()
        assert (d.cpu().numpy().view(np.uint64) == g[name]).all(), name
        assert (fl.cpu().numpy() == g[name + "_flags"]).all(), name


def _stable_cases(port, n, seed=5):
    """Seeded still-life neighbourhoods with an unknown window (mostly
    consistent) and, every fourth, random option planes (mostly
    inconsistent), as (n, 640) uint64 planes."""
    rng = np.random.default_rng(seed)
    x = np.zeros((n, 10, 64), np.uint64)
    blocks = port.parse("2o$2o!")
    for u in range(n):
        st = np.zeros(64, np.uint64)
        for _ in range(6):  # well separated blocks on a 16x16 lattice: a still life
            bx, by = int(rng.integers(4)) * 16, int(rng.integers(4)) * 16
            st |= np.roll(blocks, bx) << np.uint64(by)
        w0, h0 = int(rng.integers(4, 20)), int(rng.integers(4, 20))
        x0, y0 = int(rng.integers(0, 64 - w0)), int(rng.integers(0, 64 - h0))
        unk = np.zeros(64, np.uint64)
        unk[x0:x0 + w0] = np.uint64(((1 << h0) - 1) << y0)
        x[u, 0], x[u, 1] = st & ~unk, unk
        if u % 4 == 3:
            f = port.fill(10, seed=u)
            x[u, 2:] = f[2:] & port.fill(8, seed=u + 1000)
    return x.reshape(n, 640)


def test_stable_passes_vs_oracle(hip, port):
    """_stable_cases, every pass, then Vulnerable."""
    n = 300
    x = _stable_cases(port, n)
    results = {}
    for w, name in enumerate(hip.STABLE_PASSES):
        d = to_dev(x).reshape(n, 640)
        fl = hip.stable_pass(d, name).cpu().numpy()
        want, wfl = port.stable_pass(x, w)
        assert (d.cpu().numpy().view(np.uint64) == want).all(), name
        assert (fl == wfl).all(), name
        results[name] = (want, wfl)
    want, wfl = results["propagate"]
    assert (wfl & 1).sum() > n // 3  # the propagate loop ran to a fixpoint on many
    # Vulnerable (LifeStable.hpp:366-412) on the raw and on the propagated planes
    for planes in (x, want):
        got = hip.stable_vulnerable(to_dev(planes).reshape(n, 640))
        exp = port.stable_vulnerable(planes)
        assert (to_host(got) == exp).all()
    assert exp.any()


def test_stable_passes_chunked_grid_ragged(hip, port):
    """The passes deal each XCD a contiguous eighth of the batch
    (device.hpp xcd_chunk_block) on any grid: 20003 LifeStables (5001
    blocks, not a multiple of 8), every pass against the oracle."""
    n = 20003
    x = _stable_cases(port, n, seed=9)
    for w, name in enumerate(hip.STABLE_PASSES):
        d = to_dev(x).reshape(n, 640)
        fl = hip.stable_pass(d, name).cpu().numpy()
        want, wfl = port.stable_pass(x, w)
        assert (d.cpu().numpy().view(np.uint64) == want).all(), name
        assert (fl == wfl).all(), name
        if name == "propagate":
            assert (wfl & 1).sum() > n // 3
    got = hip.stable_vulnerable(to_dev(x).reshape(n, 640))
    assert (to_host(got) == port.stable_vulnerable(x)).all()


def test_step_contains_final_states_capped_grid(hip, port):
    """With final states the split pair runs on grids of at most 32 blocks
    per CU looping over the batch (step.hip kSplitIterBlocksPerCU): 200003
    universes (more than one pass of the capped grid, ragged), 9 and 40
    generations, first hits and final states against the oracle."""
    n = 200003
    x = port.fill(n, seed=77) & port.fill(n, seed=78)
    w, u = np.zeros(64, np.uint64), np.zeros(64, np.uint64)
    w[10] = w[11] = np.uint64(3 << 40)
    for c in (9, 10, 11, 12):
        u[c] = np.uint64(15 << 39)
    u &= ~w
    x[::5] = (x[::5] & ~(w | u)) | w
    for gens in (9, 40):
        fin = torch.empty((n, 64), dtype=torch.int64, device="cuda")
        first, _ = hip.step_contains(to_dev(x).reshape(n, 64), to_dev(w[None]), to_dev(u[None]), gens, final=fin)
        want, s = np.zeros(n, np.int64), x.copy()
        for g in range(1, gens + 1):
            s = port.step_batch(s, 1, nthreads=8)
            hit = (((s ^ w) & (w | u)) == 0).all(axis=1)
            want[(want == 0) & hit] = g
        assert (first.cpu().numpy() == want).all(), gens
        assert (to_host(fin) == s).all(), gens
        assert (want > 0).sum() > 500  # hits (the planted blocks that survive their neighbours)


def test_stable_passes_next_node_changed_lines(hip, port):
    """The passes store only the 128-byte lines holding a changed column
    (stable_kernels.hpp): on a search's next node -- _stable_cases propagated
    to their fixpoint by the oracle, then one unknown cell decided (ON or OFF
    by turns) -- a few columns change, so nearly every line is skipped, and a
    change the kernel failed to record would leave its line stale.  Every
    pass in place against the oracle, and the host-pointer form too."""
    n = 1000
    x, _ = port.stable_pass(_stable_cases(port, n, seed=21), 4)
    x = x.reshape(n, 10, 64).copy()
    decided = 0
    for u in range(n):
        cols = np.nonzero(x[u, 1])[0]
        if len(cols) == 0:
            continue
        c = int(cols[len(cols) // 2])
        low = x[u, 1, c] & (~x[u, 1, c] + np.uint64(1))
        x[u, 1, c] &= ~low
        if u % 2:
            x[u, 0, c] |= low
        decided += 1
    assert decided > n // 2
    x = x.reshape(n, 640)
    for w, name in enumerate(hip.STABLE_PASSES):
        want, wfl = port.stable_pass(x, w)
        changed_cols = (want.reshape(n, 10, 64) != x.reshape(n, 10, 64)).any(axis=1).sum(axis=1)
        d = to_dev(x).reshape(n, 640)
        fl = hip.stable_pass(d, name).cpu().numpy()
        assert (d.cpu().numpy().view(np.uint64) == want).all(), name
        assert (fl == wfl).all(), name
        if name == "propagate":
            assert 0 < np.median(changed_cols) <= 16  # few columns change: most lines are skipped
            h = np.ascontiguousarray(x).copy()
            flags = np.zeros(n, np.uint8)
            hip._check(hip.lib.lifeapi_stable_pass_batch(h.ctypes.data, flags.ctypes.data, n, w, 0, 0))
            assert (h == want).all() and (flags == wfl).all()


def test_stable_sync_clears_unknown_without_reference_change(hip, port):
    """SynchroniseStateKnown (LifeStable.hpp:526-556) clears `unknown` where
    live2 and live3 are both ruled out (the cell becomes known-off), but the
    reference's `changes` mask does not include those cells, so its flag says
    "no change".  The kernel's changed-line stores must still write the
    line: one such unknown cell per LifeStable, everything else
    already synchronised, at every column of the board."""
    n = 64 * 3
    x = np.zeros((n, 10, 64), np.uint64)
    x[:, 2] = x[:, 3] = ~np.uint64(0)  # live2 = live3 = 1 everywhere: known-off cells settled
    for u in range(n):
        c, r = u % 64, (7 * u) % 64
        x[u, 1, c] = np.uint64(1) << np.uint64(r)
    x = x.reshape(n, 640)
    want, wfl = port.stable_pass(x, 0)
    assert not want.reshape(n, 10, 64)[:, 1].any()  # the reference clears every unknown bit
    assert (wfl == 1).all()  # ... and reports no change
    for name in ("sync", "step", "propagate", "stabilise"):
        if name not in hip.STABLE_PASSES:
            continue
        w = hip.STABLE_PASSES.index(name)
        want, wfl = port.stable_pass(x, w)
        d = to_dev(x).reshape(n, 640)
        fl = hip.stable_pass(d, name).cpu().numpy()
        assert (d.cpu().numpy().view(np.uint64) == want).all(), name
        assert (fl == wfl).all(), name


def test_stable_options_then_sync_on_device(hip, port):
    """The sequence ADVICE r04 named: UpdateOptions then SynchroniseStateKnown,
    both on the device in place, on _stable_cases with fresh options (the
    sync clears unknown bits the options pass ruled live2 and live3 out of),
    then PropagateStep on the result; planes and flags against the oracle
    after every pass."""
    n = 2000
    x = _stable_cases(port, n, seed=33)
    d = to_dev(x).reshape(n, 640)
    cur = x
    for name in ("options", "sync", "step", "options", "sync"):
        w = hip.STABLE_PASSES.index(name)
        want, wfl = port.stable_pass(cur, w)
        fl = hip.stable_pass(d, name).cpu().numpy()
        assert (d.cpu().numpy().view(np.uint64) == want).all(), name
        assert (fl == wfl).all(), name
        cur = want


@pytest.mark.parametrize("density", [0.2, 0.5, 0.8])
def test_stable_step_and_propagate_dense_counts(hip, port, density):
    """PropagateStep counts the state once and derives NeighbourCount(state |
    unknown) as 9 - NeighbourCount(~(state | unknown)) (stable_kernels.hpp
    StableCounts): random state / unknown planes of every density, so the
    counts cover 0..9, and options mostly open, against the oracle's
    four-count restatement of LifeStable.hpp:526-729"""
    rng = np.random.default_rng(int(density * 100))
    n = 512
    bits = lambda p: np.packbits(rng.random((n, 64, 64)) < p, axis=2, bitorder="little").view(np.uint64)[..., 0]  # noqa: E731
    x = np.zeros((n, 10, 64), np.uint64)
    x[:, 0] = bits(density)
    x[:, 1] = bits(density) & ~x[:, 0]
    for k in range(2, 10):
        x[:, k] = bits(0.1)
    x = x.reshape(n, 640)
    for w, name in ((3, "step"), (4, "propagate")):
        d = to_dev(x).reshape(n, 640)
        fl = hip.stable_pass(d, name).cpu().numpy()
        want, wfl = port.stable_pass(x, w)
        assert (d.cpu().numpy().view(np.uint64) == want).all(), name
        assert (fl == wfl).all(), name


def test_stable_vulnerable_golden_gpu(hip):
    import os
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "stable.npz"))
    got = hip.stable_vulnerable(to_dev(g["input"]).reshape(-1, 640))
    assert (to_host(got) == g["vulnerable"]).all()
    # host-pointer twin
    out = np.zeros((g["input"].shape[0], 64), np.uint64)
    inp = np.ascontiguousarray(g["input"], dtype=np.uint64)
    hip._check(hip.lib.lifeapi_stable_vulnerable_batch(inp.ctypes.data, out.ctypes.data, inp.shape[0], 0))
    assert (out == g["vulnerable"]).all()


# ---- config 5: unknown_step_refined ternary step ----

def test_refined_step_golden(hip, port):
    import os
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "refined_step.npz"))
    got = hip.refined_step(to_dev(g["input"]).reshape(-1, 11 * 64))
    torch.cuda.synchronize()
    assert (got.cpu().numpy().view(np.uint64) == g["output"]).all()


@pytest.mark.parametrize("n", [1, 5, 1000, 4099])
def test_refined_step_vs_oracle(hip, port, n):
    x = port.fill(n * 11, seed=500 + n).reshape(n, 11 * 64)
    if n > 5:  # realistic-ish planes: sparse states, dense option masks
        x[: n // 2, :64] &= port.fill(n // 2, seed=1)[:, :] & port.fill(n // 2, seed=2)
    got = hip.refined_step(to_dev(x).reshape(n, 11 * 64))
    torch.cuda.synchronize()
    assert (got.cpu().numpy().view(np.uint64) == port.refined_step(x)).all()


def test_refined_step_full_size_sample(hip, port):
    """Config 5 at full size (256K universes): prefix and strided sample vs the oracle."""
    n = 1 << 18
    d = hip.fill_random(n * 11, seed=6).reshape(n, 11 * 64)
    got = hip.refined_step(d)
    torch.cuda.synchronize()
    idx = np.r_[0:512, 511 * np.arange(1, 500)]
    x = d.cpu().numpy().view(np.uint64)[idx]
    assert (got.cpu().numpy().view(np.uint64)[idx] == port.refined_step(x)).all()


def test_stable_passes_8_byte_aligned_batch(hip, port):
    """SynchroniseStateKnown, UpdateOptions, SignalNeighbours, PropagateStep
    and StabiliseOptions (passes 0, 1, 2, 3, 5) move a 16-byte aligned batch
    through LDS with 16-byte accesses (stencils.hip, k_stable_dma); Propagate
    keeps k_stable, and a batch that is only 8-byte aligned (the ABI's
    requirement) takes k_stable for every pass.  Both forms, every pass, against the oracle,
    on a search's next node and on fresh options."""
    n = 777
    fresh = _stable_cases(port, n, seed=41)
    nxt, _ = port.stable_pass(fresh, 4)
    nxt = nxt.reshape(n, 10, 64).copy()
    for u in range(n):
        cols = np.nonzero(nxt[u, 1])[0]
        if len(cols):
            c = int(cols[0])
            low = nxt[u, 1, c] & (~nxt[u, 1, c] + np.uint64(1))
            nxt[u, 1, c] &= ~low
            nxt[u, 0, c] |= low
    for x in (fresh, nxt.reshape(n, 640)):
        for w, name in enumerate(hip.STABLE_PASSES):
            want, wfl = port.stable_pass(x, w)
            for offset in (0, 1):  # int64 words: 16-byte aligned, then 8-byte aligned only
                buf = torch.empty(n * 640 + 2, dtype=torch.int64, device="cuda")
                d = buf[offset: offset + n * 640].view(n, 640)
                assert (d.data_ptr() % 16 == 0) == (offset == 0)
                d.copy_(to_dev(x).reshape(n, 640))
                fl = hip.stable_pass(d, name).cpu().numpy()
                assert (to_host(d).reshape(n, 640) == want).all(), (name, offset)
                assert (fl == wfl).all(), (name, offset)


def test_filter_launch_form_follows_the_target(hip, port):
    """One pair of target buffers rewritten in place between calls, as a
    search loop does: round 5 picked the launch form from the last call's
    report on the same pointers (a stale form had to stay exact); from round 6
    no form depends on a report -- every wave of the one launch picks its pass
    from the target it reads (step.hip: k_cone_adapt's DMA form at 1-2
    generations, the merged split kernel from 3) -- and every call must be
    exact whatever the previous target was.  Every call against the oracle,
    at 1, 2, 3 and 5 generations, ragged n."""
    n = 70001
    x = port.fill(n, seed=91) & port.fill(n, seed=92)
    d = to_dev(x)
    whole_u = np.zeros(64, np.uint64)
    whole_u[0::3] = np.uint64(1 << 10)
    small_w, small_u = np.zeros(64, np.uint64), np.zeros(64, np.uint64)
    small_w[10] = small_w[11] = np.uint64(3 << 40)
    small_u[9:13] = np.uint64(15 << 39)
    small_u &= ~small_w
    tw = torch.zeros((1, 64), dtype=torch.int64, device="cuda")
    tu = torch.zeros((1, 64), dtype=torch.int64, device="cuda")

    def want(w, u, gens):
        res, s = np.zeros(n, np.uint32), x.copy()
        for g in range(1, gens + 1):
            s = port.step_batch(s, 1, nthreads=8)
            hit = (((s ^ w) & (w | u)) == 0).all(axis=1)
            res[(res == 0) & hit] = g
        return res
    row10_u = np.zeros(64, np.uint64)  # care row 10 in four columns: fits a whole-board report's row window
    row10_u[20:24] = np.uint64(1 << 10)
    zero = np.zeros(64, np.uint64)
    for gens in (1, 2, 3, 5):
        for w, u in ((zero, whole_u), (small_w, small_u), (zero, whole_u), (zero, row10_u), (zero, whole_u)):
            tw.copy_(to_dev(w[None]).reshape(1, 64))
            tu.copy_(to_dev(u[None]).reshape(1, 64))
            exp = want(w, u, gens)
            for _ in range(3):  # first call: the last report is stale or absent; then the target's own form
                first, _ = hip.step_contains(d, tw, tu, gens)
                torch.cuda.synchronize()
                assert (first.cpu().numpy().astype(np.uint32) == exp).all(), (gens, int(w.any()), int(np.count_nonzero(u)))


def _rows_target(rows, cols, wanted_at=None):
    """care cells at `rows` of every column in `cols` (unwanted), and one
    wanted cell (row, column) if given"""
    w, u = np.zeros(64, np.uint64), np.zeros(64, np.uint64)
    m = np.uint64(0)
    for r in rows:
        m |= np.uint64(1) << np.uint64(r % 64)
    for c in cols:
        u[c] = m
    if wanted_at is not None:
        r, c = wanted_at
        w[c] = np.uint64(1) << np.uint64(r)
        u[c] &= ~w[c]
    return w, u


@pytest.mark.parametrize("rows,gens_list", [
    ((10,), (1, 2, 3, 4, 6, 8, 12, 15, 16)),  # 8-row fields up to 3 generations, 16 to 7, 32 to 15
    ((61, 62, 63, 0, 1), (1, 2, 5, 8)),       # a window across row 63 (8, 16, 32 rows)
    ((30, 31, 32, 33), (1, 2, 6, 10)),        # across the two 32-bit halves
    (tuple(range(40, 54)), (1, 2, 3, 9, 10)),  # 16-row fields at 1, 32 to 9 (no slack), then the full pass
    (tuple(range(64)), (1, 2)),            # every row: the full pass
])
def test_filter_whole_board_row_windows(hip, port, rows, gens_list):
    """A whole-board target whose care rows, widened by the light cone, fit 8,
    16 or 32 rows takes the packed row-window pass (cone_kernels.hpp
    cone_wave_rows_dma: 4, 2 or 1 universes per 32-bit register, shifts for
    the vertical neighbours) in the LDS form; windows across row 63 and across
    the 32-bit halves; every call against the oracle, three calls each
    (round 5's calls differed by the launch report; round 6's are one form),
    ragged n.  From 3 generations the merged split kernel (step.hip): the
    LDS-DMA packed pass below kConeWholeWinGens, the window split layout
    (cone_split.hpp) from it on."""
    n = 70001
    x = port.fill(n, seed=93) & port.fill(n, seed=94) & port.fill(n, seed=95)
    d = to_dev(x)
    tw = torch.zeros((1, 64), dtype=torch.int64, device="cuda")
    tu = torch.zeros((1, 64), dtype=torch.int64, device="cuda")
    targets = [_rows_target(rows, range(0, 64, 3)),
               _rows_target(rows, range(0, 64, 2), wanted_at=(rows[len(rows) // 2] % 64, 8))]
    for gens in gens_list:
        for w, u in targets:
            tw.copy_(to_dev(w[None]).reshape(1, 64))
            tu.copy_(to_dev(u[None]).reshape(1, 64))
            res, s = np.zeros(n, np.uint32), x.copy()
            for g in range(1, gens + 1):
                s = port.step_batch(s, 1, nthreads=8)
                hit = (((s ^ w) & (w | u)) == 0).all(axis=1)
                res[(res == 0) & hit] = g
            for call in range(3):
                first, _ = hip.step_contains(d, tw, tu, gens)
                torch.cuda.synchronize()
                got = first.cpu().numpy().astype(np.uint32)
                assert (got == res).all(), (rows, gens, call, int(w.any()), int((got != res).sum()))


def test_propagate_window_sensitive_fixture(hip):
    """Propagate on the LifeStables of tests/golden/stable_window.npz --
    next nodes on which a window trusting fewer rows than the analysis's
    RHO = 3 goes wrong (found by tools/stable_window_mutant_search.py) --
    against the reference's answers; both alignments"""
    import os
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "stable_window.npz"))
    x, n = g["input"], g["input"].shape[0]
    for aligned in (True, False):
        if aligned:
            d = to_dev(x).reshape(n, 640)
        else:
            t8 = torch.zeros(x.size + 1, dtype=torch.int64, device="cuda")
            d = t8[1:].view(n, 640)
            d.copy_(to_dev(x).reshape(n, 640))
        fl = hip.stable_pass(d, "propagate").cpu().numpy()
        got = to_host(d).reshape(n, 640)
        assert (got == g["propagate"]).all() and (fl == g["flags"]).all(), aligned
