"""GPU parity pinned DIRECTLY to the reference: the shipped HIP kernels
against the reference's own code, compiled from /root/reference into
oracle/_ref/libref_v{3,4}.so (oracle/Makefile, target ref; the .so travels to
the GPU box prebuilt).  No restatement in between:

* Step() / Step(n) (LifeAPI.hpp:1196-1216, 877-886) for the shipped
  configurations -- gens 1 and 2 (k_step, natural layout), 3, 31 and 1024
  (k_step_split, the assembly loop; nontemporal below 32) -- on a prefix of
  the config-2 input generated on the device, plus seam cases, the
  reference-shaped RandomState() draws and ragged batch sizes;
* the full config-2 batch (1M universes x 1 gen) word for word;
* LifeWeld::Step (LifeWeld.hpp:169-186) and the config-5 harness around the
  reference's own unknown_step_refined fragment.

Bit-exact on every word (integer work, no tolerance).
"""
import os

import numpy as np
import pytest
import torch

from test_gpu_parity import seam_cases, to_dev, to_host

pytestmark = pytest.mark.gpu

THREADS = max(1, min(16, len(os.sched_getaffinity(0))))


@pytest.fixture(scope="module")
def R(hip):
    from oracle.oracle import Ref
    assert Ref.available(), "oracle/_ref was not built: run __graft_entry__.build() where /root/reference exists"
    return Ref()


def _check(got, want, what):
    bad = np.nonzero((got != want).any(axis=1))[0]
    assert bad.size == 0, f"{what}: {bad.size} universes differ from the reference, first {bad[:8]}"


@pytest.mark.parametrize("gens", [1, 2, 3, 31, 1024])
def test_shipped_step_vs_reference(hip, R, port, gens):
    n = 1 << 14 if gens < 1024 else 1 << 12
    d = hip.fill_random(n, seed=2)                      # config-2 prefix, generated on the device
    x = np.concatenate([seam_cases(port), to_host(d),
                        np.load(os.path.join(os.path.dirname(__file__), "golden", "randomstate_kat.npz"))["input"]])
    got = to_host(hip.step(to_dev(x), generations=gens))
    _check(got, R.step_batch(x, gens, nthreads=THREADS), f"Step^{gens} ({hip.step_kernel_name(gens)})")


@pytest.mark.parametrize("n", [1, 3, 5, 63, 65, 4099])
@pytest.mark.parametrize("gens", [1, 7])
def test_ragged_vs_reference(hip, R, port, n, gens):
    x = port.fill(n, seed=100 + n)
    _check(to_host(hip.step(to_dev(x), generations=gens)), R.step_batch(x, gens, nthreads=THREADS),
           f"n={n} gens={gens}")


def test_inplace_vs_reference(hip, R, port):
    x = port.fill(5003, seed=5)
    d = to_dev(x)
    hip.step(d, out=d, generations=1)
    hip.step(d, out=d, generations=40)
    _check(to_host(d), R.step_batch(x, 41, nthreads=THREADS), "in-place Step^1 then Step^40")


def test_full_config2_vs_reference(hip, R):
    n = 1 << 20
    d = hip.fill_random(n, seed=2)
    x = to_host(d)
    _check(to_host(hip.step(d, generations=1)), R.step_batch(x, 1, nthreads=THREADS), "config 2, 1M x 1")


def test_weld_vs_reference(hip, R, port):
    rw = port.fill(300 * 4, seed=606).reshape(300, 256)
    rw[:, 64:] &= port.fill(300 * 3, seed=607).reshape(300, 192) & port.fill(300 * 3, seed=608).reshape(300, 192)
    for gens in (1, 5, 12, 40):
        d = torch.from_numpy(rw.view(np.int64).copy()).cuda()
        hip.weld_step(d, generations=gens)
        got = d.cpu().numpy().view(np.uint64).reshape(-1, 256)
        _check(got, R.weld_step(rw, gens), f"LifeWeld::Step^{gens}")


def test_refined_vs_reference(hip, R):
    n = 4096
    d = hip.fill_random(n * 11, seed=66).reshape(n, 11 * 64)
    got = hip.refined_step(d)
    torch.cuda.synchronize()
    x = d.cpu().numpy().view(np.uint64)
    _check(got.cpu().numpy().view(np.uint64), R.refined_step(x), "unknown_step_refined harness")


@pytest.mark.parametrize("gens", [1, 3])
def test_batch_beyond_2_32_words(hip, R, port, gens):
    """A batch of 2^26 + 5 universes (2^32 + 320 words, 32 GiB per buffer):
    every index in the fill, the step kernels and their grid arithmetic must be
    64-bit.  Universes on both sides of the 2^32-word boundary and the ragged
    tail are checked against the reference (the fill is indexable, so the
    oracle regenerates exactly those universes)."""
    n = (1 << 26) + 5
    d = hip.fill_random(n, seed=77)
    out = hip.step(d, generations=gens)
    torch.cuda.synchronize()
    for first in (0, (1 << 26) - 3, n - 40):
        k = min(40, n - first)
        x = port.fill(k, seed=77, first_universe=first)
        assert (to_host(d[first:first + k]) == x).all(), f"fill differs at universe {first}"
        _check(to_host(out[first:first + k]), R.step_batch(x, gens), f"Step^{gens} at universe {first}")
    del d, out
    torch.cuda.empty_cache()


def _targets():
    """a 2 x 2 block + empty ring (4-row window: the low-layout kernel) and a
    loaf + its 6 x 6 box (6 rows: the other kernel of the shipped pair);
    both still lifes"""
    blk_w, blk_u = np.zeros(64, np.uint64), np.zeros(64, np.uint64)
    blk_w[10] = blk_w[11] = np.uint64(3 << 40)
    for c in (9, 10, 11, 12):
        blk_u[c] = np.uint64(15 << 39)
    loaf_w, loaf_u = np.zeros(64, np.uint64), np.zeros(64, np.uint64)
    for c, rows in zip(range(21, 25), ((1,), (0, 2), (0, 3), (1, 2))):  # .oo. / o..o / .o.o / ..o.
        loaf_w[c] = np.uint64(sum(1 << (31 + r) for r in rows))
    for c in range(20, 26):
        loaf_u[c] = np.uint64(0x3F << 30)
    return [(blk_w, blk_u & ~blk_w), (loaf_w, loaf_u & ~loaf_w)]


@pytest.mark.parametrize("which", [0, 1])
@pytest.mark.parametrize("gens", [1, 2, 9, 64])
def test_step_contains_vs_reference(hip, R, port, which, gens):
    """the shipped fused Step + Contains pair against the reference's own
    Step() + Contains(LifeTarget) loop (ref_shim.cpp, LifeTarget.hpp:44-51):
    first-hit generations and final states, with planted targets"""
    w, u = _targets()[which]
    n = 4099
    x = port.fill(n, seed=31 + which) & port.fill(n, seed=41 + which) & port.fill(n, seed=51 + which)
    clear = np.zeros(64, np.uint64)
    clear[2:30] = np.uint64(((1 << 28) - 1) << 22)   # an empty region around both targets
    x[::7] = (x[::7] & ~clear) | w                   # contained from generation 1 (still lifes)
    fin = torch.empty((n, 64), dtype=torch.int64, device="cuda")
    first, _ = hip.step_contains(to_dev(x), to_dev(w[None]), to_dev(u[None]), gens, final=fin)
    exp_first, exp_fin = R.step_contains_batch(x, w, u, gens, nthreads=THREADS)
    assert (first.cpu().numpy().astype(np.uint32) == exp_first).all()
    assert (exp_first > 0).sum() >= n // 14
    _check(to_host(fin), exp_fin, f"final states after the fused kernel, gens={gens}")


def test_config3_search_loop_vs_reference_digest(hip):
    """config 3 as the search loop, full size (64K x 1024): the digests the
    reference's own loop produced (tests/golden/make_golden.py)"""
    import json
    from lifeapi_amd.digest import batch_digest
    with open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")) as f:
        gold = json.load(f)["digests"]["config3_contains"]
    w, u = (np.array([int(v, 16) for v in gold[k]], dtype=np.uint64) for k in ("wanted", "unwanted"))
    d = hip.fill_random(gold["universes"], seed=gold["seed"])
    fin = torch.empty_like(d)
    first, _ = hip.step_contains(d, to_dev(w[None]), to_dev(u[None]), gold["generations"], final=fin)
    assert int((first > 0).sum().item()) == gold["hits"]
    assert f"{batch_digest(first.cpu().numpy().astype(np.uint64)):016x}" == gold["first_digest"]
    assert f"{batch_digest(hip.hashes(fin).cpu().numpy()):016x}" == gold["output_digest"]


def test_step_contains_random_windows_vs_reference(hip, R, port):
    """the shipped filter (round 6: one launch of the merged split kernel,
    whose waves pick the pass from the target they read -- no launch report)
    on 48 targets with random row windows (1..12 rows, also
    20 and 64, anywhere including across the row seam) and columns:
    each target is universe 0's box after 3 generations, so universe 0 hits;
    first-hit generations and final states against the reference's loop"""
    rng = np.random.default_rng(4242)
    n, gens = 257, 6
    x = port.fill(n, seed=91) & port.fill(n, seed=92)
    for t in range(48):
        h = int(rng.choice([1, 2, 3, 4, 5, 6, 7, 8, 9, 12, 20, 64]))
        y0 = int(rng.integers(64))
        rows = np.uint64(sum(1 << ((y0 + i) % 64) for i in range(h)))
        cols = sorted({int(c) for c in rng.integers(0, 64, size=int(rng.integers(1, 6)))})
        box = np.zeros(64, np.uint64)
        box[cols] = rows
        ahead = port.step_batch(x[:1], 3)[0]
        w, u = ahead & box, box & ~ahead
        first, _ = hip.step_contains(to_dev(x), to_dev(w[None]), to_dev(u[None]), gens)
        exp, _ = R.step_contains_batch(x, w, u, gens)
        got = first.cpu().numpy().astype(np.uint32)
        assert (got == exp).all(), (t, h, y0, cols, np.nonzero(got != exp)[0][:8])
        assert 1 <= exp[0] <= 3


@pytest.mark.parametrize("gens", [3, 4, 5, 7, 8, 11, 15])
def test_filter_shrinking_windows_vs_reference(hip, R, port, gens):
    """the window split pass that halves its lanes once the light cone's
    columns fit (cone_split.hpp SHRINK): column windows of every lane class
    (K = w + 2 gens in 9..16, 17..32, 33..63), row windows of 32 and (up to
    7 generations) 16 rows, across the column and row seams; universes that
    are universe 0 stepped 1..k - 1 generations hit before and after the
    merge, in both halves of a chunk, at a ragged batch end"""
    rng = np.random.default_rng(1000 + gens)
    n = 1000 + gens
    x = port.fill(n, seed=gens) & port.fill(n, seed=gens + 50)
    lanes = [(9, 16), (17, 32), (33, 63)]
    for t in range(18):
        lo, hi = lanes[t % 3]
        w = int(rng.integers(max(1, lo - 2 * gens), max(2, hi - 2 * gens + 1)))
        w = min(w, 64 - 2 * gens - 1)
        x0 = int(rng.integers(64)) if t % 2 else 64 - w // 2  # across column 63 every other target
        rmax = 16 if gens <= 7 and t % 4 == 1 else 32
        h = int(rng.integers(1, rmax - 2 * gens + 1))
        y0 = int(rng.integers(64)) if t % 3 else 64 - h // 2
        rows = np.uint64(sum(1 << ((y0 + i) % 64) for i in range(h)))
        box = np.zeros(64, np.uint64)
        box[[(x0 + i) % 64 for i in range(w)]] = rows
        k = int(rng.integers(1, gens + 1))
        at = rng.choice(n, size=k, replace=False)  # at[d]: x[src] stepped d generations
        src = int(at[0])
        for d in range(1, k):
            x[at[d]] = port.step_batch(x[src:src + 1], d)[0]
        ahead = port.step_batch(x[src:src + 1], k)[0]
        wv, uv = ahead & box, box & ~ahead
        first, _ = hip.step_contains(to_dev(x), to_dev(wv[None]), to_dev(uv[None]), gens)
        exp, _ = R.step_contains_batch(x, wv, uv, gens, nthreads=THREADS)
        got = first.cpu().numpy().astype(np.uint32)
        assert (got == exp).all(), (t, w, x0, h, y0, k, np.nonzero(got != exp)[0][:8])
        assert 1 <= exp[src] <= k


@pytest.mark.parametrize("gens", [1, 2, 13])
@pytest.mark.parametrize("which", [0, 1])
def test_step_contains_in_place_vs_reference(hip, R, port, which, gens):
    """d_final == d_in (the search loop stepping its own batch): each wave
    reads its universes before it writes them, in the one-generation filter
    kernel (8 universes per wave) and in both kernels of the pair"""
    w, u = _targets()[which]
    n = 2053
    x = port.fill(n, seed=61 + which) & port.fill(n, seed=71 + which)
    d = to_dev(x)
    first, _ = hip.step_contains(d, to_dev(w[None]), to_dev(u[None]), gens, final=d)
    exp_first, exp_fin = R.step_contains_batch(x, w, u, gens, nthreads=THREADS)
    assert (first.cpu().numpy().astype(np.uint32) == exp_first).all()
    _check(to_host(d), exp_fin, "in-place final states")


def test_eater_pairs_vs_reference(hip, R):
    """tests/InteractionTest.cpp:7-27's workload: two eaters, the second at
    every offset in [-10, 10)^2, stepped once -- 400 interacting
    configurations on the GPU against the reference's own Step(); and
    InteractionCountsAndNext's 'next' plane equal to that step
    (LifeAPI.hpp:997-1040)."""
    eater = R.parse("2b2o$bobo$bo$2o!")   # Parse, not ConstantParse

    def moved(s, dx, dy):
        s = np.roll(s, dx)
        dy %= 64
        return (s << np.uint64(dy)) | (s >> np.uint64((64 - dy) % 64)) if dy else s.copy()

    base = moved(eater, 20, 20)
    x = np.stack([base | moved(base, dx, dy) for dx in range(-10, 10) for dy in range(-10, 10)])
    want = R.step_batch(x, 1)
    _check(to_host(hip.step(to_dev(x), generations=1)), want, "eater pairs, Step()")
    nxt = hip.interaction_counts(to_dev(x), with_next=True)[:, 3].cpu().numpy().view(np.uint64)
    _check(nxt, want, "eater pairs, InteractionCountsAndNext next")


@pytest.mark.parametrize("gens", [1, 5])
def test_search_loop_beyond_2_32_words(hip, R, port, gens):
    """the fused search loop on 2^26 + 5 universes (2^32 + 320 words): the
    filter (1 generation) and the split-layout pair (5) index 64-bit; the
    universes on both sides of the 2^32-word boundary and the ragged tail
    against the reference's loop (the fill is indexable)"""
    # two care cells (one alive, one dead): random universes hit it at varying
    # generations, so a universe read from the wrong place would show
    w, u = np.zeros(64, np.uint64), np.zeros(64, np.uint64)
    w[10] = np.uint64(1 << 40)
    u[11] = np.uint64(1 << 40)
    n = (1 << 26) + 5
    d = hip.fill_random(n, seed=78)
    first, _ = hip.step_contains(d, to_dev(w[None]), to_dev(u[None]), gens)
    torch.cuda.synchronize()
    seen = set()
    for lo in (0, (1 << 26) - 20, n - 40):   # the 2^32-word boundary is at universe 2^26
        k = min(40, n - lo)
        x = port.fill(k, seed=78, first_universe=lo)
        want, _ = R.step_contains_batch(x, w, u, gens)
        assert (first[lo:lo + k].cpu().numpy().astype(np.uint32) == want).all(), lo
        seen |= set(want.tolist())
    assert len(seen) >= 2, seen
    del d, first
    torch.cuda.empty_cache()


def _column_box_target(rng, state, x0, w):
    """a target whose care cells (wanted | unwanted) span exactly the cyclic
    columns [x0, x0 + w): the box of those columns x random rows, wanted =
    the state's live cells in it, unwanted = its dead cells"""
    cols = [(x0 + i) % 64 for i in range(w)]
    keep = [cols[0], cols[-1]] + [c for c in cols[1:-1] if rng.random() < 0.6]
    box = np.zeros(64, np.uint64)
    for c in keep:
        box[c] = np.uint64(int(rng.integers(1, 1 << 63)) | 1 << int(rng.integers(64)))
    return state & box, box & ~state


CONE_WIDTHS = [1, 2, 3, 4, 5, 6, 7, 8, 9, 12, 14, 15, 16, 17, 28, 30, 31, 32, 33, 40, 60, 61, 62, 63, 64]


@pytest.mark.parametrize("w", CONE_WIDTHS)
def test_cone_contains_and_filter_vs_reference(hip, R, port, w):
    """The light-cone kernels (cone_kernels.hpp): batched Contains(LifeTarget)
    and the 1-2 generation search filter with first hits only, against the
    reference's own Contains (LifeTarget.hpp:44-51) and Step() + Contains loop,
    on targets whose care columns span exactly w columns -- every lane layout
    (P = 4 .. 64 lanes per universe, margins included), windows straddling
    the column seam 63|0, and w + 2g >= 64 (the whole board).  Universe 0's
    own future is the target, and every 5th universe is a copy of it, so hits
    and misses both occur."""
    rng = np.random.default_rng(1000 + w)
    n = 4099                                     # ragged against 32 universes per wave
    x = port.fill(n, seed=200 + w) & port.fill(n, seed=300 + w)
    x[::5] = x[0]
    for x0 in (int(rng.integers(64)), 64 - w // 2 if w > 1 else 63, 0):
        for g in (0, 1, 2):
            ahead = R.step_batch(x[:1], g)[0] if g else x[0]
            tw, tu = _column_box_target(rng, ahead, x0, w)
            dw, du = to_dev(tw[None]), to_dev(tu[None])
            if g == 0:
                got = hip.contains(to_dev(x), dw, du).cpu().numpy()
                want = R.contains_batch(x, tw, tu)
                assert (got == want).all(), (w, x0, np.nonzero(got != want)[0][:8])
                assert want[0] == 1 and 0 < want.sum() < n
            for gens in (0, 1, 2):
                first, _ = hip.step_contains(to_dev(x), dw, du, gens)
                exp, _ = R.step_contains_batch(x, tw, tu, gens, nthreads=THREADS)
                got = first.cpu().numpy().astype(np.uint32)
                assert (got == exp).all(), (w, x0, g, gens, np.nonzero(got != exp)[0][:8])
                if gens >= g >= 1:
                    assert 1 <= exp[0] <= g


@pytest.mark.parametrize("n", [1, 2, 15, 16, 17, 31, 33, 65, 127])
def test_cone_ragged_and_empty_target_vs_reference(hip, R, port, n):
    """ragged batches (partial register sets and waves) for a narrow and a
    wide window, and the empty target (contained by every state)"""
    rng = np.random.default_rng(n)
    x = port.fill(n, seed=900 + n) & port.fill(n, seed=901 + n)
    zero = np.zeros(64, np.uint64)
    targets = [_column_box_target(rng, x[0], 62, 3), _column_box_target(rng, x[-1], 5, 40), (zero, zero)]
    for tw, tu in targets:
        dw, du = to_dev(tw[None]), to_dev(tu[None])
        assert (hip.contains(to_dev(x), dw, du).cpu().numpy() == R.contains_batch(x, tw, tu)).all()
        for gens in (1, 2):
            first, _ = hip.step_contains(to_dev(x), dw, du, gens)
            exp, _ = R.step_contains_batch(x, tw, tu, gens)
            assert (first.cpu().numpy().astype(np.uint32) == exp).all(), (n, gens)
    first, _ = hip.step_contains(to_dev(x), to_dev(zero[None]), to_dev(zero[None]), 2)
    assert (first.cpu().numpy() == 1).all()


@pytest.mark.parametrize("w,gens", [(1, 3), (4, 3), (4, 8), (4, 14), (6, 9), (6, 13), (6, 14), (10, 11), (16, 8),
                                    (20, 6), (26, 3), (30, 1), (3, 15), (2, 16), (1, 40)])
def test_iterated_search_loop_cone_and_split_vs_reference(hip, R, port, w, gens):
    """gens > 2 with no final states: targets whose light cone spans at most
    32 columns are answered by the cone kernel, the rest by the split-layout
    pair (each wave of each launch checks), with final states always by the
    pair; both against the reference's own Step() + Contains loop, windows
    straddling the seam, ragged n"""
    rng = np.random.default_rng(7 * w + gens)
    n = 1031
    x = port.fill(n, seed=500 + w) & port.fill(n, seed=600 + gens)
    x[::4] = x[0]
    for x0 in (int(rng.integers(64)), 62):
        tw, tu = _column_box_target(rng, R.step_batch(x[:1], max(1, gens // 2))[0], x0, w)
        dw, du = to_dev(tw[None]), to_dev(tu[None])
        exp_first, exp_fin = R.step_contains_batch(x, tw, tu, gens, nthreads=THREADS)
        dx = to_dev(x)
        for call in range(2):  # (round 5: the second call took the form the first one's report picked)
            first, _ = hip.step_contains(dx, dw, du, gens)
            got = first.cpu().numpy().astype(np.uint32)
            assert (got == exp_first).all(), (w, gens, x0, call, np.nonzero(got != exp_first)[0][:8])
        fin = torch.empty((n, 64), dtype=torch.int64, device="cuda")
        first, _ = hip.step_contains(to_dev(x), dw, du, gens, final=fin)
        assert (first.cpu().numpy().astype(np.uint32) == exp_first).all()
        _check(to_host(fin), exp_fin, f"final states, w={w} gens={gens}")
        assert 1 <= exp_first[0] <= gens


@pytest.mark.parametrize("w,h,gens", [(2, 1, 3), (2, 2, 8), (4, 4, 13), (4, 5, 13), (6, 7, 9), (6, 8, 3),
                                      (20, 3, 5), (20, 6, 5), (27, 2, 3), (28, 4, 3), (4, 3, 15), (4, 6, 16),
                                      (12, 4, 24), (12, 6, 24),
                                      # round 6: the window split layout's shapes (cone_split.hpp):
                                      # P = 8 / 16 / 32 / 64 lanes x R = 32 / 16 rows
                                      (2, 20, 3), (1, 12, 3), (6, 14, 5), (14, 4, 6), (30, 1, 15),
                                      (40, 2, 4), (40, 12, 7), (64, 3, 14)])
def test_iterated_search_loop_short_targets_vs_reference(hip, R, port, w, h, gens):
    """gens > 2, no final states, targets of w columns x h rows (cyclic, at
    the seams), each called twice (round 5's two calls differed by the
    launch report): rows that fit 32 with the light cone take the window split
    layout (cone_split.hpp; the round-6 shapes cover P = 8 / 16 / 32 / 64
    lanes x R = 32 / 16 rows), narrower cones of taller targets the natural
    layout's cone pass, the rest the 8-way row split that their height
    picks (step_kernels.hpp kContainsAll).  Against the reference's Step() +
    Contains loop."""
    rng = np.random.default_rng(100 * w + 10 * h + gens)
    n = 777
    x = port.fill(n, seed=700 + w) & port.fill(n, seed=800 + h)
    x[::3] = x[0]
    for x0, y0 in ((int(rng.integers(64)), int(rng.integers(64))), (62, 63)):
        rows = 0
        for i in range(h):
            rows |= 1 << ((y0 + i) % 64)
        rows_mask = np.uint64(rows)
        ref_state = R.step_batch(x[:1], max(1, gens // 2))[0]
        cols = [(x0 + i) % 64 for i in range(w)]
        box = np.zeros(64, np.uint64)
        for c in cols:
            box[c] = rows_mask
        tw, tu = ref_state & box, box & ~ref_state
        dw, du = to_dev(tw[None]), to_dev(tu[None])
        exp_first, _ = R.step_contains_batch(x, tw, tu, gens, nthreads=THREADS)
        dx = to_dev(x)
        for call in range(2):  # (round 5: the second call took the form the first one's report picked)
            first, _ = hip.step_contains(dx, dw, du, gens)
            got = first.cpu().numpy().astype(np.uint32)
            assert (got == exp_first).all(), (w, h, gens, x0, y0, call, np.nonzero(got != exp_first)[0][:8])
        assert 1 <= exp_first[0] <= gens


@pytest.mark.parametrize("seed", range(8))
def test_filter_fuzz_vs_reference(hip, R, port, seed):
    """The search filter (first hits only) on 40 random targets per seed
    against the reference's own Step() + Contains loop: 1-15 generations;
    targets of one to five boxes (1-20 columns x 1-24 rows each, anywhere,
    across both seams), sometimes a row band over every column, sometimes
    wanted cells only or unwanted only; each target cut from a universe of
    the batch a few generations ahead, so that hits occur; ragged batches
    on both alignments.  Every pass the one launch picks (natural cone,
    window split with and without shrinking, whole-board rows, LDS-DMA
    chunks, 8-way split) meets targets of its class here."""
    rng = np.random.default_rng(7000 + seed)
    for t in range(40):
        n = int(rng.integers(60, 700))
        x = port.fill(n, seed=int(rng.integers(1 << 30))) & port.fill(n, seed=int(rng.integers(1 << 30)))
        gens = int(rng.integers(1, 16))
        box = np.zeros(64, np.uint64)
        if rng.random() < 0.2:  # a band of rows over every column (a whole-board target)
            y0, h = int(rng.integers(64)), int(rng.integers(1, 6))
            box[:] = np.uint64(sum(1 << ((y0 + i) % 64) for i in range(h)))
            box[rng.random(64) < 0.5] = 0
        else:
            for _ in range(int(rng.integers(1, 6))):
                x0, w = int(rng.integers(64)), int(rng.integers(1, 21))
                y0, h = int(rng.integers(64)), int(rng.integers(1, 25))
                rows = np.uint64(sum(1 << ((y0 + i) % 64) for i in range(h)))
                for c in range(w):
                    box[(x0 + c) % 64] |= rows
        src = int(rng.integers(n))
        ahead = port.step_batch(x[src:src + 1], int(rng.integers(1, gens + 1)))[0]
        tw, tu = ahead & box, box & ~ahead
        kind = rng.random()
        if kind < 0.1:
            tu[:] = 0
        elif kind < 0.2:
            tw[:] = 0
        exp, _ = R.step_contains_batch(x, tw, tu, gens, nthreads=THREADS)
        for d in (to_dev(x), None):
            if d is None:  # 8-byte aligned only
                t8 = torch.zeros(x.size + 1, dtype=torch.int64, device="cuda")
                d = t8[1:].view(n, 64)
                d.copy_(to_dev(x))
            first, _ = hip.step_contains(d, to_dev(tw[None]), to_dev(tu[None]), gens)
            got = first.cpu().numpy().astype(np.uint32)
            assert (got == exp).all(), (seed, t, gens, n, d.data_ptr() % 16, np.nonzero(got != exp)[0][:8])


def test_filter_zero_generations_vs_reference(hip, R, port):
    """generations = 0: the loop `for g in 1..gens` never runs -- every answer
    0 and d_final = Stepped(0) = the input, in every launch form (the cone
    kernel without final states, the streaming filter with them), whatever the
    target (one contained by every universe included)"""
    n = 333
    x = port.fill(n, seed=55)
    targets = [(np.zeros(64, np.uint64), np.zeros(64, np.uint64)),  # the empty target: contained by all
               (x[0].copy(), np.zeros(64, np.uint64))]
    for w, u in targets:
        exp_first, exp_fin = R.step_contains_batch(x, w, u, 0)
        assert not exp_first.any()
        first, _ = hip.step_contains(to_dev(x), to_dev(w[None]), to_dev(u[None]), 0)
        assert not first.cpu().numpy().any()
        fin = torch.empty((n, 64), dtype=torch.int64, device="cuda")
        first, _ = hip.step_contains(to_dev(x), to_dev(w[None]), to_dev(u[None]), 0, final=fin)
        assert not first.cpu().numpy().any()
        _check(to_host(fin), exp_fin, "Stepped(0)")


@pytest.mark.parametrize("gens", [3, 7, 8, 12, 15, 16, 17])
def test_filter_window_boundaries_vs_reference(hip, R, port, gens):
    """The routing edges of the iterated filter: care rows whose light cone
    needs exactly 8 / 16 / 32 rows or one more (the packed fields, R = 16 / 32
    windows, none), column windows whose cone is exactly 16 / 32 / 63 columns
    or one more (P = 16 / 32 / 64 and the whole board), a whole board at the
    kConeWholeWinGens edge, and 16 / 17 generations (the window passes stop
    at 15), each across the seams; against the reference's own loop"""
    n = 389
    x = port.fill(n, seed=900 + gens) & port.fill(n, seed=950 + gens)
    cases = []
    for need in (8, 9, 16, 17, 32, 33):
        h = need - 2 * gens
        if h >= 1:
            cases.append(("rows", h, None))
    for kc in (16, 17, 32, 33, 63, 64):
        w = kc - 2 * gens
        if 1 <= w <= 64:
            cases.append(("cols", 3, w))
    cases.append(("whole", 1, 64))
    for t, (kind, h, w) in enumerate(cases):
        y0 = (61 + 7 * t) % 64
        x0 = (62 + 5 * t) % 64
        rows = np.uint64(sum(1 << ((y0 + i) % 64) for i in range(h)))
        box = np.zeros(64, np.uint64)
        if kind == "rows":
            box[0::3] = rows  # a whole board whose rows may fit a window
        else:
            for c in range(w):
                box[(x0 + c) % 64] = rows
        src = (17 * t) % n
        ahead = port.step_batch(x[src:src + 1], max(1, gens // 2))[0]
        tw, tu = ahead & box, box & ~ahead
        exp, _ = R.step_contains_batch(x, tw, tu, gens, nthreads=THREADS)
        first, _ = hip.step_contains(to_dev(x), to_dev(tw[None]), to_dev(tu[None]), gens)
        got = first.cpu().numpy().astype(np.uint32)
        assert (got == exp).all(), (gens, kind, h, w, np.nonzero(got != exp)[0][:8])


def _stable_next_nodes(R, port, n, seed):
    """LifeStables as a search meets them: still lifes with an unknown window
    (anywhere, across the row and column seams, 4-44 rows tall), propagated
    to their fixpoint by the reference, then one unknown cell decided ON or
    OFF -- Propagate from there changes rows near that cell (the window
    steps, stable_kernels.hpp stable_iter_window), or, in tall windows,
    more rows than the window holds (the whole-column fallback)"""
    rng = np.random.default_rng(seed)
    blocks = port.parse("2o$2o!")
    x = np.zeros((n, 10, 64), np.uint64)
    for u in range(n):
        st = np.zeros(64, np.uint64)
        for _ in range(int(rng.integers(3, 9))):
            bx, by = int(rng.integers(16)) * 4, int(rng.integers(16)) * 4
            st |= np.roll(blocks, bx) << np.uint64(by) | (np.roll(blocks, bx) >> np.uint64((64 - by) % 64) if by else 0)
        w0, h0 = int(rng.integers(3, 24)), int(rng.integers(4, 45))
        x0, y0 = int(rng.integers(64)), int(rng.integers(64))
        rows = np.uint64(sum(1 << ((y0 + i) % 64) for i in range(h0)))
        unk = np.zeros(64, np.uint64)
        for c in range(w0):
            unk[(x0 + c) % 64] = rows
        x[u, 0], x[u, 1] = st & ~unk, unk
        obj = np.ascontiguousarray(x[u].reshape(640))
        R.stable_pass(obj, 4)  # the parent: propagated to its fixpoint
        x[u] = obj.reshape(10, 64)
        cols = np.nonzero(x[u, 1])[0]
        if cols.size:
            c = int(rng.choice(cols))
            bits = [b for b in range(64) if (int(x[u, 1, c]) >> b) & 1]
            b = int(rng.choice(bits))
            x[u, 1, c] &= ~np.uint64(1 << b)
            if rng.random() < 0.5:
                x[u, 0, c] |= np.uint64(1 << b)  # decided ON
            else:
                x[u, 0, c] &= ~np.uint64(1 << b)  # decided OFF
    return x.reshape(n, 640)


@pytest.mark.parametrize("seed", [1, 2])
def test_stable_next_node_passes_vs_reference(hip, R, port, seed):
    """Propagate (its steps after the first on a 32-row window, or the whole
    columns when the changed rows do not fit), StabiliseOptions and
    PropagateStep on next nodes against the reference's own LifeStable
    members (LifeStable.hpp:677-729), object by object: planes and the
    PropagateResult flags, on both alignments"""
    n = 160
    x = _stable_next_nodes(R, port, n, 500 + seed)
    for name, which in (("propagate", 4), ("stabilise", 5), ("step", 3)):
        want, wfl = x.copy(), np.zeros(n, np.uint8)
        for u in range(n):
            obj = np.ascontiguousarray(want[u])
            wfl[u] = R.stable_pass(obj, which)
            want[u] = obj
        for aligned in (True, False):
            if aligned:
                d = to_dev(x).reshape(n, 640)
            else:
                t8 = torch.zeros(x.size + 1, dtype=torch.int64, device="cuda")
                d = t8[1:].view(n, 640)
                d.copy_(to_dev(x).reshape(n, 640))
            fl = hip.stable_pass(d, name).cpu().numpy()
            got = to_host(d).reshape(n, 640)
            bad = np.nonzero((got != want).any(axis=1) | (fl != wfl))[0]
            assert bad.size == 0, (name, aligned, bad[:8], fl[bad[:4]], wfl[bad[:4]])


def test_propagate_cascades_vs_reference(hip, R, port):
    """Propagate on LifeStables whose fixpoint takes many steps: still lifes
    (blocks, beehives, loaves, boats, tubs on an 8-cell lattice) under a
    large unknown region (10-40 rows and columns, across the seams) with a
    few of its cells decided ON or OFF, so that forcing chains run through
    the region step after step -- the windowed steps (a window of the rows
    within 2 RHO = 6 of the previous step's changes, the band within RHO = 3
    trusted) must reach the reference's fixpoint and flags exactly; both
    alignments"""
    rng = np.random.default_rng(8080)
    pats = [port.parse(t) for t in ("2o$2o!", "b2o$o2bo$b2o!", "b2o$o2bo$bobo$2bo!", "2o$obo$bo!", "bo$obo$bo!")]
    n = 400
    x = np.zeros((n, 10, 64), np.uint64)
    for u in range(n):
        st = np.zeros(64, np.uint64)
        for gx in range(8):
            for gy in range(8):
                if rng.random() < 0.55:
                    pt = pats[int(rng.integers(len(pats)))]
                    st |= np.roll(pt, 8 * gx + 1) << np.uint64(8 * gy + 1)
        unk = np.zeros(64, np.uint64)
        y0, h = int(rng.integers(64)), int(rng.integers(10, 41))
        rows = np.uint64(sum(1 << ((y0 + i) % 64) for i in range(h)))
        x0, w = int(rng.integers(64)), int(rng.integers(10, 41))
        for c in range(w):
            unk[(x0 + c) % 64] = rows
        state = st & ~unk
        for _ in range(int(rng.integers(1, 4))):  # decided cells inside the region
            c, b = (x0 + int(rng.integers(w))) % 64, (y0 + int(rng.integers(h))) % 64
            unk[c] &= ~np.uint64(1 << b)
            if rng.random() < 0.5:
                state[c] |= np.uint64(1 << b)
        x[u, 0], x[u, 1] = state, unk
    x = x.reshape(n, 640)
    want, wfl = x.copy(), np.zeros(n, np.uint8)
    for u in range(n):
        obj = np.ascontiguousarray(want[u])
        wfl[u] = R.stable_pass(obj, 4)
        want[u] = obj
    assert (wfl & 1).sum() > n // 10, int((wfl & 1).sum())  # consistent ones among them
    for aligned in (True, False):
        if aligned:
            d = to_dev(x).reshape(n, 640)
        else:
            t8 = torch.zeros(x.size + 1, dtype=torch.int64, device="cuda")
            d = t8[1:].view(n, 640)
            d.copy_(to_dev(x).reshape(n, 640))
        fl = hip.stable_pass(d, "propagate").cpu().numpy()
        got = to_host(d).reshape(n, 640)
        bad = np.nonzero((got != want).any(axis=1) | (fl != wfl))[0]
        assert bad.size == 0, (aligned, bad[:8], fl[bad[:4]], wfl[bad[:4]])


def test_propagate_window_at_every_row_offset_vs_reference(hip, R, port):
    """The window's first row y0 at every offset: next nodes rolled down the
    torus by each of 0..63 rows (every plane's column words rotated), so that
    the window steps start on both sides of the columns' 64-row seam and
    exactly on it (y0 = 0 and 32, where stable_kernels.hpp place_rows leaves
    one word half to the band mask) -- Propagate and StabiliseOptions against
    the reference's own members, planes and flags"""
    base = _stable_next_nodes(R, port, 12, 777).reshape(12, 10, 64)
    rolled = []
    for r in range(64):
        s = np.uint64(r)
        rolled.append(base if r == 0 else (base << s) | (base >> np.uint64(64 - r)))
    x = np.ascontiguousarray(np.stack(rolled, 1).reshape(-1, 640))
    n = x.shape[0]
    for name, which in (("propagate", 4), ("stabilise", 5)):
        want, wfl = x.copy(), np.zeros(n, np.uint8)
        for u in range(n):
            obj = np.ascontiguousarray(want[u])
            wfl[u] = R.stable_pass(obj, which)
            want[u] = obj
        d = to_dev(x).reshape(n, 640)
        fl = hip.stable_pass(d, name).cpu().numpy()
        got = to_host(d).reshape(n, 640)
        bad = np.nonzero((got != want).any(axis=1) | (fl != wfl))[0]
        assert bad.size == 0, (name, bad[:8] // 64, bad[:8] % 64, fl[bad[:4]], wfl[bad[:4]])
