"""CPU: the light-cone kernels' data flow (lifeapi_amd/csrc/cone_kernels.hpp),
modelled lane for lane and checked against the oracle's direct answer.

k_cone packs 64 / P universes into one 64-lane register set, lane j of group
q holding column (xs + j) mod 64 of its universe (zero for j >= K), and steps
the set with the streaming network, whose neighbour exchange is a 64-lane
rotate.  A register set is therefore stepped exactly as Step()
(LifeAPI.hpp:1196-1216) steps a LifeState whose column l is lane l -- so the
model assembles those "lane states", steps them with the oracle, and applies
the kernel's per-group test.  Agreement with Contains of the true state
(LifeTarget.hpp:44-51) on every window shape is the light-cone argument,
checked without a GPU: the neighbouring groups' columns that the rotate
brings into a group's margins never reach its care columns within g
generations.  The window search restates care_window (step_kernels.hpp).
"""
import numpy as np
import pytest

M64 = (1 << 64) - 1


def care_window(mask: int):
    """(x0, w): step_kernels.hpp care_window -- the complement of the longest
    cyclic run of empty positions, the lowest-starting run on ties; (0, 1)
    for an empty mask"""
    if mask == 0:
        return 0, 1
    best_len, best_start = 0, 0
    for p in range(64):
        run = 0
        while run < 64 and not (mask >> ((p + run) % 64)) & 1:
            run += 1
        if run > best_len:
            best_len, best_start = run, p
    if best_len == 0:
        return 0, 64
    return (best_start + best_len) % 64, 64 - best_len


def cone_layout(wanted, unwanted, gens):
    cols = 0
    for x in range(64):
        if int(wanted[x]) | int(unwanted[x]):
            cols |= 1 << x
    x0, w = care_window(cols)
    K, xs = w + 2 * gens, (x0 - gens) % 64
    if K >= 64:
        K, xs = 64, 0
    P = 4
    while P < K:
        P *= 2
    return xs, K, P


def cone_model(port, states, wanted, unwanted, gens, upw=32):
    """first generation 1..gens containing the target (gens >= 1), or
    Contains of the state as loaded (gens == 0), as k_cone computes them"""
    n = len(states)
    xs, K, P = cone_layout(wanted, unwanted, gens)
    gps = 64 // P
    lanes = np.arange(64)
    j, q = lanes % P, lanes // P
    col = (xs + j) % 64
    live = j < K
    tw = np.where(live, wanted[col], np.uint64(0))
    tm = np.where(live, wanted[col] | unwanted[col], np.uint64(0))
    n_sets = -(-n // gps)
    u = np.arange(n_sets)[:, None] * gps + q[None, :]            # universe of each (set, lane)
    ok = live[None, :] & (u < n)
    sets = np.where(ok, states[np.minimum(u, n - 1), col[None, :]], np.uint64(0))
    res = np.zeros((n_sets, gps), np.uint32)

    def clean(s):
        bad = ((s ^ tw) & tm) != 0                               # per lane
        return ~bad.reshape(n_sets, gps, P).any(axis=2)          # per group

    if gens == 0:
        res = clean(sets).astype(np.uint32)
    for g in range(1, gens + 1):
        sets = port.step_batch(sets, 1)                         # the 64-lane rotate = the torus of a lane state
        c = clean(sets)
        res[(res == 0) & c] = g
    return res.reshape(-1)[:n]


def direct(port, states, wanted, unwanted, gens):
    if gens == 0:
        return (((states ^ wanted) & (wanted | unwanted)) == 0).all(axis=1).astype(np.uint32)
    first, s = np.zeros(len(states), np.uint32), states
    for g in range(1, gens + 1):
        s = port.step_batch(s, 1)
        hit = (((s ^ wanted) & (wanted | unwanted)) == 0).all(axis=1)
        first[(first == 0) & hit] = g
    return first


def test_care_window_is_the_smallest_cyclic_window():
    rng = np.random.default_rng(3)
    for _ in range(400):
        k = int(rng.integers(1, 10))
        mask = 0
        for c in rng.integers(0, 64, size=k):
            mask |= 1 << int(c)
        if rng.random() < 0.3:                                   # a dense block across the seam
            a = int(rng.integers(64))
            for i in range(int(rng.integers(1, 64))):
                mask |= 1 << ((a + i) % 64)
        x0, w = care_window(mask)
        cover = sum(1 << ((x0 + i) % 64) for i in range(w))
        assert mask & ~cover == 0
        assert w == 64 or (mask >> x0) & 1 and (mask >> ((x0 + w - 1) % 64)) & 1
        # nothing shorter covers it
        assert not any(mask & ~sum(1 << ((s + i) % 64) for i in range(w - 1)) == 0 for s in range(64)) or w == 1
    assert care_window(0) == (0, 1) and care_window(M64) == (0, 64)
    assert care_window((1 << 63) | 1) == (63, 2)


def rotr64(v: int, k: int) -> int:
    return ((v >> k) | (v << ((64 - k) % 64))) & M64


def cone_fits(mask: int, gens: int, kmax: int) -> bool:
    """step_kernels.hpp cone_fits: a cyclic run of >= 64 - kmax + 2 gens empty
    columns, by doubling to runs of 32 and one shifted AND"""
    run = ~mask & M64
    for k in range(5):
        run &= rotr64(run, 1 << k)
    return run & rotr64(run, 64 - kmax + 2 * gens - 32) != 0


def has_run(e: int, L: int) -> bool:
    """step_kernels.hpp has_run: a cyclic run of >= L set bits in e"""
    if L >= 64:
        return e == M64
    run = [e]
    for k in range(1, 6):
        run.append(run[-1] & rotr64(run[-1], 1 << (k - 1)))
    cur, ln = M64, 0
    for k in range(5, -1, -1):
        if (L >> k) & 1:
            cur &= rotr64(run[k], ln)
            ln += 1 << k
    return cur != 0


def test_cone_whole_is_cone_window_k_64():
    """k_cone's quick whole-board test (cone_whole) agrees with cone_window's
    K = 64 for every gens 0..40 on every mask family"""
    rng = np.random.default_rng(12)
    masks = [0, M64, 1, (1 << 63) | 1, M64 ^ 1, M64 ^ (3 << 20)]
    for _ in range(500):
        m = M64
        for _ in range(int(rng.integers(0, 4))):             # a few empty runs
            a, ln = int(rng.integers(64)), int(rng.integers(1, 40))
            for i in range(ln):
                m &= ~(1 << ((a + i) % 64))
        masks.append(m)
        masks.append(int(rng.integers(0, 1 << 63)))
    for m in masks:
        _, w = care_window(m)
        for g in range(0, 41):
            whole = g >= 32 or not has_run(~m & M64, 2 * g + 1)
            assert whole == (g >= 32 or w + 2 * g >= 64), (hex(m), g)


def test_cone_fits_is_cone_window_k_at_most_kmax():
    """the split kernels' quick test agrees with cone_window's K <= kmax
    (K = w + 2 gens) on every mask family, 2 gens < kmax <= 32"""
    rng = np.random.default_rng(11)
    masks = [0, M64, 1, (1 << 63) | 1]
    for _ in range(600):
        w = int(rng.integers(1, 65))
        a = int(rng.integers(64))
        m = (1 << a) | (1 << ((a + w - 1) % 64))                 # a window of exactly w columns
        for c in rng.integers(0, w, size=int(rng.integers(0, 6))):
            m |= 1 << ((a + int(c)) % 64)
        masks.append(m)
        masks.append(int(rng.integers(0, 1 << 63)) & int(rng.integers(0, 1 << 63)))
    for m in masks:
        _, w = care_window(m)
        for kmax in (4, 8, 17, 24, 32):
            for g in range(0, (kmax + 1) // 2):
                if 2 * g >= kmax:
                    continue
                assert cone_fits(m, g, kmax) == (w + 2 * g <= kmax), (hex(m), g, kmax)


@pytest.mark.parametrize("w", [1, 2, 3, 4, 5, 6, 7, 8, 9, 13, 15, 16, 17, 28, 30, 31, 32, 33, 47, 60, 61, 62, 63, 64])
def test_cone_model_equals_contains(port, w):
    rng = np.random.default_rng(w)
    n = 97                                                       # ragged: partial sets and groups
    x = port.fill(n, seed=w) & port.fill(n, seed=w + 100)
    x[::4] = x[0]
    for x0 in (int(rng.integers(64)), (64 - w // 2) % 64, 63):
        box = np.zeros(64, np.uint64)
        for i in range(w):
            if i in (0, w - 1) or rng.random() < 0.5:
                box[(x0 + i) % 64] = np.uint64(int(rng.integers(1, 1 << 63)))
        for g in (0, 1, 2):
            ahead = port.step_batch(x[:1], g)[0] if g else x[0]
            tw, tu = ahead & box, box & ~ahead
            for gens in (0, 1, 2):
                want = direct(port, x, tw, tu, gens)
                got = cone_model(port, x, tw, tu, gens)
                assert (got == want).all(), (w, x0, g, gens, np.nonzero(got != want)[0][:8])
                if gens == g:
                    assert want[0] != 0


def test_cone_model_without_margins_is_wrong(port):
    """The margins are necessary: the same model with K = w (no light cone)
    gets the 1-generation filter wrong on random states -- the check above
    would notice a kernel that dropped them."""
    x = port.fill(400, seed=5)
    tw = np.zeros(64, np.uint64)
    tu = np.zeros(64, np.uint64)
    tw[20] = np.uint64(1 << 30)                                   # one live and one dead cell
    tu[21] = np.uint64(1 << 30)
    global cone_layout
    keep = cone_layout
    try:
        cone_layout = lambda w_, u_, gens: (20, 2, 4)            # noqa: E731  (no margins)
        got = cone_model(port, x, tw, tu, 1)
    finally:
        cone_layout = keep
    want = direct(port, x, tw, tu, 1)
    assert 0 < want.sum() < len(x) and (got != want).any()


@pytest.mark.parametrize("w,gens", [(1, 3), (2, 8), (4, 5), (4, 13), (6, 7), (6, 13), (10, 11), (16, 8), (20, 6),
                                    (3, 15), (1, 31), (30, 17)])
def test_cone_model_iterated(port, w, gens):
    """The iterated search loop on the light cone (gens > 2, no final
    states): the margins grow with g (K = w + 2g), and a cone that reaches 64
    columns (or g >= 32) is the whole board; equal to the direct loop"""
    rng = np.random.default_rng(100 * w + gens)
    n = 65
    x = port.fill(n, seed=w + gens) & port.fill(n, seed=3 * w + gens)
    x[::3] = x[0]
    x0 = int(rng.integers(64))
    box = np.zeros(64, np.uint64)
    for i in range(w):
        if i in (0, w - 1) or rng.random() < 0.5:
            box[(x0 + i) % 64] = np.uint64(int(rng.integers(1, 1 << 63)))
    ahead = port.step_batch(x[:1], gens // 2)[0]
    tw, tu = ahead & box, box & ~ahead
    want = direct(port, x, tw, tu, gens)
    assert (cone_model(port, x, tw, tu, gens) == want).all()
    assert want[0] != 0
