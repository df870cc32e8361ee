"""GPU: the multi-device branch of the host-pointer lifeapi_step_batch and
lifeapi_step_contains_batch (device = -1: contiguous shards, one host thread
each, the arrays pinned once for all shards; host.hip over_devices).  A 1-GPU box has one device, so the shard count is
forced with LIFEAPI_HOST_SHARDS (shard s on device s mod ndev): the threads,
the shard arithmetic and the shared pins all run as they would over 8 GPUs.  Checked against the reference's own Step() (oracle/_ref)
where built, else the C port."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture
def shards(monkeypatch):
    def set_(k):
        monkeypatch.setenv("LIFEAPI_HOST_SHARDS", str(k))
    return set_


@pytest.fixture(scope="module")
def stepper():
    from oracle.oracle import Port, Ref
    return Ref() if Ref.available() else Port()


@pytest.mark.parametrize("k", [2, 3, 8])
@pytest.mark.parametrize("n,gens", [(1, 1), (7, 3), (4099, 1), (20001, 5), (70000, 1)])
def test_sharded_host_step(hip, stepper, shards, k, n, gens):
    shards(k)
    from oracle.oracle import Port
    x = Port().fill(n, seed=900 + n + k)
    got = hip.step_host(x, gens, device=-1)
    assert (got == stepper.step_batch(x, gens)).all()


def test_sharded_in_place_large(hip, stepper, shards):
    # > kPinMinBytes, so the call pins the arrays once for all 4 shard threads
    shards(4)
    from oracle.oracle import Port
    x = Port().fill(40000, seed=4242)
    want = stepper.step_batch(x, 2)
    hip.step_host(x, 2, device=-1, out=x)
    assert (x == want).all()


@pytest.mark.parametrize("k", [2, 3])
@pytest.mark.parametrize("n,gens,keep", [(5, 1, True), (4099, 2, False), (20001, 13, True)])
def test_sharded_host_search_loop(hip, shards, k, n, gens, keep):
    """the search loop (Step + Contains every generation) sharded the same
    way: first-hit generations and final states against the reference's own
    loop (oracle/_ref ref_step_contains_batch) where built, else the port"""
    shards(k)
    from oracle.oracle import Port, Ref
    P = Port()
    w, u = np.zeros(64, np.uint64), np.zeros(64, np.uint64)
    w[10] = w[11] = np.uint64(3 << 40)
    for c in (9, 10, 11, 12):
        u[c] = np.uint64(15 << 39)
    u &= ~w
    x = P.fill(n, seed=300 + n) & P.fill(n, seed=301 + n) & P.fill(n, seed=302 + n)
    clear = np.zeros(64, np.uint64)
    clear[2:20] = np.uint64(0x3FFFF << 32)
    x[::5] = (x[::5] & ~clear) | w
    fin = np.empty_like(x) if keep else None
    first = hip.step_contains_host(x, w, u, gens, final=fin, device=-1)
    if Ref.available():
        want_first, want_fin = Ref().step_contains_batch(x, w, u, gens, nthreads=4)
    else:
        want_first, s = np.zeros(n, np.uint32), x.copy()
        for g in range(1, gens + 1):
            s = P.step_batch(s, 1)
            hit = np.array([P.contains(s[i], w, u) for i in range(n)])
            want_first[(want_first == 0) & hit] = g
        want_fin = s
    assert (first == want_first).all()
    assert (want_first > 0).any()
    if keep:
        assert (fin == want_fin).all()


@pytest.mark.parametrize("k", [2, 3])
def test_sharded_host_forms(hip, shards, k):
    """every other host form (pop, contains, counts, weld, refined, LifeStable
    pass and Vulnerable) sharded the same way equals its one-device result"""
    from oracle.oracle import Port
    P = Port()
    n = 3001
    x = P.fill(n, seed=77) & P.fill(n, seed=78)
    w = x[5].copy()
    one = {"pop": hip.pop_host(x, device=0)}
    shards(k)
    assert (hip.pop_host(x, device=-1) == one["pop"]).all()
    lib, c = hip.lib, __import__("ctypes")

    def call(name, *args):
        hip._check(getattr(lib, name)(*args))

    def host_twice(fn):
        a, b = fn(0), fn(-1)
        assert all((p == q).all() for p, q in zip(a, b))
        return a

    def contains(dev):
        out = np.zeros(n, np.uint8)
        call("lifeapi_contains_batch", x.ctypes.data, w.ctypes.data, w.ctypes.data, out.ctypes.data, n, dev)
        return (out,)
    assert host_twice(contains)[0][5] == 1

    def counts(dev):
        out = np.zeros((n, 4, 64), np.uint64)
        call("lifeapi_neighbour_count_batch", x.ctypes.data, out.ctypes.data, n, dev)
        out3 = np.zeros((n, 3, 64), np.uint64)
        call("lifeapi_interaction_counts_batch", x.ctypes.data, out3.ctypes.data, n, 0, dev)
        return out, out3
    host_twice(counts)

    welds0 = P.fill(n * 4, seed=79).reshape(n, 256)

    def weld(dev):
        wd = welds0.copy()
        call("lifeapi_weld_step_batch", wd.ctypes.data, n, 3, dev)
        return (wd,)
    host_twice(weld)

    planes11 = P.fill(n * 11, seed=80).reshape(n, 11 * 64)

    def refined(dev):
        out = np.zeros((n, 3 * 64), np.uint64)
        call("lifeapi_refined_step_batch", planes11.ctypes.data, out.ctypes.data, n, dev)
        return (out,)
    host_twice(refined)

    st0 = P.fill(n * 10, seed=81).reshape(n, 640)
    st0[:, 128:] &= P.fill(n * 8, seed=82).reshape(n, 512)

    def stable(dev):
        st = st0.copy()
        flags = np.zeros(n, np.uint8)
        call("lifeapi_stable_pass_batch", st.ctypes.data, flags.ctypes.data, n, 3, 0, dev)
        vul = np.zeros((n, 64), np.uint64)
        call("lifeapi_stable_vulnerable_batch", st0.ctypes.data, vul.ctypes.data, n, dev)
        return st, flags, vul
    host_twice(stable)


def test_bad_device_index(hip):
    x = np.zeros((2, 64), np.uint64)
    with pytest.raises(hip.LifeApiError) as e:
        hip.step_host(x, 1, device=hip.device_count())
    assert e.value.code == -2
    with pytest.raises(hip.LifeApiError):
        hip.step_host(x, 1, device=-2)


@pytest.mark.parametrize("bad", ["0", "65", "100000", "-3", "4x", " "])
def test_shard_override_rejects_bad_values(hip, shards, bad):
    """LIFEAPI_HOST_SHARDS outside 1..64 (or not an integer) is a caller
    error, not a request for that many threads (host.hip over_devices)"""
    shards(bad)
    from oracle.oracle import Port
    x = Port().fill(5, seed=5)
    with pytest.raises(hip.LifeApiError) as e:
        hip.step_host(x, 1, device=-1)
    assert e.value.code == -1 and "LIFEAPI_HOST_SHARDS" in str(e.value)  # LIFEAPI_E_INVALID


def test_shard_override_empty_means_unset(hip, stepper, shards):
    """`export LIFEAPI_HOST_SHARDS=` leaves the variable set but empty: that
    is no override (one shard per visible device), not an error"""
    shards("")
    from oracle.oracle import Port
    x = Port().fill(7, seed=77)
    assert (hip.step_host(x, 3, device=-1) == stepper.step_batch(x, 3)).all()


def test_shard_override_capped_at_n(hip, stepper, shards):
    """more shards than universes: one shard per universe, no empty shards"""
    shards(64)
    from oracle.oracle import Port
    x = Port().fill(3, seed=33)
    assert (hip.step_host(x, 2, device=-1) == stepper.step_batch(x, 2)).all()
