"""GPU: the launch policies that change speed but never results.

* occupancy caps (host.hip occupancy_lds): the dynamic LDS the product adds
  to cap the resident blocks per CU must give exactly the requested count on
  the occupancy API (round 2 rounded the share up, so a cap of 6 ran 5);
* the launch order keyed on the batch (host.hip launch_reverse): a launch
  reverses exactly when its input is a batch an earlier order-keyed launch
  wrote forward, and interleaved loops over several batches (A, B, A, B)
  keep the alternation per batch -- with results equal to the reference's
  own Step() (oracle/_ref) whatever the order."""
import os
import sys

import numpy as np
import pytest
import torch

from test_gpu_parity import to_dev, to_host

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "tune"))


@pytest.fixture(scope="module")
def tune():
    import tune_hip
    return tune_hip


@pytest.fixture(scope="module")
def stepper():
    from oracle.oracle import Port, Ref
    return Ref() if Ref.available() else Port()


def test_shipped_occupancy_caps_are_exact(tune):
    """the streaming k_step's cap (7 blocks, step.hip kStreamResidentBlocks)
    and the LifeStable kernels' (3 for the single passes and 4 for
    StabiliseOptions and Vulnerable, stencils.hip kStablePassResident)"""
    assert tune.capped_occupancy(0, 7) == 7
    for which in range(1, 8):
        for want in (3, 4):
            assert tune.capped_occupancy(which, want) == want, (which, want)


@pytest.mark.parametrize("want", [2, 3, 4, 5, 6, 7, 8])
def test_occupancy_cap_every_count(tune, want):
    """every cap from 2 to 8 on the streaming step (28 VGPRs: 8 blocks fit
    without a cap), including the counts that do not divide 160 KiB"""
    assert tune.capped_occupancy(0, want) == want


def test_order_book_alternates_per_batch(tune):
    """A and B ping-ponged in turn: each launch reverses the order its input
    was written in, so each batch alternates on its own"""
    nb = 4096 * 512
    a0, a1, b0, b1 = (torch.empty((4096, 64), dtype=torch.int64, device="cuda") for _ in range(4))
    p = lambda t: t.data_ptr()  # noqa: E731
    tune.order_note(p(a0), nb)  # a0 / b0 written forward (the book is process-wide)
    tune.order_note(p(b0), nb)
    seq = []
    for _ in range(3):
        seq.append(tune.order_probe(p(a0), p(a1), nb))   # A: a0 -> a1
        seq.append(tune.order_probe(p(b0), p(b1), nb))   # B: b0 -> b1
        seq.append(tune.order_probe(p(a1), p(a0), nb))   # A: a1 -> a0
        seq.append(tune.order_probe(p(b1), p(b0), nb))   # B: b1 -> b0
    assert seq == [True, True, False, False] * 3


def test_order_book_in_place_and_foreign_writes(tune):
    w = torch.empty((1024, 4, 64), dtype=torch.int64, device="cuda")
    p, nb = w.data_ptr(), 1024 * 2048
    tune.order_note(p, nb)
    assert [tune.order_probe(p, p, nb) for _ in range(4)] == [True, False, True, False]
    # a write of another extent over the same memory forgets the batch
    tune.order_note(p, 512)
    assert tune.order_probe(p, p, nb) is False
    # an input the book holds at another extent runs forward
    x = torch.empty((1024, 64), dtype=torch.int64, device="cuda")
    tune.order_note(x.data_ptr(), 512)
    assert tune.order_probe(x.data_ptr(), p, nb) is False


def test_every_device_writer_records_its_output(tune, hip):
    """A batch the book holds as written in reverse is read forward next;
    once another kernel rewrites it (the fill, the counts, a LifeStable
    pass, the split weld, the refined step), the book must hold it as written
    forward, so the next reader of that extent reverses (only the
    step, the filter and k_weld below 12 generations used to record)"""
    n = 4096
    big = torch.empty(n * 16 * 64, dtype=torch.int64, device="cuda")
    src = big.data_ptr()                       # a stand-in input address (the book never reads memory)
    zp = src + 8 * n * 512

    def check(ptr, nbytes, write):
        tune.order_note(src, nbytes)
        assert tune.order_probe(src, ptr, nbytes) is True     # ptr recorded as written in reverse
        write()
        torch.cuda.synchronize()
        assert tune.order_probe(ptr, zp, nbytes) is True      # rewritten forward: the next reader reverses

    y = torch.zeros((n, 64), dtype=torch.int64, device="cuda")
    check(y.data_ptr(), n * 512, lambda: hip.fill_random(n, seed=1, out=y))
    counts = torch.empty((n, 4, 64), dtype=torch.int64, device="cuda")
    check(counts.data_ptr(), n * 2048,
          lambda: hip._check(hip.lib.lifeapi_neighbour_count_batch_dev(y.data_ptr(), counts.data_ptr(), n,
                                                                       hip._stream(None))))
    st = torch.zeros((n // 8, 640), dtype=torch.int64, device="cuda")
    check(st.data_ptr(), (n // 8) * 5120, lambda: hip.stable_pass(st, "sync"))
    welds = torch.zeros((n // 4, 256), dtype=torch.int64, device="cuda")
    check(welds.data_ptr(), (n // 4) * 2048, lambda: hip.weld_step(welds, 12))
    planes = torch.zeros((n // 8, 11 * 64), dtype=torch.int64, device="cuda")
    out = torch.empty((n // 8, 3 * 64), dtype=torch.int64, device="cuda")
    check(out.data_ptr(), (n // 8) * 1536, lambda: hip.refined_step(planes, out=out))


@pytest.mark.parametrize("n", [1, 4099, 300000])
def test_interleaved_batches_equal_reference(hip, stepper, n):
    """the streaming step over two batches in turn (A, B, A, B, ...), ping-pong
    and in place, every launch equal to the reference whichever order the
    book gave it"""
    from oracle.oracle import Port
    xa, xb = Port().fill(n, seed=n + 1), Port().fill(n, seed=n + 2)
    want_a, want_b = [xa], [xb]
    for _ in range(4):
        want_a.append(stepper.step_batch(want_a[-1], 1))
        want_b.append(stepper.step_batch(want_b[-1], 1))
    a, a2 = to_dev(xa), torch.empty((n, 64), dtype=torch.int64, device="cuda")
    b, b2 = to_dev(xb), torch.empty((n, 64), dtype=torch.int64, device="cuda")
    for k in range(1, 5):
        hip.step(a, out=a2, generations=1)
        hip.step(b, out=b2, generations=1)
        assert (to_host(a2) == want_a[k]).all(), ("A", k)
        assert (to_host(b2) == want_b[k]).all(), ("B", k)
        a, a2, b, b2 = a2, a, b2, b
    a, b = to_dev(xa), to_dev(xb)
    for k in range(1, 4):
        hip.step(a, out=a, generations=1)
        hip.step(b, out=b, generations=1)
        assert (to_host(a) == want_a[k]).all() and (to_host(b) == want_b[k]).all(), k


def test_interleaved_filter_and_step(hip, stepper):
    """the search filter with final states (order-keyed up to 2M universes)
    reading what the step wrote, and the step reading the filter's output"""
    from oracle.oracle import Port
    n = 20001
    x = Port().fill(n, seed=77)
    w, u = np.zeros(64, np.uint64), np.zeros(64, np.uint64)
    w[3] = np.uint64(6)
    u[3] = np.uint64(9)
    dw, du = (torch.from_numpy(t[None].view(np.int64).copy()).cuda() for t in (w, u))
    a, b = to_dev(x), torch.empty((n, 64), dtype=torch.int64, device="cuda")
    want = x
    for k in range(4):
        if k % 2:
            first, fin = hip.step_contains(a, dw, du, 1, final=b)
            want = stepper.step_batch(want, 1)
            hit = (((want ^ w) & (w | u)) == 0).all(axis=1)
            assert (first.cpu().numpy() == np.where(hit, 1, 0)).all(), k
        else:
            hip.step(a, out=b, generations=1)
            want = stepper.step_batch(want, 1)
        assert (to_host(b) == want).all(), k
        a, b = b, a
