"""GPU parity of the RLE batch I/O kernels (Parsing.hpp:8-63,143-204):
k_rle (LifeState::RLE) and k_parse_rle (LifeState::Parse) through the C ABI,
against the reference-generated fixture (tests/golden/rle.npz) and the C
oracle; byte-exact.  The parser reads 64 bytes per step, so the fuzz cases
put digits, header lines and CR/LF across those boundaries."""
import os
import random

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def to_dev(a: np.ndarray) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64).reshape(-1, 64).copy()).cuda()


def to_host(t: torch.Tensor) -> np.ndarray:
    torch.cuda.synchronize()
    return t.cpu().numpy().view(np.uint64).reshape(-1, 64)


def blob_dev(strs):
    bs = [s.encode() if isinstance(s, str) else s for s in strs]
    offs = np.zeros(len(bs) + 1, np.int64)
    offs[1:] = np.cumsum([len(b) for b in bs])
    text = torch.from_numpy(np.frombuffer(b"".join(bs) or b"\0", np.uint8).copy()).cuda()
    return text, torch.from_numpy(offs).cuda()


def moved32(s):
    s = np.roll(np.asarray(s, np.uint64).reshape(-1, 64), 32, axis=1)
    return (s << np.uint64(32)) | (s >> np.uint64(32))


def test_rle_golden(hip):
    g = np.load(os.path.join(GOLD, "rle.npz"))
    text, offs = hip.rle(to_dev(g["states"]))
    torch.cuda.synchronize()
    assert offs.cpu().numpy().tolist() == g["rle_offsets"].astype(np.int64).tolist()
    assert text.cpu().numpy().tobytes() == g["rle_text"].tobytes()


def test_parse_golden(hip):
    g = np.load(os.path.join(GOLD, "rle.npz"))
    text = torch.from_numpy(g["parse_text"].copy()).cuda()
    offs = torch.from_numpy(g["parse_offsets"].astype(np.int64)).cuda()
    out, status = hip.parse_rle(text, offs)
    assert (to_host(out) == g["parsed"]).all()
    st = status.cpu().numpy()
    pt = g["parse_text"].tobytes()
    for u in range(len(st)):
        s = pt[g["parse_offsets"][u]:g["parse_offsets"][u + 1]]
        assert st[u] == (2 if s.startswith(b"o129$") else 0), (s, st[u])


def fuzz(rle: str, rng: random.Random) -> str:
    """Same pattern, new bytes: header and 'x' lines, CR/LF and spaces
    anywhere (also inside counts, which GenericParse accumulates across)."""
    out = ["x = 64, y = 64, rule = B3/S23\r\n" if rng.random() < 0.5 else ""]
    for ch in rle:
        r = rng.random()
        if r < 0.05:
            out.append("\r\n")
        elif r < 0.08:
            out.append(" ")
        elif r < 0.09:
            out.append("\nx this line is dropped 12o$\n")
        out.append(ch)
    return "".join(out)


def test_parse_fuzz_vs_oracle(hip, port):
    rng = random.Random(5)
    x = port.fill(300, seed=51)
    x[100:200] &= port.fill(100, seed=52) & port.fill(100, seed=53)
    x[200:] &= port.fill(100, seed=54) & port.fill(100, seed=55) & port.fill(100, seed=56)
    strs = [fuzz(port.rle(s), rng) for s in x]
    out, status = hip.parse_rle(*blob_dev(strs))
    got = to_host(out)
    assert not status.any().item()
    for u, s in enumerate(strs):
        assert (got[u] == port.parse(s)).all(), u
    assert (got == moved32(x)).all()


def test_parse_edges(hip, port):
    cases = ["", "!", "o", "64o!", "65o!", "o$" * 63 + "o!", "o$" * 64 + "o!", "b63o$63bo!", "o128$o!",
             "o129$o!", "5$", "x", "x\n", "\n\n3o!", "2o!ooo", "9" * 70 + "b!", "1" + " " * 70 + "2o!",
             "x" + "b" * 100 + "\n2o!", "#comment\no!", "o\r\no\r\n!", "0o$o!", "$" * 70 + "o!"]
    out, status = hip.parse_rle(*blob_dev(cases))
    got, st = to_host(out), status.cpu().numpy()
    for u, c in enumerate(cases):
        try:
            want, off_board = port.parse(c), False
        except ValueError:
            want, off_board = None, True
        assert bool(st[u] & 1) == off_board, (c, st[u])
        if want is not None:
            assert (got[u] == want).all(), c
    assert st[cases.index("o129$o!")] == 2
    # in-board cells of an off-board run are kept
    assert got[cases.index("65o!")][:64].tolist() == [1] * 64


def test_rle_round_trip_full_size(hip, port):
    n = 1 << 18
    x = hip.fill_random(n, seed=61)
    y = hip.fill_random(n, seed=62)
    x[n // 2:] &= y[n // 2:]
    text, offs = hip.rle(x)
    back, status = hip.parse_rle(text, offs)
    torch.cuda.synchronize()
    assert not status.any().item()
    xs = to_host(x)
    assert (to_host(back) == moved32(xs)).all()
    o = offs.cpu().numpy()
    t = text.cpu().numpy().tobytes()
    for u in list(range(0, n, 9973)) + [n - 1]:
        assert t[o[u]:o[u + 1]].decode() == port.rle(xs[u]), u


def test_rle_host_twins(hip, port):
    x = port.fill(1000, seed=71)
    x[500:] &= port.fill(500, seed=72)
    strs = hip.rle_host(x)
    assert strs[:50] == [port.rle(s) for s in x[:50]]
    back, st = hip.parse_rle_host(strs)
    assert not st.any() and (back == moved32(x)).all()
    assert hip.rle_host(x[:0]) == []
    with pytest.raises(hip.LifeApiError):
        offs = np.zeros(3, np.uint64)
        hip.lib.lifeapi_rle_batch(x.ctypes.data, 2, b"tiny", 4, offs.ctypes.data, 0)
        hip._check(hip.lib.lifeapi_rle_batch(x.ctypes.data, 2, b"tiny", 4, offs.ctypes.data, 0))
