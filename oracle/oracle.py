"""ctypes bindings for the parity oracle.  TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline
leg import this module, and only as the checker / the timed CPU baseline.
The product package ``lifeapi_amd`` never imports it.

Two oracles live here:

* ``Port``  -- ``oracle/liboracle.so``: the plain-C restatement
  (``lifeapi_oracle.c``) of LifeAPI.hpp:822-907,1196-1254 and
  NeighbourCount.hpp:25-102.
* ``Ref``   -- ``oracle/_ref/libref_v{3,4}.so``: the reference's OWN
  ``LifeState::Step()`` etc., compiled from /root/reference by
  ``oracle/Makefile`` (target ``ref``).  Present on the GPU box only as the
  prebuilt .so (the reference tree itself is not there).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_u64p = ctypes.POINTER(ctypes.c_uint64)
_u32p = ctypes.POINTER(ctypes.c_uint32)


def _p64(a: np.ndarray):
    assert a.dtype == np.uint64 and a.flags.c_contiguous
    return a.ctypes.data_as(_u64p)


def _cpu_has_avx512() -> bool:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("flags"):
                    fl = set(line.split(":", 1)[1].split())
                    return {"avx512f", "avx512bw", "avx512dq", "avx512vl", "avx512cd"} <= fl
    except OSError:
        pass
    return False


def universes(n: int) -> np.ndarray:
    """Zeroed, 64-byte aligned (n, 64) uint64 array (LifeState[] layout)."""
    raw = np.zeros(n * 64 + 8, dtype=np.uint64)
    off = (-raw.ctypes.data % 64) // 8
    return raw[off:off + n * 64].reshape(n, 64)


class Port:
    """The C restatement (oracle/lifeapi_oracle.c)."""

    ROKICKI, FULLADD, NCOUNT = 0, 1, 2

    def __init__(self, path: str | None = None):
        path = path or os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: run `make -C oracle`")
        L = self.lib = ctypes.CDLL(path)
        L.oracle_step_batch.argtypes = [_u64p, _u64p, ctypes.c_size_t, ctypes.c_uint,
                                        ctypes.c_int, ctypes.c_int]
        L.oracle_pop_batch.argtypes = [_u64p, _u32p, ctypes.c_size_t]
        L.oracle_contains_target.argtypes = [_u64p, _u64p, _u64p]
        L.oracle_parse_rle.argtypes = [ctypes.c_char_p, _u64p]
        L.oracle_rle.argtypes = [_u64p, ctypes.c_char_p, ctypes.c_size_t]
        L.oracle_rle.restype = ctypes.c_size_t
        L.oracle_fill.argtypes = [_u64p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint64,
                                  ctypes.c_int]
        L.oracle_hash_batch.argtypes = [_u64p, _u64p, ctypes.c_size_t]
        L.oracle_batch_digest.argtypes = [_u64p, ctypes.c_size_t, ctypes.c_uint64]
        L.oracle_batch_digest.restype = ctypes.c_uint64
        L.oracle_neighbour_count.argtypes = [_u64p] * 5
        L.oracle_interaction_counts.argtypes = [_u64p] * 5
        L.oracle_weld_step.argtypes = [_u64p, ctypes.c_uint]
        L.oracle_stable_vulnerable.argtypes = [_u64p, _u64p, ctypes.POINTER(ctypes.c_uint8)]
        L.oracle_stable_pass.argtypes = [_u64p, ctypes.c_int, ctypes.POINTER(ctypes.c_uint8),
                                         ctypes.POINTER(ctypes.c_uint8)]
        L.oracle_refined_step_batch.argtypes = [_u64p, _u64p, ctypes.c_size_t,
                                                ctypes.POINTER(ctypes.c_uint8)]
        self._tt = None
        for name in ("oracle_step", "oracle_step_alt", "oracle_step_nc"):
            getattr(L, name).argtypes = [_u64p]

    def step_batch(self, states: np.ndarray, gens: int = 1, formulation: int = 0,
                   nthreads: int = 1) -> np.ndarray:
        src = np.ascontiguousarray(states, dtype=np.uint64).reshape(-1, 64)
        out = universes(src.shape[0])
        self.lib.oracle_step_batch(_p64(src), _p64(out), src.shape[0], gens, formulation, nthreads)
        return out

    def fill(self, n: int, seed: int, first_universe: int = 0, mode: int = 0) -> np.ndarray:
        out = universes(n)
        self.lib.oracle_fill(_p64(out), n, seed, first_universe, mode)
        return out

    def pop(self, states: np.ndarray) -> np.ndarray:
        src = np.ascontiguousarray(states, dtype=np.uint64).reshape(-1, 64)
        out = np.zeros(src.shape[0], dtype=np.uint32)
        self.lib.oracle_pop_batch(_p64(src), out.ctypes.data_as(_u32p), src.shape[0])
        return out

    def hashes(self, states: np.ndarray) -> np.ndarray:
        src = np.ascontiguousarray(states, dtype=np.uint64).reshape(-1, 64)
        out = np.zeros(src.shape[0], dtype=np.uint64)
        self.lib.oracle_hash_batch(_p64(src), _p64(out), src.shape[0])
        return out

    def digest(self, hashes: np.ndarray, first_universe: int = 0) -> int:
        h = np.ascontiguousarray(hashes, dtype=np.uint64)
        return int(self.lib.oracle_batch_digest(_p64(h), h.shape[0], first_universe))

    def contains(self, state, wanted, unwanted) -> bool:
        a, w, u = (np.ascontiguousarray(x, dtype=np.uint64).reshape(64) for x in (state, wanted, unwanted))
        return bool(self.lib.oracle_contains_target(_p64(a), _p64(w), _p64(u)))

    def parse(self, rle: str) -> np.ndarray:
        out = np.zeros(64, dtype=np.uint64)
        rc = self.lib.oracle_parse_rle(rle.encode(), _p64(out))
        if rc != 0:
            raise ValueError(f"RLE places a cell outside the 64x64 board: {rle!r}")
        return out

    def rle(self, state) -> str:
        s = np.ascontiguousarray(state, dtype=np.uint64).reshape(64)
        buf = ctypes.create_string_buffer(8192)
        n = self.lib.oracle_rle(_p64(s), buf, 8192)
        return buf.raw[:n].decode()

    def neighbour_count(self, state) -> np.ndarray:
        s = np.ascontiguousarray(state, dtype=np.uint64).reshape(64)
        b = np.zeros((4, 64), dtype=np.uint64)
        self.lib.oracle_neighbour_count(_p64(s), _p64(b[0]), _p64(b[1]), _p64(b[2]), _p64(b[3]))
        return b  # bit3, bit2, bit1, bit0

    def interaction_counts(self, state, with_next: bool = True) -> np.ndarray:
        """(4, 64): out1, out2, outMore, next (LifeAPI.hpp:956-1040)."""
        s = np.ascontiguousarray(state, dtype=np.uint64).reshape(64)
        b = np.zeros((4, 64), dtype=np.uint64)
        self.lib.oracle_interaction_counts(_p64(s), _p64(b[0]), _p64(b[1]), _p64(b[2]),
                                           _p64(b[3]) if with_next else None)
        return b if with_next else b[:3]

    def weld_step(self, welds: np.ndarray, gens: int = 1) -> np.ndarray:
        """LifeWeld::Step^gens on (n, 4*64) {state, frozen2, frozen1, frozen0}."""
        out = np.ascontiguousarray(welds, dtype=np.uint64).reshape(-1, 256).copy()
        for u in range(out.shape[0]):
            self.lib.oracle_weld_step(_p64(out[u]), gens)
        return out

    STABLE_PASSES = ("sync", "options", "signal", "step", "propagate", "stabilise")

    def stable_pass(self, planes: np.ndarray, which: int):
        """LifeStable pass `which` (0..5, see lifeapi_oracle.h) on (n, 640)
        planes; returns (planes, flags: bit0 consistent, bit1 changed)."""
        gold = os.path.join(os.path.dirname(HERE), "tests", "golden")
        if not hasattr(self, "_stt"):
            self._stt = tuple(np.ascontiguousarray(np.load(os.path.join(gold, f))["tt"].astype(np.uint8))
                              for f in ("stable_count_tt.npz", "stable_signal_tt.npz"))
        u8 = ctypes.POINTER(ctypes.c_uint8)
        out = np.ascontiguousarray(planes, dtype=np.uint64).reshape(-1, 640).copy()
        flags = np.zeros(out.shape[0], np.uint8)
        for u in range(out.shape[0]):
            flags[u] = self.lib.oracle_stable_pass(_p64(out[u]), which, self._stt[0].ctypes.data_as(u8),
                                                   self._stt[1].ctypes.data_as(u8))
        return out, flags

    def stable_vulnerable(self, planes: np.ndarray) -> np.ndarray:
        """LifeStable::Vulnerable() (LifeStable.hpp:366-412) of (n, 640) planes."""
        if not hasattr(self, "_vtt"):
            gold = os.path.join(os.path.dirname(HERE), "tests", "golden", "stable_vulnerable_tt.npz")
            self._vtt = np.ascontiguousarray(np.load(gold)["tt"].astype(np.uint8))
        src = np.ascontiguousarray(planes, dtype=np.uint64).reshape(-1, 640)
        out = universes(src.shape[0])
        u8 = ctypes.POINTER(ctypes.c_uint8)
        for u in range(src.shape[0]):
            self.lib.oracle_stable_vulnerable(_p64(src[u]), _p64(out[u]), self._vtt.ctypes.data_as(u8))
        return out

    def refined_truth_table(self) -> np.ndarray:
        if self._tt is None:
            path = os.path.join(os.path.dirname(HERE), "tests", "golden", "unknown_step_refined_tt.npz")
            self._tt = np.ascontiguousarray(np.load(path)["tt"].astype(np.uint8))
        return self._tt

    def refined_step(self, planes: np.ndarray) -> np.ndarray:
        """Config-5 harness: (n, 11*64) input planes -> (n, 3*64) output planes."""
        src = np.ascontiguousarray(planes, dtype=np.uint64).reshape(-1, 11 * 64)
        out = np.zeros((src.shape[0], 3 * 64), dtype=np.uint64)
        tt = self.refined_truth_table()
        self.lib.oracle_refined_step_batch(_p64(src), _p64(out), src.shape[0],
                                           tt.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))
        return out


class Ref:
    """The reference's own code (oracle/_ref/libref_v*.so)."""

    def __init__(self, path: str | None = None):
        if path is None:
            v = "v4" if _cpu_has_avx512() else "v3"
            path = os.path.join(HERE, "_ref", f"libref_{v}.so")
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: run `make -C oracle ref` where /root/reference exists")
        self.path = path
        L = self.lib = ctypes.CDLL(path)
        for name in ("ref_step", "ref_step_alt", "ref_step_nc", "ref_random_state"):
            getattr(L, name).argtypes = [_u64p]
        L.ref_step_n.argtypes = [_u64p, ctypes.c_uint]
        L.ref_step_batch.argtypes = [_u64p, _u64p, ctypes.c_size_t, ctypes.c_uint, ctypes.c_int]
        L.ref_pop.argtypes = [_u64p]
        L.ref_pop.restype = ctypes.c_uint
        L.ref_contains_target.argtypes = [_u64p, _u64p, _u64p]
        L.ref_parse.argtypes = [ctypes.c_char_p, _u64p]
        L.ref_rle.argtypes = [_u64p, ctypes.c_char_p, ctypes.c_size_t]
        L.ref_rle.restype = ctypes.c_size_t
        L.ref_neighbour_count.argtypes = [_u64p] * 5
        L.ref_count_neighbourhood.argtypes = [_u64p] * 5
        L.ref_interaction_counts.argtypes = [_u64p] * 5
        L.ref_weld_step.argtypes = [_u64p, ctypes.c_uint]
        L.ref_unknown_step_refined.argtypes = [_u64p, _u64p]
        L.ref_refined_step_batch.argtypes = [_u64p, _u64p, ctypes.c_size_t]
        L.ref_stable_pass.argtypes = [_u64p, ctypes.c_int]
        L.ref_stable_vulnerable.argtypes = [_u64p, _u64p]
        L.ref_contains_batch.argtypes = [_u64p, ctypes.c_size_t, _u64p, _u64p, ctypes.c_char_p]
        L.ref_pattern_batch.argtypes = [_u64p, ctypes.c_size_t, _u64p, _u64p, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_int, ctypes.c_char_p]
        L.ref_target_from_state.argtypes = [_u64p, ctypes.c_int, ctypes.c_int, _u64p, _u64p]
        L.ref_step_contains_batch.argtypes = [_u64p, _u64p, ctypes.c_size_t, ctypes.c_uint, _u64p, _u64p,
                                              ctypes.POINTER(ctypes.c_uint32), ctypes.c_int]

    @staticmethod
    def available() -> bool:
        v = "v4" if _cpu_has_avx512() else "v3"
        return os.path.exists(os.path.join(HERE, "_ref", f"libref_{v}.so"))

    def step_batch(self, states: np.ndarray, gens: int = 1, nthreads: int = 1) -> np.ndarray:
        src = np.ascontiguousarray(states, dtype=np.uint64).reshape(-1, 64)
        out = universes(src.shape[0])
        self.lib.ref_step_batch(_p64(src), _p64(out), src.shape[0], gens, nthreads)
        return out

    def step_contains_batch(self, states, wanted, unwanted, gens: int, nthreads: int = 1):
        """(first, final): the reference's Step() then Contains(LifeTarget)
        after every generation (ref_shim.cpp ref_step_contains_batch)"""
        src = np.ascontiguousarray(states, dtype=np.uint64).reshape(-1, 64)
        w, u = (np.ascontiguousarray(x, dtype=np.uint64).reshape(64) for x in (wanted, unwanted))
        out = universes(src.shape[0])
        first = np.zeros(src.shape[0], dtype=np.uint32)
        self.lib.ref_step_contains_batch(_p64(src), _p64(out), src.shape[0], gens, _p64(w), _p64(u),
                                         first.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), nthreads)
        return first, out

    def _each(self, fn, states):
        out = universes(np.asarray(states).reshape(-1, 64).shape[0])
        out[:] = np.asarray(states, dtype=np.uint64).reshape(-1, 64)
        for u in range(out.shape[0]):
            fn(_p64(out[u]))
        return out

    def step_alt(self, states):
        return self._each(self.lib.ref_step_alt, states)

    def step_nc(self, states):
        return self._each(self.lib.ref_step_nc, states)

    def random_state(self) -> np.ndarray:
        out = np.zeros(64, dtype=np.uint64)
        self.lib.ref_random_state(_p64(out))
        return out

    def parse(self, rle: str) -> np.ndarray:
        out = np.zeros(64, dtype=np.uint64)
        self.lib.ref_parse(rle.encode(), _p64(out))
        return out

    def rle(self, state) -> str:
        s = np.ascontiguousarray(state, dtype=np.uint64).reshape(64)
        buf = ctypes.create_string_buffer(8192)
        n = self.lib.ref_rle(_p64(s), buf, 8192)
        return buf.raw[:n].decode()

    def pop(self, state) -> int:
        s = np.ascontiguousarray(state, dtype=np.uint64).reshape(64)
        return int(self.lib.ref_pop(_p64(s)))

    def contains(self, state, wanted, unwanted) -> bool:
        a, w, u = (np.ascontiguousarray(x, dtype=np.uint64).reshape(64) for x in (state, wanted, unwanted))
        return bool(self.lib.ref_contains_target(_p64(a), _p64(w), _p64(u)))

    def contains_batch(self, states, wanted, unwanted) -> np.ndarray:
        """uint8 per universe: the reference's Contains(LifeTarget) (LifeTarget.hpp:44-51)"""
        src = np.ascontiguousarray(states, dtype=np.uint64).reshape(-1, 64)
        w, u = (np.ascontiguousarray(x, dtype=np.uint64).reshape(64) for x in (wanted, unwanted))
        out = ctypes.create_string_buffer(max(1, src.shape[0]))
        self.lib.ref_contains_batch(_p64(src), src.shape[0], _p64(w), _p64(u), out)
        return np.frombuffer(out.raw[:src.shape[0]], dtype=np.uint8).copy()

    PATTERN_KINDS = ("contains", "disjoint", "contains_at", "disjoint_at", "target_at")

    def pattern_batch(self, states, kind: str, pat, pat2=None, dx: int = 0, dy: int = 0) -> np.ndarray:
        """uint8 per universe: Contains(pat) / AreDisjoint(pat) / their (dx, dy)
        forms / Contains(LifeTarget{pat, pat2}, dx, dy) (LifeAPI.hpp:378-422,
        LifeTarget.hpp:38-42)"""
        src = np.ascontiguousarray(states, dtype=np.uint64).reshape(-1, 64)
        p = np.ascontiguousarray(pat, dtype=np.uint64).reshape(64)
        p2 = np.zeros(64, np.uint64) if pat2 is None else np.ascontiguousarray(pat2, dtype=np.uint64).reshape(64)
        out = ctypes.create_string_buffer(max(1, src.shape[0]))
        self.lib.ref_pattern_batch(_p64(src), src.shape[0], _p64(p), _p64(p2), self.PATTERN_KINDS.index(kind),
                                   dx, dy, out)
        return np.frombuffer(out.raw[:src.shape[0]], dtype=np.uint8).copy()

    def target_from_state(self, state, dx: int = 0, dy: int = 0):
        """(wanted, unwanted) of LifeTarget(state).Moved({dx, dy}) (LifeTarget.hpp:10-13,33-35)"""
        s = np.ascontiguousarray(state, dtype=np.uint64).reshape(64)
        w, u = np.zeros(64, np.uint64), np.zeros(64, np.uint64)
        self.lib.ref_target_from_state(_p64(s), dx, dy, _p64(w), _p64(u))
        return w, u

    def neighbour_count(self, state) -> np.ndarray:
        s = np.ascontiguousarray(state, dtype=np.uint64).reshape(64)
        b = np.zeros((4, 64), dtype=np.uint64)
        self.lib.ref_neighbour_count(_p64(s), _p64(b[0]), _p64(b[1]), _p64(b[2]), _p64(b[3]))
        return b

    def interaction_counts(self, state) -> np.ndarray:
        s = np.ascontiguousarray(state, dtype=np.uint64).reshape(64)
        b = np.zeros((4, 64), dtype=np.uint64)
        self.lib.ref_interaction_counts(_p64(s), _p64(b[0]), _p64(b[1]), _p64(b[2]), _p64(b[3]))
        return b

    def weld_step(self, welds: np.ndarray, gens: int = 1) -> np.ndarray:
        out = np.ascontiguousarray(welds, dtype=np.uint64).reshape(-1, 256).copy()
        for u in range(out.shape[0]):
            self.lib.ref_weld_step(_p64(out[u]), gens)
        return out

    def stable_pass(self, planes: np.ndarray, which: int) -> int:
        """one LifeStable pass in place on one object's 10 x 64 planes
        (ref_shim.cpp ref_stable_pass): returns consistent | changed << 1"""
        assert planes.dtype == np.uint64 and planes.flags.c_contiguous and planes.size == 640
        return int(self.lib.ref_stable_pass(_p64(planes), which))

    def stable_vulnerable(self, planes: np.ndarray) -> np.ndarray:
        s = np.ascontiguousarray(planes, dtype=np.uint64).reshape(640)
        out = np.zeros(64, np.uint64)
        self.lib.ref_stable_vulnerable(_p64(s), _p64(out))
        return out

    def refined_step(self, planes: np.ndarray) -> np.ndarray:
        """Config-5 harness around the reference's own fragment (ref_shim.cpp)."""
        src = np.ascontiguousarray(planes, dtype=np.uint64).reshape(-1, 11 * 64)
        out = np.zeros((src.shape[0], 3 * 64), dtype=np.uint64)
        self.lib.ref_refined_step_batch(_p64(src), _p64(out), src.shape[0])
        return out
