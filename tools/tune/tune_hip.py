"""ctypes binding of the TUNING build (tools/tune/liblifeapi_tune.so,
lifeapi_tune.h): batched Step() with an explicit launch configuration.
Loads the product binding (lifeapi_amd.hip) first, so both libraries share
torch's HIP runtime and the product's error state."""
from __future__ import annotations

import ctypes
import os

import torch

import lifeapi_amd.hip as hip

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "liblifeapi_tune.so")
if not os.path.exists(LIB_PATH):
    raise ImportError(f"{LIB_PATH} is missing: build it with __graft_entry__.build()")
lib = ctypes.CDLL(LIB_PATH)

XCHG_DPP, XCHG_LDS, XCHG_BPERM, XCHG_MIX, XCHG_MIX1, XCHG_MIX3, XCHG_LDSR, XCHG_LDSR3, XCHG_ASM = range(9)
XCHG_LDS_PIPE = 9


def XCHG_ASM_V(k: int) -> int:
    return 24 + k


def XCHG_LDS_DPP(d: int) -> int:
    return 16 + d


class LaunchCfg(ctypes.Structure):
    """lifeapi_launch_cfg (tools/tune/lifeapi_tune.h)."""

    _fields_ = [("xchg", ctypes.c_int), ("universes_per_wave", ctypes.c_int),
                ("blocks_per_cu", ctypes.c_int), ("nontemporal", ctypes.c_int),
                ("rule", ctypes.c_int)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


_vp, _sz, _u32, _int = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_int
lib.lifeapi_tune_default_cfg.argtypes = [ctypes.POINTER(LaunchCfg), _u32]
lib.lifeapi_tune_default_cfg.restype = None
lib.lifeapi_tune_step_batch_dev_cfg.argtypes = [_vp, _vp, _sz, _u32, _vp, ctypes.POINTER(LaunchCfg)]
lib.lifeapi_tune_step_batch_dev_cfg.restype = _int


def default_cfg(generations: int = 1) -> LaunchCfg:
    c = LaunchCfg()
    lib.lifeapi_tune_default_cfg(ctypes.byref(c), generations)
    return c


def step(states: torch.Tensor, out: torch.Tensor | None = None, generations: int = 1,
         cfg: LaunchCfg | None = None, stream=None) -> torch.Tensor:
    n = hip._universes(states)
    if out is None:
        out = torch.empty_like(states)
    if hip._universes(out, "out") != n:
        raise ValueError("out has a different number of universes")
    hip._check(lib.lifeapi_tune_step_batch_dev_cfg(states.data_ptr(), out.data_ptr(), n, generations,
                                                   hip._stream(stream),
                                                   ctypes.byref(cfg) if cfg is not None else None))
    return out


lib.lifeapi_tune_step_clock.argtypes = [_vp, _vp, _sz, _u32, _vp, _vp]
lib.lifeapi_tune_step_clock.restype = _int


def step_clock(states: torch.Tensor, out: torch.Tensor, generations: int, stream=None):
    """The shipped gens > 2 kernel with clock stamps; returns (out, stamps
    int64 (waves, 4): t0, q0, t1, q1)."""
    n = hip._universes(states)
    stamps = torch.zeros(((n + 3) // 4, 4), dtype=torch.int64, device=states.device)
    hip._check(lib.lifeapi_tune_step_clock(states.data_ptr(), out.data_ptr(), n, generations,
                                           hip._stream(stream), stamps.data_ptr()))
    return out, stamps


lib.lifeapi_tune_step_order.argtypes = [_vp, _vp, _sz, _u32, _vp, _int, _int, _int, ctypes.c_uint64]
lib.lifeapi_tune_step_order.restype = _int


def step_order(states: torch.Tensor, out: torch.Tensor, generations: int = 1, reverse: bool = False,
               nts: bool = True, resident: int = 6, upw: int = 4, plain_bytes: int = 0,
               stream=None, xcd_chunk: bool = False) -> torch.Tensor:
    """The shipped gens <= 2 kernel with nontemporal or plain stores, at most
    `resident` blocks per CU, `upw` universes per wave, universes taken in
    reverse order if asked; plain stores for the groups that store the last
    `plain_bytes` of the launch's order whatever `nts` says."""
    n = hip._universes(states)
    hip._check(lib.lifeapi_tune_step_order(states.data_ptr(), out.data_ptr(), n,
                                           generations | ((1 << 31) if reverse else 0) |
                                           ((1 << 30) if xcd_chunk else 0), hip._stream(stream),
                                           1 if nts else 0, resident, upw, plain_bytes))
    return out


lib.lifeapi_tune_hash.argtypes = [_vp, _vp, _sz, _int, _int, _vp]
lib.lifeapi_tune_hash.restype = _int


def hash_variant(states: torch.Tensor, variant: int, blocks_per_cu: int = 0, out=None, stream=None):
    n = hip._universes(states)
    if out is None:
        out = torch.empty(n, dtype=torch.int64, device=states.device)
    hip._check(lib.lifeapi_tune_hash(states.data_ptr(), out.data_ptr(), n, variant, blocks_per_cu,
                                     hip._stream(stream)))
    return out


lib.lifeapi_tune_stable_pass.argtypes = [_vp, _vp, _sz, _int, _u32, _int, _vp, _int]
lib.lifeapi_tune_stable_pass.restype = _int
lib.lifeapi_tune_stable_vulnerable.argtypes = [_vp, _vp, _sz, _int, _vp]
lib.lifeapi_tune_stable_vulnerable.restype = _int


def stable_pass(planes: torch.Tensor, which: int, blocks_per_cu: int, max_iters: int = 0, stream=None,
                reverse: bool = False, xcd_chunk: bool = False, store_all: bool = False, upw: int = 0,
                no_store: bool = False):
    """store_all: every line stored (round 3's k_stable), else only the lines
    holding a changed column (the shipped form); no_store (k_stable only): no
    plane stored -- a timing probe, the planes are left wrong"""
    n = planes.numel() // (10 * 64)
    flags = torch.empty(n, dtype=torch.uint8, device=planes.device)
    hip._check(lib.lifeapi_tune_stable_pass(planes.data_ptr(), flags.data_ptr(), n, which, max_iters,
                                            blocks_per_cu, hip._stream(stream),
                                            (1 if reverse else 0) | (2 if xcd_chunk else 0) | (4 if store_all else 0)
                                            | (8 if no_store else 0) | (upw << 8)))
    return flags


lib.lifeapi_tune_reduce.argtypes = [_int, _vp, _vp, _vp, _vp, _sz, _int, _int, _vp]
lib.lifeapi_tune_reduce.restype = _int


def reduce(kind: int, states, out, upw: int, blocks_per_cu: int, wanted=None, unwanted=None, stream=None):
    """kind 0 GetPop (out int32), 1 Contains (out uint8)"""
    n = hip._universes(states)
    hip._check(lib.lifeapi_tune_reduce(kind, states.data_ptr(), None if wanted is None else wanted.data_ptr(),
                                       None if unwanted is None else unwanted.data_ptr(), out.data_ptr(), n, upw,
                                       blocks_per_cu, hip._stream(stream)))
    return out


lib.lifeapi_tune_weld_order.argtypes = [_vp, _sz, _int, ctypes.c_uint64, _vp]
lib.lifeapi_tune_weld_order.restype = _int


def weld_order(welds: torch.Tensor, reverse: bool = False, plain_welds: int = 0, stream=None):
    """k_weld one generation in place, order reversed if asked, the last
    `plain_welds` welds of the launch's order loaded and stored plain."""
    hip._check(lib.lifeapi_tune_weld_order(welds.data_ptr(), welds.shape[0], 1 if reverse else 0, plain_welds,
                                           hip._stream(stream)))
    return welds


lib.lifeapi_tune_stencil.argtypes = [_int, _vp, _vp, _sz, _int, _vp]
lib.lifeapi_tune_stencil.restype = _int


def stencil(kind: int, inp: torch.Tensor, out, n: int, resident: int, stream=None):
    """kind 0..2 k_counts, 3 k_weld (1 gen, in place on inp), 4 k_refined"""
    hip._check(lib.lifeapi_tune_stencil(kind, inp.data_ptr(), None if out is None else out.data_ptr(), n, resident,
                                        hip._stream(stream)))


def stable_vulnerable(planes: torch.Tensor, blocks_per_cu: int, out=None, stream=None):
    n = planes.numel() // (10 * 64)
    if out is None:
        out = torch.empty((n, 64), dtype=torch.int64, device=planes.device)
    hip._check(lib.lifeapi_tune_stable_vulnerable(planes.data_ptr(), out.data_ptr(), n, blocks_per_cu,
                                                  hip._stream(stream)))
    return out


lib.lifeapi_tune_step_pair.argtypes = [_vp, _vp, _sz, _u32, _int, _vp]
lib.lifeapi_tune_step_pair.restype = _int


def step_pair(states: torch.Tensor, out: torch.Tensor, generations: int, variant: int = 0, stream=None):
    n = hip._universes(states)
    hip._check(lib.lifeapi_tune_step_pair(states.data_ptr(), out.data_ptr(), n, generations, variant,
                                          hip._stream(stream)))
    return out


lib.lifeapi_tune_step_contains.argtypes = [_vp, _vp, _vp, _vp, _vp, _sz, _u32, _int, _vp]
lib.lifeapi_tune_step_contains.restype = _int


def step_contains(states, wanted, unwanted, generations, variant, final=None, stream=None):
    n = hip._universes(states)
    first = torch.empty(n, dtype=torch.int32, device=states.device)
    hip._check(lib.lifeapi_tune_step_contains(states.data_ptr(), None if final is None else final.data_ptr(),
                                              wanted.data_ptr(), unwanted.data_ptr(), first.data_ptr(), n,
                                              generations, variant, hip._stream(stream)))
    return first


lib.lifeapi_tune_step_contains_nat.argtypes = [_vp, _vp, _vp, _vp, _vp, _sz, _u32, _int, _int, _vp]
lib.lifeapi_tune_step_contains_nat.restype = _int


def step_contains_nat(states, wanted, unwanted, generations, upw, resident, final=None, stream=None):
    """the natural-layout fused kernel (gens <= 2), upw universes per wave"""
    n = hip._universes(states)
    first = torch.empty(n, dtype=torch.int32, device=states.device)
    hip._check(lib.lifeapi_tune_step_contains_nat(
        states.data_ptr(), None if final is None else final.data_ptr(), wanted.data_ptr(), unwanted.data_ptr(),
        first.data_ptr(), n, generations, upw, resident, hip._stream(stream)))
    return first


lib.lifeapi_tune_step_contains_pair.argtypes = [_vp, _vp, _vp, _vp, _vp, _sz, _u32, _int, _int, _vp]
lib.lifeapi_tune_step_contains_pair.restype = _int


def step_contains_pair(states, wanted, unwanted, generations, cap_lo, cap_hi, final=None, stream=None):
    """the shipped fused pair with each grid capped (blocks per CU, 0 = none)"""
    n = hip._universes(states)
    first = torch.empty(n, dtype=torch.int32, device=states.device)
    hip._check(lib.lifeapi_tune_step_contains_pair(
        states.data_ptr(), None if final is None else final.data_ptr(), wanted.data_ptr(), unwanted.data_ptr(),
        first.data_ptr(), n, generations, cap_lo, cap_hi, hip._stream(stream)))
    return first


lib.lifeapi_tune_capped_occupancy.argtypes = [_int, _int, ctypes.POINTER(_int)]
lib.lifeapi_tune_capped_occupancy.restype = _int


def capped_occupancy(which: int, want: int) -> int:
    """resident blocks per CU (occupancy API) of a shipped kernel under the
    cap the product sets for `want`: which 0 = the streaming k_step, 1..6 =
    k_stable<which-1>, 7 = k_stable_vulnerable"""
    got = _int(0)
    hip._check(lib.lifeapi_tune_capped_occupancy(which, want, ctypes.byref(got)))
    return got.value


lib.lifeapi_tune_order_probe.argtypes = [_vp, _vp, ctypes.c_uint64]
lib.lifeapi_tune_order_probe.restype = _int


def order_probe(d_in: int, d_out: int, nbytes: int) -> bool:
    """the product's launch-order book: would a launch reading d_in and
    writing d_out run in reverse?  (records d_out as such a launch does)"""
    return bool(lib.lifeapi_tune_order_probe(d_in, d_out, nbytes))


lib.lifeapi_tune_order_note.argtypes = [_vp, ctypes.c_uint64]
lib.lifeapi_tune_order_note.restype = None


def order_note(d_out: int, nbytes: int) -> None:
    """record d_out (nbytes) in the product's order book as written forward"""
    lib.lifeapi_tune_order_note(d_out, nbytes)


lib.lifeapi_tune_fill16.argtypes = [_vp, _sz, ctypes.c_uint64, ctypes.c_uint64, _int, _int, _vp]
lib.lifeapi_tune_fill16.restype = _int


def fill16(out: torch.Tensor, seed: int, first_universe: int = 0, mode: int = 0, blocks_per_cu: int = 0,
           stream=None) -> torch.Tensor:
    """the seeded fill with 16-byte stores into out (n, 64)"""
    hip._check(lib.lifeapi_tune_fill16(out.data_ptr(), hip._universes(out), seed, first_universe, mode,
                                       blocks_per_cu, hip._stream(stream)))
    return out


lib.lifeapi_tune_step_split_wpb.argtypes = [_vp, _vp, _sz, _u32, _int, _vp]
lib.lifeapi_tune_step_split_wpb.restype = _int


def step_split_wpb(states: torch.Tensor, out: torch.Tensor, generations: int, wpb: int, stream=None):
    """the shipped gens > 2 kernel with wpb waves per block (1, 2, 4 = shipped)"""
    n = hip._universes(states)
    hip._check(lib.lifeapi_tune_step_split_wpb(states.data_ptr(), out.data_ptr(), n, generations, wpb,
                                               hip._stream(stream)))
    return out


lib.lifeapi_tune_cone.argtypes = [_int, _vp, _vp, _vp, _vp, _sz, _u32, _int, _int, _vp]
lib.lifeapi_tune_cone.restype = _int


def cone(states, wanted, unwanted, generations, upw, rmax, first=True, out=None, stream=None):
    """the light-cone kernel (k_cone) with `upw` universes per wave and `rmax`
    register sets per pass: first generations (int32, first=True, gens <= 2)
    or Contains (uint8)"""
    n = hip._universes(states)
    if out is None:
        out = torch.empty(n, dtype=torch.int32 if first else torch.uint8, device=states.device)
    hip._check(lib.lifeapi_tune_cone(1 if first else 0, states.data_ptr(), wanted.data_ptr(), unwanted.data_ptr(),
                                     out.data_ptr(), n, generations, upw, rmax, hip._stream(stream)))
    return out


lib.lifeapi_tune_weld_u.argtypes = [_vp, _sz, _int, _int, _int, _vp]
lib.lifeapi_tune_weld_u.restype = _int


def weld_u(welds, u: int, resident: int = 0, chunk: bool = False, stream=None):
    """k_weld one generation in place with u welds per wave (tune_stencils.hip)"""
    hip._check(lib.lifeapi_tune_weld_u(welds.data_ptr(), welds.shape[0], u, resident, 1 if chunk else 0,
                                       hip._stream(stream)))
    return welds


lib.lifeapi_tune_search_iter.argtypes = [_vp, _vp, _vp, _vp, _sz, _u32, _int, _int, _vp]
lib.lifeapi_tune_search_iter.restype = _int


def search_iter(states, wanted, unwanted, generations, cone_cap, split_cap, stream=None):
    """step.hip's gens > 2 launch sequence without final states, caps given"""
    n = hip._universes(states)
    first = torch.empty(n, dtype=torch.int32, device=states.device)
    hip._check(lib.lifeapi_tune_search_iter(states.data_ptr(), wanted.data_ptr(), unwanted.data_ptr(), first.data_ptr(),
                                            n, generations, cone_cap, split_cap, hip._stream(stream)))
    return first


lib.lifeapi_tune_line_read.argtypes = [_vp, _vp, _sz, _int, _vp]
lib.lifeapi_tune_line_read.restype = _int


def line_read(states, line, out=None, stream=None):
    """one 128-byte line of each universe read, one uint32 written per universe"""
    n = hip._universes(states)
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=states.device)
    hip._check(lib.lifeapi_tune_line_read(states.data_ptr(), out.data_ptr(), n, line, hip._stream(stream)))
    return out


lib.lifeapi_tune_stable_rep.argtypes = [_vp, _vp, _sz, _int, _u32, _vp]
lib.lifeapi_tune_stable_rep.restype = _int


def stable_rep(planes: torch.Tensor, which: int, reps: int, stream=None):
    """the LifeStable pass `which` repeated `reps` times per LifeStable in
    registers (k_stable_rep: a VALU probe; the planes get one result)"""
    n = planes.numel() // (10 * 64)
    flags = torch.empty(n, dtype=torch.uint8, device=planes.device)
    hip._check(lib.lifeapi_tune_stable_rep(planes.data_ptr(), flags.data_ptr(), n, which, reps, hip._stream(stream)))
    return flags


lib.lifeapi_tune_rows_probe.argtypes = [_vp, _vp, _vp, _vp, _sz, _u32, _u32, _int, _vp]
lib.lifeapi_tune_rows_probe.restype = _int


def rows_probe(states, wanted, unwanted, generations, y0, sleep=0, out=None, stream=None):
    """the row-window filter pass, window given, s_sleep(sleep) after each
    next-pass fetch (tune_cone.hip k_rows_probe)"""
    n = hip._universes(states)
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=states.device)
    hip._check(lib.lifeapi_tune_rows_probe(states.data_ptr(), wanted.data_ptr(), unwanted.data_ptr(), out.data_ptr(),
                                           n, generations, y0, sleep, hip._stream(stream)))
    return out


lib.lifeapi_tune_filter_iter.argtypes = [_vp, _vp, _vp, _vp, _sz, _u32, _int, _vp]
lib.lifeapi_tune_filter_iter.restype = _int
# tools/filter_iter_probe.py's forms of the round-6 A/B: blocks per CU | PF | Hi / Lo alone
FILTER_ITER_FORMS = {"pair32": 32, "all32_pf": 32 | 0x900, "all14_pf": 14 | 0x900,
                     "all16_pf_win": 16 | 0x1900, "all32_pf_win": 32 | 0x1900, "all8_pf_win": 8 | 0x1900,
                     "all16_win": 16 | 0x1800}


def filter_iter(states, wanted, unwanted, generations, variant, stream=None):
    """the split pair without final states, round 6 variants (tune_step.hip)"""
    n = hip._universes(states)
    first = torch.empty(n, dtype=torch.int32, device=states.device)
    hip._check(lib.lifeapi_tune_filter_iter(states.data_ptr(), wanted.data_ptr(), unwanted.data_ptr(),
                                            first.data_ptr(), n, generations, variant, hip._stream(stream)))
    return first
