"""ctypes binding of the C ABI in include/lifeapi_hip.h.

Import order matters: torch is imported first so that its bundled HIP runtime
(SONAME ``libamdhip64.so.7``) is the one ``liblifeapi_hip.so`` binds to --
device pointers and streams handed over from torch then belong to the same
runtime.  There is no fallback of any kind: a missing or unloadable library
raises ImportError, and every failed call raises :class:`LifeApiError`.

Universes are int64 tensors of shape (n, 64) holding the reference's
``LifeState::state`` words bit-for-bit (LifeAPI.hpp:39-40).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch  # noqa: F401  (must precede loading the HIP library)

from .layout import N

# (LIFEAPI_HIP_LIB: another build of the same library, for A/B probes under tools/)
LIB_PATH = os.environ.get("LIFEAPI_HIP_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                             "liblifeapi_hip.so")

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"{LIB_PATH} is missing: build it with "
        "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc --offload-arch=gfx950)")
lib = ctypes.CDLL(LIB_PATH)

class LifeApiError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"lifeapi error {code}: {msg}")
        self.code = code


_vp, _sz, _u32, _u64, _int = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
_SIGS = {
    "lifeapi_abi_version": ([], _int),
    "lifeapi_last_error": ([], ctypes.c_char_p),
    "lifeapi_device_count": ([], _int),
    "lifeapi_step_kernel_name": ([_u32], ctypes.c_char_p),
    "lifeapi_step_kernel_name_n": ([_u32, _sz], ctypes.c_char_p),
    "lifeapi_step_batch_dev": ([_vp, _vp, _sz, _u32, _vp], _int),
    "lifeapi_pop_batch_dev": ([_vp, _vp, _sz, _vp], _int),
    "lifeapi_hash_batch_dev": ([_vp, _vp, _sz, _vp], _int),
    "lifeapi_contains_batch_dev": ([_vp, _vp, _vp, _vp, _sz, _vp], _int),
    "lifeapi_step_contains_batch_dev": ([_vp, _vp, _vp, _vp, _vp, _sz, _u32, _vp], _int),
    "lifeapi_fill_random_dev": ([_vp, _sz, _u64, _u64, _int, _vp], _int),
    "lifeapi_weld_step_batch_dev": ([_vp, _sz, _u32, _vp], _int),
    "lifeapi_stable_pass_batch_dev": ([_vp, _vp, _sz, _int, _u32, _vp], _int),
    "lifeapi_neighbour_count_batch_dev": ([_vp, _vp, _sz, _vp], _int),
    "lifeapi_interaction_counts_batch_dev": ([_vp, _vp, _sz, _int, _vp], _int),
    "lifeapi_refined_step_batch_dev": ([_vp, _vp, _sz, _vp], _int),
    "lifeapi_step_batch": ([_vp, _vp, _sz, _u32, _int], _int),
    "lifeapi_host_register": ([_vp, _sz], _int),
    "lifeapi_step_contains_batch": ([_vp, _vp, _vp, _vp, _vp, _sz, _u32, _int], _int),
    "lifeapi_host_unregister": ([_vp], _int),
    "lifeapi_pop_batch": ([_vp, _vp, _sz, _int], _int),
    "lifeapi_weld_step_batch": ([_vp, _sz, _u32, _int], _int),
    "lifeapi_stable_pass_batch": ([_vp, _vp, _sz, _int, _u32, _int], _int),
    "lifeapi_neighbour_count_batch": ([_vp, _vp, _sz, _int], _int),
    "lifeapi_interaction_counts_batch": ([_vp, _vp, _sz, _int, _int], _int),
    "lifeapi_refined_step_batch": ([_vp, _vp, _sz, _int], _int),
    "lifeapi_contains_batch": ([_vp, _vp, _vp, _vp, _sz, _int], _int),
    "lifeapi_stable_vulnerable_batch_dev": ([_vp, _vp, _sz, _vp], _int),
    "lifeapi_stable_vulnerable_batch": ([_vp, _vp, _sz, _int], _int),
    "lifeapi_rle_lengths_batch_dev": ([_vp, _vp, _sz, _vp], _int),
    "lifeapi_rle_write_batch_dev": ([_vp, _vp, _vp, _sz, _vp], _int),
    "lifeapi_parse_rle_batch_dev": ([_vp, _vp, _sz, _vp, _vp, _vp], _int),
    "lifeapi_rle_batch": ([_vp, _sz, _vp, _sz, _vp, _int], _int),
    "lifeapi_parse_rle_batch": ([_vp, _vp, _sz, _vp, _vp, _int], _int),
}
for _name, (_args, _res) in _SIGS.items():
    _f = getattr(lib, _name)
    _f.argtypes = _args
    _f.restype = _res

EXPORTS = tuple(_SIGS)


def _check(rc: int) -> None:
    if rc != 0:
        raise LifeApiError(rc, lib.lifeapi_last_error().decode(errors="replace"))


def abi_version() -> int:
    return lib.lifeapi_abi_version()


def device_count() -> int:
    return lib.lifeapi_device_count()


def step_kernel_name(generations: int = 1, n: int | None = None) -> str:
    """The shipped kernel configuration a step of `generations` runs on a
    batch of `n` universes (None: the name for batches of at most 4M)."""
    if n is None:
        return lib.lifeapi_step_kernel_name(generations).decode()
    return lib.lifeapi_step_kernel_name_n(generations, n).decode()


def _stream(stream) -> int:
    if stream is None:
        stream = torch.cuda.current_stream()
    return stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream)


def _universes(t: torch.Tensor, name: str = "states") -> int:
    if not t.is_cuda:
        raise ValueError(f"{name} must be a device tensor")
    if t.dtype not in (torch.int64, torch.uint64) or not t.is_contiguous() or t.numel() % N:
        raise ValueError(f"{name} must be a contiguous int64 tensor of shape (n, 64)")
    return t.numel() // N


def empty_universes(n: int, device=None) -> torch.Tensor:
    return torch.empty((n, N), dtype=torch.int64, device=device or "cuda")


def step(states: torch.Tensor, out: torch.Tensor | None = None, generations: int = 1,
         stream=None) -> torch.Tensor:
    """Batched ``Stepped(generations)`` (LifeAPI.hpp:882-886); ``out`` may be ``states``."""
    n = _universes(states)
    if out is None:
        out = torch.empty_like(states)
    if _universes(out, "out") != n:
        raise ValueError("out has a different number of universes")
    _check(lib.lifeapi_step_batch_dev(states.data_ptr(), out.data_ptr(), n, generations, _stream(stream)))
    return out


def pop(states: torch.Tensor, stream=None) -> torch.Tensor:
    """Per-universe ``GetPop()`` (LifeAPI.hpp:290-298) as int32."""
    n = _universes(states)
    out = torch.empty(n, dtype=torch.int32, device=states.device)
    _check(lib.lifeapi_pop_batch_dev(states.data_ptr(), out.data_ptr(), n, _stream(stream)))
    return out


def hashes(states: torch.Tensor, stream=None) -> torch.Tensor:
    """Per-universe build-defined 64-bit hash (bit pattern in an int64 tensor)."""
    n = _universes(states)
    out = torch.empty(n, dtype=torch.int64, device=states.device)
    _check(lib.lifeapi_hash_batch_dev(states.data_ptr(), out.data_ptr(), n, _stream(stream)))
    return out


def contains(states: torch.Tensor, wanted: torch.Tensor, unwanted: torch.Tensor,
             stream=None) -> torch.Tensor:
    """Per-universe ``Contains(LifeTarget{wanted, unwanted})`` (LifeTarget.hpp:44-51)."""
    n = _universes(states)
    _universes(wanted, "wanted"), _universes(unwanted, "unwanted")
    out = torch.empty(n, dtype=torch.uint8, device=states.device)
    _check(lib.lifeapi_contains_batch_dev(states.data_ptr(), wanted.data_ptr(), unwanted.data_ptr(),
                                          out.data_ptr(), n, _stream(stream)))
    return out


def step_contains(states: torch.Tensor, wanted: torch.Tensor, unwanted: torch.Tensor,
                  generations: int, final: torch.Tensor | None = None, stream=None):
    """First generation (1..gens, 0 = never) at which each universe contains the target."""
    n = _universes(states)
    first = torch.empty(n, dtype=torch.int32, device=states.device)
    fptr = 0 if final is None else final.data_ptr()
    if final is not None and _universes(final, "final") != n:
        raise ValueError("final has a different number of universes")
    _check(lib.lifeapi_step_contains_batch_dev(states.data_ptr(), fptr or None, wanted.data_ptr(),
                                               unwanted.data_ptr(), first.data_ptr(), n,
                                               generations, _stream(stream)))
    return first, final


def fill_random(n: int, seed: int, first_universe: int = 0, mode: int = 0,
                out: torch.Tensor | None = None, device=None, stream=None) -> torch.Tensor:
    """Seeded synthetic universes (see lifeapi_fill_random_dev)."""
    if out is None:
        out = empty_universes(n, device)
    if _universes(out, "out") != n:
        raise ValueError("out has a different number of universes")
    _check(lib.lifeapi_fill_random_dev(out.data_ptr(), n, seed & (2**64 - 1), first_universe,
                                       mode, _stream(stream)))
    return out


def _host_u64(a: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.uint64)
    if a.size % N:
        raise ValueError("host batch must hold whole universes (multiples of 64 words)")
    return a


def step_host(states: np.ndarray, generations: int = 1, device: int = 0,
              out: np.ndarray | None = None) -> np.ndarray:
    """Host-pointer ``lifeapi_step_batch`` (synchronous, PCIe-staged)."""
    src = _host_u64(states)
    dst = np.empty_like(src) if out is None else out
    _check(lib.lifeapi_step_batch(src.ctypes.data, dst.ctypes.data, src.size // N, generations, device))
    return dst


def step_contains_host(states: np.ndarray, wanted: np.ndarray, unwanted: np.ndarray, generations: int,
                       final: np.ndarray | None = None, device: int = 0) -> np.ndarray:
    """Host-pointer ``lifeapi_step_contains_batch``: first generation (1..gens,
    0 = never) containing the target; ``final`` (may be ``states``) gets
    Stepped(gens)."""
    src = _host_u64(states)
    w, u = _host_u64(wanted), _host_u64(unwanted)
    first = np.empty(src.size // N, dtype=np.uint32)
    fptr = None if final is None else final.ctypes.data
    _check(lib.lifeapi_step_contains_batch(src.ctypes.data, fptr, w.ctypes.data, u.ctypes.data,
                                           first.ctypes.data, src.size // N, generations, device))
    return first


class host_pinned:
    """Context manager: page-lock numpy arrays (lifeapi_host_register) for
    the host-pointer calls inside the block."""

    def __init__(self, *arrays: np.ndarray):
        self.arrays = arrays

    def __enter__(self):
        done = []
        try:
            for a in self.arrays:
                _check(lib.lifeapi_host_register(a.ctypes.data, a.nbytes))
                done.append(a)
        except Exception:
            for a in done:
                lib.lifeapi_host_unregister(a.ctypes.data)
            raise
        return self

    def __exit__(self, *exc):
        for a in self.arrays:
            _check(lib.lifeapi_host_unregister(a.ctypes.data))
        return False


def pop_host(states: np.ndarray, device: int = 0) -> np.ndarray:
    src = _host_u64(states)
    out = np.empty(src.size // N, dtype=np.uint32)
    _check(lib.lifeapi_pop_batch(src.ctypes.data, out.ctypes.data, src.size // N, device))
    return out


def loaded_hip_runtimes() -> list[str]:
    """Paths of every libamdhip64 mapped into this process (must be exactly one)."""
    paths = set()
    with open("/proc/self/maps") as f:
        for line in f:
            p = line.split()[-1] if len(line.split()) >= 6 else ""
            if "libamdhip64" in p:
                paths.add(p)
    return sorted(paths)


def refined_step(planes: torch.Tensor, out: torch.Tensor | None = None, stream=None) -> torch.Tensor:
    """Config-5 ternary step: (n, 11*64) int64 planes -> (n, 3*64) planes
    (see lifeapi_refined_step_batch_dev)."""
    if not planes.is_cuda or planes.dtype not in (torch.int64, torch.uint64) or \
            not planes.is_contiguous() or planes.numel() % (11 * N):
        raise ValueError("planes must be a contiguous int64 device tensor of shape (n, 11*64)")
    n = planes.numel() // (11 * N)
    if out is None:
        out = torch.empty((n, 3 * N), dtype=torch.int64, device=planes.device)
    _check(lib.lifeapi_refined_step_batch_dev(planes.data_ptr(), out.data_ptr(), n, _stream(stream)))
    return out


def weld_step(welds: torch.Tensor, generations: int = 1, stream=None) -> torch.Tensor:
    """LifeWeld::Step()^generations in place on (n, 4*64) {state, frozen2,
    frozen1, frozen0} planes (LifeWeld.hpp:169-186)."""
    if not welds.is_cuda or welds.dtype not in (torch.int64, torch.uint64) or \
            not welds.is_contiguous() or welds.numel() % (4 * N):
        raise ValueError("welds must be a contiguous int64 device tensor of shape (n, 4*64)")
    _check(lib.lifeapi_weld_step_batch_dev(welds.data_ptr(), welds.numel() // (4 * N), generations,
                                           _stream(stream)))
    return welds


STABLE_PASSES = ("sync", "options", "signal", "step", "propagate", "stabilise")


def stable_pass(planes: torch.Tensor, which: str | int, max_iters: int = 0,
                stream=None) -> torch.Tensor:
    """LifeStable pass in place on (n, 10*64) planes; returns uint8 flags
    (bit0 consistent, bit1 changed, bit2 stopped by max_iters)."""
    w = STABLE_PASSES.index(which) if isinstance(which, str) else int(which)
    if not planes.is_cuda or planes.dtype not in (torch.int64, torch.uint64) or \
            not planes.is_contiguous() or planes.numel() % (10 * N):
        raise ValueError("planes must be a contiguous int64 device tensor of shape (n, 10*64)")
    n = planes.numel() // (10 * N)
    flags = torch.empty(n, dtype=torch.uint8, device=planes.device)
    _check(lib.lifeapi_stable_pass_batch_dev(planes.data_ptr(), flags.data_ptr(), n, w, max_iters,
                                             _stream(stream)))
    return flags


def stable_vulnerable(planes: torch.Tensor, stream=None) -> torch.Tensor:
    """LifeStable::Vulnerable() (LifeStable.hpp:366-412) of (n, 10*64) planes -> (n, 64)."""
    if not planes.is_cuda or planes.dtype not in (torch.int64, torch.uint64) or \
            not planes.is_contiguous() or planes.numel() % (10 * N):
        raise ValueError("planes must be a contiguous int64 device tensor of shape (n, 10*64)")
    n = planes.numel() // (10 * N)
    out = torch.empty((n, N), dtype=torch.int64, device=planes.device)
    _check(lib.lifeapi_stable_vulnerable_batch_dev(planes.data_ptr(), out.data_ptr(), n, _stream(stream)))
    return out


def neighbour_count(states: torch.Tensor, stream=None) -> torch.Tensor:
    """NeighbourCount planes (NeighbourCount.hpp:40-70): (n, 4, 64) = bit3..bit0."""
    n = _universes(states)
    out = torch.empty((n, 4, N), dtype=torch.int64, device=states.device)
    _check(lib.lifeapi_neighbour_count_batch_dev(states.data_ptr(), out.data_ptr(), n, _stream(stream)))
    return out


def interaction_counts(states: torch.Tensor, with_next: bool = False, stream=None) -> torch.Tensor:
    """InteractionCounts[AndNext] (LifeAPI.hpp:956-1040): (n, 3|4, 64) planes
    out1, out2, outMore[, next]."""
    n = _universes(states)
    out = torch.empty((n, 4 if with_next else 3, N), dtype=torch.int64, device=states.device)
    _check(lib.lifeapi_interaction_counts_batch_dev(states.data_ptr(), out.data_ptr(), n,
                                                    1 if with_next else 0, _stream(stream)))
    return out


def rle(states: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """``LifeState::RLE()`` (Parsing.hpp:8-63,200-204) of every universe on
    the device, on torch's current stream: (text uint8 tensor, offsets int64
    tensor of n+1; pattern u = text[offsets[u]:offsets[u+1]])."""
    n = _universes(states)
    s = _stream(None)
    lens = torch.empty(n, dtype=torch.int32, device=states.device)
    _check(lib.lifeapi_rle_lengths_batch_dev(states.data_ptr(), lens.data_ptr(), n, s))
    offs = torch.zeros(n + 1, dtype=torch.int64, device=states.device)
    if n:
        torch.cumsum(lens, 0, out=offs[1:])
    total = int(offs[-1].item()) if n else 0
    text = torch.empty(max(total, 1), dtype=torch.uint8, device=states.device)
    _check(lib.lifeapi_rle_write_batch_dev(states.data_ptr(), offs.data_ptr(), text.data_ptr(), n, s))
    return text[:total], offs


def parse_rle(text: torch.Tensor, offsets: torch.Tensor, stream=None) -> tuple[torch.Tensor, torch.Tensor]:
    """``LifeState::Parse`` (Parsing.hpp:143-198) of every pattern of a device
    text blob: (states (n, 64) int64, status uint8; bit 0 = cells off the
    board dropped, bit 1 = stopped at a "$" count of 129)."""
    if not (text.is_cuda and offsets.is_cuda) or text.dtype != torch.uint8 or offsets.dtype != torch.int64:
        raise ValueError("text must be a device uint8 tensor, offsets a device int64 tensor")
    n = offsets.numel() - 1
    out = torch.empty((max(n, 0), N), dtype=torch.int64, device=text.device)
    status = torch.empty(max(n, 0), dtype=torch.uint8, device=text.device)
    buf = text if text.numel() else torch.zeros(1, dtype=torch.uint8, device=text.device)
    _check(lib.lifeapi_parse_rle_batch_dev(buf.data_ptr(), offsets.data_ptr(), max(n, 0), out.data_ptr(),
                                           status.data_ptr(), _stream(stream)))
    return out, status


def rle_host(states: np.ndarray, device: int = 0) -> list[str]:
    """Host-pointer ``lifeapi_rle_batch``: size query, then the write."""
    src = _host_u64(states)
    n = src.size // N
    offs = np.zeros(n + 1, dtype=np.uint64)
    _check(lib.lifeapi_rle_batch(src.ctypes.data, n, None, 0, offs.ctypes.data, device))
    text = ctypes.create_string_buffer(max(int(offs[-1]), 1))
    _check(lib.lifeapi_rle_batch(src.ctypes.data, n, text, int(offs[-1]), offs.ctypes.data, device))
    raw = text.raw
    return [raw[int(offs[u]):int(offs[u + 1])].decode() for u in range(n)]


def parse_rle_host(patterns: list[str | bytes], device: int = 0) -> tuple[np.ndarray, np.ndarray]:
    """Host-pointer ``lifeapi_parse_rle_batch``."""
    bs = [p.encode() if isinstance(p, str) else bytes(p) for p in patterns]
    offs = np.zeros(len(bs) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(b) for b in bs])
    blob = b"".join(bs) or b"\0"
    out = np.zeros((len(bs), N), dtype=np.uint64)
    status = np.zeros(len(bs), dtype=np.uint8)
    _check(lib.lifeapi_parse_rle_batch(blob, offs.ctypes.data, len(bs), out.ctypes.data, status.ctypes.data,
                                       device))
    return out, status
