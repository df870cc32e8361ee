"""CPU: the C-ABI library loads, exports exactly what include/lifeapi_hip.h
declares, and validates arguments before touching any device (no compute
calls here -- there is no GPU in the CPU suite)."""
import ctypes
import os
import re
import subprocess

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "lifeapi_hip.h")


def declared():
    src = open(HDR).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(lifeapi_\w+)\s*\(", src, re.M)))


def test_header_declares_entry_points():
    names = declared()
    for must in ("lifeapi_step_batch_dev", "lifeapi_step_batch", "lifeapi_last_error",
                 "lifeapi_device_count", "lifeapi_pop_batch_dev", "lifeapi_contains_batch_dev",
                 "lifeapi_fill_random_dev", "lifeapi_hash_batch_dev"):
        assert must in names


def test_library_exports_every_declared_symbol():
    import lifeapi_amd.hip as hip
    lib = ctypes.CDLL(hip.LIB_PATH)
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing
    # and the python binding covers the whole ABI
    assert sorted(hip.EXPORTS) == declared()
    nm = subprocess.run(["nm", "-D", "--defined-only", hip.LIB_PATH], capture_output=True,
                        text=True, check=True).stdout
    exported = sorted(set(re.findall(r"\bT (lifeapi_\w+)", nm)))
    assert exported == declared()


def test_single_hip_runtime_after_torch():
    import lifeapi_amd.hip as hip
    rts = hip.loaded_hip_runtimes()
    assert len(rts) == 1, rts
    assert "torch" in rts[0]


def test_gfx950_code_object_present():
    """The fat binary carries exactly one device code object, for gfx950."""
    import lifeapi_amd.hip as hip
    data = open(hip.LIB_PATH, "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx\w+)", data))
    assert targets == {b"gfx950"}, targets


def test_abi_version_and_shipped_kernels():
    import lifeapi_amd.hip as hip
    assert hip.abi_version() == 2
    assert hip.step_kernel_name(1).startswith("k_step<dpp")
    assert hip.step_kernel_name(3).startswith("k_step_split<8-way")
    assert "nt" in hip.step_kernel_name(31) and "nt" not in hip.step_kernel_name(32).split(",")[2]
    # the launch above 4M universes is a different shape, and named so
    assert hip.step_kernel_name(1, 1 << 22) == hip.step_kernel_name(1)
    assert "XCD" in hip.step_kernel_name(1, (1 << 22) + 1) and "alternating" not in hip.step_kernel_name(1, 1 << 24)
    assert hip.step_kernel_name(3, 1 << 24) == hip.step_kernel_name(3)


def test_no_tuning_knobs_in_product_library():
    """The product exports only the drop-in entry points: the measured
    alternatives live in the tuning build (tools/tune/liblifeapi_tune.so)."""
    import lifeapi_amd.hip as hip
    for name in ("lifeapi_step_batch_dev_cfg", "lifeapi_default_cfg", "lifeapi_refined_step_batch_dev_cfg",
                 "lifeapi_tune_step_batch_dev_cfg"):
        assert not hasattr(hip.lib, name), name


def test_argument_validation_without_device():
    import lifeapi_amd.hip as hip
    L = hip.lib
    # null pointers
    assert L.lifeapi_step_batch_dev(None, None, 4, 1, None) == -1
    assert b"null" in L.lifeapi_last_error()
    # misaligned
    assert L.lifeapi_step_batch_dev(8 * 1000 + 4, 8 * 5000, 4, 1, None) == -1
    # overlapping but not identical batches
    assert L.lifeapi_step_batch_dev(4096, 4096 + 512, 4, 1, None) == -1
    assert b"overlap" in L.lifeapi_last_error()
    # n == 0 is a no-op success even with null pointers
    assert L.lifeapi_step_batch_dev(None, None, 0, 1, None) == 0
    assert L.lifeapi_fill_random_dev(4096, 1, 0, 0, 5, None) == -1


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-device error path")
def test_host_api_reports_no_device():
    import numpy as np

    import lifeapi_amd.hip as hip
    assert hip.device_count() == 0
    with pytest.raises(hip.LifeApiError) as e:
        hip.step_host(np.zeros((2, 64), np.uint64), 1)
    assert e.value.code == -2
