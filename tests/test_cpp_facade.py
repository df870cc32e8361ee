"""Runs the C++ facade tests (tests/cpp/*.cpp, built by __graft_entry__.build())."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_facade_compiles_without_gpu():
    """The facade header is self-contained C++20 (CPU: syntax + layout asserts)."""
    src = os.path.join(ROOT, "tests", "cpp", "step_batch_test.cpp")
    subprocess.run(["g++", "-std=c++20", "-fsyntax-only", "-Wall", "-Wextra", "-Werror",
                    "-I" + os.path.join(ROOT, "include"), src], check=True)


def test_facade_members_equal_reference_cpu():
    """The standalone facade's single-state members (Step, StepAlt, ZOI,
    GetBoundary, Move(d), Contains / AreDisjoint with and without offsets,
    LifeTarget(state), LifeTarget::Moved) against the reference's own, on the
    CPU (tests/cpp/facade_cpu_test.cpp, built against the reference headers by
    oracle/Makefile, target ref)."""
    exe = os.path.join(ROOT, "oracle", "_ref", "facade_cpu_test")
    if not os.path.exists(exe):
        pytest.skip("oracle/_ref/facade_cpu_test needs the reference headers at build time")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    print(r.stdout, r.stderr[-4000:])
    assert r.returncode == 0, r.stderr[-4000:]


@pytest.mark.gpu
def test_step_batch_cpp():
    exe = os.path.join(ROOT, "build", "step_batch_test")
    if not os.path.exists(exe):
        import __graft_entry__ as g
        g.build_cpp_tests()
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stderr[-4000:]


@pytest.mark.gpu
def test_step_batch_cpp_asan():
    """The same facade tests with the library's host code (every csrc/*.hip,
    host side only) and the test under ASan + UBSan."""
    exe = os.path.join(ROOT, "build", "step_batch_test_asan")
    if not os.path.exists(exe):
        pytest.skip("build/step_batch_test_asan not built (__graft_entry__.build())")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:protect_shadow_gap=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    print(r.stdout, r.stderr[-4000:])
    assert r.returncode == 0, r.stderr[-4000:]


@pytest.mark.gpu
def test_reference_types_dropin():
    """The batch header on the REFERENCE's own ::LifeState / ::LifeTarget /
    ::LifeWeld / ::NeighbourCount / ::LifeStable (tests/cpp/ref_dropin_test.cpp,
    compiled against the reference headers in the build container by
    oracle/Makefile, target ref) gives
    exactly what their member functions give."""
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_dropin_test")  # oracle/Makefile, target ref
    if not os.path.exists(exe):
        pytest.skip("oracle/_ref/ref_dropin_test needs the reference headers at build time")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    print(r.stdout, r.stderr[-4000:])
    assert r.returncode == 0, r.stderr[-4000:]
