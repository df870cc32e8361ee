"""Host code under ASan + UBSan: the C++ facade's CPU members
and the C oracle, compiled with -fsanitize=address,undefined and
-fno-sanitize-recover, checked against each other (tests/cpp/host_sanitize_test.cpp).
CPU only; the GPU-side host library is exercised under the same sanitizers by
tests/test_cpp_facade.py::test_step_batch_cpp_asan."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]


def test_host_code_under_asan_ubsan(tmp_path):
    obj = tmp_path / "oracle.o"
    exe = tmp_path / "host_sanitize_test"
    subprocess.run(["gcc", "-std=c11", "-c", *SAN, "-Wall", "-Wextra",
                    os.path.join(ROOT, "oracle", "lifeapi_oracle.c"), "-o", str(obj)], check=True)
    subprocess.run(["g++", "-std=c++20", *SAN, "-Wall", "-Wextra", "-I" + os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "host_sanitize_test.cpp"), str(obj), "-pthread",
                    "-o", str(exe)], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    print(r.stdout, r.stderr[-4000:])
    assert r.returncode == 0, r.stderr[-4000:]
    assert "failures" in r.stdout and " 0 failures" in r.stdout
