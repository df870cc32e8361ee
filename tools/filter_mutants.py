"""Build the filter mutants tools/gpu_r06m.sh runs the GPU tests on: copies of
lifeapi_amd/csrc with one deliberate fault each, linked with the in-tree
objects but step.o into build/abs/liblifeapi_hip_m?.so.  Every mutant must
fail the filter tests (profiles/r06/mutants/)."""
import glob
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"

MUTANTS = {
    # the window test ORs 7 of the 8 difference registers
    "A": ("cone_split.hpp", "lut3<kOr3>(d[3], d[4], d[5]), d[6] | d[7]);",
          "lut3<kOr3>(d[3], d[4], d[5]), d[6]);"),
    # the whole-board LDS-DMA chunk read takes the neighbouring universe's word
    "B": ("cone_split.hpp", "e[u] = cut(img[u * kWave + lane]);",
          "e[u] = cut(img[(u ^ 1) * kWave + lane]);"),
    # the packed row window starts one row late
    "C": ("step_kernels.hpp", "  y0 = (cy0 - gens) & 63u;", "  y0 = (cy0 - gens + 1u) & 63u;"),
    # the column light cone one column narrower on each side
    "D": ("step_kernels.hpp",
          "K = gens >= (uint32_t)kWave / 2 ? (uint32_t)kWave : w + 2 * gens;\n  xs = (x0 - gens) & (kWave - 1);",
          "K = gens >= (uint32_t)kWave / 2 ? (uint32_t)kWave : w + 2 * gens - 2;\n  xs = (x0 - gens + 1) & (kWave - 1);"),
}


def build(name, tmp):
    path, old, new = MUTANTS[name]
    src = os.path.join(tmp, name)
    shutil.copytree(os.path.join(ROOT, "lifeapi_amd", "csrc"), src)
    f = os.path.join(src, path)
    text = open(f).read()
    assert text.count(old) == 1, (name, old)
    open(f, "w").write(text.replace(old, new))
    obj = os.path.join(src, "step_m.o")
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                    "-I" + os.path.join(ROOT, "include"), "-c", os.path.join(src, "step.hip"), "-o", obj],
                   check=True)
    others = [o for o in sorted(glob.glob(os.path.join(ROOT, "build", "obj", "*.o")))
              if os.path.basename(o) != "step.o"]
    out = os.path.join(ROOT, "build", "abs", f"liblifeapi_hip_m{name}.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out, obj, *others], check=True)
    print(out)


if __name__ == "__main__":
    with tempfile.TemporaryDirectory() as tmp:
        for m in sys.argv[1:] or sorted(MUTANTS):
            build(m, tmp)
