"""Build libscgpu.so (HIP kernels + C ABI) in-tree for gfx950.

    python gym-supplychain_amd/build_native.py [--debug]

Output: gym-supplychain_amd/gym_supplychain_amd/libscgpu.so (git-ignored, but it
travels to the GPU box with the gpurun snapshot). Cross-compiles without a GPU.
"""
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "gym_supplychain_amd", "libscgpu.so")
SOURCES = ["scg_common.hip", "scg_beergame.hip", "scg_supplychain.hip"]
ARCH = "gfx950"


def hipcc():
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found")


def build_binding(verbose=True):
    """_scgpu_fast: METH_FASTCALL CPython binding of the per-step entry points."""
    import sysconfig
    src = os.path.join(CSRC, "scg_pybind.c")
    out = os.path.join(HERE, "gym_supplychain_amd", "_scgpu_fast" + sysconfig.get_config_var("EXT_SUFFIX"))
    deps = [src, OUT, os.path.join(REPO, "include", "scgpu.h")]
    if os.path.exists(out) and all(os.path.getmtime(out) >= os.path.getmtime(d) for d in deps):
        return out
    cmd = ["gcc", "-O2", "-shared", "-fPIC", "-Wall", "-I", sysconfig.get_paths()["include"],
           "-I", os.path.join(REPO, "include"), src, "-L", os.path.dirname(OUT), "-lscgpu",
           "-Wl,-rpath,$ORIGIN", "-o", out + ".tmp"]
    if verbose:
        print("[build_native]", " ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


def build(debug=False, verbose=True):
    lib = build_library(debug, verbose)
    build_binding(verbose)
    return lib


# hipcc flags of libscgpu.so (tools/exp_build.py builds its variants with the same ones)
HIP_FLAGS = ["-std=c++17", "-fPIC", "-shared", "-fvisibility=hidden", "-ffp-contract=off",
             # leading scalar kernel arguments preloaded into SGPRs at wave launch (gfx950);
             # kernels whose first argument is a struct are unaffected
             "-mllvm", "-amdgpu-kernarg-preload-count=7",
             "-fhip-fp32-correctly-rounded-divide-sqrt", "-Wall", "-Wno-unused-function"]


def build_library(debug=False, verbose=True):
    srcs = [os.path.join(CSRC, s) for s in SOURCES]
    deps = srcs + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")] + \
        [os.path.join(REPO, "include", "scgpu.h")]
    if os.path.exists(OUT) and all(os.path.getmtime(OUT) >= os.path.getmtime(d) for d in deps):
        if verbose:
            print(f"[build_native] {OUT} up to date")
        return OUT
    cmd = [hipcc(), f"--offload-arch={ARCH}"] + HIP_FLAGS + [
        "-I", os.path.join(REPO, "include"), "-I", CSRC, "-O1" if debug else "-O3", "-o", OUT + ".tmp"] + srcs
    if verbose:
        print("[build_native]", " ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    build(debug="--debug" in sys.argv)
