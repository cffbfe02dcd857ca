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
SOURCES = ["scg_common.hip", "scg_beergame.hip", "scg_bg_levels_1.hip", "scg_bg_levels_2.hip", "scg_bg_levels_3.hip",
           "scg_bg_levels_4.hip", "scg_supplychain.hip", "scg_sc_nodes.hip"]
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
HIP_FLAGS = ["-std=c++17", "-fPIC", "-fvisibility=hidden", "-ffp-contract=off",
             # leading scalar kernel arguments preloaded into SGPRs at wave launch (gfx950);
             # kernels whose first argument is a struct are unaffected
             "-mllvm", "-amdgpu-kernarg-preload-count=9",
             "-fhip-fp32-correctly-rounded-divide-sqrt", "-Wall", "-Wno-unused-function"]


def compile_library(out, srcs, include_dirs, extra=(), opt="-O3", verbose=True):
    """Each source to an object concurrently (the template instantiations dominate), then one
    shared-library link; the TUs share no device symbols, so no relocatable device code."""
    from concurrent.futures import ThreadPoolExecutor
    objdir = out + ".objs"
    os.makedirs(objdir, exist_ok=True)
    inc = [x for d in include_dirs for x in ("-I", d)]
    objs = [os.path.join(objdir, os.path.splitext(os.path.basename(s))[0] + ".o") for s in srcs]
    # an object is reused when it is newer than its source, every header and this script
    hdr = [os.path.join(d, f) for d in include_dirs for f in os.listdir(d) if f.endswith(".h")]
    newest_dep = max([os.path.getmtime(h) for h in hdr] + [os.path.getmtime(__file__)])

    def cc(src_obj):
        src, obj = src_obj
        if os.path.exists(obj) and os.path.getmtime(obj) >= max(newest_dep, os.path.getmtime(src)):
            return
        cmd = [hipcc(), f"--offload-arch={ARCH}"] + HIP_FLAGS + inc + [opt, *extra, "-c", src, "-o", obj]
        if verbose:
            print("[build_native]", " ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)

    with ThreadPoolExecutor(max_workers=min(len(srcs), os.cpu_count() or 1)) as pool:
        list(pool.map(cc, zip(srcs, objs)))
    link = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out + ".tmp"] + objs
    if verbose:
        print("[build_native]", " ".join(link), flush=True)
    subprocess.run(link, check=True)
    os.replace(out + ".tmp", out)
    return out


def build_library(debug=False, verbose=True):
    srcs = [os.path.join(CSRC, s) for s in SOURCES]
    deps = srcs + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")] + \
        [os.path.join(REPO, "include", "scgpu.h")]
    if os.path.exists(OUT) and all(os.path.getmtime(OUT) >= os.path.getmtime(d) for d in deps):
        if verbose:
            print(f"[build_native] {OUT} up to date")
        return OUT
    return compile_library(OUT, srcs, [os.path.join(REPO, "include"), CSRC], opt="-O1" if debug else "-O3",
                           verbose=verbose)


if __name__ == "__main__":
    build(debug="--debug" in sys.argv)
