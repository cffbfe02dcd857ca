"""Build experiment variants of libscgpu.so side by side (for A/B timing on the GPU box).

    python tools/exp_build.py NAME [--rev GIT_REV] [--file csrc/X.h=REV ...] [-D MACRO=V ...]
                              [--replace csrc/X.h OLD NEW ...]

Writes exp/NAME/gym_supplychain_amd/ — a copy of the package whose libscgpu.so is built
from the working-tree csrc/ (or from GIT_REV, or per-file revisions) with extra -D flags.
Run a tool against it with SCG_PKG_ROOT=exp/NAME (bench.py and tools/bench_sc.py,
tools/bg_variants.py honour it). exp/ is git-ignored scratch.
"""
import argparse
import os
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "gym-supplychain_amd")
sys.path.insert(0, PKG)
import build_native  # noqa: E402


def git_show(rev, path):
    return subprocess.run(["git", "-C", REPO, "show", f"{rev}:{path}"], check=True, capture_output=True,
                          text=True).stdout


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("name")
    ap.add_argument("--rev", default=None, help="take every csrc file and include/scgpu.h from this revision")
    ap.add_argument("--file", action="append", default=[], help="csrc/FILE=REV: one file from a revision")
    ap.add_argument("-D", dest="defines", action="append", default=[])
    ap.add_argument("--xflag", action="append", default=[],
                    help="an extra compiler flag for every source (e.g. --xflag=-mllvm "
                         "--xflag=-amdgpu-sched-strategy=max-ilp); disables --reuse-objs")
    ap.add_argument("--replace", nargs=3, action="append", default=[], metavar=("FILE", "OLD", "NEW"),
                    help="csrc/FILE: replace the exact text OLD by NEW (it must occur); for ablations")
    ap.add_argument("--reuse-objs", action="store_true",
                    help="reuse the tree's up-to-date objects for sources whose text (and every header) is "
                         "unchanged and names none of the -D macros")
    a = ap.parse_args()
    root = os.path.join(REPO, "exp", a.name)
    shutil.rmtree(root, ignore_errors=True)
    csrc = os.path.join(root, "csrc")
    inc = os.path.join(root, "include")
    os.makedirs(csrc)
    os.makedirs(inc)
    for f in os.listdir(os.path.join(PKG, "csrc")):
        src = os.path.join(PKG, "csrc", f)
        try:
            text = git_show(a.rev, f"gym-supplychain_amd/csrc/{f}") if a.rev else open(src).read()
        except subprocess.CalledProcessError:  # a file the revision does not have yet
            continue
        open(os.path.join(csrc, f), "w").write(text)
    hdr = git_show(a.rev, "include/scgpu.h") if a.rev else open(os.path.join(REPO, "include", "scgpu.h")).read()
    open(os.path.join(inc, "scgpu.h"), "w").write(hdr)
    for spec in a.file:
        path, rev = spec.split("=")
        open(os.path.join(csrc, os.path.basename(path)), "w").write(git_show(rev, f"gym-supplychain_amd/{path}"))
    for f, old, new in a.replace:
        path = os.path.join(csrc, os.path.basename(f))
        text = open(path).read()
        old, new = old.encode().decode("unicode_escape"), new.encode().decode("unicode_escape")
        if old not in text:
            sys.exit(f"--replace: text not found in {f}: {old!r}")
        open(path, "w").write(text.replace(old, new))
    pkg = os.path.join(root, "gym_supplychain_amd")
    if a.rev:  # the Python package of that revision too (it must match the library's ABI)
        files = subprocess.run(["git", "-C", REPO, "ls-tree", "-r", "--name-only", a.rev,
                                "gym-supplychain_amd/gym_supplychain_amd"], check=True, capture_output=True,
                               text=True).stdout.split()
        for f in files:
            dst = os.path.join(pkg, os.path.relpath(f, "gym-supplychain_amd/gym_supplychain_amd"))
            os.makedirs(os.path.dirname(dst), exist_ok=True)
            open(dst, "w").write(git_show(a.rev, f))
    else:
        shutil.copytree(os.path.join(PKG, "gym_supplychain_amd"), pkg,
                        ignore=shutil.ignore_patterns("*.so", "__pycache__"))
    out = os.path.join(pkg, "libscgpu.so")
    srcs = [os.path.join(csrc, s) for s in build_native.SOURCES]
    if a.reuse_objs and not a.xflag:
        tree_csrc, tree_objs = os.path.join(PKG, "csrc"), build_native.OUT + ".objs"
        same = lambda f: open(os.path.join(csrc, f)).read() == open(os.path.join(tree_csrc, f)).read()  # noqa: E731
        headers_same = all(same(f) for f in os.listdir(csrc) if f.endswith(".h")) and \
            open(os.path.join(inc, "scgpu.h")).read() == open(os.path.join(REPO, "include", "scgpu.h")).read()
        os.makedirs(out + ".objs", exist_ok=True)
        macros = [d.split("=")[0] for d in a.defines]
        for s_ in build_native.SOURCES:
            obj = os.path.splitext(s_)[0] + ".o"
            tobj = os.path.join(tree_objs, obj)
            # a macro named by the source or by any header counts (headers reach every source)
            text = open(os.path.join(csrc, s_)).read() + "".join(
                open(os.path.join(csrc, h)).read() for h in os.listdir(csrc) if h.endswith(".h"))
            fresh = os.path.exists(tobj) and os.path.getmtime(tobj) >= os.path.getmtime(os.path.join(tree_csrc, s_))
            if headers_same and same(s_) and fresh and not any(m in text for m in macros):
                shutil.copyfile(os.path.join(tree_objs, obj), os.path.join(out + ".objs", obj))  # fresh mtime
    build_native.compile_library(out, srcs, [inc, csrc], extra=[f"-D{d}" for d in a.defines] + a.xflag,
                                 verbose=False)
    import sysconfig
    bout = os.path.join(pkg, "_scgpu_fast" + sysconfig.get_config_var("EXT_SUFFIX"))
    subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-I", sysconfig.get_paths()["include"], "-I", inc,
                    os.path.join(csrc, "scg_pybind.c"), "-L", pkg, "-lscgpu", "-Wl,-rpath,$ORIGIN", "-o", bout],
                   check=True)
    print(f"[exp_build] {root}")


if __name__ == "__main__":
    main()
