"""Static instruction mix of the SupplyChain / BeerGame kernels (gfx950 assembly).

    python tools/isa_stats.py [csrc/scg_supplychain.hip] [-D MACRO=V ...] [--filter sc_step]

Compiles one source to device assembly with the library's flags and prints, per kernel
whose name contains --filter: static instruction counts by class (VALU / SALU / LDS /
VMEM / SMEM / branch / waitcnt), VGPR / SGPR counts, scratch and LDS use. A quick CPU-side
check of what a code change does to the kernel before spending GPU time on it.
"""
import argparse
import collections
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "gym-supplychain_amd")
sys.path.insert(0, PKG)
import build_native  # noqa: E402


def classify(op):
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith(("s_cbranch", "s_branch", "s_setpc", "s_swappc")):
        return "branch"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("v_"):
        return "valu"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src", nargs="?", default=os.path.join(PKG, "csrc", "scg_supplychain.hip"))
    ap.add_argument("-D", action="append", default=[])
    ap.add_argument("--filter", default="sc_step")
    ap.add_argument("--save", default=None, help="also write the assembly here")
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "k.s")
        cmd = [build_native.hipcc(), f"--offload-arch={build_native.ARCH}", "--cuda-device-only", "-S"] + \
            [f for f in build_native.HIP_FLAGS if f != "-fPIC"] + \
            ["-I", os.path.join(REPO, "include"), "-I", os.path.join(PKG, "csrc"), "-O3"] + \
            [f"-D{x}" for x in a.D] + [a.src, "-o", out]
        subprocess.run(cmd, check=True)
        text = open(out).read()
    if a.save:
        open(a.save, "w").write(text)
    kernels = {}
    cur = None
    for line in text.splitlines():
        m = re.match(r"^(_Z\S+):\s*(;.*)?$", line)
        if m and not line.startswith("\t"):
            cur = m.group(1)
            kernels[cur] = collections.Counter()
            continue
        if cur is None:
            continue
        if line.startswith("\t.size") or line.startswith("\t.end_amdhsa_kernel"):
            cur = None
            continue
        s = line.strip()
        if not s or s.startswith((";", ".", "//")) or s.endswith(":"):
            continue
        kernels[cur][classify(s.split()[0])] += 1
    for name, cnt in kernels.items():
        dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        if a.filter not in dem:
            continue
        blk = re.search(re.escape(name) + r"[\s\S]*?\.amdhsa_next_free_vgpr (\d+)[\s\S]*?\.amdhsa_next_free_sgpr (\d+)",
                        text)
        scr = re.search(r"; ScratchSize: (\d+)", text[text.find(name + ":"):])
        total = sum(cnt.values())
        print(f"{dem}: total {total}  " + "  ".join(f"{k} {v}" for k, v in sorted(cnt.items())) +
              (f"  vgpr {blk.group(1)} sgpr {blk.group(2)}" if blk else "") +
              (f"  scratch {scr.group(1)}" if scr else ""))


if __name__ == "__main__":
    main()
