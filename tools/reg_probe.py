"""Register-pressure probe for the SupplyChain kernels (device compile only, no GPU).

    python tools/reg_probe.py ["FILE|OLD|NEW" ...]

Copies csrc/ to /tmp/probe, keeps only the MAXD=16 instantiations of scg_supplychain.hip (so a
compile takes under a minute), applies each exact-text edit FILE|OLD|NEW (an ablation, a
noinline marker, a -D default), compiles to gfx950 assembly with the library's flags and prints
NumVgprs / ScratchSize of the staged kernels and of any out-of-line helper. Used to find where
the staged kernel's registers go: e.g. marking sc_staged_heap noinline shows the
heap phase alone at 212 VGPRs.
"""
import os, re, shutil, subprocess, sys
REPO = "/root/repo"
src = os.path.join(REPO, "gym-supplychain_amd/csrc")
dst = "/tmp/probe/csrc"
shutil.rmtree(dst, ignore_errors=True)
shutil.copytree(src, dst)
p = os.path.join(dst, "scg_supplychain.hip")
s = open(p).read()
s = re.sub(r"_LAUNCH\((2|4|8|32)\)", "_LAUNCH(16)", s)
s = re.sub(r"sc_step_kernel<(2|4|8|32)>", "sc_step_kernel<16>", s)
open(p, "w").write(s)
# edits: "file|old|new" triples from argv
for arg in sys.argv[1:]:
    f, old, new = arg.split("|")
    q = os.path.join(dst, f)
    t = open(q).read()
    assert old in t, (f, old)
    t = t.replace(old, new, 1)
    open(q, "w").write(t)
sys.path.insert(0, os.path.join(REPO, "gym-supplychain_amd"))
import build_native
out = os.path.join(os.path.dirname(dst), "p.s")
cmd = [build_native.hipcc(), f"--offload-arch={build_native.ARCH}", "--cuda-device-only", "-S"] + \
    [f for f in build_native.HIP_FLAGS if f != "-fPIC"] + \
    ["-I", os.path.join(REPO, "include"), "-I", dst, "-O3", p, "-o", out]
subprocess.run(cmd, check=True, stderr=subprocess.DEVNULL)
name = None
for line in open(out):
    m = re.match(r"^(_Z\S+):", line)
    if m:
        name = m.group(1)
    m = re.match(r"^; (NumVgprs|ScratchSize|NumSgprs): (\d+)", line)
    if m and name and ("staged" in name or "sc_node_act" in name or "receive" in name or "observe_bins" in name or "heappush" in name):
        dem = subprocess.run(["c++filt"], input=name, capture_output=True, text=True).stdout.strip()
        dem = re.sub(r"\(scg::.*", "", dem)[:110]
        print(f"{m.group(1)}={m.group(2)}  {dem}")
