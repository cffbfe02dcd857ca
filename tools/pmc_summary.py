"""Summarise rocprofv3 --pmc CSVs (tools/gpu_pmc.sh) per kernel.

    python tools/pmc_summary.py gpurun_out/pmc_r01 --meta bench=beergame-v0 n_envs=65536 --family bg \
        > profiles/r01_pmc_summary.json

For every pass directory, averages each counter per kernel name over its dispatches.
HBM traffic per launch follows MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are
KiB; on gfx950 FETCH_SIZE reads 1/2 of the bytes of wide coalesced streaming reads, so
`read_bytes_corrected` doubles it (WRITE_SIZE is exact for 16-B/lane stores).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(pass_dir):
    files = glob.glob(os.path.join(pass_dir, "**", "*counter_collection*.csv"), recursive=True)
    acc = defaultdict(lambda: defaultdict(list))
    for f in files:
        for row in csv.DictReader(open(f)):
            acc[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} | {"dispatches": max(len(v) for v in d.values())}
            for k, d in acc.items()}


def main(root, meta=None, families=()):
    out = {}
    for d in sorted(glob.glob(os.path.join(root, "*"))):
        if os.path.isdir(d):
            out[os.path.basename(d)] = load(d)
    traffic = {}
    for prefix in ("bg", "sc"):
        fetch, write = out.get(f"{prefix}_fetch", {}), out.get(f"{prefix}_write", {})
        for k in set(fetch) | set(write):
            f = fetch.get(k, {}).get("FETCH_SIZE")
            w = write.get(k, {}).get("WRITE_SIZE")
            traffic[k] = {"FETCH_SIZE_KiB": f, "WRITE_SIZE_KiB": w,
                          "read_bytes_corrected": None if f is None else 2 * f * 1024,
                          "write_bytes": None if w is None else w * 1024,
                          "hbm_bytes_per_launch": None if (f is None or w is None) else (2 * f + w) * 1024}
    summ = {"passes": out, "traffic": traffic}
    if meta:
        summ["workload"] = meta
    # the kernel sources the passes ran: written by the GPU script next to the passes
    # (src_hash_<family>.txt), else this tree's (bench.kernel_sources_hash)
    if families:
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from bench import kernel_sources_hash
        summ["src_hash"] = {}
        for fam in families:
            p = os.path.join(root, f"src_hash_{fam}.txt")
            summ["src_hash"][fam] = open(p).read().strip() if os.path.exists(p) else kernel_sources_hash(fam)
    json.dump(summ, sys.stdout, indent=1, sort_keys=True)
    print()


def _value(v):
    if v in ("true", "false"):
        return v == "true"
    try:
        return int(v)
    except ValueError:
        return v


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--meta", nargs="*", default=[], help="workload key=value pairs (bench.pmc_lookup matches them)")
    ap.add_argument("--family", nargs="*", default=[], help="kernel families whose source hash to record (bg, sc)")
    a = ap.parse_args()
    main(a.root, {k: _value(v) for k, v in (x.split("=", 1) for x in a.meta)}, a.family)
