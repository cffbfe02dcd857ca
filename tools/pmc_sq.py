"""Per-wave SQ counter summary of rocprofv3 --pmc runs (tools/gpu_sc_*.sh output).

    python tools/pmc_sq.py DIR [DIR ...] [--filter step]

Each DIR holds a pmc_counter_collection.csv; counters are averaged over the dispatches of
every kernel whose name contains --filter, then divided by SQ_WAVES when that counter is in
the same run (per-wave figures; SQ_WAVE_CYCLES and SQ_WAIT_* / SQ_ACTIVE_* are quad-cycles).
"""
import argparse
import collections
import csv
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--filter", default="step")
    a = ap.parse_args()
    waves = {}
    rows = collections.defaultdict(dict)
    for d in a.dirs:
        agg = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(os.path.join(d, "pmc_counter_collection.csv"))):
            if a.filter in r["Kernel_Name"]:
                agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, cs in agg.items():
            for c, v in cs.items():
                rows[k][c] = sum(v) / len(v)
            if "SQ_WAVES" in cs:
                waves[k] = rows[k]["SQ_WAVES"]
    for k, cs in rows.items():
        w = waves.get(k)
        print(k[:70])
        for c in sorted(cs):
            print(f"  {c:24s} {cs[c]:16.0f}" + (f"  per wave {cs[c] / w:10.1f}" if w and c != "SQ_WAVES" else ""))


if __name__ == "__main__":
    main()
