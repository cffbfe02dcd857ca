"""Generate tests/golden/demand_models.npz from the REFERENCE demand generators — build
container only.

Runs gym_supplychain/envs/demands_generator.py (imported read-only from /root/reference)
with RandomState and records value histograms of its normal and sinusoidal generators, for
the distribution tests of the device's inverse-CDF / base-plus-perturbation draws
(tests/test_demand_models.py). Nothing is written under /root/reference; without it the
script exits leaving the committed fixture alone.

    python oracle/gen_golden_demand.py
"""
import importlib.util
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REFERENCE = "/root/reference"
OUT = os.path.join(REPO, "tests", "golden", "demand_models.npz")
sys.dont_write_bytecode = True

HORIZON = 360
PERIODS = list(range(0, HORIZON + 1, 30))
# (name, generate_demand keywords): the seasonal 2-per-stage scenario
# (supplychain_2perstage_env.py:67-80), the multi-product by-product ones
# (supplychain_multiproduct_env.py:157-209) and generic ones
MODELS = {
    "normal": dict(minv=0, maxv=400, std=50.0),
    "normal_narrow": dict(minv=10, maxv=20, std=2.5),
    "seasonal": dict(minv=0, maxv=400, std=10, sen_peaks=4, minavg=150, maxavg=250, perturb_norm=True),
    "sine_normal": dict(minv=0, maxv=400, std=30.0, sen_peaks=4, minavg=100, maxavg=300, perturb_norm=True),
    "sine_uniform": dict(minv=0, maxv=400, std=5, sen_peaks=4, minavg=100, maxavg=300, perturb_norm=False),
    "sine_flat": dict(minv=0, maxv=400, std=None, sen_peaks=2, minavg=100, maxavg=300, perturb_norm=False),
}
SAMPLES = 400000       # normal: draws pooled over one period
PER_PERIOD = 20000     # sinusoids: draws per period (the reference loops per element)


def main():
    path = os.path.join(REFERENCE, "gym_supplychain", "envs", "demands_generator.py")
    if not os.path.exists(path):
        print("gen_golden_demand: /root/reference absent; keeping the committed fixture")
        return 0
    spec = importlib.util.spec_from_file_location("ref_demands_generator", path)
    gen = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gen)
    rec, meta = {}, {"horizon": HORIZON, "periods": PERIODS, "models": {}}
    for i, (name, kw) in enumerate(MODELS.items()):
        rng = np.random.RandomState(100 + i)
        lo, hi = kw["minv"], kw["maxv"]
        if kw.get("sen_peaks") is None:
            data = gen.generate_demand(rng, (SAMPLES,), HORIZON, **kw)
            rec[name] = np.bincount(data - lo, minlength=hi - lo + 1).astype(np.int64)[None, :]
        else:
            data = gen.generate_demand(rng, (HORIZON + 1, PER_PERIOD), HORIZON, **kw)
            rec[name] = np.stack([np.bincount(data[t] - lo, minlength=hi - lo + 1) for t in PERIODS]).astype(np.int64)
        meta["models"][name] = kw
        print(f"{name}: {rec[name].shape}, {int(rec[name].sum())} draws", flush=True)
    np.savez_compressed(OUT, meta=np.array(json.dumps(meta)), **rec)
    print(f"wrote {OUT} ({os.path.getsize(OUT)} B)")
    return 0


if __name__ == "__main__":
    sys.exit(main())
