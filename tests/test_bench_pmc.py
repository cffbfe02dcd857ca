"""bench.pmc_lookup: a committed PMC summary counts for a bench line only when its recorded
workload matches every key of the line's workload and it was collected on the current tree's
kernel sources (round 3's SupplyChain lines took the two-product chain's summary, whose kernel
symbol is the same, and a reverted variant's)."""
import json
import os

import bench


def _summary(path, family, src, workload, kernel, nbytes):
    with open(path, "w") as f:
        json.dump({"traffic": {kernel: {"hbm_bytes_per_launch": nbytes}}, "workload": workload,
                   "src_hash": {family: src}}, f)


def test_pmc_lookup_matches_workload_and_sources(tmp_path, monkeypatch):
    prof = tmp_path / "profiles"
    prof.mkdir()
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    monkeypatch.setattr(bench, "kernel_sources_hash", lambda family: {"sc": "aaaa", "bg": "bbbb"}[family])
    k = "void scg::sc_step_nodes_kernel<2, false, false>(scg::ScArgs, int, int)"
    base = {"bench": "bench_sc", "scenario": "2perstage", "n_envs": 65536, "kernel": "auto", "build_info": False}
    _summary(prof / "r04a_sc_2perstage_pmc_summary.json", "sc", "aaaa", base, k, 72e6)
    # newer, same kernel symbol, another scenario (the two-product chain)
    _summary(prof / "r04b_sc_mp_pmc_summary.json", "sc", "aaaa", dict(base, scenario="2perstage_mp"), k, 141e6)
    # newest, right workload, collected on other sources (a kernel since changed)
    _summary(prof / "r04c_sc_2perstage_pmc_summary.json", "sc", "cccc", base, k, 99e6)
    got, src = bench.pmc_lookup("sc", base, "sc_step_nodes_kernel<2, false, false>")
    assert got == 72e6 and os.path.basename(src) == "r04a_sc_2perstage_pmc_summary.json"
    got, _ = bench.pmc_lookup("sc", dict(base, scenario="2perstage_mp"), "sc_step_nodes_kernel<2")
    assert got == 141e6
    assert bench.pmc_lookup("sc", dict(base, n_envs=4096), "sc_step_nodes_kernel") == (None, None)
    assert bench.pmc_lookup("sc", dict(base, build_info=True), "sc_step_nodes_kernel") == (None, None)
    assert bench.pmc_lookup("bg", base, "sc_step_nodes_kernel") == (None, None)      # other family's hash


def test_profile_tag_order():
    keys = sorted(["r04a_x", "r03ak_x", "r04g_x", "r04_x", "r04aa_x"], key=bench.profile_tag_key)
    assert keys == ["r03ak_x", "r04_x", "r04a_x", "r04g_x", "r04aa_x"]


def test_kernel_sources_hash_is_stable_and_family_specific():
    assert bench.kernel_sources_hash("bg") == bench.kernel_sources_hash("bg")
    assert bench.kernel_sources_hash("bg") != bench.kernel_sources_hash("sc")
