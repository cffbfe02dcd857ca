"""Checkpoint format logic (gym_supplychain_amd/checkpoint.py) on CPU tensors: fingerprints
of the ABI config structs, the checks load_state_dict() makes, strided views saved
contiguous and restored through the view, and the torch.save / weights_only round trip.
The device vec envs' resume is tested on the GPU (test_gpu_checkpoint.py)."""
import ctypes
import io

import pytest
import torch

from gym_supplychain_amd import _native as nat
from gym_supplychain_amd import checkpoint as ckpt


def test_fingerprint_skips_pointers_and_named_fields():
    c = nat.ScConfig()
    c.n_nodes, c.kernel, c.layout = 8, 3, 1
    c.level_start[2] = 5
    c.nodes = 12345
    fp = dict((k, v) for k, v in ckpt.config_fingerprint(c, skip=("kernel", "layout")))
    assert fp["n_nodes"] == 8 and fp["level_start"][2] == 5
    assert "kernel" not in fp and "layout" not in fp and "nodes" not in fp
    b = nat.BgConfig()
    b.initial_inventory[1] = 7
    fpb = dict((k, v) for k, v in ckpt.config_fingerprint(b))
    assert fpb["initial_inventory"][1] == 7 and "plan" not in fpb


def _env():
    stock = torch.arange(12, dtype=torch.float64).reshape(3, 4)  # [NP][N], saved env-major
    return {"stock": stock.t(), "size": torch.zeros(4, dtype=torch.int32), "ledger": None}, stock


def test_snapshot_check_restore_roundtrip():
    bufs, stock = _env()
    fp = [["n_envs", 4]]
    sd = ckpt.snapshot("X", fp, {"seed": 2 ** 63 + 5, "episode": 3, "week": 7}, bufs)
    assert "ledger" not in sd["tensors"] and sd["tensors"]["stock"].is_contiguous()
    assert torch.equal(sd["tensors"]["stock"], stock.t())
    buf = io.BytesIO()
    torch.save(sd, buf)
    buf.seek(0)
    sd2 = torch.load(buf, weights_only=True)
    bufs2, stock2 = _env()
    stock2.zero_()
    ckpt.check(sd2, "X", fp, bufs2)
    cnt = ckpt.restore(sd2, bufs2)
    assert cnt == {"seed": 2 ** 63 + 5, "episode": 3, "week": 7}
    assert torch.equal(stock2, stock)  # written through the transposed view


def test_check_refuses_mismatches():
    bufs, _ = _env()
    fp = [["n_envs", 4], ["levels", 4]]
    sd = ckpt.snapshot("X", fp, {"seed": 1}, bufs)
    with pytest.raises(ValueError, match="not a"):
        ckpt.check({"format": "other"}, "X", fp, bufs)
    with pytest.raises(ValueError, match="version"):
        ckpt.check(dict(sd, version=99), "X", fp, bufs)
    with pytest.raises(ValueError, match="a X, this env is a Y"):
        ckpt.check(sd, "Y", fp, bufs)
    with pytest.raises(ValueError, match="levels: 4 vs 3"):
        ckpt.check(sd, "X", [["n_envs", 4], ["levels", 3]], bufs)
    with pytest.raises(ValueError, match="tracking options"):
        ckpt.check(sd, "X", fp, dict(bufs, ledger=torch.zeros(4)))
    other = dict(bufs, size=torch.zeros(5, dtype=torch.int32))
    with pytest.raises(ValueError, match="'size'"):
        ckpt.check(sd, "X", fp, other)
    other = dict(bufs, size=torch.zeros(4, dtype=torch.int64))
    with pytest.raises(ValueError, match="'size'"):
        ckpt.check(sd, "X", fp, other)


def test_vec_envs_expose_the_checkpoint_api():
    from gym_supplychain_amd import BeerGame2VecEnv, BeerGameVecEnv, SupplyChainVecEnv
    for cls in (BeerGameVecEnv, BeerGame2VecEnv, SupplyChainVecEnv):
        assert callable(cls.state_dict) and callable(cls.load_state_dict)
    assert ctypes.sizeof(nat.BgConfig) > 0
