"""Multi-GPU sharding for the vectorised envs: one process per GPU, envs never interact.

Rank r owns global env ids [r * n_per_rank, (r + 1) * n_per_rank). Every per-env draw
(Philox counter = global env id, episode, week) depends only on the global id, so a
trajectory is identical at 1, 2, 4 or 8 GPUs (tests/test_gpu_beergame.py
test_sharding_is_invariant). The data path has no collective; the only exchange is the
end-of-episode metric gather, an RCCL all-gather over xGMI issued asynchronously so it
overlaps the next episode's steps (the north star's "all-gather for the end-of-episode
reward/metric reduction").
"""
import os

import torch
import torch.distributed as dist


def rank_world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))


def shard_offset(n_per_rank, rank=None):
    """Global id of this rank's first env."""
    if rank is None:
        rank = rank_world()[0]
    return int(rank) * int(n_per_rank)


def entropy_seed(seed, seed_group=None):
    """A 64-bit Philox key: `seed`, or fresh OS entropy for None (RandomState(None) semantics).

    The entropy is this process's own unless `seed_group` names a torch.distributed process
    group (True: the default group): then the group's rank 0 draws it and every member
    adopts it, so the shards of one seed=None batch draw what one big batch would
    (env_offset). That is a collective: every rank of the group must make the same call."""
    if seed is not None:
        return int(seed) & 0xFFFFFFFFFFFFFFFF
    key = [int.from_bytes(os.urandom(8), "little")]
    if seed_group is not None and seed_group is not False:
        if not (dist.is_available() and dist.is_initialized()):
            raise RuntimeError("seed_group needs an initialised torch.distributed process group")
        group = None if seed_group is True else seed_group
        if dist.get_world_size(group) > 1:
            src = 0 if group is None else dist.get_global_rank(group, 0)
            dist.broadcast_object_list(key, src=src, group=group)
    return key[0]


def _async_copy(dst, src):
    """dst <- src, async on the current stream. On the GPU one hipMemcpyAsync (device to
    device) through torch's HIP runtime: a torch copy_ costs the host ≈10 µs of dispatch,
    a quarter of a 35-week episode's step budget at 65,536 envs."""
    if dst.device.type != "cuda" or not (dst.is_contiguous() and src.is_contiguous()) or dst.dtype != src.dtype \
            or dst.numel() != src.numel() or src.device != dst.device:
        dst.copy_(src, non_blocking=True)
        return
    import ctypes

    from . import _native as nat
    hip = nat.hip_runtime()
    if not getattr(hip, "_scg_memcpy_async", False):
        hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
        hip._scg_memcpy_async = True
    rc = hip.hipMemcpyAsync(dst.data_ptr(), src.data_ptr(), src.numel() * src.element_size(), 3,  # D2D
                            ctypes.c_void_p(nat.raw_stream(dst.device.index)))
    if rc != 0:
        raise RuntimeError(f"hipMemcpyAsync failed ({rc})")


class EpisodeReturnGather:
    """All-gather of every env's finished-episode return, overlapped with compute.

    on_episode_end(final_return) snapshots the per-env int64 returns on the producing
    stream (so the next episode may overwrite the env's buffer) and launches an async
    all-gather; result() waits for the latest one and returns the global [world * N]
    tensor. With one process it degenerates to the snapshot, unless `collective` asks for
    the all-gather anyway (a one-rank rehearsal of the RCCL path; default: world > 1).
    """

    def __init__(self, n_per_rank, device, group=None, collective=None):
        self.rank, self.world = rank_world()
        self.group = group
        self.n = int(n_per_rank)
        self.device = torch.device(device)
        self.collective = self.world > 1 if collective is None else bool(collective)
        if self.collective and not (dist.is_available() and dist.is_initialized()):
            raise RuntimeError("the return all-gather needs an initialised torch.distributed process group")
        self._stage = torch.zeros(self.n, dtype=torch.int64, device=self.device) if self.collective else None
        self._out = torch.zeros(self.world * self.n, dtype=torch.int64, device=self.device)
        self._work = None
        self.gathers = 0

    def on_episode_end(self, final_return):
        if not self.collective:  # the snapshot is the result: one device copy per episode
            _async_copy(self._out, final_return)
            self.gathers += 1
            return
        if self._work is not None:
            self._work.wait()  # previous gather still reading _stage
        _async_copy(self._stage, final_return)
        self._work = dist.all_gather_into_tensor(self._out, self._stage, group=self.group, async_op=True)
        self.gathers += 1

    def result(self):
        if self._work is not None:
            self._work.wait()
            self._work = None
        return self._out
