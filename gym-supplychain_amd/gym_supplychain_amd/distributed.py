"""Multi-GPU sharding for the vectorised envs: one process per GPU, envs never interact.

Rank r owns global env ids [r * n_per_rank, (r + 1) * n_per_rank). Every per-env draw
(Philox counter = global env id, episode, week) depends only on the global id, so a
trajectory is identical at 1, 2, 4 or 8 GPUs (tests/test_gpu_beergame.py
test_sharding_is_invariant). The data path has no collective; the only exchange is the
end-of-episode metric gather, an RCCL all-gather over xGMI issued asynchronously so it
overlaps the next episode's steps (the north star's "all-gather for the end-of-episode
reward/metric reduction").
"""
import ctypes
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


def agree(ok, group=None, device=None):
    """True on every rank of the group iff `ok` is true on every rank (an all_reduce MIN; on
    an nccl group the flag travels on `device`). Every rank must call it: the setup steps
    below use it so that a failure on any rank takes every rank down the same fallback
    instead of leaving the others waiting in a collective."""
    on = device if (device is not None and dist.get_backend(group) == "nccl") else "cpu"
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=on)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(t.item())


class _RcclAllGather:
    """An RCCL communicator of our own over torch's librccl, for the episode-return
    all-gather: ncclAllGather goes straight onto a side HIP stream ordered by two events, with
    none of torch.distributed's per-collective bookkeeping (Work objects, stream syncs,
    watchdog records: ≈30 µs of host time per call through dist.all_gather_into_tensor,
    profiles/r04p_gather_probe.log, against ≈ a launch here). The unique id travels over the
    torch.distributed group; every rank of the group builds it (a collective)."""

    class _UniqueId(ctypes.Structure):
        _fields_ = [("internal", ctypes.c_char * 128)]

    NCCL_INT64 = 4

    def __init__(self, group, device):
        from . import _native as nat
        self.comm = ctypes.c_void_p()
        lib_dir = os.path.join(os.path.dirname(torch.__file__), "lib")
        path = os.path.join(lib_dir, "librccl.so")
        try:
            lib = ctypes.CDLL(path if os.path.exists(path) else "librccl.so")
        except OSError:
            lib = None
        if not agree(lib is not None, group, device):
            raise RuntimeError("librccl.so did not load on every rank")
        self.lib = lib
        lib.ncclGetUniqueId.argtypes = [ctypes.POINTER(self._UniqueId)]
        lib.ncclCommInitRank.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, self._UniqueId, ctypes.c_int]
        lib.ncclAllGather.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p,
                                      ctypes.c_void_p]
        lib.ncclCommDestroy.argtypes = [ctypes.c_void_p]
        lib.ncclGetErrorString.restype = ctypes.c_char_p
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        uid = self._UniqueId()
        box = [None]
        if rank == 0 and lib.ncclGetUniqueId(ctypes.byref(uid)) == 0:
            box = [bytes(uid)]  # the raw 128 bytes (the field itself reads up to a NUL)
        src = 0 if group is None else dist.get_global_rank(group, 0)
        dist.broadcast_object_list(box, src=src, group=group, device=device)
        if box[0] is None:  # every rank sees the same box
            raise RuntimeError("ncclGetUniqueId failed on rank 0")
        uid = self._UniqueId.from_buffer_copy(box[0])
        with torch.cuda.device(device):
            rc = lib.ncclCommInitRank(ctypes.byref(self.comm), world, uid, rank)
            if not agree(rc == 0, group, device):
                if rc == 0:
                    lib.ncclCommDestroy(self.comm)
                self.comm = ctypes.c_void_p()
                raise RuntimeError(f"ncclCommInitRank failed on some rank (here: {rc})")
            self.stream = torch.cuda.Stream(device)  # from torch's pool: non-blocking
        hip = nat.hip_runtime()
        hip.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
        hip.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        hip.hipStreamWaitEvent.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint]
        hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
        self.hip = hip
        self._src = (None, None)  # (tensor, data_ptr) of the last snapshot source, checked once
        self.ready, self.done = ctypes.c_void_p(), ctypes.c_void_p()
        for ev in (self.ready, self.done):  # hipEventDisableTiming: a record is a marker only
            if hip.hipEventCreateWithFlags(ctypes.byref(ev), 2) != 0:
                raise RuntimeError("hipEventCreateWithFlags failed")
        self.gstream = ctypes.c_void_p(self.stream.cuda_stream)
        self.pending = False

    def _check(self, rc, what):
        if rc != 0:
            raise RuntimeError(f"{what}: {self.lib.ncclGetErrorString(rc).decode()} ({rc})")

    def gather(self, out, stage, src, stream):
        """out <- all ranks' src (via stage), ordered after the work on `stream` (raw handle)
        and, for the next snapshot into stage, before it."""
        hip = self.hip
        if self._src[0] is not src or self._src[1] != src.data_ptr():
            if not (src.is_cuda and src.is_contiguous() and src.dtype == stage.dtype and src.numel() == stage.numel()
                    and src.device == stage.device):
                raise ValueError("the returns to gather must be a contiguous int64 tensor of n_per_rank on the device")
            self._src = (src, src.data_ptr())
        if self.pending:  # the previous gather may still read stage
            hip.hipStreamWaitEvent(stream, self.done, 0)
        if hip.hipMemcpyAsync(stage.data_ptr(), self._src[1], stage.numel() * 8, 3, stream) != 0:  # D2D snapshot
            raise RuntimeError("hipMemcpyAsync failed")
        hip.hipEventRecord(self.ready, stream)
        hip.hipStreamWaitEvent(self.gstream, self.ready, 0)
        self._check(self.lib.ncclAllGather(stage.data_ptr(), out.data_ptr(), stage.numel(), self.NCCL_INT64,
                                           self.comm, self.gstream), "ncclAllGather")
        hip.hipEventRecord(self.done, self.gstream)
        self.pending = True

    def wait(self, stream):
        """Order `stream` after the latest gather."""
        if self.pending:
            self.hip.hipStreamWaitEvent(stream, self.done, 0)
            self.pending = False

    def close(self):
        if self.comm:
            torch.cuda.current_stream().synchronize()
            self.stream.synchronize()
            self.lib.ncclCommDestroy(self.comm)
            self.comm = ctypes.c_void_p()


class EpisodeReturnGather:
    """All-gather of every env's finished-episode return, overlapped with compute.

    on_episode_end(final_return) snapshots the per-env int64 returns on the producing
    stream (so the next episode may overwrite the env's buffer) and launches an async
    all-gather; result() waits for the latest one and returns the global [world * N]
    tensor. With one process it degenerates to the snapshot, unless `collective` asks for
    the all-gather anyway (a one-rank rehearsal of the RCCL path; default: world > 1).

    The gather runs on dist.all_gather_into_tensor (RCCL on an nccl group, gloo on the
    CPU). SCG_GATHER=rccl puts it on a communicator of the package's own instead
    (_RcclAllGather: ≈10 µs less host time per episode end, profiles/r04p_gather_probe.log),
    which has run at one rank only; it stays opt-in until a multi-GPU record shows it agreeing
    with torch's. `path` names the one in use ("torch", "rccl-own", or "local" without a
    collective) and verify() checks the latest gather's content.
    """

    def __init__(self, n_per_rank, device, group=None, collective=None):
        self.rank, self.world = rank_world()
        self.group = group
        self.n = int(n_per_rank)
        self.device = torch.device(device)
        self.collective = self.world > 1 if collective is None else bool(collective)
        if self.collective and not (dist.is_available() and dist.is_initialized()):
            raise RuntimeError("the return all-gather needs an initialised torch.distributed process group")
        if self.collective:  # the rank of this process within the gather's group
            self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        self._stage = torch.zeros(self.n, dtype=torch.int64, device=self.device) if self.collective else None
        self._out = torch.zeros(self.world * self.n, dtype=torch.int64, device=self.device)
        self._work = None
        self._rccl = None
        self._last = None  # the tensor handed to the latest on_episode_end
        self.path = "torch" if self.collective else "local"
        if self.collective and self.device.type == "cuda" and dist.get_backend(group) == "nccl" \
                and os.environ.get("SCG_GATHER", "torch") == "rccl":
            try:  # every rank takes the same branch (agree() inside)
                self._rccl = _RcclAllGather(group, self.device)
                self.path = "rccl-own"
            except RuntimeError as exc:
                import warnings
                warnings.warn(f"episode-return gather falls back to dist.all_gather_into_tensor: {exc}")
        self.gathers = 0

    def on_episode_end(self, final_return):
        self._last = final_return
        if not self.collective:  # the snapshot is the result: one device copy per episode
            _async_copy(self._out, final_return)
            self.gathers += 1
            return
        if self._rccl is not None:
            from . import _native as nat
            self._rccl.gather(self._out, self._stage, final_return, nat.raw_stream(self.device.index))
            self.gathers += 1
            return
        if self._work is not None:
            self._work.wait()  # previous gather still reading _stage
        _async_copy(self._stage, final_return)
        self._work = dist.all_gather_into_tensor(self._out, self._stage, group=self.group, async_op=True)
        self.gathers += 1

    def result(self):
        if self._rccl is not None:
            from . import _native as nat
            self._rccl.wait(nat.raw_stream(self.device.index))
            return self._out
        if self._work is not None:
            self._work.wait()
            self._work = None
        return self._out

    @staticmethod
    def _checksums(x):
        """(sum, sum of (j + 1) * x_j) of an int64 vector: position-sensitive, so a slice that
        is shifted, reordered or another rank's shard does not match (int64 wraps alike)."""
        w = torch.arange(1, x.numel() + 1, dtype=torch.int64, device=x.device)
        return torch.stack([x.sum(), (x * w).sum()])

    def verify(self):
        """Check the latest gather (a collective when the gather is: every rank calls it).

        * this rank's slice of the gathered tensor equals its local snapshot, and the snapshot
          equals the tensor it was taken from (still holding the last episode's returns when
          no episode ended since, as in bench.py after its last gather);
        * slice r equals rank r's own snapshot, compared through per-rank checksums that
          travel on dist.all_gather_into_tensor — an independent collective from the one
          checked when the gather runs on the package's own communicator.
        Returns {"allgather_ok": bool, "gather_path": str, "envs_checked": int}; the flag is
        the same on every rank (agree)."""
        out = self.result()
        if self.gathers == 0:
            return {"allgather_ok": True, "gather_path": self.path, "envs_checked": 0}
        local = self._stage if self.collective else out
        mine = out[self.rank * self.n:(self.rank + 1) * self.n]
        ok = bool(torch.equal(mine, local))
        if self._last is not None and self._last.numel() == self.n:
            ok &= bool(torch.equal(local, self._last.to(local.device)))
        if self.collective:
            on = self.device if dist.get_backend(self.group) == "nccl" else torch.device("cpu")
            cs = self._checksums(local).to(on)
            every = torch.empty(self.world * 2, dtype=torch.int64, device=on)
            dist.all_gather_into_tensor(every, cs, group=self.group)
            want = every.view(self.world, 2).cpu()
            got = torch.stack([self._checksums(out[r * self.n:(r + 1) * self.n]) for r in range(self.world)]).cpu()
            ok &= bool(torch.equal(got, want))
            ok = agree(ok, self.group, self.device)
        return {"allgather_ok": ok, "gather_path": self.path, "envs_checked": self.world * self.n}

    def close(self):
        """Release the RCCL communicator (synchronises)."""
        if self._rccl is not None:
            self._rccl.close()
            self._rccl = None
