"""The resident step-server waves of this process (include/scgpu.h scg_bg_server_*,
scg_sc_server_*): at most one per device at a time.

A parked server wave holds its hardware queue until it exits (its idle time-out). The
servers' streams are of the highest priority, which keeps them off the hardware queues of
normal-priority streams (torch's, RCCL's), but HIP spreads the streams of one priority over
a few queues (GPU_MAX_HW_QUEUES), so two servers' streams may share one: a launch behind a
parked wave would wait for its time-out. So before a server posts, `claim` stops whichever
other server of the device may be resident. The BeerGame server serves every drop-in
BeerGameEnv of a level count from one wave, so envs of one kind stepped in turn never
switch; only stepping different kinds in turn costs a stop and a launch per switch.
"""
import ctypes
import threading

import torch

from .. import _native as nat

_LOCK = threading.Lock()
_RESIDENT = {}  # device index -> the server whose wave may be resident


def claim(dev_index, server):
    """Make `server` the device's resident server, stopping the previous one (if any)."""
    if _RESIDENT.get(dev_index) is server:
        return
    with _LOCK:
        cur = _RESIDENT.get(dev_index)
        if cur is not server:
            if cur is not None:
                cur.stop()
            _RESIDENT[dev_index] = server


def release(dev_index, server):
    with _LOCK:
        if _RESIDENT.get(dev_index) is server:
            del _RESIDENT[dev_index]


def server_stream(device):
    """A new non-blocking stream of the device's highest priority (raw hipStream_t)."""
    hip = nat.hip_runtime()
    hip.hipStreamCreateWithPriority.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint, ctypes.c_int]
    hip.hipDeviceGetStreamPriorityRange.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
    stream = ctypes.c_void_p()
    with torch.cuda.device(device):
        least, greatest = ctypes.c_int(0), ctypes.c_int(0)
        if hip.hipDeviceGetStreamPriorityRange(ctypes.byref(least), ctypes.byref(greatest)) != 0:
            greatest.value = 0
        if hip.hipStreamCreateWithPriority(ctypes.byref(stream), 1, greatest.value) != 0:  # hipStreamNonBlocking
            raise RuntimeError("hipStreamCreateWithPriority failed")
    return stream.value, greatest.value


def destroy_stream(stream):
    hip = nat.hip_runtime()
    hip.hipStreamDestroy.argtypes = [ctypes.c_void_p]
    hip.hipStreamDestroy(ctypes.c_void_p(stream))
