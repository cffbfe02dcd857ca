"""Checkpoint / resume of the device vec envs.

The reference keeps an env's state in plain Python attributes and serialises nothing
(`beergame_env.py:44-60`, `supplychain_env.py:556-628`); SURVEY §5 names `state_dict()` of the
SoA tensors as this build's equivalent. A vec env's whole state is its device buffers plus
three host counters — the Philox key (seed), the episode and the week / time step — because
every device draw is a function of (seed, global env id, episode, index). So a
restored env continues bit for bit as the saved one would have, whatever kernel either runs.

`state_dict()` clones the buffers on the caller's stream (ordered after every step already
enqueued; no synchronisation) and returns a dict of tensors, ints, strs and lists, which
`torch.save` / `torch.load(..., weights_only=True)` round-trip. `load_state_dict()` checks the
checkpoint against the env (class, configuration, every buffer's name, shape and dtype),
then copies into the env's own buffers, so the device pointers the C ABI was given stay valid.

What is not state, and so not saved: buffers that live only inside one step (the staged
kernel's shipment inbox, the node-parallel kernel's per-node ledger slots) and caller-owned
inputs (demand / lead-time tables passed to the constructor: build the env with the same ones).
"""
import ctypes

import torch

FORMAT = "scgpu-vecenv"
VERSION = 1


def config_fingerprint(struct, skip=()):
    """The non-pointer fields of a ctypes config struct (include/scgpu.h), as a list of
    [name, value] pairs with arrays flattened to lists; fields named in `skip` (the kernel
    choice, which does not change the state's meaning) are left out."""
    out = []
    for name, ctype in struct._fields_:
        if name in skip or ctype is ctypes.c_void_p:
            continue
        v = getattr(struct, name)
        out.append([name, list(v) if isinstance(v, ctypes.Array) else int(v)])
    return out


def snapshot(kind, fingerprint, counters, buffers):
    """The checkpoint dict: `buffers` (name -> device tensor or a strided view of one, None
    entries skipped) cloned, contiguous, on the current stream."""
    return {"format": FORMAT, "version": VERSION, "kind": kind, "fingerprint": fingerprint,
            "counters": {k: int(v) for k, v in counters.items()},
            "tensors": {k: t.detach().clone(memory_format=torch.contiguous_format)
                        for k, t in buffers.items() if t is not None}}


def _diff(a, b):
    da, db = dict((k, v) for k, v in a), dict((k, v) for k, v in b)
    keys = [k for k in list(da) + [k for k in db if k not in da] if da.get(k) != db.get(k)]
    return ", ".join(f"{k}: {da.get(k)!r} vs {db.get(k)!r}" for k in keys[:6])


def check(sd, kind, fingerprint, buffers):
    """Raise ValueError unless checkpoint `sd` was taken from an env of class `kind` with
    this configuration and exactly these buffers (names, shapes, dtypes)."""
    if not isinstance(sd, dict) or sd.get("format") != FORMAT:
        raise ValueError(f"not a {FORMAT} checkpoint")
    if sd.get("version") != VERSION:
        raise ValueError(f"checkpoint version {sd.get('version')!r}, this build reads {VERSION}")
    if sd.get("kind") != kind:
        raise ValueError(f"checkpoint of a {sd.get('kind')}, this env is a {kind}")
    if sd.get("fingerprint") != fingerprint:
        raise ValueError("checkpoint of another configuration (saved vs this env): "
                         + _diff(sd.get("fingerprint") or [], fingerprint))
    saved = sd.get("tensors") or {}
    live = {k: t for k, t in buffers.items() if t is not None}
    if set(saved) != set(live):
        raise ValueError(f"checkpoint buffers {sorted(saved)} do not match this env's {sorted(live)} "
                         "(tracking options differ)")
    for k, t in live.items():
        s = saved[k]
        if not isinstance(s, torch.Tensor) or tuple(s.shape) != tuple(t.shape) or s.dtype != t.dtype:
            raise ValueError(f"checkpoint buffer {k!r}: {getattr(s, 'dtype', type(s))} "
                             f"{tuple(getattr(s, 'shape', ()))}, this env holds {t.dtype} {tuple(t.shape)}")


def restore(sd, buffers):
    """Copy the checkpoint's tensors into the env's live buffers (on the current stream)."""
    for k, t in buffers.items():
        if t is not None:
            t.copy_(sd["tensors"][k].to(t.device), non_blocking=True)
    return sd["counters"]
