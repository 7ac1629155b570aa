"""Checkpoint I/O (parity: ``comfy/utils.py:10-44, 285-291``; C31).

* ``.safetensors`` — parsed by the in-tree C++ reader (``csrc/runtime/safetensors.cpp``: mmap,
  header JSON, zero-copy tensor views), optionally straight onto the device; falls back to the
  ``safetensors`` package when the runtime extension is not built.
* ``.ckpt/.pt/.pth/.bin`` — ``torch.load(weights_only=True)`` only (never unpickles code).
* writer for CheckpointSave / SaveLatent (safetensors with ``__metadata__``).
"""
from __future__ import annotations

import json
import logging
import os
import struct

import torch

from .. import _native

_DT = {
    "F64": torch.float64, "F32": torch.float32, "F16": torch.float16, "BF16": torch.bfloat16,
    "I64": torch.int64, "I32": torch.int32, "I16": torch.int16, "I8": torch.int8, "U8": torch.uint8,
    "BOOL": torch.bool, "F8_E4M3": torch.float8_e4m3fn, "F8_E5M2": torch.float8_e5m2,
}
_DT_INV = {v: k for k, v in _DT.items()}


def safetensors_header(path, max_size=100 * 1024 * 1024):
    with open(path, "rb") as f:
        n = struct.unpack("<Q", f.read(8))[0]
        if n > max_size:
            return None
        return f.read(n)


def read_metadata(path):
    h = safetensors_header(path)
    if h is None:
        return None
    return json.loads(h).get("__metadata__")


def _element_size(dt):
    return torch.empty(0, dtype=dt).element_size()


def load_safetensors_to_device(path, device, dtype=None):
    """Whole-file upload into one HBM arena: the mmap'ed data section streams to
    the device through pinned double buffers (``cgs_h2d_upload``); tensors are views into the
    arena. ``dtype`` converts floating tensors on the device (the arena is then released).
    Returns None when the native pieces are unavailable."""
    rt = _native.load_runtime()
    lib = _native.load_kernels()
    if rt is None or not hasattr(rt, "SafeTensorsFile") or lib is None or not hasattr(lib, "cgs_h2d_upload"):
        return None
    device = torch.device(device)
    f = rt.SafeTensorsFile(path)
    addr, size, keep = f.data_section()
    arena = torch.empty(max(int(size), 1), dtype=torch.uint8, device=device)
    with torch.cuda.device(device):
        stream = torch.cuda.current_stream(device)
        err = lib.cgs_h2d_upload(addr, arena.data_ptr(), int(size), 64 << 20, 4, stream.cuda_stream)
    del keep
    if err != 0:
        raise RuntimeError(f"cgs_h2d_upload failed with hipError {err}")
    out = {}
    for name in f.keys():
        dt_name, shape, _ = f.info(name)
        dt = _DT[dt_name]
        b, e = f.offsets(name)
        es = _element_size(dt)
        raw = arena[b:e]
        if b % es:                                   # unaligned element offset: copy out
            raw = raw.clone()
        t = raw.view(dt).reshape(shape) if e > b else torch.empty(shape, dtype=dt, device=device)
        if dtype is not None and t.is_floating_point() and t.dtype != dtype:
            t = t.to(dtype)
        out[name] = t
    return out


def _load_safetensors(path, device="cpu"):
    if str(device) != "cpu" and torch.device(device).type == "cuda" and os.environ.get("CGS_DIRECT_LOAD", "1") != "0":
        sd = load_safetensors_to_device(path, device)
        if sd is not None:
            return sd
    rt = _native.load_runtime()
    if rt is not None and hasattr(rt, "SafeTensorsFile") and os.environ.get("CGS_PY_SAFETENSORS") != "1":
        f = rt.SafeTensorsFile(path)
        out = {}
        for name in f.keys():
            dtype, shape, buf = f.tensor(name)   # buf: memoryview over the mmap
            t = torch.frombuffer(buf, dtype=_DT[dtype]) if len(buf) else torch.empty(0, dtype=_DT[dtype])
            t = t.reshape(shape)
            out[name] = t.to(device) if str(device) != "cpu" else t.clone()
        return out
    import safetensors.torch
    return safetensors.torch.load_file(path, device=str(device))


FILE_READS: list = []     # paths this process read from disk (serving metrics / the R3 broadcast tests)


def _trace_read(path):
    FILE_READS.append(path)
    tr = os.environ.get("CGS_TRACE_LOADS")
    if tr:
        with open(tr, "a") as fh:
            fh.write(f"{os.environ.get('RANK', '0')} {path}\n")


def load_state_dict(path, safe_load=True, device=None, return_metadata=False):
    """A checkpoint's state dict. Inside an SPMD prompt of several ranks (``sched/spmd.py``) only rank 0
    reads the file; the other ranks receive the tensors over the data plane (one disk
    read per node, RCCL over xGMI into each rank's HBM)."""
    device = device or torch.device("cpu")
    if os.environ.get("CGS_SPMD_BCAST_LOAD", "1") != "0":
        from ..sched import spmd as _spmd
        ctx = _spmd.active()
        if ctx is not None and ctx.world > 1 and ctx.comm.enabled:
            return ctx.load_state_dict(path, device, return_metadata,
                                       lambda: _load_local(path, device, return_metadata))
    return _load_local(path, device, return_metadata)


def _load_local(path, device, return_metadata=False):
    _trace_read(path)
    meta = None
    if path.lower().endswith(".safetensors") or path.lower().endswith(".sft"):
        sd = _load_safetensors(path, device)
        if return_metadata:
            meta = read_metadata(path)
    else:
        pl = torch.load(path, map_location=device, weights_only=True)
        if isinstance(pl, dict) and "global_step" in pl:
            logging.debug("Global Step: %s", pl["global_step"])
        if isinstance(pl, dict) and "state_dict" in pl:
            sd = pl["state_dict"]
        else:
            sd = pl
    return (sd, meta) if return_metadata else sd


load_torch_file = load_state_dict


def save_state_dict(sd, path, metadata=None):
    """Write a safetensors file (C++ writer when built, else pure Python)."""
    rt = _native.load_runtime()
    tensors = {k: v.detach().contiguous().cpu() for k, v in sd.items()}
    if rt is not None and hasattr(rt, "save_safetensors"):
        items = [(k, _DT_INV[t.dtype], list(t.shape), t.view(torch.uint8).numpy().tobytes() if t.numel() else b"")
                 for k, t in tensors.items()]
        rt.save_safetensors(path, items, metadata or {})
        return
    header = {}
    off = 0
    blobs = []
    for k, t in tensors.items():
        b = t.view(torch.uint8).numpy().tobytes() if t.numel() else b""
        header[k] = {"dtype": _DT_INV[t.dtype], "shape": list(t.shape), "data_offsets": [off, off + len(b)]}
        off += len(b)
        blobs.append(b)
    if metadata:
        header["__metadata__"] = {str(k): str(v) for k, v in metadata.items()}
    hb = json.dumps(header, separators=(",", ":")).encode("utf-8")
    hb += b" " * ((8 - len(hb) % 8) % 8)
    with open(path, "wb") as f:
        f.write(struct.pack("<Q", len(hb)))
        f.write(hb)
        for b in blobs:
            f.write(b)


save_torch_file = save_state_dict


def calculate_parameters(sd, prefix=""):
    return sum(v.nelement() for k, v in sd.items() if k.startswith(prefix))


def weight_dtype(sd, prefix=""):
    dtypes = {}
    for k, v in sd.items():
        if k.startswith(prefix):
            dtypes[v.dtype] = dtypes.get(v.dtype, 0) + 1
    return max(dtypes, key=dtypes.get) if dtypes else None
