"""HBM weight arena (C27; SURVEY §7.1 runtime/): every resident model's parameters and buffers live
in ONE device slab per GPU, placed by the C++ offset allocator ``_cgs_runtime.Arena`` (best fit,
coalescing free list, 256-B aligned blocks -- csrc/runtime/arena.cpp).

Why a slab: 288 GB of HBM holds several SDXL-class pipelines at once; with per-tensor caching-
allocator blocks, weights interleave with activation blocks of every resolution the server has
seen, and evicting a model leaves holes the activation pools cannot reuse. The slab keeps weights
contiguous, makes residency accounting exact (``stats()``), and eviction / reload of a model is a
block free / best-fit placement without touching the activation pools or the hipGraph pools.

On by default on a GPU with at least 128 GB of HBM (a 48 GiB slab, allocated when the first model
is placed); ``--weight-arena-gb N`` / env ``CGS_WEIGHT_ARENA_GB`` sets the size, 0 disables.
``ModelPatcher.patch_model`` places modules here instead of ``module.to(device)`` (a model that does
not fit falls back to the caching allocator), and ``unpatch_model`` evicts them.
"""
from __future__ import annotations

import os
import threading

import torch

from .. import _native


class ArenaFull(RuntimeError):
    pass


class _PyArena:
    """Same interface as the C++ allocator (used only when _cgs_runtime is not built)."""

    def __init__(self, capacity, align=256):
        self.align = align
        self.cap = capacity - capacity % align
        self.free_list = [(0, self.cap)]
        self.used = {}
        self.peak = 0

    def alloc(self, n):
        need = (max(n, 1) + self.align - 1) // self.align * self.align
        fits = [(s, o) for o, s in self.free_list if s >= need]
        if not fits:
            return -1
        s, o = min(fits)
        self.free_list.remove((o, s))
        if s > need:
            self.free_list.append((o + need, s - need))
        self.used[o] = need
        self.peak = max(self.peak, sum(self.used.values()))
        return o

    def free(self, o):
        if o not in self.used:
            return False
        size = self.used.pop(o)
        blocks = sorted(self.free_list + [(o, size)])
        merged = []
        for bo, bs in blocks:
            if merged and merged[-1][0] + merged[-1][1] == bo:
                merged[-1] = (merged[-1][0], merged[-1][1] + bs)
            else:
                merged.append((bo, bs))
        self.free_list = merged
        return True

    def stats(self):
        return {"capacity": self.cap, "used": sum(self.used.values()), "peak": self.peak,
                "largest_free": max((s for _, s in self.free_list), default=0),
                "free_blocks": len(self.free_list), "live_blocks": len(self.used)}


class WeightArena:
    def __init__(self, capacity_bytes: int, device, align: int = 256):
        rt = _native.load_runtime()
        self.alloc = rt.Arena(int(capacity_bytes), align) if rt is not None and hasattr(rt, "Arena") \
            else _PyArena(int(capacity_bytes), align)
        self.device = torch.device(device)
        self.slab = torch.empty(int(capacity_bytes), dtype=torch.uint8, device=self.device)
        self.base = self.slab.data_ptr()
        self.blocks: dict[int, dict[str, int]] = {}      # id(module) -> {tensor name: offset}
        self.lock = threading.Lock()

    def owns(self, t: torch.Tensor) -> bool:
        return t.device == self.device and self.base <= t.data_ptr() < self.base + self.slab.numel()

    def _view(self, off: int, t: torch.Tensor) -> torch.Tensor:
        """A contiguous ``t``-shaped tensor on the slab's storage at byte ``off``, created in the same
        inference mode as ``t``: ``t.data = view`` with mismatched inference-ness leaves a tensor
        that no view op accepts ("Inference tensors do not track version counter")."""
        es = t.element_size()
        stride, acc = [], 1
        for d in reversed(t.shape):
            stride.append(acc)
            acc *= max(int(d), 1)
        with torch.inference_mode(t.is_inference()):
            return torch.empty(0, dtype=t.dtype, device=self.device).set_(
                self.slab.untyped_storage(), off // es, tuple(t.shape), tuple(reversed(stride)))

    def place_module(self, module: torch.nn.Module) -> int:
        """Move every parameter / buffer of ``module`` into the slab (shared tensors once); raises
        ArenaFull (after undoing this call's placements) when it does not fit."""
        placed = 0
        with self.lock:
            table = self.blocks.setdefault(id(module), {})
            seen: dict[int, torch.Tensor] = {}
            new = []          # (name, tensor, original data) of blocks allocated by this call
            tied = []         # (tensor, original data) of tied weights redirected onto those blocks
            try:
                for name, t in list(module.named_parameters(recurse=True)) + list(module.named_buffers(recurse=True)):
                    if t is None or name in table:
                        continue
                    key = t.data_ptr() if t.numel() else id(t)
                    if key in seen:                         # tied weights: one block, same view
                        tied.append((t, t.data))
                        t.data = seen[key]
                        continue
                    nbytes = t.numel() * t.element_size()
                    off = self.alloc.alloc(nbytes)
                    if off < 0:
                        raise ArenaFull(f"weight arena full: {nbytes} B for {name} ({self.stats()})")
                    v = self._view(off, t)
                    with torch.inference_mode(t.is_inference()):
                        v.copy_(t.data)
                    seen[key] = v
                    new.append((name, t, t.data))
                    t.data = v
                    table[name] = off
                    placed += nbytes
            except ArenaFull:
                for t, orig in tied:                       # never leave a view of a freed block behind
                    t.data = orig
                for name, t, orig in new:
                    t.data = orig
                    self.alloc.free(table.pop(name))
                raise
        return placed

    def evict_module(self, module: torch.nn.Module, device_to="cpu") -> int:
        """Copy the module's tensors out to ``device_to`` and free their blocks."""
        freed = 0
        with self.lock:
            table = self.blocks.pop(id(module), {})
            for name, t in list(module.named_parameters(recurse=True)) + list(module.named_buffers(recurse=True)):
                if t is not None and self.owns(t):
                    with torch.inference_mode(t.is_inference()):
                        t.data = t.data.to(device_to, copy=True)
            for off in table.values():
                self.alloc.free(off)
                freed += 1
        return freed

    def stats(self) -> dict:
        return dict(self.alloc.stats())


_ARENAS: dict = {}
_LOCK = threading.Lock()


DEFAULT_GB = 48.0


def configured_gb(device) -> float:
    """Slab size for ``device``: CGS_WEIGHT_ARENA_GB, else DEFAULT_GB on >= 128 GB devices, else 0."""
    v = os.environ.get("CGS_WEIGHT_ARENA_GB", "auto") or "auto"
    if v != "auto":
        return float(v)
    try:
        total = torch.cuda.get_device_properties(device).total_memory
    except Exception:
        return 0.0
    return DEFAULT_GB if total >= (128 << 30) else 0.0


def get(device) -> WeightArena | None:
    """The arena of ``device`` when enabled, created on first use."""
    device = torch.device(device)
    if device.type != "cuda":
        return None
    gb = configured_gb(device)
    if gb <= 0:
        return None
    key = device.index if device.index is not None else torch.cuda.current_device()
    with _LOCK:
        a = _ARENAS.get(key)
        if a is None:
            a = _ARENAS[key] = WeightArena(int(gb * (1 << 30)), torch.device("cuda", key))
        return a
