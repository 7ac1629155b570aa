"""Measured per-shape kernel selection ("find" step) for the device op layer.

The first time an op sees a new problem key (op, shape, epilogue, dtype) on the GPU it times every
legal candidate — the hand-written HIP variants (GEMM v1/v3/v5, conv v2/v3/v5, flash attention) and,
where legal, the vendor library through ATen (hipBLASLt GEMM, SDPA) — with HIP events on the
current stream, and caches the winner. Later calls (and hipGraph capture) reuse the cached choice;
a key first seen *during* capture gets the default candidate (no timing inside a capture).

Parity: the reference picks one attention backend globally at import time
(``comfy/model_management.py:132-202``, ``attention.py:352-368``); here the choice is per shape and
measured, like MIOpen's find mode.

A measured table for MI355X ships with the package (``data/tune_mi355x.json``) and is loaded by
default, so a fresh box runs the recorded choices instead of re-tuning inside the first job (and
two boxes cannot drift apart through different timing-noise picks). Keys missing from it are
still tuned on first use.

Env:
  CGS_AUTOTUNE=0          disable (always the first/default candidate: the HIP kernel)
  CGS_TUNE_FILE=path      persist choices as JSON (loaded after the packaged table, rewritten on new
                          entries; the packaged table itself is never written)
  CGS_TUNE_DEFAULT=0      do not load the packaged table
  CGS_TUNE_REPS=n         timed repetitions per candidate (default 3)
  CGS_TUNE_DUMP=path      at exit, write every choice made in this process with its per-candidate ms
  CGS_TUNE_OVERRIDE=json  {key: choice} merged over the loaded tables (A/B runs of one kernel choice)
"""
from __future__ import annotations

import json
import os
import threading

import torch

DEFAULT_TABLE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data",
                             "tune_mi355x.json")
_cache: dict[str, str] = {}
_lock = threading.Lock()
_loaded = False
_timings: dict[str, dict[str, float]] = {}


def enabled() -> bool:
    return os.environ.get("CGS_AUTOTUNE", "1") != "0"


def _key(parts) -> str:
    return "|".join(str(p) for p in parts)


def _load():
    global _loaded
    if _loaded:
        return
    _loaded = True
    paths = []
    if os.environ.get("CGS_TUNE_DEFAULT", "1") != "0":
        paths.append(DEFAULT_TABLE)
    if os.environ.get("CGS_TUNE_FILE"):
        paths.append(os.environ["CGS_TUNE_FILE"])
    for path in paths:
        if not os.path.exists(path):
            continue
        try:
            with open(path) as f:
                data = json.load(f)
            if isinstance(data, dict):
                _cache.update({str(k): str(v) for k, v in data.items() if not str(k).startswith("_")})
        except (OSError, ValueError):
            pass


def _save():
    path = os.environ.get("CGS_TUNE_FILE")
    if not path:
        return
    tmp = path + ".tmp"
    try:
        with open(tmp, "w") as f:
            json.dump(_cache, f, indent=0, sort_keys=True)
        os.replace(tmp, path)
    except OSError:
        pass


def _dump_at_exit():
    path = os.environ.get("CGS_TUNE_DUMP")
    if not path:
        return
    try:
        with open(path, "w") as f:
            json.dump(table(), f, indent=1, sort_keys=True)
    except OSError:
        pass


if os.environ.get("CGS_TUNE_DUMP"):
    import atexit
    atexit.register(_dump_at_exit)


def _capturing() -> bool:
    try:
        return torch.cuda.is_current_stream_capturing()
    except Exception:
        return False


_ov = ("", {})


def _override(key):
    """CGS_TUNE_OVERRIDE (re-read when the variable changes: ab_bench flips it between jobs)."""
    global _ov
    src = os.environ.get("CGS_TUNE_OVERRIDE", "")
    if not src:
        return None
    if src != _ov[0]:
        try:
            txt = open(src[1:]).read() if src.startswith("@") else src     # "@file.json" or inline JSON
            _ov = (src, {str(k): str(v) for k, v in json.loads(txt).items()})
        except (OSError, ValueError):
            _ov = (src, {})
    return _ov[1].get(key)


def choose(key_parts, candidates, default: str | None = None) -> str:
    """Return the name of the fastest candidate for this key.

    ``candidates``: list of (name, fn) where fn() runs the op once on the current stream.
    """
    names = [n for n, _ in candidates]
    if default is None:
        default = names[0]
    if not enabled():               # explicit opt-out: the default kernel, table entries included
        return default
    key = _key(key_parts)
    ov = _override(key)
    if ov is not None and ov in names:
        return ov
    with _lock:
        _load()
        hit = _cache.get(key)
    if hit is not None and hit in names:
        return hit
    if len(candidates) == 1 or _capturing():
        return default
    reps = max(1, int(os.environ.get("CGS_TUNE_REPS", "3")))
    stream = torch.cuda.current_stream()
    times = {}
    for name, fn in candidates:
        try:
            fn()                      # warm (JIT / library heuristics / allocator)
            stream.synchronize()
            s = torch.cuda.Event(enable_timing=True)
            e = torch.cuda.Event(enable_timing=True)
            s.record(stream)
            for _ in range(reps):
                fn()
            e.record(stream)
            e.synchronize()
            times[name] = s.elapsed_time(e) / reps
        except Exception:            # an illegal candidate simply drops out
            continue
    best = min(times, key=times.get) if times else default
    with _lock:
        _cache[key] = best
        _timings[key] = times
        _save()
    return best


def table() -> dict:
    """Choices made so far (key -> candidate) and their measured ms."""
    with _lock:
        return {k: {"choice": v, "ms": _timings.get(k, {})} for k, v in _cache.items()}


def reset():
    with _lock:
        _cache.clear()
        _timings.clear()
