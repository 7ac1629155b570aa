"""Content hashing for ``IS_CHANGED`` / proto ``WorkflowFile.blake3_hash`` (parity: ``nodes.py:9,
586-600, 1895-1909``; SURVEY §2.3 blake3 row). BLAKE3 comes from the in-tree C++ runtime
(``csrc/runtime/blake3.cpp``); without the runtime a SHA-256 digest (prefixed ``sha256:``) keeps
cache invalidation correct."""
from __future__ import annotations

import hashlib

from .. import _native


def blake3_hex(data: bytes) -> str | None:
    rt = _native.load_runtime()
    if rt is not None and hasattr(rt, "blake3_hex"):
        return rt.blake3_hex(data)
    return None


def file_digest(path: str) -> str:
    rt = _native.load_runtime()
    if rt is not None and hasattr(rt, "blake3_file_hex"):
        return rt.blake3_file_hex(path)
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return "sha256:" + h.hexdigest()


def bytes_digest(data: bytes) -> str:
    b = blake3_hex(data)
    return b if b is not None else "sha256:" + hashlib.sha256(data).hexdigest()
