"""Shared output map (the fork's Yjs ``workflows`` map: ``server.py:144-145, 825-832``,
``execution.py:334-345``; C02).

The reference writes each ``prompt["outputs"][key]`` result into a y_py ``YMap`` and broadcasts the
encoded doc over WS — broken at runtime (``ws.send`` does not exist on aiohttp, ``json.dumps(bytes)``
raises). Here the map is a last-writer-wins register map with a Lamport clock per
key; ``encode_update`` produces a JSON delta ``{"clock": n, "entries": {key: [clock, value]}}`` that
clients merge by per-key clock (the same convergence rule a Yjs map gives single-writer keys).
y_py is not available in this image, so the binary lib0 encoding is not produced.
"""
from __future__ import annotations

import threading


class OutputMap:
    def __init__(self, server=None):
        self._lock = threading.Lock()
        self._clock = 0
        self._entries = {}
        self._dirty = set()
        self.server = server

    def set(self, key, value):
        with self._lock:
            self._clock += 1
            self._entries[key] = (self._clock, value)
            self._dirty.add(key)

    def get(self, key, default=None):
        with self._lock:
            e = self._entries.get(key)
            return default if e is None else e[1]

    def to_json(self):
        with self._lock:
            return {k: v[1] for k, v in self._entries.items()}

    def encode_update(self, full=False):
        with self._lock:
            keys = list(self._entries) if full else list(self._dirty)
            self._dirty.clear()
            return {"clock": self._clock, "entries": {k: list(self._entries[k]) for k in keys}}

    def apply_update(self, upd):
        with self._lock:
            for k, (c, v) in upd.get("entries", {}).items():
                cur = self._entries.get(k)
                if cur is None or c > cur[0]:
                    self._entries[k] = (c, v)
            self._clock = max(self._clock, upd.get("clock", 0))
