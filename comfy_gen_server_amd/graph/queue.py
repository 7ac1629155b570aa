"""Prompt queue + history (C07; API parity with the reference ``PromptQueue``, ``execution.py:920-1044``).

State: a min-heap of pending items ``(number, prompt_id, prompt, extra_data, outputs_to_execute)``
(``front`` submissions carry negative numbers), the items currently executing keyed by their task id,
the bounded history (oldest entry evicted first) and the flags channel for ``/free``. The attribute
names (``queue``, ``currently_running``, ``history``, ``mutex``, ``not_empty``, ``flags``) are what
custom nodes and the API layer read, so they are kept.

Persistence: with ``journal_path`` every state change is one record of an append-only JSONL
journal, written by the same ``_mutate`` call that applies it; a restart replays the records through
``_mutate`` with journaling off, so the replayed state is by construction the state the records
describe: items that were queued or running and never finished come back queued, finished ones come
back as history, deleted / wiped ones stay gone.
"""
from __future__ import annotations

import copy
import heapq
import json
import os
import threading
import time
from typing import List, Literal, NamedTuple

MAXIMUM_HISTORY_SIZE = 10000


class PromptQueue:
    class ExecutionStatus(NamedTuple):
        status_str: Literal["success", "error"]
        completed: bool
        messages: List[str]

    def __init__(self, server, journal_path=None):
        self.server = server
        self.mutex = threading.RLock()
        self.not_empty = threading.Condition(self.mutex)
        self.task_counter = 0
        self.queue: list = []
        self.currently_running: dict = {}
        self.history: dict = {}
        self.flags: dict = {}
        self.enqueue_time: dict = {}
        self.journal_path = journal_path
        self._journaling = False
        server.prompt_queue = self
        if journal_path and os.path.exists(journal_path):
            with self.mutex:
                for rec in self._read_journal():
                    self._mutate(rec)
            with open(journal_path, "rb+") as f:     # a torn last line: end it, so new records start clean
                f.seek(0, os.SEEK_END)
                if f.tell() > 0:
                    f.seek(-1, os.SEEK_END)
                    if f.read(1) != b"\n":
                        f.write(b"\n")
        self._journaling = bool(journal_path)

    # ------------------------------------------------------------------ the one mutation point
    def _mutate(self, rec: dict):
        """Apply one state change (``rec["op"]``) and, when journaling, append it to the journal. Caller
        holds the mutex."""
        op, pid = rec["op"], rec.get("prompt_id")
        if op == "put":
            heapq.heappush(self.queue, tuple(rec["item"]))
        elif op == "done":
            self._drop_pending(pid)         # a replayed journal never saw this item's start
            if len(self.history) >= MAXIMUM_HISTORY_SIZE:
                self.history.pop(next(iter(self.history)))
            self.history[pid] = rec["history"]
        elif op == "delete":
            self._drop_pending(pid)
        elif op == "history_delete":
            self.history.pop(pid, None)
        elif op == "history_wipe":
            self.history = {}
        else:
            raise ValueError(f"unknown queue record {op!r}")
        if self._journaling:
            try:
                with open(self.journal_path, "a") as f:
                    f.write(json.dumps(rec, default=str) + "\n")
            except OSError:
                pass

    def _drop_pending(self, pid):
        keep = [it for it in self.queue if it[1] != pid]
        if len(keep) != len(self.queue):
            heapq.heapify(keep)
            self.queue = keep

    def _read_journal(self):
        with open(self.journal_path) as f:
            for line in f:
                try:
                    rec = json.loads(line)
                except ValueError:          # a torn last line (crash mid-write): everything before it counts
                    continue
                if isinstance(rec, dict) and "op" in rec:
                    yield rec

    # ------------------------------------------------------------------ queue
    def put(self, item):
        with self.mutex:
            self._mutate({"op": "put", "prompt_id": item[1], "item": list(item)})
            self.enqueue_time[item[1]] = time.time()
            self.server.queue_updated()
            self.not_empty.notify()

    def get(self, timeout=None):
        """Pop the next item (lowest number) -> (item, task id); None if ``timeout`` passes first. Starting a
        prompt is not journaled: after a crash a started, unfinished prompt runs again."""
        with self.not_empty:
            deadline = None if timeout is None else time.monotonic() + timeout
            while not self.queue:
                left = None if deadline is None else deadline - time.monotonic()
                if left is not None and left <= 0:
                    return None
                self.not_empty.wait(timeout=left)
            item = heapq.heappop(self.queue)
            task_id = self.task_counter
            self.task_counter += 1
            self.currently_running[task_id] = copy.deepcopy(item)
            self.server.queue_updated()
            return item, task_id

    def task_done(self, item_id, outputs, status=None):
        with self.mutex:
            item = self.currently_running.pop(item_id)
            pid = item[1]
            entry = {"prompt": item, "outputs": copy.deepcopy(outputs),
                     "status": copy.deepcopy(status._asdict()) if status is not None else None}
            self._mutate({"op": "done", "prompt_id": pid, "history": entry})
            t0 = self.enqueue_time.pop(pid, None)
            if t0 is not None:
                self.history[pid]["metrics"] = {"total_seconds": time.time() - t0}
            self.server.queue_updated()

    def get_current_queue(self):
        with self.mutex:
            return list(self.currently_running.values()), copy.deepcopy(self.queue)

    def get_tasks_remaining(self):
        with self.mutex:
            return len(self.queue) + len(self.currently_running)

    def wipe_queue(self):
        with self.mutex:
            for pid in [it[1] for it in self.queue]:
                self._mutate({"op": "delete", "prompt_id": pid})
            self.server.queue_updated()

    def delete_queue_item(self, function):
        """Remove the first pending item ``function`` accepts; True if one was removed."""
        with self.mutex:
            for it in self.queue:
                if function(it):
                    self._mutate({"op": "delete", "prompt_id": it[1]})
                    self.enqueue_time.pop(it[1], None)
                    self.server.queue_updated()
                    return True
        return False

    # ------------------------------------------------------------------ history
    def get_history(self, prompt_id=None, max_items=None, offset=-1):
        """One entry (``prompt_id``), or a window of the history in insertion order: from ``offset``
        (default: the last ``max_items`` entries), at most ``max_items`` of them."""
        with self.mutex:
            if prompt_id is not None:
                return {prompt_id: copy.deepcopy(self.history[prompt_id])} if prompt_id in self.history else {}
            keys = list(self.history)
            if offset < 0:
                offset = max(0, len(keys) - max_items) if max_items is not None else 0
            keys = keys[offset:]
            if max_items is not None:
                keys = keys[:max_items]
            return {k: self.history[k] for k in keys}

    def wipe_history(self):
        with self.mutex:
            self._mutate({"op": "history_wipe"})

    def delete_history_item(self, id_to_delete):
        with self.mutex:
            if id_to_delete in self.history:
                self._mutate({"op": "history_delete", "prompt_id": id_to_delete})

    # ------------------------------------------------------------------ /free flags
    def set_flag(self, name, data):
        with self.mutex:
            self.flags[name] = data
            self.not_empty.notify()

    def get_flags(self, reset=True):
        with self.mutex:
            if not reset:
                return self.flags.copy()
            out, self.flags = self.flags, {}
            return out
