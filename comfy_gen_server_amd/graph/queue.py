"""Prompt queue + history (parity: ``execution.py:920-1044``; C07).

Thread-safe min-heap of (number, prompt_id, prompt, extra_data, outputs_to_execute); ``front``
submissions use negative numbers; in-memory history capped at MAXIMUM_HISTORY_SIZE; flags channel
for /free. Extra (SURVEY §5.4 'New'): an optional append-only JSONL journal so queued prompts and
history survive a restart (``journal_path``).
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
        self.queue = []
        self.currently_running = {}
        self.history = {}
        self.flags = {}
        self.journal_path = journal_path
        self.enqueue_time = {}
        server.prompt_queue = self
        if journal_path:
            self._replay_journal()

    # ---------------------------------------------------------------- journal
    def _journal(self, rec):
        if not self.journal_path:
            return
        try:
            with open(self.journal_path, "a") as f:
                f.write(json.dumps(rec, default=str) + "\n")
        except OSError:
            pass

    def _replay_journal(self):
        if not os.path.exists(self.journal_path):
            return
        pending = {}
        with open(self.journal_path) as f:
            for line in f:
                try:
                    rec = json.loads(line)
                except ValueError:
                    continue
                if rec.get("op") == "put":
                    pending[rec["item"][1]] = tuple(rec["item"])
                elif rec.get("op") in ("done", "delete"):
                    pending.pop(rec.get("prompt_id"), None)
                    if rec.get("op") == "done" and "history" in rec:
                        self.history[rec["prompt_id"]] = rec["history"]
        for item in pending.values():
            heapq.heappush(self.queue, item)

    # ---------------------------------------------------------------- queue ops
    def put(self, item):
        with self.mutex:
            heapq.heappush(self.queue, item)
            self.enqueue_time[item[1]] = time.time()
            self._journal({"op": "put", "item": list(item)})
            self.server.queue_updated()
            self.not_empty.notify()

    def get(self, timeout=None):
        with self.not_empty:
            while len(self.queue) == 0:
                self.not_empty.wait(timeout=timeout)
                if timeout is not None and len(self.queue) == 0:
                    return None
            item = heapq.heappop(self.queue)
            i = self.task_counter
            self.currently_running[i] = copy.deepcopy(item)
            self.task_counter += 1
            self.server.queue_updated()
            return item, i

    def task_done(self, item_id, outputs, status=None):
        with self.mutex:
            prompt = self.currently_running.pop(item_id)
            if len(self.history) > MAXIMUM_HISTORY_SIZE:
                self.history.pop(next(iter(self.history)))
            sd = copy.deepcopy(status._asdict()) if status is not None else None
            self.history[prompt[1]] = {"prompt": prompt, "outputs": copy.deepcopy(outputs), "status": sd}
            t0 = self.enqueue_time.pop(prompt[1], None)
            if t0 is not None:
                self.history[prompt[1]]["metrics"] = {"total_seconds": time.time() - t0}
            self._journal({"op": "done", "prompt_id": prompt[1],
                           "history": {"prompt": prompt, "outputs": outputs, "status": sd}})
            self.server.queue_updated()

    def get_current_queue(self):
        with self.mutex:
            return list(self.currently_running.values()), copy.deepcopy(self.queue)

    def get_tasks_remaining(self):
        with self.mutex:
            return len(self.queue) + len(self.currently_running)

    def wipe_queue(self):
        with self.mutex:
            for it in self.queue:
                self._journal({"op": "delete", "prompt_id": it[1]})
            self.queue = []
            self.server.queue_updated()

    def delete_queue_item(self, function):
        with self.mutex:
            for x in range(len(self.queue)):
                if function(self.queue[x]):
                    self._journal({"op": "delete", "prompt_id": self.queue[x][1]})
                    if len(self.queue) == 1:
                        self.wipe_queue()
                    else:
                        self.queue.pop(x)
                        heapq.heapify(self.queue)
                    self.server.queue_updated()
                    return True
        return False

    def get_history(self, prompt_id=None, max_items=None, offset=-1):
        with self.mutex:
            if prompt_id is None:
                out = {}
                if offset < 0 and max_items is not None:
                    offset = len(self.history) - max_items
                for i, k in enumerate(self.history):
                    if i >= offset:
                        out[k] = self.history[k]
                        if max_items is not None and len(out) >= max_items:
                            break
                return out
            if prompt_id in self.history:
                return {prompt_id: copy.deepcopy(self.history[prompt_id])}
            return {}

    def wipe_history(self):
        with self.mutex:
            self.history = {}

    def delete_history_item(self, id_to_delete):
        with self.mutex:
            self.history.pop(id_to_delete, None)

    def set_flag(self, name, data):
        with self.mutex:
            self.flags[name] = data
            self.not_empty.notify()

    def get_flags(self, reset=True):
        with self.mutex:
            if reset:
                r = self.flags
                self.flags = {}
                return r
            return self.flags.copy()
