"""Tracing, metrics and fault injection (SURVEY §5.1, §5.3, §5.5 "New" rows).

* **Markers.** ``span(name)`` opens a ``torch.profiler.record_function`` range (visible in the
  Perfetto trace below) and a ROCTx range (``torch.cuda.nvtx`` is the roctx shim on ROCm builds;
  ``rocprofv3 --marker-trace`` shows it). The executor wraps every node, the sampler every step.
* **Per-prompt traces.** ``--profile-dir DIR`` (or ``CGS_PROFILE_DIR``): the worker runs each prompt
  under ``torch.profiler`` (CPU + GPU activity) and writes ``DIR/<prompt_id>.json`` — a Chrome /
  Perfetto trace with the node and step ranges on top of the HIP kernels.
* **Counters.** sampler steps / step wall time, per-node-class execution time, images produced,
  HBM allocated / reserved; exported through ``/metrics`` (Prometheus text) and ``/system_stats``.
* **Fault injection.** ``CGS_FAULT`` = comma list of ``node:<ClassType>`` (raise inside that
  node), ``oom:<ClassType>`` (raise an out-of-memory error there), ``step:<n>`` (raise at sampler
  step n), ``rank_exit:<rank>`` (that DP rank exits at its next heartbeat), ``node_exit:<ClassType>``
  (the process dies inside that node). ``<key>@<rank>`` limits an entry to one rank of a multi-rank
  job (``RANK``). Each entry fires once per process unless suffixed ``!`` (always). Used by the
  failure-handling tests.
"""
from __future__ import annotations

import contextlib
import json
import logging
import os
import threading
import time
from collections import defaultdict

import torch

_lock = threading.Lock()
_counters: dict = defaultdict(float)
_node_seconds: dict = defaultdict(float)
_node_calls: dict = defaultdict(int)
_last_step_s = 0.0


# ----------------------------------------------------------------------------------------------
# markers
# ----------------------------------------------------------------------------------------------
def _roctx_push(name):
    try:
        if torch.cuda.is_available():
            torch.cuda.nvtx.range_push(name)
            return True
    except Exception:
        pass
    return False


def _roctx_pop():
    try:
        torch.cuda.nvtx.range_pop()
    except Exception:
        pass


@contextlib.contextmanager
def span(name: str):
    pushed = _roctx_push(name)
    try:
        with torch.profiler.record_function(name):
            yield
    finally:
        if pushed:
            _roctx_pop()


# ----------------------------------------------------------------------------------------------
# counters
# ----------------------------------------------------------------------------------------------
def record_node(class_type: str, seconds: float):
    with _lock:
        _node_seconds[class_type] += seconds
        _node_calls[class_type] += 1


def record_step(seconds: float):
    global _last_step_s
    with _lock:
        _counters["sampler_steps_total"] += 1
        _counters["sampler_step_seconds_total"] += seconds
        _last_step_s = seconds


def add(name: str, value: float = 1.0):
    with _lock:
        _counters[name] += value


def step_timer(callback=None):
    """Wrap a sampler callback ``cb(step, x0, x, total)``: records the wall time between steps
    and opens a ``sampler_step`` marker per step; fault site ``step:<n>``."""
    state = {"t": time.perf_counter()}

    def cb(step, x0, x, total):
        now = time.perf_counter()
        record_step(now - state["t"])
        state["t"] = now
        maybe_fault("step", str(step))
        if callback is not None:
            return callback(step, x0, x, total)
    return cb


def snapshot() -> dict:
    with _lock:
        out = dict(_counters)
        steps = out.get("sampler_steps_total", 0.0)
        out["sampler_step_ms_avg"] = 1e3 * out.get("sampler_step_seconds_total", 0.0) / steps if steps else 0.0
        out["sampler_step_ms_last"] = 1e3 * _last_step_s
        nodes = {k: {"seconds": _node_seconds[k], "calls": _node_calls[k]} for k in _node_seconds}
    if torch.cuda.is_available():
        try:
            out["hbm_allocated_bytes"] = float(torch.cuda.memory_allocated())
            out["hbm_reserved_bytes"] = float(torch.cuda.memory_reserved())
        except Exception:
            pass
    out["nodes"] = nodes
    return out


def prometheus_lines(prefix: str = "cgs_") -> list:
    snap = snapshot()
    lines = []
    for k, v in snap.items():
        if k == "nodes":
            continue
        kind = "counter" if k.endswith("_total") else "gauge"
        lines += [f"# TYPE {prefix}{k} {kind}", f"{prefix}{k} {v}"]
    if snap["nodes"]:
        lines.append(f"# TYPE {prefix}node_seconds_total counter")
        for cls, d in sorted(snap["nodes"].items()):
            lines.append(f'{prefix}node_seconds_total{{class_type="{cls}"}} {d["seconds"]}')
        lines.append(f"# TYPE {prefix}node_calls_total counter")
        for cls, d in sorted(snap["nodes"].items()):
            lines.append(f'{prefix}node_calls_total{{class_type="{cls}"}} {d["calls"]}')
    return lines


# ----------------------------------------------------------------------------------------------
# per-prompt profiler traces
# ----------------------------------------------------------------------------------------------
def profile_dir():
    return os.environ.get("CGS_PROFILE_DIR") or None


@contextlib.contextmanager
def maybe_profile(prompt_id: str):
    d = profile_dir()
    if not d:
        yield None
        return
    os.makedirs(d, exist_ok=True)
    acts = [torch.profiler.ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(torch.profiler.ProfilerActivity.CUDA)
    with torch.profiler.profile(activities=acts, record_shapes=False) as prof:
        with span(f"prompt:{prompt_id}"):
            yield prof
    path = os.path.join(d, f"{prompt_id}.json")
    try:
        prof.export_chrome_trace(path)
        logging.info("profile trace written to %s", path)
    except Exception as e:   # trace export must never fail a prompt
        logging.warning("profile export failed: %s", e)


# ----------------------------------------------------------------------------------------------
# structured logs
# ----------------------------------------------------------------------------------------------
class JsonFormatter(logging.Formatter):
    def format(self, record):
        d = {"ts": round(record.created, 3), "level": record.levelname, "logger": record.name,
             "msg": record.getMessage()}
        if record.exc_info:
            d["exc"] = self.formatException(record.exc_info)
        return json.dumps(d)


def use_json_logs(level=logging.INFO):
    h = logging.StreamHandler()
    h.setFormatter(JsonFormatter())
    root = logging.getLogger()
    root.handlers = [h]
    root.setLevel(level)


# ----------------------------------------------------------------------------------------------
# fault injection
# ----------------------------------------------------------------------------------------------
class InjectedFault(RuntimeError):
    pass


_fired: set = set()


def _faults():
    spec = os.environ.get("CGS_FAULT", "")
    out = []
    for item in spec.split(","):
        item = item.strip()
        if ":" in item:
            kind, _, arg = item.partition(":")
            always = arg.endswith("!")
            out.append((kind, arg.rstrip("!"), always, item))
    return out


def maybe_fault(site: str, key: str):
    """Raise / exit if ``CGS_FAULT`` names this (site, key)."""
    if "CGS_FAULT" not in os.environ:
        return
    for kind, arg, always, item in _faults():
        if "@" in arg:   # "<key>@<rank>": only on that rank of a multi-rank job (RANK env)
            arg, _, on_rank = arg.partition("@")
            if os.environ.get("RANK", "0") != on_rank:
                continue
        if arg != key:
            continue
        if site == "node" and kind == "node_exit":     # the process dies inside the node (lost rank)
            logging.error("injected process exit in node %s", key)
            os._exit(17)
        if not always and item in _fired:
            continue
        if site == "node" and kind == "node":
            _fired.add(item)
            raise InjectedFault(f"injected fault in node {key}")
        if site in ("node", "vae") and kind == "oom":
            _fired.add(item)
            raise torch.cuda.OutOfMemoryError(f"injected out-of-memory in node {key}")
        if site == "step" and kind == "step":
            _fired.add(item)
            raise InjectedFault(f"injected fault at sampler step {key}")
        if site == "teardown" and kind == "teardown_hang":    # a process-group teardown that never returns
            _fired.add(item)
            logging.error("injected hang in the process-group teardown (rank %s)", key)
            time.sleep(3600)
        if site == "rank" and kind == "rank_exit":
            _fired.add(item)
            logging.error("injected rank exit (rank %s)", key)
            os._exit(17)
