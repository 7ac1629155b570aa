"""Rank-0 front end + per-GPU workers: one ``/prompt`` API for the whole node.

The reference serves a prompt on one process and one GPU (``main.py:93-146`` worker thread ->
``execution.py:526``). Here ``python -m comfy_gen_server_amd.main --gpus N`` starts N ranks (one process
per GPU, ``torch.distributed`` over RCCL/xGMI for tensors, Gloo for host control). Rank 0 runs the
HTTP/WS server, the prompt queue and this ``Coordinator``; ranks 1..N-1 run ``worker_main``.

Per queued prompt the coordinator picks a mode (``choose_mode``):

* ``spmd`` -- the prompt's latent batch is at least the number of live ranks: every rank executes the
  graph, the samplers and decoders split the batch by global image index (``spmd.py``), rank 0 writes
  the outputs. A batch-64 prompt uses the whole node;
* ``single`` -- the prompt runs whole on ONE idle rank (rank 0 included). Independent prompts run
  concurrently on different GPUs, so N small prompts keep N GPUs busy.

Transport: JSON messages over ``multiprocessing.connection`` (authenticated local socket) -- run
requests and interrupts down, WS events and completions up. Rank 0 forwards a worker's events to the
submitting client (``sid``): JSON events as they are; binary frames (latent previews, ``SaveImageWebsocket``
images) encoded on the worker and shipped as ``op: "binary"`` (base64 of the frame payload); writes to the
Yjs ``outputs`` map as ``op: "yjs"`` / ``"yjs_flush"``, applied to rank 0's map and broadcast from there
(reference ``main.py:152-160``, ``server.py:754-791`` / ``:825-832``, ``execution.py:334-345``).

Ranks keep one executor for single prompts (its own cross-prompt cache) and one per SPMD rank prefix
[0, k) (k = 2..N): a prefix's executor only sees that prefix's prompts, so its caches stay identical on
its members and they all reach the same collectives. A batch b < N runs SPMD on the prefix of size b while
the other ranks keep serving single prompts; an SPMD prompt waits only for its own ranks.

Scheduling: the dispatch loop never runs a prompt itself. A single prompt goes to an idle rank (workers
first); an SPMD prompt reserves its prefix in queue order and runs on its own thread once those ranks are
idle, while the loop keeps handing single prompts to the ranks outside the prefix (reserved ranks take
none, so a waiting SPMD prompt is not starved).

Elastic: a worker whose connection drops is marked dead -- its single prompt re-runs on a survivor, an
SPMD prompt it was part of re-runs on the prefix below it (shards re-queued to the surviving GPUs,
SURVEY §5.3) -- and a replacement process is started. Once it has connected and no rank is busy, a
re-rendezvous runs on its own thread, all or nothing: every rank leaves the broken process group (bounded:
a worker whose teardown hangs exits and is replaced), and only if all left cleanly does every rank join
generation + 1. Until it succeeds prompts run single (any live rank). Nothing re-execs a process that
touched the GPU.
"""
from __future__ import annotations

import json
import logging
import os
import queue
import secrets
import socket
import subprocess
import sys
import threading
import time
from multiprocessing.connection import Client, Listener

SAMPLER_TYPES = ("KSampler", "KSamplerAdvanced")
GC_INTERVAL_S = 10.0          # the reference worker's model cleanup + GC cadence (main.py:139-146)
MAX_RETRIES = 1               # re-runs of a prompt whose rank died under it
SPMD_REPORT_TIMEOUT_S = 30.0  # rank 0 waits this long for the workers' reports of a finished SPMD prompt


def _housekeeping():
    """Between prompts on every rank: drop models nobody holds, collect, return cached HBM."""
    import gc
    from ..runtime import device as dm
    dm.cleanup_models()
    gc.collect()
    dm.soft_empty_cache()


def _default(o):
    try:
        import torch
        if torch.is_tensor(o):
            return o.tolist() if o.numel() <= 64 else f"tensor{tuple(o.shape)}"
    except Exception:  # pragma: no cover
        pass
    return str(o)


def send_msg(conn, obj, lock=None):
    data = json.dumps(obj, default=_default).encode()
    if lock is None:
        conn.send_bytes(data)
    else:
        with lock:
            conn.send_bytes(data)


def recv_msg(conn):
    return json.loads(conn.recv_bytes().decode())


def prompt_batch(prompt: dict) -> int:
    """Image batch at the samplers' latent inputs, traced upstream through the graph: latent / image
    constructors (``batch_size``), repeats (``amount`` x upstream), batch concatenations (sum of both
    inputs), batch slices (``length``), and for every other node (VAEEncode / inpaint encoders, upscales,
    masks, ...) the largest batch among its linked inputs. A node this cannot see through counts as 1:
    an under-estimate only costs parallelism (the prompt runs on one rank), never correctness."""
    memo: dict = {}

    def batch_of(nid, depth=0):
        if nid in memo:
            return memo[nid]
        node = prompt.get(nid)
        if not isinstance(node, dict) or depth > 64:
            return 1
        memo[nid] = 1       # cycle guard
        ct, inputs = node.get("class_type", ""), node.get("inputs", {})
        links = {k: v[0] for k, v in inputs.items() if isinstance(v, list) and len(v) == 2}
        up = [batch_of(v, depth + 1) for v in links.values()]
        if isinstance(inputs.get("batch_size"), int):
            b = inputs["batch_size"]
        elif ct.startswith("Repeat") and isinstance(inputs.get("amount"), int):
            b = inputs["amount"] * max(up, default=1)
        elif ct.endswith("FromBatch") and isinstance(inputs.get("length"), int):
            b = inputs["length"]
        elif ct in ("LatentBatch", "ImageBatch"):
            b = sum(up) if up else 1
        else:
            b = max(up, default=1)
        memo[nid] = max(1, b)
        return memo[nid]

    best = 1
    for node in prompt.values():
        if isinstance(node, dict) and node.get("class_type") in SAMPLER_TYPES:
            src = node.get("inputs", {}).get("latent_image")
            if isinstance(src, list) and len(src) == 2:
                best = max(best, batch_of(src[0]))
    return best


def choose_mode(prompt: dict, extra_data: dict | None, world: int, latency_default: bool = False,
                subsets: bool = False) -> str:
    """``spmd`` when the batch covers every live rank (``subsets``: at least two ranks -- the coordinator
    then runs it on a rank prefix) and the prompt samples; ``latency`` for a smaller batch when the server
    runs with ``--latency-mode`` (one image sooner instead of more images per second); else ``single``.
    ``extra_data["dp"]`` (``"spmd"`` / ``"latency"`` / ``"single"``) overrides."""
    want = (extra_data or {}).get("dp", "auto")
    if world <= 1:
        return "single"
    if want in ("spmd", "single", "latency"):
        return want
    has_sampler = any(isinstance(n, dict) and n.get("class_type") in SAMPLER_TYPES for n in prompt.values())
    if not has_sampler:
        return "single"
    b = prompt_batch(prompt)
    if b >= world:
        return "spmd"
    if latency_default:
        return "latency"
    return "spmd" if subsets and b >= 2 else "single"


# ------------------------------------------------------------------------------------------------
# worker side
# ------------------------------------------------------------------------------------------------
PREVIEW_IMAGE, UNENCODED_PREVIEW_IMAGE = 1, 2     # api.server.BinaryEventTypes (the WS binary frame types)


def encode_preview(image_data) -> bytes:
    """(image type, PIL image, max size) -> the PREVIEW_IMAGE payload: a big-endian image-type word (1 JPEG,
    2 PNG) and the encoded image, as ``PromptServer.send_image`` frames it."""
    import io
    import struct
    from PIL import Image
    image_type, image, max_size = image_data
    if max_size is not None:
        image = image.copy()
        image.thumbnail((max_size, max_size), Image.LANCZOS if hasattr(Image, "LANCZOS") else Image.Resampling.LANCZOS)
    bio = io.BytesIO()
    bio.write(struct.pack(">I", 2 if image_type == "PNG" else 1))
    image.save(bio, format=image_type, quality=95, compress_level=1)
    return bio.getvalue()


class RemoteOutputMap:
    """Worker-side stand-in for the server's Yjs ``outputs`` map: writes go up to rank 0, whose map holds
    the node's state and broadcasts it (``yjs_flush``)."""

    def __init__(self, server):
        self.server = server

    def set(self, key, value):
        self.server._up({"op": "yjs", "key": key, "value": value})


class RemoteServer:
    """Worker-side stand-in for ``PromptServer``: WS events (JSON and binary) and Yjs writes go up to rank 0."""

    def __init__(self, conn, lock):
        self.conn, self.lock = conn, lock
        self.client_id = None
        self.last_node_id = None
        self.last_prompt_id = None
        self.metrics = {}
        self.output_map = RemoteOutputMap(self)

    def _up(self, msg):
        try:
            send_msg(self.conn, msg, self.lock)
        except (OSError, EOFError):
            pass

    def send_sync(self, event, data, sid=None):
        if isinstance(event, str):
            self._up({"op": "event", "event": event, "data": data, "sid": sid})
            return
        import base64
        if event == UNENCODED_PREVIEW_IMAGE:    # encoded here: the worker's CPU, not rank 0's, pays for it
            event, data = PREVIEW_IMAGE, encode_preview(data)
        if isinstance(data, (bytes, bytearray)):
            self._up({"op": "binary", "event": int(event), "data": base64.b64encode(bytes(data)).decode("ascii"),
                      "sid": sid})

    def queue_updated(self):
        pass

    def broadcast_yjs_updates(self):
        self._up({"op": "yjs_flush"})


def _forward_progress(server):
    from ..runtime import device as dm
    from ..utils import progress

    def hook(value, total, preview_image):
        dm.throw_exception_if_processing_interrupted()
        server.send_sync("progress", {"value": value, "max": total, "prompt_id": server.last_prompt_id,
                                      "node": server.last_node_id}, server.client_id)
        if preview_image is not None:
            server.send_sync(UNENCODED_PREVIEW_IMAGE, preview_image, server.client_id)
    progress.set_progress_bar_global_hook(hook)


def _spmd_sizes(world: int):
    """Rank prefixes that get their own SPMD groups: every size 2..world (``CGS_SPMD_PREFIXES=pow2``: the powers
    of two below the node size, and the node). A batch b < world runs on the prefix of size b (SPMD over a
    subset: a batch of 3 on an 8-GPU node uses 3 ranks, not 2) and leaves the other ranks to single prompts.
    Each prefix keeps its own executor (identical caches on its members), i.e. its own cached model copies
    once used: with 288 GB of HBM per MI355X, seven SDXL-sized copies (~7 GB each) fit beside the working set."""
    if world <= 1:
        return []
    if os.environ.get("CGS_SPMD_PREFIXES", "all") == "pow2":
        out, k = [], 2
        while k < world:
            out.append(k)
            k *= 2
        return out + [world]
    return list(range(2, world + 1))


def worker_main(comm, address, authkey: bytes, respawned: bool = False):
    """Rank >= 1: execute what rank 0 sends until it says stop. A respawned rank (replacing one that died)
    connects first and joins the process group at the coordinator's next re-rendezvous (``regroup``)."""
    from ..graph.executor import PromptExecutor
    from ..runtime import device as dm
    from ..utils import imageio
    from . import spmd
    conn = None
    for _ in range(600):
        try:
            conn = Client(tuple(address), authkey=authkey)
            break
        except (ConnectionRefusedError, OSError):
            time.sleep(0.1)
    if conn is None:
        raise RuntimeError(f"rank {comm.rank}: cannot reach the coordinator at {address}")
    lock = threading.Lock()
    send_msg(conn, {"op": "hello", "rank": comm.rank, "respawned": respawned}, lock)
    server = RemoteServer(conn, lock)
    _forward_progress(server)
    ctxs: dict = {}                  # k -> SPMD context of the rank prefix [0, k)
    ex_spmd: dict = {}               # k -> executor that only sees that prefix's SPMD prompts

    def build():
        comm.build_subsets(_spmd_sizes(comm.world))
        ctxs.clear()
        ex_spmd.clear()
        for k, c in sorted(comm.subsets.items()):
            ctxs[k] = spmd.SPMD(c)   # collective for the whole node (latency-mode groups)
    if not respawned:
        build()
    ex_single = PromptExecutor(server)
    inbox: queue.Queue = queue.Queue()

    def reader():
        while True:
            try:
                m = recv_msg(conn)
            except (EOFError, OSError):
                inbox.put({"op": "stop"})
                return
            if m.get("op") == "interrupt":
                dm.interrupt_current_processing(True)
            else:
                inbox.put(m)
    threading.Thread(target=reader, daemon=True).start()
    last_gc, need_gc = time.perf_counter(), False
    while True:
        try:
            m = inbox.get(timeout=1.0)
        except queue.Empty:
            m = {"op": "idle"}
        op = m.get("op")
        if op == "stop":
            break
        if op == "exit":              # the coordinator replaces this process (its group state is unknown)
            break
        if op == "teardown":          # re-rendezvous, phase 1: leave the broken process group (bounded)
            ctxs.clear()
            ex_spmd.clear()
            ok = comm.leave(float(m.get("timeout", TEARDOWN_TIMEOUT_S)))
            send_msg(conn, {"op": "torn_down", "rank": comm.rank, "gen": int(m["gen"]), "ok": ok}, lock)
            if not ok:                # a teardown that hangs: this process is replaced by a fresh child
                logging.error("rank %d: process-group teardown hung; exiting for a replacement", comm.rank)
                try:
                    conn.close()
                finally:
                    os._exit(75)
            continue
        if op == "join":              # phase 2: every rank left cleanly -> join generation m["gen"]
            ok, err = True, ""
            try:
                comm.join(int(m["port"]), int(m["gen"]), timeout_s=float(m.get("timeout", REGROUP_TIMEOUT_S)))
                build()
            except Exception as ex:    # noqa: BLE001 - reported; the coordinator replaces this rank
                logging.exception("rank %d: joining generation %s failed", comm.rank, m.get("gen"))
                ok, err = False, str(ex)
            send_msg(conn, {"op": "joined", "rank": comm.rank, "gen": int(m["gen"]), "ok": ok, "error": err}, lock)
            continue
        if op == "free":              # POST /free forwarded by rank 0 (same order as the prompts)
            if m.get("unload_models") or m.get("free_memory"):
                dm.unload_all_models()
            if m.get("free_memory"):
                ex_single.reset()
                for ex in ex_spmd.values():
                    ex.reset()
            need_gc, last_gc = True, 0.0
        if op != "run":
            if need_gc and time.perf_counter() - last_gc > GC_INTERVAL_S:
                _housekeeping()
                last_gc, need_gc = time.perf_counter(), False
            continue
        pid, extra = m["prompt_id"], m.get("extra_data") or {}
        server.last_prompt_id = pid
        t0 = time.perf_counter()
        k = int(m.get("k") or comm.world)
        ctx = ctxs.get(k)
        n0, b0, l0 = (ctx.images_sampled, ctx.comm.bytes_moved, ctx.loads_received) if ctx else (0, 0, 0)
        if m["mode"] in ("spmd", "latency") and ctx is not None:
            ex = ex_spmd.get(k)
            if ex is None:
                ex = ex_spmd[k] = PromptExecutor(None, node_hook=ctx)
            with spmd.activate(ctx, m["mode"]):
                ex.execute(m["prompt"], pid, {kk: v for kk, v in extra.items() if kk == "extra_pnginfo"},
                           m["outputs"])
        else:
            ex_single.execute(m["prompt"], pid, extra, m["outputs"])
            ex = ex_single
        need_gc = True
        save_errs = imageio.wait_futures(imageio.take_pending())    # this rank's files are on disk first
        ok = ex.success and not save_errs
        msgs = ex.status_messages + ([("execution_error", {"prompt_id": pid, "exception_message": "; ".join(save_errs)})]
                                     if save_errs else [])
        send_msg(conn, {"op": "done", "prompt_id": pid, "mode": m["mode"], "rank": comm.rank, "success": ok,
                        "messages": msgs, "outputs_ui": ex.outputs_ui,
                        "seconds": time.perf_counter() - t0,
                        "images_sampled": (ctx.images_sampled - n0) if ctx else 0,
                        "comm_bytes": (ctx.comm.bytes_moved - b0) if ctx else 0,
                        "loads_received": (ctx.loads_received - l0) if ctx else 0}, lock)
    try:
        conn.close()
    except OSError:
        pass


# ------------------------------------------------------------------------------------------------
# rank 0
# ------------------------------------------------------------------------------------------------
MAX_RESPAWNS = 3              # per rank: a rank that keeps dying stays dead
SPMD_WAIT_LOG_S = 30.0        # an SPMD prompt waiting this long for its ranks to go idle is logged
REGROUP_TIMEOUT_S = 120.0
TEARDOWN_TIMEOUT_S = float(os.environ.get("CGS_TEARDOWN_TIMEOUT_S", "30"))


class Coordinator:
    """Rank 0's scheduler for the node. Elastic: a worker that dies is respawned as a fresh child process
    (never a re-exec of a process that touched the GPU) and, once every rank is idle, all ranks leave the
    broken process group and rendezvous again (``Comm.reinit``, generation + 1); meanwhile SPMD prompts
    run on the rank prefix below the dead rank and single prompts on any survivor."""

    def __init__(self, q, server, comm, listener, accept_timeout_s: float = 600.0, latency_default=False,
                 respawn: bool = True):
        from ..graph.executor import PromptExecutor
        self.q, self.server, self.comm = q, server, comm
        self.world = comm.world
        self.latency_default = latency_default
        self.respawn = respawn and os.environ.get("CGS_RESPAWN", "1") != "0"
        self.listener = listener
        self.conns: dict = {}
        self.locks: dict = {}
        self.dead: set = set()
        self.busy: dict = {}          # rank -> prompt_id
        self.cv = threading.Condition()
        self.spmd_waiting: dict = {}  # prompt_id -> {rank: done message}
        self.ran_on: dict = {}        # prompt_id -> rank(s), for /history metrics and tests
        self._inflight: dict = {}     # rank -> (queue item id, prompt id, prompt, extra, outputs): its single prompt
        self._sids: dict = {}         # prompt id -> submitting client (WS)
        self._retries: dict = {}      # prompt id -> re-runs after a rank death
        self._respawns: dict = {}     # rank -> respawns so far
        self._spawned: dict = {}      # rank -> replacement process not yet in the process group
        self._acks: dict = {}         # (op, rank) -> a worker's re-rendezvous acknowledgement
        self.procs: list = []         # replacement processes (the launcher owns the first ones)
        self.gen = 0
        self.regroups = 0
        self.regroup_failures = 0
        self.regrouping = False       # a re-rendezvous is running (its own thread): workers take no prompts
        self.groups_ok = True         # every rank is in the current generation's process groups (SPMD allowed)
        self._spmd_queue: list = []   # waiting SPMD prompts in arrival order: {"members": set of ranks}
        self._started: dict = {}      # prompt id -> wall time its rank(s) were assigned
        self._last_gc, self._need_gc = time.perf_counter(), False
        self._accepted = threading.Condition()
        threading.Thread(target=self._accept_loop, daemon=True).start()
        with self._accepted:
            deadline = time.time() + accept_timeout_s
            while len(self.conns) < self.world - 1 and time.time() < deadline:
                self._accepted.wait(timeout=1.0)
        if len(self.conns) < self.world - 1:
            raise RuntimeError(f"only {len(self.conns)} of {self.world - 1} worker ranks connected")
        self.ex_single = PromptExecutor(server)
        self._build_contexts()        # after the handshakes: collective (subset + latency-mode groups)
        if hasattr(server, "interrupt_hooks"):
            server.interrupt_hooks.append(self.interrupt_all)

    def _build_contexts(self):
        from ..graph.executor import PromptExecutor
        from . import spmd
        self.comm.build_subsets(_spmd_sizes(self.world))
        self.ctxs = {k: spmd.SPMD(c) for k, c in sorted(self.comm.subsets.items())}
        self.ex_spmds = {k: PromptExecutor(self.server, node_hook=c) for k, c in self.ctxs.items()}
        self.ctx = self.ctxs.get(self.world)
        self.ex_spmd = self.ex_spmds.get(self.world)

    # -------------------------------------------------------------- plumbing
    def _accept_loop(self):
        """Worker connections, at start-up and whenever a replacement rank comes up."""
        while True:
            try:
                conn = self.listener.accept()
                hello = recv_msg(conn)
            except (OSError, EOFError):
                return
            except Exception:       # noqa: BLE001 - a bad handshake must not stop the accept loop
                logging.exception("worker handshake failed")
                continue
            r = int(hello["rank"])
            with self._accepted:
                self.conns[r], self.locks[r] = conn, threading.Lock()
                self._accepted.notify_all()
            threading.Thread(target=self._reader, args=(r, conn), daemon=True).start()
            if hello.get("respawned"):
                logging.warning("replacement for rank %d connected", r)
                with self.cv:
                    self.cv.notify_all()

    def live(self):
        return [r for r in range(self.world) if r not in self.dead]

    def prefix(self):
        """Ranks [0, L) that are all alive (the usable SPMD prefixes are the subsets of size <= L)."""
        return min(self.dead) if self.dead else self.world

    def _reader(self, r, conn):
        while True:
            try:
                m = recv_msg(conn)
            except (EOFError, OSError):
                if self.conns.get(r) is conn:
                    self._rank_died(r)
                return
            op = m.get("op")
            if op == "event":
                self.server.send_sync(m["event"], m["data"], m.get("sid"))
            elif op == "binary":
                import base64
                self.server.send_sync(int(m["event"]), base64.b64decode(m["data"]), m.get("sid"))
            elif op == "yjs":
                om = getattr(self.server, "output_map", None)
                if om is not None:
                    om.set(m["key"], m["value"])
            elif op == "yjs_flush":
                if getattr(self.server, "output_map", None) is not None:
                    self.server.broadcast_yjs_updates()
            elif op in ("torn_down", "joined"):
                with self.cv:
                    self._acks[(op, r)] = m
                    self.cv.notify_all()
            elif op == "done":
                with self.cv:
                    pid = m["prompt_id"]
                    if pid in self.spmd_waiting:
                        self.spmd_waiting[pid][r] = m
                    elif m.get("mode", "single") == "single":
                        self._finish_single(r, m)
                    else:
                        # a survivor's report of an SPMD attempt that was already settled (a rank died
                        # under it): never let it complete the prompt's single re-run on this rank
                        logging.info("late SPMD report of prompt %s from rank %d ignored", pid, r)
                    self.cv.notify_all()

    def _rank_died(self, r):
        """A worker's connection dropped: mark it dead (SPMD prompts use the rank prefix below it until the
        next re-rendezvous), re-run its single prompt on a survivor (once), unblock a waiting SPMD prompt,
        and start a replacement process."""
        logging.error("rank %d left the cluster", r)
        retry = None
        with self.cv:
            if r in self.dead:
                return
            self.dead.add(r)
            self.conns.pop(r, None)       # a replacement says hello on a fresh connection
            try:    # SPMD agreements waiting on the dead rank fail within ~1 s (spmd.SPMD._agree)
                st = self.comm.store()
                if st is not None:
                    st.set("cgs/dead", ",".join(str(x) for x in sorted(self.dead)))
            except Exception:   # pragma: no cover - store already gone
                pass
            pid = self.busy.pop(r, None)
            rec = self._inflight.pop(r, None)
            if rec is not None:
                if self._retries.get(rec[1], 0) < MAX_RETRIES and self.live():
                    self._retries[rec[1]] = self._retries.get(rec[1], 0) + 1
                    retry = rec
                else:
                    self._complete(rec[0], rec[1], {}, False,
                                   [("execution_error", {"prompt_id": pid, "exception_message": f"rank {r} died"})])
            for w in self.spmd_waiting.values():
                w.setdefault(r, {"success": False, "messages": [], "outputs_ui": {}, "dead": True})
            self.cv.notify_all()
        self._spawn_replacement(r)
        if retry is not None:
            logging.warning("re-running prompt %s (rank %d died under it)", retry[1], r)
            threading.Thread(target=self._run_single, args=retry, daemon=True).start()

    def _spawn_replacement(self, r):
        if not self.respawn or _LAUNCH.get("argv") is None:
            return
        n = self._respawns.get(r, 0)
        if n >= MAX_RESPAWNS:
            logging.error("rank %d died %d times: not respawned", r, n)
            return
        self._respawns[r] = n + 1
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), CGS_SCHED_ROLE="worker", CGS_SCHED_RESPAWN="1",
                   PYTHONPATH=_LAUNCH["pypath"])
        env.pop("CGS_FAULT", None)    # injected faults fire once, not in the replacement
        try:
            p = subprocess.Popen([sys.executable, "-m", "comfy_gen_server_amd.main"] + list(_LAUNCH["argv"]), env=env)
        except OSError:
            logging.exception("respawning rank %d failed", r)
            return
        self.procs.append(p)
        self._spawned[r] = p
        _LAUNCH.setdefault("procs", {})[r] = p
        logging.warning("respawned rank %d (pid %d)", r, p.pid)

    def _kick_regroup(self):
        """Start the re-rendezvous (on its own thread, so the dispatch loop keeps serving) once every dead
        rank has a connected replacement and no rank is busy."""
        with self.cv:
            if self.regrouping or not self.dead or self.busy:
                return
            if any(r not in self._spawned or self._spawned[r].poll() is not None or r not in self.conns
                   for r in self.dead):
                return                    # every replacement is up and has said hello
            self.regrouping, self.groups_ok = True, False
            self._acks = {}
        threading.Thread(target=self._regroup, name="cgs-regroup", daemon=True).start()

    def _regroup(self):
        """All-or-nothing re-rendezvous as generation gen + 1 (rank 0 hosts the new TCPStore):
        phase 1 every rank leaves the old process group (bounded: a worker whose teardown hangs exits and is
        replaced), phase 2 -- only if every rank left cleanly -- every rank joins the new generation. Any
        failure leaves ``groups_ok`` False (prompts run single, on any live rank) and replaces the ranks whose
        group state is unknown; the next attempt starts once their replacements are up."""
        gen, port = self.gen + 1, _free_port()
        workers = list(range(1, self.world))
        ok = False
        try:
            logging.warning("re-rendezvous of %d ranks (generation %d): teardown", self.world, gen)
            bad = self._phase("teardown", "torn_down", workers, {"gen": gen, "timeout": TEARDOWN_TIMEOUT_S},
                              TEARDOWN_TIMEOUT_S + 15.0, lambda: self.comm.leave(TEARDOWN_TIMEOUT_S))
            if bad is None:
                logging.critical("rank 0's process-group teardown hung: SPMD stays off (single prompts only)")
                return
            if bad:
                logging.error("regroup: ranks %s did not leave the old group cleanly; replacing them", bad)
                for r in bad:
                    self._force_replace(r)
                return

            def join0():
                self.comm.join(port, gen, timeout_s=REGROUP_TIMEOUT_S)
                self._build_contexts()
                return True
            logging.warning("re-rendezvous of %d ranks (generation %d): join", self.world, gen)
            bad = self._phase("join", "joined", workers, {"gen": gen, "port": port, "timeout": REGROUP_TIMEOUT_S},
                              REGROUP_TIMEOUT_S + 15.0, join0)
            if bad is None or bad:
                logging.error("regroup: generation %d incomplete (rank 0 %s, failed workers %s)", gen,
                              "failed" if bad is None else "ok", bad or [])
                for r in bad or []:
                    self._force_replace(r)
                return
            with self.cv:
                self.gen = gen
                self.regroups += 1
                self.dead.clear()
                self._spawned.clear()
            ok = True
            logging.warning("node whole again (generation %d, %d ranks)", gen, self.world)
        except Exception:   # noqa: BLE001 - never let the regroup thread die silently
            logging.exception("regroup failed")
        finally:
            with self.cv:
                self.regrouping = False
                self.groups_ok = ok
                self.regroup_failures += 0 if ok else 1
                self.cv.notify_all()

    def _phase(self, op, ack, workers, payload, timeout_s, local):
        """Send ``op`` to every worker, run ``local()`` on rank 0, wait up to ``timeout_s`` for the ``ack``s.
        Returns the workers that failed or did not answer, or None if rank 0's own part failed."""
        bad = set()
        for r in workers:
            try:
                send_msg(self.conns[r], dict(payload, op=op), self.locks[r])
            except (OSError, KeyError):
                bad.add(r)
        try:
            ok0 = bool(local())
        except Exception:   # noqa: BLE001
            logging.exception("regroup %s failed on rank 0", op)
            ok0 = False
        deadline = time.time() + timeout_s
        # a rank whose connection drops meanwhile (_rank_died pops it) will not answer; a dead rank's connected
        # replacement will
        self._wait(lambda: all((ack, r) in self._acks or r in bad or r not in self.conns for r in workers)
                   or time.time() > deadline)
        with self.cv:
            bad |= {r for r in workers if not self._acks.get((ack, r), {}).get("ok")}
        return sorted(bad) if ok0 else None

    def _force_replace(self, r):
        """A worker whose process-group state is unknown: ask it to exit, kill it if it does not, and let
        ``_rank_died`` (its connection drops) spawn the replacement."""
        conn, proc = self.conns.get(r), _LAUNCH.get("procs", {}).get(r)
        if conn is not None:
            try:
                send_msg(conn, {"op": "exit"}, self.locks[r])
            except OSError:
                pass
        if proc is not None:
            try:
                proc.wait(timeout=10)
            except subprocess.TimeoutExpired:
                proc.kill()
        if r not in self.dead:
            self._rank_died(r)

    def interrupt_all(self):
        for r in list(self.busy):
            if r != 0 and r not in self.dead:
                try:
                    send_msg(self.conns[r], {"op": "interrupt"}, self.locks[r])
                except OSError:
                    pass

    def _complete(self, item_id, prompt_id, outputs_ui, success, messages):
        self.q.task_done(item_id, outputs_ui,
                         status=self.q.ExecutionStatus(status_str="success" if success else "error",
                                                       completed=success, messages=messages))
        with self.q.mutex:                       # which rank(s) served it, and when: /history metrics
            h = self.q.history.get(prompt_id)
            if h is not None:
                mt = h.setdefault("metrics", {})
                mt["ranks"] = self.ran_on.get(prompt_id)
                mt["started_at"] = self._started.pop(prompt_id, None)    # its rank(s) assigned (epoch s)
                mt["finished_at"] = time.time()
        sid = self._sids.pop(prompt_id, None)
        if sid is not None:
            self.server.send_sync("executing", {"node": None, "prompt_id": prompt_id}, sid)
        m = getattr(self.server, "metrics", None)
        if isinstance(m, dict):
            m["prompts_total"] = m.get("prompts_total", 0) + 1
            if not success:
                m["prompts_failed"] = m.get("prompts_failed", 0) + 1

    def _finish_single(self, r, m):
        rec = self._inflight.pop(r, None)
        self.busy.pop(r, None)
        self._need_gc = True
        if rec is None:
            return
        item_id, pid = rec[0], rec[1]
        self._complete(item_id, pid, m.get("outputs_ui") or {}, bool(m.get("success")), m.get("messages") or [])

    # -------------------------------------------------------------- scheduling
    def spmd_size(self, prompt, extra):
        """(mode, k): the execution mode of a prompt and the rank prefix [0, k) it runs on."""
        mode = choose_mode(prompt, extra, self.world, self.latency_default, subsets=True)
        if not self.groups_ok:        # a re-rendezvous is running or failed: no collectives until it succeeds
            return "single", 1
        L = self.prefix()
        if mode == "latency":
            return ("latency", self.world) if L == self.world else ("single", 1)
        if mode != "spmd":
            return "single", 1
        want = (extra or {}).get("dp", "auto")
        b = self.world if want == "spmd" else prompt_batch(prompt)
        ks = [k for k in self.ctxs if k <= min(b, L)]
        return ("spmd", max(ks)) if ks else ("single", 1)

    def run_forever(self, stop_event: threading.Event | None = None):
        while stop_event is None or not stop_event.is_set():
            got = self.q.get(timeout=1.0)
            if got is not None:
                item, item_id = got
                prompt_id, prompt, extra, outputs = item[1], item[2], item[3] or {}, item[4]
                sid = extra.get("client_id")
                if sid is not None:
                    self._sids[prompt_id] = sid
                mode, k = self.spmd_size(prompt, extra)
                if mode in ("spmd", "latency"):
                    # its own thread: the loop goes on handing single prompts to the ranks outside the prefix;
                    # the prefix is reserved now, in queue order, so later single prompts cannot starve it
                    ticket = self._reserve(k)
                    threading.Thread(target=self._run_spmd, args=(item_id, prompt_id, prompt, extra, outputs, mode,
                                                                   k, ticket), daemon=True).start()
                else:
                    self._run_single(item_id, prompt_id, prompt, extra, outputs)
            self._kick_regroup()
            self._housekeeping()

    def _housekeeping(self):
        """The reference worker's between-prompt duties (main.py:139-146) for the whole node: POST /free
        flags (applied on rank 0 once it is idle, forwarded to every worker in prompt order) and the
        periodic model cleanup + GC."""
        from ..runtime import device as dm
        flags = self.q.get_flags()
        free_memory = flags.get("free_memory", False)
        unload = flags.get("unload_models", free_memory)
        if unload or free_memory:
            self._wait(lambda: 0 not in self.busy)
            dm.unload_all_models()
            if free_memory:
                self.ex_single.reset()
                for ex in self.ex_spmds.values():
                    ex.reset()
            for r in self.live():
                if r != 0:
                    try:
                        send_msg(self.conns[r], {"op": "free", "unload_models": bool(unload),
                                                 "free_memory": bool(free_memory)}, self.locks[r])
                    except OSError:
                        self._rank_died(r)
            self._need_gc, self._last_gc = True, 0.0
        if self._need_gc and 0 not in self.busy and time.perf_counter() - self._last_gc > GC_INTERVAL_S:
            _housekeeping()
            self._last_gc, self._need_gc = time.perf_counter(), False

    def _wait(self, pred):
        with self.cv:
            while not pred():
                self.cv.wait(timeout=1.0)

    def _reserve(self, k):
        """Queue an SPMD prompt on the rank prefix [0, k): single prompts stay off those ranks from now on."""
        ticket = {"members": set(range(k))}
        with self.cv:
            self._spmd_queue.append(ticket)
        return ticket

    def _idle_for_single(self):
        """Ranks a single prompt may take: live, not busy, not reserved by a waiting SPMD prompt, and (during a
        re-rendezvous) rank 0 only -- the workers are inside it."""
        reserved = set().union(*(t["members"] for t in self._spmd_queue)) if self._spmd_queue else set()
        return [r for r in self.live() if r not in self.busy and r not in reserved
                and not (self.regrouping and r != 0)]

    def _run_single(self, item_id, prompt_id, prompt, extra, outputs):
        self._wait(lambda: bool(self._idle_for_single()))
        with self.cv:
            r = max(self._idle_for_single())    # workers first: rank 0 also serves HTTP / WS
            self.busy[r] = prompt_id
            self._inflight[r] = (item_id, prompt_id, prompt, extra, outputs)
            self.ran_on[prompt_id] = r
            self._started[prompt_id] = time.time()
        if r == 0:
            threading.Thread(target=self._local_single, args=(prompt_id, prompt, extra, outputs), daemon=True).start()
        else:
            try:
                send_msg(self.conns[r], {"op": "run", "mode": "single", "prompt_id": prompt_id, "prompt": prompt,
                                         "extra_data": extra, "outputs": outputs}, self.locks[r])
            except OSError:
                self._rank_died(r)

    def _local_single(self, prompt_id, prompt, extra, outputs):
        from ..utils import imageio
        self.server.last_prompt_id = prompt_id
        msg = {"success": False, "messages": [("execution_error", {"prompt_id": prompt_id,
                                                                   "exception_message": "executor raised"})],
               "outputs_ui": {}}
        try:
            self.ex_single.execute(prompt, prompt_id, extra, outputs)
            errs = imageio.wait_futures(imageio.take_pending())
            msg = {"success": self.ex_single.success and not errs,
                   "messages": self.ex_single.status_messages + (
                       [("execution_error", {"prompt_id": prompt_id, "exception_message": "; ".join(errs)})]
                       if errs else []),
                   "outputs_ui": self.ex_single.outputs_ui}
        except Exception as ex:     # the executor handles node errors itself: this is a bug, not a node error
            logging.exception("rank 0 executor raised")
            msg["messages"][0][1]["exception_message"] = str(ex)
        finally:
            with self.cv:
                self._finish_single(0, msg)
                self.cv.notify_all()

    def _run_spmd(self, item_id, prompt_id, prompt, extra, outputs, mode="spmd", k=None, ticket=None):
        from ..utils import imageio
        from . import spmd
        k = k or self.world
        members = list(range(k))
        if ticket is None:
            ticket = self._reserve(k)
        t_wait = time.perf_counter()
        logged = [False]

        def changed():    # a member died, or the groups went away (a re-rendezvous failed): choose again
            return any(r in self.dead for r in members) or (not self.groups_ok and not self.regrouping)

        def members_idle():
            if not logged[0] and time.perf_counter() - t_wait > SPMD_WAIT_LOG_S:
                logged[0] = True
                logging.warning("SPMD prompt %s has waited %.0f s for ranks %s (busy: %s)", prompt_id,
                                time.perf_counter() - t_wait, members, dict(self.busy))
            first = self._spmd_queue and self._spmd_queue[0] is ticket     # FIFO among SPMD prompts
            return (first and not self.regrouping and self.groups_ok and all(r not in self.busy for r in members)) \
                or changed()
        self._wait(members_idle)
        with self.cv:
            redo = changed()
            if not redo:
                for r in members:
                    self.busy[r] = prompt_id
                self._started[prompt_id] = time.time()
            if ticket in self._spmd_queue:
                self._spmd_queue.remove(ticket)
            self.cv.notify_all()
        if redo:
            mode, k = self.spmd_size(prompt, extra)
            if mode == "single":
                return self._run_single(item_id, prompt_id, prompt, extra, outputs)
            return self._run_spmd(item_id, prompt_id, prompt, extra, outputs, mode, k)
        ctx, ex_spmd = self.ctxs[k], self.ex_spmds[k]
        with self.cv:
            self.spmd_waiting[prompt_id] = {}
            self.ran_on[prompt_id] = ("all" if k == self.world else members) if mode == "spmd" else "latency"
        # the workers' SPMD executors get the PNG metadata (SaveImage's hidden EXTRA_PNGINFO: every rank
        # writes its own images), not the client id (their WS events are rank 0's to send)
        xd = {"extra_pnginfo": extra.get("extra_pnginfo")} if extra.get("extra_pnginfo") is not None else {}
        msg = {"op": "run", "mode": mode, "k": k, "prompt_id": prompt_id, "prompt": prompt, "outputs": outputs,
               "extra_data": xd}
        for r in members[1:]:
            try:
                send_msg(self.conns[r], msg, self.locks[r])
            except OSError:
                self._rank_died(r)
        self.server.last_prompt_id = prompt_id
        n0, b0, l0 = ctx.images_sampled, ctx.comm.bytes_moved, ctx.loads_received
        ctx.reserved = []
        with spmd.activate(ctx, mode):
            ex_spmd.execute(prompt, prompt_id, extra, outputs)
        save_errs = imageio.wait_futures(imageio.take_pending())
        mine, mine_b = ctx.images_sampled - n0, ctx.comm.bytes_moved - b0
        # every member's report (a survivor of a rank death fails its next agreement within ~1 s);
        # bounded, so a wedged worker cannot hold the node
        t_end = time.perf_counter() + SPMD_REPORT_TIMEOUT_S
        self._wait(lambda: all(r in self.spmd_waiting[prompt_id] for r in members[1:])
                   or time.perf_counter() > t_end)
        retry = False
        with self.cv:
            done = self.spmd_waiting.pop(prompt_id)
            ok = ex_spmd.success and not save_errs and all(bool(m.get("success")) for m in done.values())
            msgs = list(ex_spmd.status_messages)
            if save_errs:
                msgs.append(("execution_error", {"prompt_id": prompt_id, "exception_message": "; ".join(save_errs)}))
            for r, m in sorted(done.items()):
                if not m.get("success"):
                    msgs += [(e, d) for e, d in (m.get("messages") or []) if e == "execution_error"]
            for r in list(self.busy):
                if self.busy[r] == prompt_id:
                    del self.busy[r]
            self._need_gc = True
            # a member died under the prompt: run it again on the survivors (SPMD on the rank prefix below
            # the dead rank, else whole on one rank). Noise is keyed by global image index, so the images are
            # the ones the first attempt would have produced.
            lost = any(m.get("dead") for m in done.values()) or any(r in self.dead for r in members)
            if not ok:
                # once every member has reported (or is gone) no rank writes this attempt's files any more
                from ..utils import imageio as _io
                _io.flush()
                ctx.cleanup_reserved()
            if not ok and lost and self.live() and self._retries.get(prompt_id, 0) < MAX_RETRIES:
                self._retries[prompt_id] = self._retries.get(prompt_id, 0) + 1
                retry = True
            else:
                self._complete(item_id, prompt_id, ex_spmd.outputs_ui, ok, msgs)
            with self.q.mutex:
                h = self.q.history.get(prompt_id)
                if h is not None:   # images sampled per rank (the batch split), checkpoints received (R3)
                    h["metrics"]["images_per_rank"] = {0: mine, **{r: m.get("images_sampled", 0)
                                                                   for r, m in done.items()}}
                    h["metrics"]["comm_bytes_per_rank"] = {0: mine_b, **{r: m.get("comm_bytes", 0)
                                                                         for r, m in done.items()}}
                    h["metrics"]["loads_received_per_rank"] = {0: ctx.loads_received - l0,
                                                               **{r: m.get("loads_received", 0)
                                                                  for r, m in done.items()}}
            self.cv.notify_all()
        if retry:
            mode2, k2 = self.spmd_size(prompt, extra)
            logging.warning("re-running prompt %s on surviving ranks (%s, k=%d)", prompt_id, mode2, k2)
            if mode2 in ("spmd", "latency"):
                self._run_spmd(item_id, prompt_id, prompt, extra, outputs, mode2, k2)
            else:
                self._run_single(item_id, prompt_id, prompt, extra, outputs)

    def shutdown(self):
        for r, conn in self.conns.items():
            try:
                send_msg(conn, {"op": "stop"}, self.locks[r])
            except OSError:
                pass


# ------------------------------------------------------------------------------------------------
# launcher
# ------------------------------------------------------------------------------------------------
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


_LAUNCH: dict = {}     # argv / PYTHONPATH of the worker command line (replacement ranks use it)


def launch(n: int, argv):
    """Rank 0 (this process, before it touches the GPU): start ranks 1..n-1 as children running the
    same command line, set up the rendezvous env for all of them, and return (listener, procs)."""
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(_free_port()))
    key = secrets.token_hex(16)
    listener = Listener(("127.0.0.1", 0), authkey=key.encode())
    env_common = {"WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n), "CGS_SCHED_ADDR": json.dumps(listener.address),
                  "CGS_SCHED_KEY": key, "HSA_ENABLE_IPC_MODE_LEGACY": os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0")}
    os.environ.update(env_common)
    os.environ.update(RANK="0", LOCAL_RANK="0")
    procs = []
    pkg_parent = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    pypath = os.pathsep.join(p for p in (pkg_parent, os.environ.get("PYTHONPATH", "")) if p)
    _LAUNCH.update(argv=list(argv), pypath=pypath)
    for r in range(1, n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), CGS_SCHED_ROLE="worker", PYTHONPATH=pypath)
        procs.append(subprocess.Popen([sys.executable, "-m", "comfy_gen_server_amd.main"] + list(argv), env=env))
    _LAUNCH["procs"] = {r: p for r, p in zip(range(1, n), procs)}
    return listener, procs


def worker_address():
    return json.loads(os.environ["CGS_SCHED_ADDR"]), os.environ["CGS_SCHED_KEY"].encode()
