"""Communicator: one process per GPU over RCCL/xGMI (``torch.distributed`` backend ``nccl`` IS RCCL
on ROCm), Gloo on the CPU for tests. The reference has no collective call sites;
the new ones are:

  R1 job broadcast      ``broadcast_object`` (workflow JSON / seeds / prompts, rank 0 -> all) -- on the
                        Gloo CONTROL group (host memory), so the RCCL communicator only ever carries
                        device tensors and its collectives stay in one order on one stream
  R2 result gather      ``gather`` of uint8 images / latents to rank 0 only (``all_gather`` where every
                        rank needs the batch, e.g. latents feeding a replicated node)
  R3 weight broadcast   ``broadcast_module`` — bucketed (256 MB default) in-place broadcast of every
                        parameter from rank 0 so only one rank reads a checkpoint from disk
  R6 control            ``barrier`` / ``heartbeat`` (all-reduce of a liveness counter)

xGMI is point-to-point (7 links x ~153 GB/s per GPU); RCCL picks ring/tree per size. Buckets are
sized so a collective is bandwidth-bound (hundreds of MB), not latency-bound.
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist


# ``Comm.broadcast_state_dict`` on a receiving rank when the source's checkpoint is not a flat
# {name: tensor} dict (nested upscaler ``.pth`` files, A1111 hypernetworks, PhotoMaker ``.bin``): no table
# can describe it, so every rank reads the file itself.
LOAD_LOCALLY = object()


def is_flat_tensor_dict(sd) -> bool:
    return isinstance(sd, dict) and all(isinstance(k, str) and torch.is_tensor(v) for k, v in sd.items())


class Comm:
    def __init__(self):
        self.rank = 0
        self.world = 1
        self.local_rank = 0
        self.backend = None
        self.device = torch.device("cpu")
        self.group = None     # data-plane group (None: the default group)
        self.ctrl = None      # Gloo group for host-side control traffic (None: the default group)
        self.bytes_moved = 0  # tensor bytes this rank sent + received in gathers (serving metrics)
        self.load_bytes = 0   # checkpoint bytes sent / received by ``broadcast_state_dict`` (R3)
        self.gen = 0          # process-group generation (bumped by every re-rendezvous, ``reinit``)
        self.subsets = {}     # k -> SubComm over ranks [0, k) (``build_subsets``)

    degraded = False   # set by the DP engine after a rank failure: the process group is unusable

    @property
    def enabled(self):
        return self.world > 1 and not self.degraded

    def barrier(self):
        if self.enabled:
            if self.backend == "nccl":
                dist.barrier(group=self.group, device_ids=[self.local_rank])
            else:
                dist.barrier(group=self.group)

    def broadcast_object(self, obj, src=0):
        """R1 over the Gloo control group: no device sync, no RCCL op on the issuing stream."""
        if not self.enabled:
            return obj
        lst = [obj if self.rank == src else None]
        dist.broadcast_object_list(lst, src=src, group=self.ctrl)
        return lst[0]

    def send_object(self, obj, dst):
        dist.send_object_list([obj], dst=dst, group=self.ctrl)

    def recv_object(self, src=None):
        """Receive one object (from ``src``, or from any rank); returns (obj, source rank)."""
        lst = [None]
        r = dist.recv_object_list(lst, src=src, group=self.ctrl)
        return lst[0], (src if src is not None else r)

    def ctrl_barrier(self):
        if self.enabled:
            dist.barrier(group=self.ctrl)

    def broadcast_tensor(self, t, src=0):
        if self.enabled:
            dist.broadcast(t, src=src, group=self.group)
        return t

    @torch.no_grad()
    def broadcast_module(self, module, src=0, bucket_bytes=256 << 20):
        """Bucketed parameter/buffer broadcast (R3): flatten same-dtype tensors into buckets."""
        if not self.enabled:
            return module
        tensors = [p.data for p in module.parameters()] + [b for b in module.buffers()]
        groups = {}
        for t in tensors:
            groups.setdefault((t.dtype, t.device), []).append(t)
        for (dt, dev), ts in groups.items():
            bucket, size = [], 0
            for t in ts + [None]:
                if t is not None and (size + t.numel() * t.element_size() <= bucket_bytes or not bucket):
                    bucket.append(t)
                    size += t.numel() * t.element_size()
                    continue
                if bucket:
                    flat = torch.cat([b.reshape(-1) for b in bucket])
                    if flat.is_cuda and self.backend == "gloo":     # shared-GPU rehearsal: via host memory
                        h = flat.cpu()
                        if h.dtype in (torch.bfloat16, torch.float16):
                            h = h.float()                         # exact; Gloo lacks 16-bit types
                        dist.broadcast(h, src=src, group=self.group)
                        flat.copy_(h)
                    else:
                        dist.broadcast(flat, src=src, group=self.group)
                    off = 0
                    for b in bucket:
                        n = b.numel()
                        b.copy_(flat[off:off + n].view_as(b))
                        off += n
                bucket, size = ([t], t.numel() * t.element_size()) if t is not None else ([], 0)
        return module

    @torch.no_grad()
    def broadcast_state_dict(self, sd, device, src=0, bucket_bytes=256 << 20):
        """R3 for a checkpoint's raw state dict: ``src`` (which read the file) sends the key / shape / dtype
        table over the control group, then the tensors in same-dtype buckets over the data plane (RCCL over
        xGMI on the GPU); the other ranks allocate and receive them on ``device`` without touching the file.
        ``sd`` is None on the receivers. An exception object in place of ``sd`` on ``src`` is re-raised on
        every rank (a failed load fails the node everywhere). A source dict that is not flat
        (``is_flat_tensor_dict``) is not sent: the receivers get ``LOAD_LOCALLY`` and read the file
        themselves."""
        if not self.enabled:
            return sd
        if self.rank == src:
            if isinstance(sd, BaseException):
                self.broadcast_object({"error": f"{type(sd).__name__}: {sd}"}, src=src)
                raise sd
            if not is_flat_tensor_dict(sd):
                self.broadcast_object({"local": True}, src=src)
                return sd
            table = [(k, tuple(v.shape), str(v.dtype).replace("torch.", "")) for k, v in sd.items()]
            self.broadcast_object({"table": table}, src=src)
        else:
            msg = self.broadcast_object(None, src=src)
            if "error" in msg:
                raise RuntimeError(f"checkpoint load failed on rank {src}: {msg['error']}")
            if msg.get("local"):
                return LOAD_LOCALLY
            table = msg["table"]
            sd = {k: torch.empty(shape, dtype=getattr(torch, dt), device=device) for k, shape, dt in table}
        xdev = self.device if self.backend == "nccl" else torch.device("cpu")
        names = list(sd.keys())
        by_dt = {}
        for k in names:
            by_dt.setdefault(sd[k].dtype, []).append(k)
        for dt, keys in by_dt.items():
            bucket, size = [], 0
            for k in keys + [None]:
                nb = 0 if k is None else sd[k].numel() * sd[k].element_size()
                if k is not None and (size + nb <= bucket_bytes or not bucket):
                    bucket.append(k)
                    size += nb
                    continue
                if bucket:
                    n = sum(sd[b].numel() for b in bucket)
                    if self.rank == src:
                        flat = torch.cat([sd[b].reshape(-1).to(xdev) for b in bucket]) if n else \
                            torch.empty(0, dtype=dt, device=xdev)
                    else:
                        flat = torch.empty(n, dtype=dt, device=xdev)
                    dist.broadcast(flat, src=src, group=self.group)
                    self.load_bytes += flat.numel() * flat.element_size()
                    if self.rank != src:
                        off = 0
                        for b in bucket:
                            m = sd[b].numel()
                            sd[b].copy_(flat[off:off + m].view_as(sd[b]))
                            off += m
                bucket, size = ([k], nb) if k is not None else ([], 0)
        return sd

    def build_subsets(self, sizes=None):
        """Data/control groups over the rank prefixes [0, k) for every k in ``sizes`` (default 2..world-1;
        k = world is this communicator itself). Collective over the default group: every rank calls it
        with the same sizes in the same order (right after ``init_from_env`` / ``reinit``). A prompt whose
        image batch is smaller than the node then runs SPMD on k ranks while the others serve single
        prompts; after a rank death the prefixes below it stay usable until the re-rendezvous."""
        self.subsets = {}
        if self.world <= 1:
            return self.subsets
        sizes = sorted(set(sizes if sizes is not None else range(2, self.world)))
        for k in sizes:
            if not 2 <= k < self.world:
                continue
            ranks = list(range(k))
            g = dist.new_group(ranks)
            c = dist.new_group(ranks, backend="gloo") if self.backend == "nccl" else g
            if self.rank < k:
                self.subsets[k] = SubComm(self, k, g, c)
        self.subsets[self.world] = self
        return self.subsets

    def leave(self, timeout_s: float = 60.0) -> bool:
        """Tear down the process group (after a rank death its collectives can never complete), bounded:
        the teardown runs on a helper thread and this returns False if it has not finished within
        ``timeout_s`` -- an RCCL communicator with a dead peer can block in its destructor. The caller then
        replaces the process (a worker exits non-zero and the coordinator spawns a fresh child; nothing
        re-execs a process that touched the GPU). True when there was nothing to tear down."""
        import threading
        from ..utils.telemetry import maybe_fault
        if not dist.is_initialized():
            self.subsets = {}
            return True
        err = []

        def teardown():
            try:
                maybe_fault("teardown", str(self.rank))
                dist.destroy_process_group()
            except Exception as ex:  # noqa: BLE001 - a broken group may not tear down cleanly
                err.append(ex)
        t = threading.Thread(target=teardown, name="cgs-pg-teardown", daemon=True)
        t.start()
        t.join(timeout_s)
        if t.is_alive():
            return False
        self.subsets = {}
        self.group = None
        self.ctrl = None
        return True

    def join(self, port: int, gen: int, addr: str = "127.0.0.1", timeout_s: float = 600.0):
        """Join process-group generation ``gen`` over a fresh TCPStore on ``port`` (hosted by rank 0), with
        every other rank of the node (survivors and respawned ranks alike)."""
        self.degraded = False
        self.gen = gen
        self.group = None
        kw = dict(backend=self.backend or ("nccl" if self.device.type == "cuda" else "gloo"),
                  init_method=f"tcp://{addr}:{port}", rank=self.rank, world_size=self.world,
                  timeout=datetime.timedelta(seconds=timeout_s))
        if kw["backend"] == "nccl":
            kw["device_id"] = self.device
        dist.init_process_group(**kw)
        self.backend = kw["backend"]
        self.ctrl = dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=timeout_s)) \
            if self.backend == "nccl" else None
        return self

    def reinit(self, port: int, gen: int, addr: str = "127.0.0.1", timeout_s: float = 600.0,
               teardown_timeout_s: float = 60.0):
        """Re-rendezvous after a rank death: ``leave`` (bounded) then ``join`` generation ``gen``. Raises
        ``TimeoutError`` if the teardown does not finish."""
        if not self.leave(teardown_timeout_s):
            raise TimeoutError(f"rank {self.rank}: process-group teardown did not finish in {teardown_timeout_s} s")
        return self.join(port, gen, addr, timeout_s)

    def all_gather(self, t):
        """Concatenate ``t`` (same shape on every rank) along dim 0 across ranks."""
        if not self.enabled:
            return t
        t = t.contiguous()
        out = torch.empty((self.world * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, t, group=self.group)
        self.bytes_moved += out.numel() * out.element_size()      # own shard out, every other shard in
        return out

    def gather(self, t, dst=0):
        """R2: ``t`` of every rank (same shape) concatenated along dim 0 on ``dst``; None elsewhere.
        One RCCL gather: each rank's shard crosses one xGMI link once (an all-gather would ship the
        whole batch to every rank, world-1 times the bytes)."""
        if not self.enabled:
            return t
        t = t.contiguous()
        nb = t.numel() * t.element_size()
        if self.rank == dst:
            parts = [torch.empty_like(t) for _ in range(self.world)]
            dist.gather(t, gather_list=parts, dst=dst, group=self.group)
            self.bytes_moved += (self.world - 1) * nb
            return torch.cat(parts)
        dist.gather(t, dst=dst, group=self.group)
        self.bytes_moved += nb
        return None

    def all_reduce_max(self, x: float) -> float:
        if not self.enabled:
            return x
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.ctrl)
        return float(t.item())

    def heartbeat_fault_site(self):
        from ..utils.telemetry import maybe_fault
        maybe_fault("rank", str(self.rank))

    def heartbeat(self) -> int:
        """R6: returns the number of live ranks (all-reduce of ones)."""
        from ..utils.telemetry import maybe_fault
        maybe_fault("rank", str(self.rank))
        if not self.enabled:
            return 1
        t = torch.ones(1, dtype=torch.int32, device=self.device)
        dist.all_reduce(t, group=self.group)
        return int(t.item())

    # ---- control plane (R6): the c10d TCPStore (hosted by rank 0) outlives a dead peer, unlike a
    # collective ring, so liveness and degraded-mode result shipping go through it ----
    def store(self):
        return dist.distributed_c10d._get_default_store() if self.world > 1 and dist.is_initialized() else None

    def _seq(self):
        self._job_seq = getattr(self, "_job_seq", 0) + 1
        return self._job_seq

    def liveness_round(self, timeout_s: float = 30.0):
        """Every rank checks in; rank 0 waits up to ``timeout_s`` and publishes the verdict.
        Returns (round_id, dead_ranks) identically on every live rank."""
        st, rid = self.store(), self._seq()
        st.set(f"cgs/live/{rid}/{self.rank}", "1")
        if self.rank == 0:
            import time as _t
            deadline = _t.time() + timeout_s
            pending = set(range(1, self.world))
            while pending and _t.time() < deadline:
                pending = {r for r in pending if not st.check([f"cgs/live/{rid}/{r}"])}
                if pending:
                    _t.sleep(0.05)
            st.set(f"cgs/verdict/{rid}", ",".join(str(r) for r in sorted(pending)))
            return rid, sorted(pending)
        st.wait([f"cgs/verdict/{rid}"], datetime.timedelta(seconds=timeout_s * 2 + 30))
        v = st.get(f"cgs/verdict/{rid}").decode()
        return rid, [int(x) for x in v.split(",") if x]

    def store_put_tensor(self, key, t):
        import io
        buf = io.BytesIO()
        torch.save(t.cpu(), buf)
        self.store().set(key, buf.getvalue())

    def store_get_tensor(self, key, timeout_s=120.0):
        import io
        st = self.store()
        st.wait([key], datetime.timedelta(seconds=timeout_s))
        return torch.load(io.BytesIO(st.get(key)), weights_only=True)

    def shutdown(self):
        """Leave together: a barrier first (unless degraded: dead peers never arrive), so no rank
        tears its transport down while a peer still talks to it (Gloo aborts the process then)."""
        if self.world > 1 and dist.is_initialized():
            if not self.degraded:
                try:
                    dist.barrier()
                except Exception:       # pragma: no cover - peers already gone
                    pass
            dist.destroy_process_group()


class SubComm(Comm):
    """A view of ``parent`` restricted to ranks [0, k): the same rank numbers (rank 0 stays the
    coordinator), collectives on the prefix's own data / control groups, the parent's store."""

    def __init__(self, parent: Comm, k: int, group, ctrl):
        super().__init__()
        self.parent = parent
        self.rank, self.world, self.local_rank = parent.rank, k, parent.local_rank
        self.backend, self.device, self.gen = parent.backend, parent.device, parent.gen
        self.group, self.ctrl = group, ctrl

    @property
    def enabled(self):
        return self.world > 1 and not self.parent.degraded

    def store(self):
        return self.parent.store()

    def shutdown(self):     # the parent owns the process group
        pass


_COMM = Comm()


def get_comm() -> Comm:
    return _COMM


def init_from_env(backend=None, timeout_s=600, join=True) -> Comm:
    """Initialise from torchrun env (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR / MASTER_PORT).
    ``join=False``: rank, world and device only (a replacement rank joins later through ``reinit``)."""
    c = _COMM
    world = int(os.environ.get("WORLD_SIZE", "1"))
    c.rank = int(os.environ.get("RANK", "0"))
    c.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    c.world = world
    use_gpu = torch.cuda.is_available() and backend != "gloo"
    if os.environ.get("CGS_SHARED_GPU") == "1" and torch.cuda.is_available():
        # rehearsal: every rank on the SAME card over Gloo (the 1-GPU development box); device tensors in
        # the model-parallel collectives are staged through host memory (parallel/coll.py)
        backend, use_gpu = "gloo", False
        dev = c.local_rank % torch.cuda.device_count()
        torch.cuda.set_device(dev)
        c.device = torch.device("cuda", dev)
    if use_gpu:
        torch.cuda.set_device(c.local_rank)
        c.device = torch.device("cuda", c.local_rank)
    if world > 1 and not join:
        c.backend = backend or ("nccl" if use_gpu else "gloo")
    elif world > 1 and not dist.is_initialized():
        c.backend = backend or ("nccl" if use_gpu else "gloo")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = dict(backend=c.backend, timeout=datetime.timedelta(seconds=timeout_s))
        if c.backend == "nccl":
            kw["device_id"] = c.device
        dist.init_process_group(**kw)
        if c.backend == "nccl":
            c.ctrl = dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=timeout_s))
    elif dist.is_initialized():
        c.backend = dist.get_backend()
    return c
