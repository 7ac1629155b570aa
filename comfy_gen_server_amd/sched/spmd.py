"""SPMD execution of one prompt on every rank of the node, with its image batch split by GLOBAL index.

Reference path: ``server.py:633-672`` (POST /prompt) -> ``execution.py:526`` (PromptExecutor) ->
``nodes.py:1420-1439`` (``common_ksampler``): one process, one GPU, the whole batch. Here every rank
runs the same graph with the same executor state (an executor that only ever sees SPMD prompts, so its
output caches stay identical across ranks and every rank reaches the same collectives in the same
order), and:

* the sampler nodes (``common_ksampler``) take rank r's slice ``[off, off + n)`` of the latent batch.
  Initial noise (``prepare_noise`` batch-index replay) and every per-step ancestral / SDE draw are
  keyed by the image's global index (``sampling/rng.py``), so the union of the shards is bit-for-bit
  the batch a single GPU computes. The output LATENT carries ``dp_shard = (off, n, B)``;
* ``VAEDecode`` / ``VAEDecodeTiled`` decode the local shard; their IMAGE output is marked with the same
  shard (a tensor attribute);
* any other node that receives a sharded value first all-gathers it (RCCL over xGMI on the GPU, Gloo on
  the CPU) -- correctness never depends on a node knowing about sharding;
* per-image conditioning is sharded with the latent: a ControlNet hint batch, ``concat_latent_image``
  / ``concat_mask`` (inpaint) and any other conditioning tensor whose batch equals the latent batch
  is cut to the same ``[off, off + n)`` window (``shard_conds``); a batch smaller than the node runs
  replicated (every rank computes it whole), never with empty shards;
* ``SaveImage`` / ``PreviewImage`` of a sharded IMAGE: rank 0 reserves the file names of the whole
  batch and broadcasts them (a few hundred bytes on the Gloo control group); every rank PNG-encodes
  and writes its own images; rank 0 returns the ``ui`` records of all. Other output nodes gather
  their sharded inputs to rank 0 only (``gather``, not an all-gather) and run there;
* agreement: every node is bracketed by two max-reductions on the Gloo control group -- before it
  (interrupt flag, or a failure while building its inputs) and after it (failure while running it).
  A node that raises on one rank therefore stops every rank at the same collective, with the same
  number of collectives issued on each (``PeerNodeError`` on the ranks that did not fail), and the
  next prompt starts from a consistent state;
* ``mode = "latency"`` (a batch smaller than the node): nothing is sharded; every rank runs the whole
  prompt and each UNet call is split CFG- and token-parallel over the ranks (``parallel/latency.py``),
  so one image finishes sooner.
"""
from __future__ import annotations

import contextvars
import os

import torch

_CTX: contextvars.ContextVar = contextvars.ContextVar("cgs_spmd", default=None)

# node classes that consume / produce shards themselves
SHARD_AWARE = frozenset({"KSampler", "KSamplerAdvanced", "VAEDecode", "VAEDecodeTiled"})
# image savers that write a sharded IMAGE from every rank (rank 0 only names the files)
SHARDED_SAVERS = frozenset({"SaveImage", "PreviewImage"})
_SHARD_ATTR = "_cgs_dp_shard"


class PeerNodeError(RuntimeError):
    """A node of an SPMD prompt failed on another rank; this rank stops at the same node."""


class SPMD:
    def __init__(self, comm):
        self.comm = comm
        self.rank, self.world = comm.rank, comm.world
        self.images_sampled = 0       # images this rank sampled in SPMD prompts (shard sizes)
        self._seq = 0                 # agreement sequence number (identical on every rank)
        self._stage = 2
        # "spmd": split the image batch; "latency": every rank runs the whole (small) batch and each
        # UNet call is split CFG-/token-parallel over the ranks (parallel/latency.py)
        self.mode = "spmd"
        self.latency = None
        self.loads_received = 0       # checkpoints this rank got over the data plane instead of the disk
        self.reserved: list = []      # rank 0: PNG names reserved by the current prompt's sharded saves
        from ..parallel.comm import SubComm
        if comm.world > 1 and comm.enabled and not isinstance(comm, SubComm):
            from ..parallel.latency import LatencyParallel
            self.latency = LatencyParallel(comm)    # collective: every rank builds its SPMD context once

    def load_state_dict(self, path, device, return_metadata, load_local):
        """R3 inside an SPMD prompt: rank 0 reads the checkpoint, every other rank of the prompt receives
        it (``Comm.broadcast_state_dict``) -- one disk read per node. A failed read fails every rank. A
        checkpoint that is not a flat tensor dict (nested ``.pth`` upscalers, hypernetworks, ``.bin``
        files) is read by every rank itself."""
        from ..parallel.comm import LOAD_LOCALLY, is_flat_tensor_dict
        comm = self.comm
        if self.rank == 0:
            try:
                res = load_local()
            except Exception as ex:   # noqa: BLE001 - re-raised on every rank by the broadcast
                comm.broadcast_state_dict(ex, device)
                raise
            sd, meta = res if return_metadata else (res, None)
            comm.broadcast_state_dict(sd, device)
            if return_metadata and is_flat_tensor_dict(sd):
                comm.broadcast_object(meta)
        else:
            sd = comm.broadcast_state_dict(None, device)
            if sd is LOAD_LOCALLY:
                return load_local()
            meta = comm.broadcast_object(None) if return_metadata else None
            self.loads_received += 1
        return (sd, meta) if return_metadata else sd

    def cleanup_reserved(self):
        """After a failed (or re-run) prompt: remove the reserved placeholder files no rank wrote (still
        empty; a written PNG is renamed into place whole), so failures leave no zero-byte images."""
        for path in self.reserved:
            try:
                if os.path.getsize(path) == 0:
                    os.remove(path)
            except OSError:
                pass
        self.reserved = []

    def shard(self, total: int):
        """(offset, count) of this rank's images of a batch of ``total`` (even split, remainder first)."""
        return shard_range(total, self.rank, self.world)

    # -------------------------------------------------------------- gathers of sharded values
    def gather_tensor(self, t: torch.Tensor, total: int, to_all: bool = True):
        """Concatenate every rank's shard of a batch of ``total`` along dim 0: on every rank
        (``to_all``: a replicated node needs it everywhere) or on rank 0 only (``gather``: an output
        node runs there; each shard crosses one link once). Non-zero ranks get None then."""
        per = -(-total // self.world)
        dev = self.comm.device if self.comm.backend == "nccl" else torch.device("cpu")
        pad = torch.zeros((per,) + tuple(t.shape[1:]), dtype=t.dtype, device=dev)
        pad[:t.shape[0]] = t.to(dev)
        full = self.comm.all_gather(pad) if to_all else self.comm.gather(pad, dst=0)
        if full is None:
            return None
        parts = []
        for r in range(self.world):
            off, n = shard_range(total, r, self.world)
            parts.append(full[r * per:r * per + n])
        return torch.cat(parts).to(t.device)

    def unshard(self, v, to_all: bool = True):
        if isinstance(v, dict) and "dp_shard" in v:
            off, n, total = v["dp_shard"]
            out = {k: x for k, x in v.items() if k != "dp_shard"}
            out["samples"] = self.gather_tensor(v["samples"], total, to_all)
            mask = v.get("noise_mask")
            if torch.is_tensor(mask) and mask.dim() >= 1 and mask.shape[0] == n and n != total:
                out["noise_mask"] = self.gather_tensor(mask, total, to_all)
            return out
        if torch.is_tensor(v) and getattr(v, _SHARD_ATTR, None) is not None:
            off, n, total = getattr(v, _SHARD_ATTR)
            return self.gather_tensor(v, total, to_all)
        return v

    # -------------------------------------------------------------- executor hook
    def node_begin(self):
        """A node's first agreement point is next (called before its inputs are built)."""
        self._stage = 0

    def _agree(self, code: float) -> float:
        """Max of ``code`` over the ranks. Through the c10d TCPStore hosted by rank 0 rather than a
        collective: a store wait can be interrupted, so a rank that died (rank 0 publishes
        ``cgs/dead`` when a worker's connection drops) fails the agreement within ~1 s instead of
        stranding the survivors in a collective until the process-group timeout."""
        import datetime
        self._stage = getattr(self, "_stage", 0) + 1
        st = self.comm.store()
        if st is None or self.world <= 1:
            return code
        self._seq += 1
        base = f"cgs/agree/g{self.comm.gen}/k{self.world}/{self._seq}"
        st.set(f"{base}/{self.rank}", repr(float(code)))
        keys = [f"{base}/{r}" for r in range(self.world)]
        while True:
            try:
                st.wait(keys, datetime.timedelta(seconds=1.0))
                break
            except Exception:   # timed out: still waiting for a peer -- or the peer is gone
                if st.check(["cgs/dead"]):
                    dead = [int(x) for x in st.get("cgs/dead").decode().split(",") if x]
                    if any(r < self.world for r in dead):     # a member of THIS prompt's ranks
                        self._stage = 2
                        raise PeerNodeError("a rank of the SPMD prompt died (%s)" % dead)
        v = max(float(st.get(k).decode()) for k in keys)
        if self._seq > 2:       # every rank read seq - 2 before it wrote seq - 1: its key is dead
            try:
                st.delete_key(f"cgs/agree/g{self.comm.gen}/k{self.world}/{self._seq - 2}/{self.rank}")
            except Exception:   # pragma: no cover - stores without delete
                pass
        return v

    def abort(self):
        """Exception path of a node on this rank: take part in the node's remaining agreement point with
        a failure flag, so the peers stop at the same point (one agreement, whichever is pending)."""
        if getattr(self, "_stage", 2) < 2:
            try:
                self._agree(1.0)
            except PeerNodeError:
                pass
        self._stage = 2

    def execute(self, class_type, class_def, obj, input_data_all, run):
        """Run one node of an SPMD prompt: agree (interrupt / failure), unshard what it cannot take
        sharded, run it (output nodes on rank 0; sharded image savers everywhere), agree again.
        ``run(obj, inputs) -> (outputs, ui)``."""
        from ..runtime import device as dm
        v = self._agree(2.0 if dm.processing_interrupted() else 0.0)
        if v > 0:
            self._stage = 2
            if v >= 2:
                dm.interrupt_current_processing(False)
                raise dm.InterruptProcessingException()
            raise PeerNodeError(f"{class_type}: the prompt failed on another rank")
        try:
            out = self._run(class_type, class_def, obj, input_data_all, run)
        except Exception:
            self.abort()        # the peers learn at the second agreement point; this rank's error stands
            raise
        v = self._agree(0.0)
        self._stage = 2
        if v > 0:
            raise PeerNodeError(f"{class_type}: the node failed on another rank")
        return out

    def _run(self, class_type, class_def, obj, input_data_all, run):
        if class_type in SHARDED_SAVERS and self._sharded_images(input_data_all) is not None:
            return self._save_sharded(obj, input_data_all)
        output_node = bool(getattr(class_def, "OUTPUT_NODE", False))
        if class_type not in SHARD_AWARE:
            input_data_all = {k: [self.unshard(x, to_all=not output_node) for x in vals]
                              for k, vals in input_data_all.items()}
        if output_node and self.rank != 0:
            return [], {}
        out, ui = run(obj, input_data_all)
        return self.after(class_type, input_data_all, out), ui

    @staticmethod
    def _sharded_images(input_data_all):
        imgs = input_data_all.get("images") or []
        if len(imgs) == 1 and torch.is_tensor(imgs[0]) and getattr(imgs[0], _SHARD_ATTR, None) is not None:
            return imgs[0]
        return None

    def _save_sharded(self, obj, input_data_all):
        """SaveImage / PreviewImage of a sharded batch: rank 0 reserves ``{prefix}_{counter:05}_.png`` for
        every image of the batch and broadcasts the names; each rank encodes and writes its own."""
        import json
        from ..nodes import helpers as NH
        from ..utils import folder_paths
        from ..utils.imageio import write_png_files
        images = self._sharded_images(input_data_all)
        off, n, total = getattr(images, _SHARD_ATTR)
        prefix = (input_data_all.get("filename_prefix") or ["ComfyUI"])[0]
        plan = None
        if self.rank == 0:
            from ..utils.imageio import reserve_png_names
            out_dir = (folder_paths.get_output_directory() if getattr(obj, "type", "output") == "output"
                       else folder_paths.get_temp_directory())
            folder, filename, counter, subfolder, _ = folder_paths.get_save_image_path(
                prefix + getattr(obj, "prefix_append", ""), out_dir, images.shape[2], images.shape[1])
            names = reserve_png_names(folder, filename, counter, total)
            self.reserved += [os.path.join(folder, nm) for nm in names]
            plan = (folder, subfolder, names, getattr(obj, "type", "output"))
        folder, subfolder, names, typ = self.comm.broadcast_object(plan)
        from ..utils import telemetry
        telemetry.maybe_fault("node", "SaveImageWrite")   # fault site: names reserved, this rank's not written
        metadata = None
        if not NH.args_disable_metadata():
            metadata = {}
            prompt = (input_data_all.get("prompt") or [None])[0]
            extra = (input_data_all.get("extra_pnginfo") or [None])[0]
            if prompt is not None:
                metadata["prompt"] = json.dumps(prompt)
            if extra is not None:
                for x in extra:
                    metadata[x] = json.dumps(extra[x])
        write_png_files(images, [os.path.join(folder, nm) for nm in names[off:off + n]], metadata,
                        getattr(obj, "compress_level", 4))
        if self.rank != 0:
            return [], {}
        return [], {"images": [{"filename": nm, "subfolder": subfolder, "type": typ} for nm in names]}

    def after(self, class_type, input_data_all, output_data):
        """Propagate the shard mark through the shard-aware decoders (LATENT shard -> IMAGE shard)."""
        if class_type not in ("VAEDecode", "VAEDecodeTiled"):
            return output_data
        shard = None
        for vals in input_data_all.values():
            for x in vals:
                if isinstance(x, dict) and "dp_shard" in x:
                    shard = x["dp_shard"]
        if shard is None:
            return output_data
        for out in output_data:
            for t in out:
                if torch.is_tensor(t):
                    setattr(t, _SHARD_ATTR, shard)
        return output_data


def shard_range(total: int, rank: int, world: int):
    per, rem = total // world, total % world
    return rank * per + min(rank, rem), per + (1 if rank < rem else 0)


def active() -> SPMD | None:
    return _CTX.get()


def latency_model(model):
    """In a latency-mode prompt: ``model`` (ModelPatcher) with its UNet calls split over the ranks."""
    ctx = active()
    if ctx is None or ctx.mode != "latency" or ctx.latency is None:
        return model
    return ctx.latency.patch(model)


class activate:
    """``with spmd.activate(ctx[, mode]): executor.execute(...)`` -- the SPMD context of this thread."""

    def __init__(self, ctx: SPMD, mode: str = "spmd"):
        self.ctx, self.mode = ctx, mode

    def __enter__(self):
        self.prev_mode, self.ctx.mode = self.ctx.mode, self.mode
        self.tok = _CTX.set(self.ctx)
        return self.ctx

    def __exit__(self, *exc):
        _CTX.reset(self.tok)
        self.ctx.mode = self.prev_mode


def shard_latent(latent: dict):
    """In an SPMD prompt: this rank's part of a LATENT (already sharded or not) ->
    (local dict, global batch indices, (off, n, total)); outside, in latency mode or for a batch
    smaller than the node (run replicated: no empty shards): (latent, batch_index, None)."""
    ctx = active()
    if ctx is None or ctx.mode == "latency":
        return latent, latent.get("batch_index"), None
    if "dp_shard" in latent:
        off, n, total = latent["dp_shard"]
        ctx.images_sampled += n
        local = dict(latent)
        inds = latent.get("batch_index")
        inds = list(inds[off:off + n]) if inds is not None else list(range(off, off + n))
        mask = latent.get("noise_mask")   # a full-batch mask set after the first sampler
        if torch.is_tensor(mask) and mask.dim() >= 1 and mask.shape[0] == total and total > n:
            local["noise_mask"] = mask[off:off + n]
        return local, inds, (off, n, total)
    total = latent["samples"].shape[0]
    if total < ctx.world:
        ctx.images_sampled += total
        return latent, latent.get("batch_index"), None
    off, n = ctx.shard(total)
    ctx.images_sampled += n
    local = dict(latent)
    local["samples"] = latent["samples"][off:off + n]
    inds = latent.get("batch_index")
    inds = list(inds[off:off + n]) if inds is not None else list(range(off, off + n))
    mask = latent.get("noise_mask")
    if torch.is_tensor(mask) and mask.dim() >= 1 and mask.shape[0] == total and total > 1:
        local["noise_mask"] = mask[off:off + n]
    return local, inds, (off, n, total)


def _slice(v, off, n, total):
    if torch.is_tensor(v) and v.dim() >= 1 and total > n and v.shape[0] == total:
        return v[off:off + n]
    return v


def _shard_control(c, off, n, total):
    """A ControlNet / T2I-adapter chain whose hint batches equal the latent batch, cut to the shard
    (copies: the cached conditioning of other prompts / ranks is never touched)."""
    if c is None:
        return None
    prev = getattr(c, "previous_controlnet", None)
    prev2 = _shard_control(prev, off, n, total)
    hint = getattr(c, "cond_hint_original", None)
    hint2 = _slice(hint, off, n, total)
    if hint2 is hint and prev2 is prev:
        return c
    c2 = c.copy()
    c2.cond_hint_original = hint2
    c2.set_previous_controlnet(prev2)
    return c2


def shard_conds(conds, shard):
    """This rank's window of per-image conditioning (``shard = (off, n, total)`` from shard_latent):
    the cond tensor itself, ControlNet hints, ``concat_latent_image`` / ``concat_mask`` and any other
    conditioning tensor whose batch is the latent batch (the reference broadcasts those per image:
    ``controlnet.py`` ``broadcast_image_to``, ``model_base.py`` ``repeat_to_batch_size``)."""
    if shard is None or conds is None:
        return conds
    off, n, total = shard
    out = []
    for entry in conds:
        t, d = entry[0], entry[1]
        d2 = {}
        for k, v in d.items():
            if k == "control":
                d2[k] = _shard_control(v, off, n, total)
            else:
                d2[k] = _slice(v, off, n, total)
        out.append([_slice(t, off, n, total), d2] + list(entry[2:]))
    return out
