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
* output nodes (``OUTPUT_NODE``) gather their inputs to every rank (same collective on all ranks) and
  then run on rank 0 only, which writes the files and sends the WebSocket events;
* interrupts: a rank only stops at a node boundary, where the ranks agree through a max-reduction of
  their interrupt flags on the Gloo control group (an unagreed stop would strand the others in a
  collective);
* ``mode = "latency"`` (a batch smaller than the node): nothing is sharded; every rank runs the whole
  prompt and each UNet call is split CFG- and token-parallel over the ranks (``parallel/latency.py``),
  so one image finishes sooner.
"""
from __future__ import annotations

import contextvars

import torch

_CTX: contextvars.ContextVar = contextvars.ContextVar("cgs_spmd", default=None)

# node classes that consume / produce shards themselves
SHARD_AWARE = frozenset({"KSampler", "KSamplerAdvanced", "VAEDecode", "VAEDecodeTiled"})
_SHARD_ATTR = "_cgs_dp_shard"


class SPMD:
    def __init__(self, comm):
        self.comm = comm
        self.rank, self.world = comm.rank, comm.world
        self.images_sampled = 0       # images this rank sampled in SPMD prompts (shard sizes)
        # "spmd": split the image batch; "latency": every rank runs the whole (small) batch and each
        # UNet call is split CFG-/token-parallel over the ranks (parallel/latency.py)
        self.mode = "spmd"
        self.latency = None
        if comm.world > 1 and comm.enabled:
            from ..parallel.latency import LatencyParallel
            self.latency = LatencyParallel(comm)    # collective: every rank builds its SPMD context once

    def shard(self, total: int):
        """(offset, count) of this rank's images of a batch of ``total`` (even split, remainder first)."""
        return shard_range(total, self.rank, self.world)

    # -------------------------------------------------------------- gathers of sharded values
    def gather_tensor(self, t: torch.Tensor, total: int) -> torch.Tensor:
        """Concatenate every rank's shard of a batch of ``total`` along dim 0 (every rank gets it)."""
        per = -(-total // self.world)
        dev = self.comm.device if self.comm.backend == "nccl" else torch.device("cpu")
        pad = torch.zeros((per,) + tuple(t.shape[1:]), dtype=t.dtype, device=dev)
        pad[:t.shape[0]] = t.to(dev)
        full = self.comm.all_gather(pad)
        parts = []
        for r in range(self.world):
            off, n = shard_range(total, r, self.world)
            parts.append(full[r * per:r * per + n])
        return torch.cat(parts).to(t.device)

    def unshard(self, v):
        if isinstance(v, dict) and "dp_shard" in v:
            off, n, total = v["dp_shard"]
            out = {k: x for k, x in v.items() if k != "dp_shard"}
            out["samples"] = self.gather_tensor(v["samples"], total)
            return out
        if torch.is_tensor(v) and getattr(v, _SHARD_ATTR, None) is not None:
            off, n, total = getattr(v, _SHARD_ATTR)
            return self.gather_tensor(v, total)
        return v

    # -------------------------------------------------------------- executor hook
    def before(self, class_type, class_def, input_data_all):
        """Called before a node runs; returns the (possibly gathered) inputs, or None: skip on this rank."""
        from ..runtime import device as dm
        flag = self.comm.all_reduce_max(1.0 if dm.processing_interrupted() else 0.0)
        if flag > 0:
            dm.interrupt_current_processing(False)
            raise dm.InterruptProcessingException()
        if class_type not in SHARD_AWARE:
            input_data_all = {k: [self.unshard(x) for x in vals] for k, vals in input_data_all.items()}
        if getattr(class_def, "OUTPUT_NODE", False) and self.rank != 0:
            return None
        return input_data_all

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
    (local dict, global batch indices, (off, n, total)); outside: (latent, batch_index, None)."""
    ctx = active()
    if ctx is None or ctx.mode == "latency":
        return latent, latent.get("batch_index"), None
    if "dp_shard" in latent:
        off, n, total = latent["dp_shard"]
        ctx.images_sampled += n
        inds = latent.get("batch_index")
        inds = list(inds[off:off + n]) if inds is not None else list(range(off, off + n))
        return latent, inds, (off, n, total)
    total = latent["samples"].shape[0]
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
