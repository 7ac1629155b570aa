"""Data-parallel text-to-image across the GPUs of a node (BASELINE config 5).

One process per GPU. A job = (prompt, negative, batch, seed, steps, cfg, sampler, scheduler, size).
Rank 0 owns the job and broadcasts it (R1); each rank generates its slice of the batch with the
reference's per-index noise replay (``prepare_noise`` with ``batch_index`` = the image's global
index) for the initial latent, and the per-step ancestral/SDE noise keyed by the same global index
(``sampling/rng.py``), so a DP run is identical to a single-GPU run of the whole batch; the decoded
uint8 images are gathered to rank 0 (R2), which encodes/saves them.

Everything per rank is the standard single-GPU path (CLIP -> CFGGuider/KSampler -> VAE), so the
DP engine scales whatever the kernels deliver on one GPU.
"""
from __future__ import annotations

import dataclasses
import os
import time

import torch

from ..runtime import device as dm
from ..sampling import sample as S
from .comm import get_comm


@dataclasses.dataclass
class Job:
    prompt: str = "a photo of an astronaut riding a horse on mars, highly detailed"
    negative: str = "blurry, low quality"
    batch: int = 8
    seed: int = 0
    steps: int = 20
    cfg: float = 8.0
    sampler: str = "euler_ancestral"
    scheduler: str = "normal"
    width: int = 1024
    height: int = 1024


def encode_prompt(clip, text, width, height):
    """CLIPTextEncode (+ SDXL size conds) -> CONDITIONING list."""
    tokens = clip.tokenize(text)
    cond, pooled = clip.encode_from_tokens(tokens, return_pooled=True)
    meta = {"pooled_output": pooled}
    return [[cond, meta]]


STAGE_TIMES: dict = {}


class _stage:
    """Optional per-stage wall time (CGS_STAGE_TIMING=1): synchronises the device at both ends."""

    def __init__(self, name):
        self.name = name
        self.on = os.environ.get("CGS_STAGE_TIMING", "0") == "1"

    def __enter__(self):
        if self.on:
            dm.synchronize()
            self.t = time.perf_counter()

    def __exit__(self, *a):
        if self.on:
            dm.synchronize()
            STAGE_TIMES.setdefault(self.name, []).append(time.perf_counter() - self.t)


def generate_local(patcher, clip, vae, job: Job, index_offset: int, local_batch: int, conds=None, decode=True):
    """Generate images [index_offset, index_offset+local_batch) of ``job`` on this rank
    (``decode=False``: return the sampled latents instead of decoded images)."""
    lat_c = 4
    latent = torch.zeros([local_batch, lat_c, job.height // 8, job.width // 8])
    with _stage("clip"):
        if conds is None:
            pos = encode_prompt(clip, job.prompt, job.width, job.height)
            neg = encode_prompt(clip, job.negative, job.width, job.height)
        else:
            pos, neg = conds
    # per-image noise replay (latent "batch_index" semantics): identical for any rank split
    inds = list(range(index_offset, index_offset + local_batch))
    noise = S.prepare_noise(latent, job.seed, noise_inds=inds)
    with _stage("sample"):
        samples = S.sample(patcher, noise, job.steps, job.cfg, job.sampler, job.scheduler, pos, neg, latent,
                           denoise=1.0, seed=job.seed, noise_inds=inds)
    if not decode:
        return samples
    with _stage("vae"):
        if decode == "uint8":
            return vae.decode_uint8(samples)
        return vae.decode(samples)


def to_uint8(images: torch.Tensor) -> torch.Tensor:
    return (images.clamp(0, 1) * 255.0 + 0.5).to(torch.uint8)


class DataParallelGenerator:
    def __init__(self, patcher, clip, vae):
        self.patcher, self.clip, self.vae = patcher, clip, vae
        self.comm = get_comm()

    def sync_weights(self):
        """R3: make every rank's weights identical to rank 0's (one disk read per node)."""
        c = self.comm
        if not c.enabled:
            return
        c.broadcast_module(self.patcher.model.diffusion_model)
        if self.clip is not None:
            c.broadcast_module(self.clip.cond_stage_model)
        if self.vae is not None:
            c.broadcast_module(self.vae.first_stage_model)

    def _shard(self, job, r):
        c = self.comm
        per, rem = job.batch // c.world, job.batch % c.world
        return r * per + min(r, rem), per + (1 if r < rem else 0)

    def run(self, job: Job, gather=True, fault_tolerant=None):
        """Whole-node job: ``job.batch`` images split evenly across ranks -> uint8 [B,H,W,3] on rank 0.

        ``fault_tolerant`` (default: env ``CGS_DP_FAULT_TOLERANT=1``): before gathering, liveness is
        checked on the gloo control group; if ranks died, the survivors ship their shards to rank 0
        point-to-point and rank 0 regenerates the dead ranks' shards itself (per-image noise replay
        makes them identical to what the dead rank would have produced) — the job completes, and
        the engine marks itself degraded (later jobs run on rank 0 alone)."""
        c = self.comm
        if fault_tolerant is None:
            fault_tolerant = os.environ.get("CGS_DP_FAULT_TOLERANT", "0") == "1"
        if getattr(self, "degraded", False):
            # degraded (after a rank failure): rank 0 alone serves whole jobs; other survivors idle
            if c.rank != 0:
                return None
            return generate_local(self.patcher, self.clip, self.vae, job, 0, job.batch, decode="uint8")
        job = c.broadcast_object(job)
        c.heartbeat_fault_site()
        offset, local = self._shard(job, c.rank)
        u8 = generate_local(self.patcher, self.clip, self.vae, job, offset, local, decode="uint8")
        if gather and c.enabled and fault_tolerant:
            rid, dead = c.liveness_round(float(os.environ.get("CGS_DP_LIVENESS_TIMEOUT", "30")))
            if dead:
                return self._recover(job, u8, dead, rid)
        if gather and c.enabled:
            return self._gather_plain(job, u8)
        return u8

    def _gather_plain(self, job, u8):
        """Shards -> rank 0 (None on the other ranks)."""
        c = self.comm
        if not c.enabled:
            return u8
        per, rem = job.batch // c.world, job.batch % c.world
        local = u8.shape[0]
        if rem:
            pad = torch.zeros((per + 1 - local,) + tuple(u8.shape[1:]), dtype=u8.dtype, device=u8.device)
            u8 = torch.cat([u8, pad])
        allimgs = c.gather(u8.to(c.device), dst=0)
        if allimgs is None:
            return None
        if rem:
            keep = []
            for r in range(c.world):
                n = per + (1 if r < rem else 0)
                keep.append(allimgs[r * (per + 1): r * (per + 1) + n])
            allimgs = torch.cat(keep)
        return allimgs

    def run_many(self, jobs, pipeline=None):
        """Serve a stream of jobs; yields each job's uint8 images (rank 0: the whole batch).

        ``pipeline`` (default: env ``CGS_DP_PIPELINE=1``): prompt-level multi-stream overlap (SURVEY
        §2.5 "multi-stream" row, §7.2 step 9). Job n's VAE decode + image all-gather are issued on a
        side HIP stream, ordered after job n's sampling by an event, while the host goes on to issue
        job n+1's CLIP encode and sampler steps on the main stream -- the two share the GPU, so the
        VAE's low-occupancy phases (small-spatial convs, GroupNorm reductions, the one-workgroup-
        per-CU mid attention) and the host gaps between jobs are filled with UNet work. Results come
        out one job late, in order, with the main stream made to wait for them. The liveness /
        recovery protocol of ``run(fault_tolerant=True)`` is not used on this path.

        Multi-rank ordering: the job broadcast goes over the Gloo control group (host), so the ONLY
        RCCL collective inside the loop is the image gather, always issued on the side stream --
        one communicator, one stream, the same order on every rank. Anything issued on the main
        stream after the loop (barrier, timing reduce) follows ``_collect``'s wait on the last
        gather's event."""
        c = self.comm
        if pipeline is None:
            pipeline = os.environ.get("CGS_DP_PIPELINE", "0") == "1"
        use_side = pipeline and torch.cuda.is_available() and dm.get_torch_device().type == "cuda"
        side = torch.cuda.Stream(device=dm.get_torch_device()) if use_side else None
        pending = None
        for job in jobs:
            job = c.broadcast_object(job)
            c.heartbeat_fault_site()
            offset, local = self._shard(job, c.rank)
            if side is None:
                u8 = generate_local(self.patcher, self.clip, self.vae, job, offset, local, decode="uint8")
                yield self._gather_plain(job, u8)
                continue
            samples = generate_local(self.patcher, self.clip, self.vae, job, offset, local, decode=False)
            sampled = torch.cuda.Event()
            sampled.record()
            with torch.cuda.stream(side):
                side.wait_event(sampled)
                samples.record_stream(side)
                with _stage("vae"):
                    out = self._gather_plain(job, self.vae.decode_uint8(samples))
                done = torch.cuda.Event()
                done.record(side)
            if pending is not None:
                yield self._collect(*pending)
            pending = (out, done)
        if pending is not None:
            yield self._collect(*pending)

    @staticmethod
    def _collect(out, done):
        cur = torch.cuda.current_stream()
        cur.wait_event(done)
        if out is not None and out.is_cuda:      # gloo gathers return host tensors (no stream to record)
            out.record_stream(cur)
        return out

    def _recover(self, job, u8, dead, rid):
        """Degraded gather: survivors hand their shards to rank 0 through the store,
        rank 0 recomputes the dead ranks' shards and assembles the whole batch."""
        import logging
        c = self.comm
        self.degraded = True
        c.degraded = True     # collectives over the broken group become local no-ops from here on
        if c.rank != 0:
            c.store_put_tensor(f"cgs/shard/{rid}/{c.rank}", u8)
            return None
        logging.error("DP ranks %s failed; recomputing their shards on rank 0", dead)
        parts = {0: u8.cpu()}
        for r in range(1, c.world):
            if r in dead:
                off, n = self._shard(job, r)
                parts[r] = generate_local(self.patcher, self.clip, self.vae, job, off, n, decode="uint8").cpu()
            else:
                parts[r] = c.store_get_tensor(f"cgs/shard/{rid}/{r}")
        return torch.cat([parts[r] for r in range(c.world)])


def images_per_sec(batch, seconds):
    return batch / seconds if seconds > 0 else 0.0


def device_sync():
    dm.synchronize()
