"""Latency mode: one prompt's images across the GPUs of a node (SURVEY §2.5 SP rows, §5.7).

Data parallelism has nothing to split when a single image (B = 1) is wanted fast, or when one very
large image does not fit a throughput schedule. The reference has no multi-device path at all; here
a UNet call of batch B (= 2 x images: cond + uncond, CFG-batched by ``calc_cond_batch``) runs on P
ranks as

* **batch split** (CFG parallel): the P ranks form G = gcd(P, B) batch groups; group g evaluates rows
  [g*B/G, (g+1)*B/G) -- for one image at P = 2, rank 0 the conditional pass and rank 1 the
  unconditional one -- and the outputs are all-gathered (one collective per UNet call);
* **spatial parallel** inside a group of Q = P/G ranks (``spatial.py``, the default when the latent
  height divides into Q bands at every UNet level and no model patch is installed): every layer of
  the UNet -- ResBlocks included -- runs on the rank's band of rows (halo rows for 3 x 3 convs,
  group-summed GroupNorm statistics, self-attention over the whole image through ``SeqParallel``),
  and the output rows are all-gathered: ~1/Q of the UNet FLOPs per rank;
* otherwise **token parallel** in the group (``SeqParallel``): every SpatialTransformer keeps only the
  rank's token shard through its blocks (self-attention via Ulysses all-to-all or K/V all-gather,
  cross-attention local), then all-gathers the tokens back for the ResBlocks, which run replicated.
  ``CGS_LATENCY_SPATIAL=0`` forces this form.

Every rank runs the same sampler loop on the same latents (same seed, same noise: the per-image
Philox streams of ``sampling/rng.py``), so the results are bit-compatible with each other and match
the single-GPU run to kernel-rounding. The whole mode is a ``model_function_wrapper`` +
``transformer_options["sp"]`` on a patcher clone: ``LatencyParallel(comm).patch(patcher)``.
"""
from __future__ import annotations

import math
import os

import torch
import torch.distributed as dist

from . import coll, spatial
from .sp import SeqParallel


class LatencyParallel:
    def __init__(self, comm, batch: int = 2):
        """``batch``: the UNet batch the mode is laid out for (2 = one image with CFG). Creates the
        batch-group / token-group process groups (collective: every rank calls this)."""
        self.comm = comm
        P = comm.world if comm.enabled else 1
        self.P = P
        self.G = math.gcd(P, batch) if P > 1 else 1       # batch groups
        self.Q = P // self.G                               # ranks per token group
        self.rank = comm.rank if comm.enabled else 0
        self.bg = self.rank // self.Q                      # my batch group
        self.tok_group = None
        self.cross_group = None                            # the G ranks holding the same token shard
        if P > 1:
            for g in range(self.G):
                ranks = list(range(g * self.Q, (g + 1) * self.Q))
                pg = dist.new_group(ranks) if self.Q > 1 else None
                if g == self.bg:
                    self.tok_group = pg
            for q in range(self.Q):
                ranks = [g * self.Q + q for g in range(self.G)]
                pg = dist.new_group(ranks) if self.G > 1 else None
                if q == self.rank % self.Q:
                    self.cross_group = pg
        self.sp = SeqParallel(self.tok_group) if self.Q > 1 else None
        self.spatial = None
        if self.Q > 1:
            ranks = [self.bg * self.Q + q for q in range(self.Q)]
            self.spatial = spatial.SpatialShard(self.tok_group, self.Q, self.rank % self.Q, ranks)
        self.spatial_calls = 0
        self.calls = 0

    @staticmethod
    def _row_shardable(apply_model):
        """Only networks whose every layer is band-aware: the openaimodel UNet (``UNetModel.row_shardable``).
        Cascade's depthwise convs / GRN and any other family would treat band edges as image edges."""
        owner = getattr(apply_model, "__self__", None)
        net = getattr(owner, "diffusion_model", None)
        return getattr(net, "row_shardable", False) is True

    def _spatial_ok(self, x, c, apply_model=None):
        """Row sharding applies: a row-shardable network (see ``_row_shardable``), a band per rank at every
        level (height divisible by Q * 8: up to three 2x downsamples, >= 1 row per band), no model patches
        (their hooks see whole images)."""
        if self.spatial is None or os.environ.get("CGS_LATENCY_SPATIAL", "1") == "0":
            return False
        if not self._row_shardable(apply_model):
            return False
        to = c.get("transformer_options", {})
        if to.get("patches") or to.get("patches_replace"):
            return False
        return x.dim() == 4 and x.shape[2] % (self.Q * 8) == 0

    def _apply_spatial(self, apply_model, x, t, c):
        """One UNet call on this rank's band of rows (latent, c_concat and ControlNet residuals cut to
        the band), the output rows all-gathered over the token group."""
        sc = self.spatial
        c = dict(c)
        if torch.is_tensor(c.get("c_concat")) and c["c_concat"].dim() == 4:
            c["c_concat"] = sc.shard_rows(c["c_concat"])
        ctrl = c.get("control")
        if isinstance(ctrl, dict):
            c["control"] = {k: [sc.shard_rows(v) if torch.is_tensor(v) and v.dim() == 4 else v for v in vs]
                            for k, vs in ctrl.items()}
        self.spatial_calls += 1
        with spatial.active(sc):
            out = apply_model(sc.shard_rows(x).contiguous(), t, **c)
        return sc.gather_rows(out)

    # --------------------------------------------------------------------------------------------
    def _slice(self, v, B, lo, hi):
        if isinstance(v, torch.Tensor) and v.dim() > 0 and v.shape[0] == B:
            return v[lo:hi]
        if isinstance(v, dict):
            return {k: self._slice(x, B, lo, hi) for k, x in v.items()}
        if isinstance(v, list):
            return [self._slice(x, B, lo, hi) for x in v]
        return v

    def wrapper(self, apply_model, args):
        """``model_function_wrapper``: evaluate this rank's batch slice, all-gather the rest."""
        x, t, c = args["input"], args["timestep"], dict(args["c"])
        self.calls += 1
        B = x.shape[0]
        to = dict(c.get("transformer_options", {}))
        if self.sp is not None:
            to["sp"] = self.sp
        c["transformer_options"] = to
        if self.G == 1 or B % self.G:
            if self._spatial_ok(x, c, apply_model):
                return self._apply_spatial(apply_model, x, t, c)
            return apply_model(x, t, **c)
        n = B // self.G
        lo, hi = self.bg * n, (self.bg + 1) * n
        cs = self._slice(c, B, lo, hi)
        if self._spatial_ok(x, cs, apply_model):
            out = self._apply_spatial(apply_model, x[lo:hi], t[lo:hi], cs)
        else:
            out = apply_model(x[lo:hi], t[lo:hi], **cs)
        parts = [torch.empty_like(out) for _ in range(self.G)]
        coll.all_gather(parts, out.contiguous(), group=self.cross_group)
        return torch.cat(parts, 0)

    def patch(self, patcher):
        """A clone of ``patcher`` whose UNet calls run in latency mode (graph capture stays off for
        it: the wrapper's collectives run eagerly)."""
        m = patcher.clone()
        if self.P > 1:
            m.set_model_unet_function_wrapper(self.wrapper)
        return m
