"""Spatial (row-sharded) UNet for latency mode: every layer of the UNet -- ResBlocks included -- runs on
this rank's band of latent rows, so a batch-1 image is split over the token group with ~1/P of the
FLOPs per rank (the token-parallel form of ``sp.py`` shards only the SpatialTransformers and replicates
the ResBlocks, about a third of SDXL's UNet time).

Reference semantics (``comfy/ldm/modules/diffusionmodules/openaimodel.py:235-264`` ResBlock,
``:87-131`` Up/Downsample, ``attention.py`` SpatialTransformer) are preserved exactly: every rank holds
rows ``[r * H / P, (r + 1) * H / P)`` of every feature map at every level and

* 3 x 3 convolutions exchange halo rows with the neighbouring ranks (one row each way for stride 1;
  two rows from above for the stride-2 downsample; one row each way BEFORE the fused nearest-2x
  upsample), convolve the extended band and keep the interior -- the first / last rank's halo is
  zeros, which is the convolution's zero padding;
* GroupNorm statistics are summed over the group (one all-reduce of [N, groups, 2] fp64 per norm);
* the SpatialTransformers take their local rows as their token shard: self-attention runs over the
  whole image through ``SeqParallel.attention`` (Ulysses all-to-all or K/V all-gather), everything
  else is token-local;
* 1 x 1 convolutions, the timestep embedding and the skip concatenations are local.

``LatencyParallel`` (latency.py) enters ``active(ctx)`` around the UNet call, shards the latent (and a
``c_concat`` / ControlNet residuals) by rows and all-gathers the output rows. Needs the latent height
divisible by P * 2^(levels - 1) (SDXL at 1024^2: 128 rows, P <= 8 -> >= 4 rows per rank at level 2).
"""
from __future__ import annotations

import contextvars

import torch
import torch.distributed as dist

_CTX: contextvars.ContextVar = contextvars.ContextVar("cgs_spatial", default=None)


class SpatialShard:
    def __init__(self, group, P: int, rank: int, ranks):
        self.group, self.P, self.rank, self.ranks = group, P, rank, list(ranks)
        self.stats = {"halo": 0, "gn": 0, "gather_fallback": 0}

    # ---- rows ------------------------------------------------------------------------------------
    def band(self, H: int):
        n = H // self.P
        return self.rank * n, (self.rank + 1) * n

    def shard_rows(self, t, dim=2):
        lo, hi = self.band(t.shape[dim])
        return t.narrow(dim, lo, hi - lo)

    def gather_rows(self, t, dim=2):
        if self.P == 1:
            return t
        t = t.contiguous()
        parts = [torch.empty_like(t) for _ in range(self.P)]
        dist.all_gather(parts, t, group=self.group)
        return torch.cat(parts, dim=dim)

    def halo(self, x, top: int, bottom: int):
        """[N, C, top + R + bottom, W]: ``top`` rows from the rank above and ``bottom`` rows from the rank
        below around the local band (zeros at the image edge)."""
        self.stats["halo"] += 1
        N, C, R, W = x.shape
        above, below = self.rank - 1, self.rank + 1
        ops = []
        recv_top = recv_bot = None
        if top:
            recv_top = torch.zeros((N, C, top, W), dtype=x.dtype, device=x.device)
            if above >= 0:
                ops.append(dist.P2POp(dist.irecv, recv_top, self.ranks[above], self.group))
            if below < self.P:    # my last `top` rows are the lower neighbour's top halo
                ops.append(dist.P2POp(dist.isend, x[:, :, R - top:].contiguous(), self.ranks[below], self.group))
        if bottom:
            recv_bot = torch.zeros((N, C, bottom, W), dtype=x.dtype, device=x.device)
            if below < self.P:
                ops.append(dist.P2POp(dist.irecv, recv_bot, self.ranks[below], self.group))
            if above >= 0:        # my first `bottom` rows are the upper neighbour's bottom halo
                ops.append(dist.P2POp(dist.isend, x[:, :, :bottom].contiguous(), self.ranks[above], self.group))
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        parts = [p for p in (recv_top, x, recv_bot) if p is not None]
        out = torch.cat(parts, dim=2)
        return out.contiguous(memory_format=torch.channels_last) if x.is_cuda else out

    # ---- layers ----------------------------------------------------------------------------------
    def conv2d(self, conv_fn, x, kh, stride, padding, upsample2x, x2):
        """A conv of the row-sharded band. ``conv_fn(x, x2) -> y`` runs the single-GPU conv with the
        layer's own padding on whatever band it is given."""
        if x2 is not None:
            x = torch.cat([x, x2.to(x.dtype)], dim=1)
            if x.is_cuda:
                x = x.contiguous(memory_format=torch.channels_last)
        R = x.shape[2]
        if kh == 1 and padding == 0 and stride == 1:
            return conv_fn(x, None)
        if kh == 3 and padding == 1 and stride == 1 and not upsample2x:
            return conv_fn(self.halo(x, 1, 1), None)[:, :, 1:1 + R]
        if kh == 3 and padding == 1 and stride == 2 and not upsample2x and R % 2 == 0:
            return conv_fn(self.halo(x, 2, 0), None)[:, :, 1:1 + R // 2]
        if kh == 3 and padding == 1 and stride == 1 and upsample2x:
            return conv_fn(self.halo(x, 1, 1), None)[:, :, 2:2 + 2 * R]
        # anything else: the whole image, then this rank's rows of the output
        self.stats["gather_fallback"] += 1
        return self.shard_rows(conv_fn(self.gather_rows(x), None))

    def group_norm(self, x, groups, weight, bias, eps, silu=False, pre_add=None, x2=None):
        """GroupNorm over the whole image from band-local sums (fp64 all-reduce of [N, G, 2])."""
        self.stats["gn"] += 1
        if x2 is not None:
            x = torch.cat([x, x2.to(x.dtype)], dim=1)
        xf = x.float()
        if pre_add is not None:
            xf = xf + pre_add.float()[:, :, None, None]
        N, C, R, W = xf.shape
        g = xf.reshape(N, groups, C // groups, R, W)
        s = torch.stack([g.sum(dim=(2, 3, 4), dtype=torch.float64),
                         (g.double() ** 2).sum(dim=(2, 3, 4))], dim=-1)
        dist.all_reduce(s, group=self.group)
        cnt = float((C // groups) * R * W * self.P)
        mean = s[..., 0] / cnt
        var = (s[..., 1] / cnt - mean * mean).clamp_min(0.0)
        rstd = torch.rsqrt(var + eps)
        y = (g - mean.float()[:, :, None, None, None]) * rstd.float()[:, :, None, None, None]
        y = y.reshape(N, C, R, W)
        if weight is not None:
            y = y * weight.float()[None, :, None, None]
        if bias is not None:
            y = y + bias.float()[None, :, None, None]
        if silu:
            y = torch.nn.functional.silu(y)
        y = y.to(x.dtype)
        return y.contiguous(memory_format=torch.channels_last) if x.is_cuda else y


def current() -> SpatialShard | None:
    return _CTX.get()


class active:
    """``with spatial.active(ctx): unet(...)`` -- convs / GroupNorms of this thread run row-sharded."""

    def __init__(self, ctx: SpatialShard | None):
        self.ctx = ctx

    def __enter__(self):
        self.tok = _CTX.set(self.ctx)
        return self.ctx

    def __exit__(self, *exc):
        _CTX.reset(self.tok)
