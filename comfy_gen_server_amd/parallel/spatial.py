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
* GroupNorm statistics: each rank computes its band's per-(image, group) (mean, M2) with the native
  statistics kernel (``cgs_groupnorm_band_stats``), the [P, N, groups, 2] fp32 partials are all-gathered
  (a few KB) and Chan-combined (no cancellation, no fp64), and the native apply kernel normalises the band
  (``cgs_groupnorm_apply_stats``, SiLU / timestep pre-add / dual-source skip concat fused as in the
  single-GPU GroupNorm); on the CPU the same two steps run in fp32 torch;
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

from . import coll

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
        coll.all_gather(parts, t, group=self.group)
        return torch.cat(parts, dim=dim)

    def halo(self, x, top: int, bottom: int):
        """[N, C, top + R + bottom, W]: ``top`` rows from the rank above and ``bottom`` rows from the rank
        below around the local band (zeros at the image edge). The extended band is allocated once and the
        neighbours' rows are received straight into it (NHWC: for one image a row range is one contiguous
        block), so the only copy is the band itself."""
        self.stats["halo"] += 1
        N, C, R, W = x.shape
        above, below = self.rank - 1, self.rank + 1
        cl = x.is_cuda
        ext = torch.empty((N, C, top + R + bottom, W), dtype=x.dtype, device=x.device,
                          memory_format=torch.channels_last if cl else torch.contiguous_format)
        ext[:, :, top:top + R] = x
        sends, recvs, fix = [], [], []

        fmt = torch.channels_last if cl else torch.contiguous_format

        def slot(lo, n):
            v = ext[:, :, lo:lo + n]
            if v.is_contiguous(memory_format=fmt):
                return v, None            # receive in place
            return torch.empty((N, C, n, W), dtype=x.dtype, device=x.device, memory_format=fmt), v
        if top:
            if above >= 0:
                buf, dst = slot(0, top)
                recvs.append((buf, self.ranks[above]))
                if dst is not None:
                    fix.append((dst, buf))
            else:
                ext[:, :, :top].zero_()
            if below < self.P:    # my last `top` rows are the lower neighbour's top halo
                sends.append((x[:, :, R - top:].contiguous(), self.ranks[below]))
        if bottom:
            if below < self.P:
                buf, dst = slot(top + R, bottom)
                recvs.append((buf, self.ranks[below]))
                if dst is not None:
                    fix.append((dst, buf))
            else:
                ext[:, :, top + R:].zero_()
            if above >= 0:        # my first `bottom` rows are the upper neighbour's bottom halo
                sends.append((x[:, :, :bottom].contiguous(), self.ranks[above]))
        for req in coll.exchange(sends, recvs, self.group):
            req.wait()
        for dst, buf in fix:
            dst.copy_(buf)
        return ext

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

    def _gather_stats(self, st):
        """[N, G, 2] (mean, M2) of every rank of the group -> [P, N, G, 2]."""
        if self.P == 1:
            return st[None]
        parts = [torch.empty_like(st) for _ in range(self.P)]
        coll.all_gather(parts, st.contiguous(), group=self.group)
        return torch.stack(parts)

    def group_norm(self, x, groups, weight, bias, eps, silu=False, pre_add=None, x2=None):
        """GroupNorm over the whole image from the bands' (mean, M2) (Chan combine of the all-gathered
        [P, N, G, 2] fp32 partials; equal band sizes)."""
        from ..ops import core
        self.stats["gn"] += 1
        N, C1, R, W = x.shape
        C = C1 + (0 if x2 is None else x2.shape[1])
        native = (x.is_cuda and x.dtype in (torch.bfloat16, torch.float16) and weight is not None and C % 8 == 0
                  and C1 % 8 == 0 and C % groups == 0 and C <= 8192 and C % (8 * ((C + 2047) // 2048)) == 0
                  and (x2 is None or (x2.dtype == x.dtype and x2.is_cuda))
                  and core._native.has_kernel("cgs_groupnorm_band_stats"))
        cnt = float((C // groups) * R * W)
        if native:
            lib, dt = core._lib(), core._DT[x.dtype]
            xc = x.contiguous(memory_format=torch.channels_last)
            x2c = None if x2 is None else x2.contiguous(memory_format=torch.channels_last)
            pa = None if pre_add is None else pre_add.to(x.dtype).contiguous()
            ws = torch.empty((int(lib.cgs_groupnorm_workspace(N, R * W, C)) + 3) // 4, device=x.device,
                             dtype=torch.float32)
            st = torch.empty((N, groups, 2), device=x.device, dtype=torch.float32)
            core._check(lib.cgs_groupnorm_band_stats(xc.data_ptr(), core._ptr(x2c), C1, core._ptr(pa), ws.data_ptr(),
                                                     st.data_ptr(), N, R * W, C, groups, dt, core._stream()),
                        "cgs_groupnorm_band_stats")
        else:
            xf = x.float() if x2 is None else torch.cat([x.float(), x2.float()], dim=1)
            if pre_add is not None:
                xf = xf + pre_add.float()[:, :, None, None]
            g = xf.reshape(N, groups, -1)
            mean = g.mean(-1)
            st = torch.stack([mean, ((g - mean[..., None]) ** 2).sum(-1)], dim=-1)
        allst = self._gather_stats(st)
        mean = allst[..., 0].mean(0)
        m2 = allst[..., 1].sum(0) + cnt * ((allst[..., 0] - mean) ** 2).sum(0)
        rstd = torch.rsqrt((m2 / (cnt * self.P)).clamp_min(0.0) + eps)
        if native:
            core.count("groupnorm", "hip")
            self.stats["gn_native"] = self.stats.get("gn_native", 0) + 1
            w = weight.to(device=x.device, dtype=x.dtype).contiguous()
            b = None if bias is None else bias.to(device=x.device, dtype=x.dtype).contiguous()
            mr = torch.stack([mean, rstd], dim=-1).contiguous()
            ab = torch.empty(N * C * 2, device=x.device, dtype=torch.float32)
            y = torch.empty((N, C, R, W), device=x.device, dtype=x.dtype, memory_format=torch.channels_last)
            core._check(lib.cgs_groupnorm_apply_stats(xc.data_ptr(), core._ptr(x2c), C1, y.data_ptr(), w.data_ptr(),
                                                      core._ptr(b), core._ptr(pa), mr.data_ptr(), ab.data_ptr(), N,
                                                      R * W, C, groups, 1 if silu else 0, dt, core._stream()),
                        "cgs_groupnorm_apply_stats")
            return y
        y = ((g - mean[..., None]) * rstd[..., None]).reshape(N, C, R, W)
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
