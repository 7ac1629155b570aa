"""Stable Cascade (Würstchen v3): Stage C prior, Stage B decoder, Stage A VQGAN, the EfficientNet
encoder / previewer pair and the Cascade ControlNet (parity: ``comfy/ldm/cascade/{common,stage_a,
stage_b,stage_c,stage_c_coder,controlnet}.py`` and ``comfy/model_base.py:512-559``).

MI355X layout: every stage runs channels-last end to end. Activations are NHWC ``[B, H, W, C]``
tensors, so the reference's ``LayerNorm2d`` (permute -> LN -> permute) is one row-LayerNorm
kernel over C, every 1x1 conv / "channelwise" MLP is a plain GEMM on ``[B*H*W, C]`` (residual add
fused in its epilogue), the 2x2/stride-2 down/up convs of Stage B are patchify GEMMs, the
attention blocks feed ``[B, HW, C]`` views straight to the flash kernel, and the depthwise 3x3 of
each ResBlock is the NHWC depthwise HIP kernel. NCHW only exists at the model boundary.
Parameter names match the released checkpoints.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from . import layers
from .layers import Conv2d, DerivedMixin, LayerNorm, Linear, module_epoch


# ------------------------------------------------------------------------------------------------
# NHWC helpers
# ------------------------------------------------------------------------------------------------
def _ln(x, eps=1e-6):
    h = getattr(x, "_cgs_ln", None)       # LN(x) already produced with x (TimestepBlock.forward_ln)
    if h is not None and h[1] == x.data_ptr() and h[2] == eps:
        return h[0]
    return ops.layer_norm(x, None, None, eps)


# all off by default: each measured 0.1-0.8 % SLOWER than the separate passes at batch 1 (in-process A/B,
# profiles/r04/cascade_fusion_ab_r04k.json) -- the GRN / LayerNorm passes they remove are small at these
# grids while the extra epilogue work sits on the GEMM's critical path
_FUSE_DEFAULTS = {"GELU_EPI": "auto", "LNFOLD": "auto", "GRNFOLD": "0", "DWLN": "0", "ATTNLN": "0", "AFFLN": "1", "TSBATCH": "1"}


def _fuse(name: str, rows: int = 0) -> bool:
    """Cascade block fusions (``CGS_CASCADE_<NAME>=0/1`` overrides the default, for A/B runs): GELU_EPI
    (GELU in the first ChannelMLP GEMM), LNFOLD (LayerNorm folded into it), DWLN (its statistics from the
    depthwise kernel: off -- at Stage C's 1152-pixel grids the per-pixel reduction leaves the kernel
    latency-bound, 33 us vs 11 + 9 us for the two passes, profiles/r04/cascade_fusion_profile.md),
    GRNFOLD (GRN folded into per-image second-GEMM weights), ATTNLN (the AttnBlock's LayerNorm folded into
    its fused QKV GEMM: statistics pass + LN-fold epilogue instead of the materialised LN; off -- measured
    +1.3 % per batch-4 job and +2.5 % at batch 1: the LN-fold epilogue costs the fused QKV GEMM what the
    statistics-only pass saves, and at batch 1 the plain GEMM's fastest 256x160 tile has no LN-fold form
    for N = 6144, profiles/r05/cascade_attnln.md), AFFLN (a TimestepBlock followed by an AttnBlock also
    writes the attention's LayerNorm from the same pass, ops.channel_affine_layernorm_nhwc), TSBATCH (every
    TimestepBlock's mapper pair of a stage in one GEMM per call, _UNetStage._ts_mapped). "auto": on from ``CGS_CASCADE_FUSE_MIN_ROWS``
    (default 4096) pixels per call -- GELU_EPI + LNFOLD measured 2.5 % faster at batch 4 and 0.6 % slower
    at batch 1 (profiles/r04/cascade_fusion_ab_b4_r04av.json, cascade_fusion_ab_r04k.json)."""
    v = os.environ.get(f"CGS_CASCADE_{name}", _FUSE_DEFAULTS[name])
    if v == "auto":
        return rows >= int(os.environ.get("CGS_CASCADE_FUSE_MIN_ROWS", "4096"))
    return v != "0"


def _rows(x) -> int:
    return x.numel() // max(1, x.shape[-1])


def _cast(w, x):
    return None if w is None else (w if (w.dtype == x.dtype and w.device == x.device) else
                                   w.to(device=x.device, dtype=x.dtype))


def _pw(conv, x, residual=None, act=None):
    """1x1 conv on an NHWC tensor as a GEMM over the channel dim (``act="gelu"``: fused GELU epilogue)."""
    w = _cast(conv.weight, x).reshape(conv.out_channels, conv.in_channels)
    if x.is_cuda and conv.in_channels % 32:
        # narrow K (Stage A's 4-channel latent in): zero-pad K to 32 so the HIP GEMM takes it
        kp = (conv.in_channels + 31) // 32 * 32
        w = F.pad(w, (0, kp - conv.in_channels))
        x = F.pad(x, (0, kp - conv.in_channels))
    return ops.linear(x, w, _cast(conv.bias, x), residual=residual, act=act)


def _to_nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


def _to_nchw(x):
    return x.permute(0, 3, 1, 2).contiguous()


def _resize_nhwc(x, size, mode="bilinear"):
    y = F.interpolate(x.permute(0, 3, 1, 2), size=size, mode=mode, align_corners=True if mode == "bilinear" else None)
    return _to_nhwc(y)


class DepthwiseConv2d(Conv2d):
    """groups == channels conv evaluated on NHWC activations (K11)."""

    def __init__(self, c, kernel_size=3, bias=True, replicate=False, dtype=None, device=None):
        super().__init__(c, c, kernel_size, padding=kernel_size // 2, groups=c, bias=bias, dtype=dtype, device=device)
        self.replicate = replicate

    def w_kkc(self, x):
        def make():
            k = self.kernel_size[0]
            return self.weight.reshape(self.out_channels, k * k).t().contiguous()
        w = self._derived_get("w_kkc", make)
        return _cast(w, x)

    def forward_nhwc(self, x):
        return ops.depthwise_conv2d_nhwc(x, self.w_kkc(x), _cast(self.bias, x), self.kernel_size[0], self.replicate)


class GlobalResponseNorm(nn.Module):
    """ConvNeXt-V2 GRN on NHWC: x * (1 + gamma * N(x)) + beta, N = ||x||_HW / mean_C ||x||_HW."""

    def __init__(self, dim, dtype=None, device=None):
        super().__init__()
        self.gamma = nn.Parameter(torch.zeros(1, 1, 1, dim, dtype=dtype, device=device), requires_grad=False)
        self.beta = nn.Parameter(torch.zeros(1, 1, 1, dim, dtype=dtype, device=device), requires_grad=False)

    def forward(self, x):
        return ops.grn_nhwc(x, _cast(self.gamma, x), _cast(self.beta, x))


class _ChannelMLP(nn.Sequential):
    """Linear -> GELU -> GRN -> (Dropout) -> Linear; Sequential indices 0/2/4 match the checkpoints."""

    def __init__(self, c_in, c_hidden, c_out, dtype=None, device=None):
        super().__init__(Linear(c_in, c_hidden, dtype=dtype, device=device), nn.GELU(),
                         GlobalResponseNorm(c_hidden, dtype=dtype, device=device), nn.Identity(),
                         Linear(c_hidden, c_out, dtype=dtype, device=device))

    def forward(self, x, residual=None):
        grn = self[2]
        if not (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4) or not _fuse("GELU_EPI", _rows(x)):
            h = ops.grn_nhwc(self[0](x), _cast(grn.gamma, x), _cast(grn.beta, x), pre_gelu=True)
            return self[4](h, residual=residual)
        return self._grn_linear2(self[0](x, act="gelu"), x, residual)

    def lnfold_ok(self, x) -> bool:
        """LayerNorm (no affine) of ``x`` can fold into the first GEMM (device bf16, unhooked weights)."""
        return (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and not layers._hooked(self[0])
                and self[0].weight.dtype == torch.bfloat16 and ops.lnfold_available(x, x.shape[-1])
                and _fuse("LNFOLD", _rows(x)) and _fuse("GELU_EPI", _rows(x)))

    def forward_ln(self, x, eps=1e-6, residual=None, rs=None):
        """``forward(LN(x))`` with the LayerNorm folded into the first GEMM: only the per-pixel statistics
        pass reads ``x`` (or none: ``rs`` from the producer, ops.depthwise_conv2d_nhwc_lnstats); the
        normalised tensor is never written (K07 as in the SDXL transformer)."""
        if not self.lnfold_ok(x):
            return self(_ln(x, eps), residual=residual)
        lin1 = self[0]
        w2, cs, b2 = lin1._derived_get(("lnfold_noaffine", x.device), lambda: ops.lnfold_weights(
            _cast(lin1.weight, x), _cast(lin1.bias, x), None, None))
        if rs is None:
            rs = ops.layernorm_stats(x, eps)
        # the GEMM epilogue also leaves the GRN statistics partials of h (per image of H * W rows)
        h = ops.linear_lnfold(x, rs, w2, cs, b2, act="gelu", gns_hw=x.shape[1] * x.shape[2])
        return self._grn_linear2(h, x, residual)

    def _grn_linear2(self, h, x, residual):
        # device: GELU already in the first GEMM's epilogue; then either the GRN pass over h, or -- when the
        # output width is below the pixel count, i.e. rewriting W2 per image moves fewer bytes than
        # rewriting h (Stage B's 64^2..256^2 levels) -- the GRN scale folded into per-image copies of W2
        # and W2 beta folded into the bias (ops.grn_fold_weight)
        grn = self[2]
        N, H, W, _ = x.shape
        lin2 = self[4]
        if lin2.out_features < H * W and N <= 64 and h.shape[-1] % 8 == 0 and _fuse("GRNFOLD"):
            w2, b2 = lin2.weight_bias_for(h)
            wn = ops.grn_fold_weight(h, w2, _cast(grn.gamma, h))
            bias = ops.linear(_cast(grn.beta, h).reshape(1, -1), w2, b2).reshape(-1)      # b2 + W2 beta
            out = torch.empty((N, H, W, lin2.out_features), device=x.device, dtype=x.dtype)
            for n in range(N):
                ops.linear(h[n], wn[n], bias, residual=None if residual is None else residual[n], out=out[n])
            return out
        h = ops.grn_nhwc(h, _cast(grn.gamma, x), _cast(grn.beta, x))
        return lin2(h, residual=residual)


# ------------------------------------------------------------------------------------------------
# Blocks shared by Stage B / Stage C (common.py)
# ------------------------------------------------------------------------------------------------
class ResBlock(nn.Module):
    def __init__(self, c, c_skip=0, kernel_size=3, dropout=0.0, dtype=None, device=None):
        super().__init__()
        self.depthwise = DepthwiseConv2d(c, kernel_size, dtype=dtype, device=device)
        self.channelwise = _ChannelMLP(c + c_skip, c * 4, c, dtype=dtype, device=device)

    def forward(self, x, x_skip=None):
        if x_skip is None and self.channelwise.lnfold_ok(x) and _fuse("DWLN"):
            # depthwise conv + LayerNorm statistics in one pass, LayerNorm folded into the first GEMM
            dw = self.depthwise
            d, rs = ops.depthwise_conv2d_nhwc_lnstats(x, dw.w_kkc(x), _cast(dw.bias, x), dw.kernel_size[0], 1e-6,
                                                      dw.replicate)
            return self.channelwise.forward_ln(d, residual=x, rs=rs)
        d = self.depthwise.forward_nhwc(x)
        if x_skip is None:
            return self.channelwise.forward_ln(d, residual=x)
        h = torch.cat([_ln(d), x_skip.to(d.dtype)], dim=-1)
        return self.channelwise(h, residual=x)


class OptimizedAttention(nn.Module, DerivedMixin):
    def __init__(self, c, nhead, dtype=None, device=None):
        super().__init__()
        self.heads = nhead
        self.to_q = Linear(c, c, dtype=dtype, device=device)
        self.to_k = Linear(c, c, dtype=dtype, device=device)
        self.to_v = Linear(c, c, dtype=dtype, device=device)
        self.out_proj = Linear(c, c, dtype=dtype, device=device)

    def _fused(self, names, x):
        """[W_a; W_b; ...] / [b_a; b_b; ...] in x's dtype (cached, dropped on weight patches)."""
        def build():
            mods = [getattr(self, n) for n in names]
            w = torch.cat([_cast(m.weight, x) for m in mods], 0).contiguous()
            b = torch.cat([_cast(m.bias, x) if m.bias is not None else
                           torch.zeros(m.out_features, device=x.device, dtype=x.dtype) for m in mods], 0).contiguous()
            return w, b
        return self._derived_get(("fused",) + tuple(names) + (x.dtype, x.device), build)

    def forward(self, q, k, v, residual=None):
        o = ops.attention(self.to_q(q), self.to_k(k), self.to_v(v), self.heads)
        return self.out_proj(o, residual=residual)

    def fused_ok(self, x):
        C = x.shape[-1]
        return x.is_cuda and x.dtype == torch.bfloat16 and C % 64 == 0 and C // self.heads == 64

    def forward_self_ln(self, xs, rs, kv, residual=None, kvp=None):
        """``forward_self(LN(xs), ...)`` with the LayerNorm (no affine) folded into the fused QKV GEMM: ``rs``
        the per-row (mean, rstd) of xs (ops.layernorm_stats); the normalised rows are never written."""
        C = xs.shape[-1]
        wq, bq = self._fused(("to_q", "to_k", "to_v"), xs)
        w2, cs, b2 = self._derived_get(("lnfold_qkv", xs.dtype, xs.device),
                                       lambda: ops.lnfold_weights(wq, bq, None, None))
        qkv = ops.linear_lnfold(xs, rs, w2, cs, b2)
        kv2 = kvp if kvp is not None else self.project_kv(kv.to(xs.dtype))
        o = ops.attention_kv2(qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:], kv2[..., :C], kv2[..., C:],
                              self.heads)
        return self.out_proj(o, residual=residual)

    def project_kv(self, kv):
        """[K | V] of the conditioning tokens: the part of forward_self's keys / values that does not
        depend on the image tokens (one fused GEMM)."""
        wk, bk = self._fused(("to_k", "to_v"), kv)
        return ops.linear(kv, wk, bk)

    def forward_self(self, xs, kv, residual=None, kvp=None):
        """Stable Cascade self-attention: q from xs, keys / values over cat([xs, kv]) (common.py
        Attention2D). One fused QKV GEMM over xs and one fused KV GEMM over kv; the attention kernel reads
        the keys from the two projections directly, so neither the input nor the K / V concat is built.
        ``kvp``: the conditioning's [K | V] already projected (``project_kv``; static across steps)."""
        C = xs.shape[-1]
        if self.fused_ok(xs):
            wq, bq = self._fused(("to_q", "to_k", "to_v"), xs)
            qkv = ops.linear(xs, wq, bq)
            kv2 = kvp if kvp is not None else self.project_kv(kv.to(xs.dtype))
            o = ops.attention_kv2(qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:], kv2[..., :C], kv2[..., C:],
                                  self.heads)
            return self.out_proj(o, residual=residual)
        if kvp is not None:
            k = torch.cat([self.to_k(xs), kvp[..., :C].to(xs.dtype)], dim=1)
            v = torch.cat([self.to_v(xs), kvp[..., C:].to(xs.dtype)], dim=1)
            return self.out_proj(ops.attention(self.to_q(xs), k, v, self.heads), residual=residual)
        kvc = torch.cat([xs, kv.to(xs.dtype)], dim=1)
        return self.forward(xs, kvc, kvc, residual=residual)


class Attention2D(nn.Module):
    def __init__(self, c, nhead, dropout=0.0, dtype=None, device=None):
        super().__init__()
        self.attn = OptimizedAttention(c, nhead, dtype=dtype, device=device)

    def forward(self, x_norm, kv, self_attn=False, residual=None, kvp=None):
        B, H, W, C = x_norm.shape
        xs = x_norm.reshape(B, H * W, C)
        res = None if residual is None else residual.reshape(B, H * W, C)
        if self_attn:
            return self.attn.forward_self(xs, kv, residual=res, kvp=kvp).reshape(B, H, W, C)
        return self.attn(xs, kv, kv, residual=res).reshape(B, H, W, C)


class AttnBlock(nn.Module):
    def __init__(self, c, c_cond, nhead, self_attn=True, dropout=0.0, dtype=None, device=None):
        super().__init__()
        self.self_attn = self_attn
        self.attention = Attention2D(c, nhead, dropout, dtype=dtype, device=device)
        self.kv_mapper = nn.Sequential(nn.SiLU(), Linear(c_cond, c, dtype=dtype, device=device))

    def _map(self, kv):
        return self.kv_mapper[1](ops.silu(kv) if kv.is_contiguous() else F.silu(kv))

    def static_kv(self, clip):
        """This block's conditioning [K | V] (kv_mapper, then the fused K/V projection); None for a
        cross-attention-only block."""
        if not self.self_attn:
            return None
        return self.attention.attn.project_kv(self._map(clip))

    def forward(self, x, kv):
        at = self.attention.attn
        if self.self_attn and x.dim() == 4 and at.fused_ok(x) and _fuse("ATTNLN", _rows(x)) \
                and not any(layers._hooked(getattr(at, n)) for n in ("to_q", "to_k", "to_v")) \
                and ops.lnfold_available(x, x.shape[-1]):
            B, H, W, C = x.shape
            xs = x.reshape(B, H * W, C)
            kvp = kv[id(self)] if isinstance(kv, dict) else None
            o = at.forward_self_ln(xs, ops.layernorm_stats(x, 1e-6), None if kvp is not None else self._map(kv),
                                   residual=xs, kvp=kvp)
            return o.reshape(B, H, W, C)
        if isinstance(kv, dict):        # static conditioning K/V of a captured step (_UNetStage._static_cond)
            return self.attention(_ln(x), None, self_attn=True, residual=x, kvp=kv[id(self)])
        return self.attention(_ln(x), self._map(kv), self_attn=self.self_attn, residual=x)


class FeedForwardBlock(nn.Module):
    def __init__(self, c, dropout=0.0, dtype=None, device=None):
        super().__init__()
        self.channelwise = _ChannelMLP(c, c * 4, c, dtype=dtype, device=device)

    def forward(self, x):
        return self.channelwise.forward_ln(x, residual=x)


class TimestepBlock(nn.Module):
    def __init__(self, c, c_timestep, conds=("sca",), dtype=None, device=None):
        super().__init__()
        self.mapper = Linear(c_timestep, c * 2, dtype=dtype, device=device)
        self.conds = list(conds)
        for name in self.conds:
            setattr(self, f"mapper_{name}", Linear(c_timestep, c * 2, dtype=dtype, device=device))

    def forward_ln(self, x, t, eps=1e-6):
        """``forward`` whose output also carries its LayerNorm (no affine) for the next AttnBlock (``_ln``
        picks it up), from one pass over x."""
        if not (x.dim() == 4 and x.is_contiguous()):
            return self.forward(x, t)
        a, b = self._ab(t)
        xa, ln = ops.channel_affine_layernorm_nhwc(x, a, b, add=1.0, eps=eps)
        xa._cgs_ln = (ln, xa.data_ptr(), eps)
        return xa

    def _mappers(self):
        return [self.mapper] + [getattr(self, f"mapper_{name}") for name in self.conds]

    def _ab(self, t):
        pre = getattr(t, "_cgs_ts", None)          # all mappers of the stage in one GEMM (_ts_mapped)
        if pre is not None and id(self) in pre:
            return pre[id(self)].chunk(2, dim=-1)
        t = t.chunk(len(self.conds) + 1, dim=1)
        ab = self.mapper(t[0])
        for i, name in enumerate(self.conds):      # the sum rides the GEMMs' residual epilogue
            ab = getattr(self, f"mapper_{name}")(t[i + 1], residual=ab)
        return ab.chunk(2, dim=-1)

    def forward(self, x, t):
        a, b = self._ab(t)
        if x.dim() == 4 and x.is_contiguous():
            return ops.channel_affine_nhwc(x, a, b, add=1.0)
        return torch.addcmul(b[:, None, None, :], x, 1 + a[:, None, None, :])


def _r_embedding(r, c_r, max_positions=10000):
    """Stable Cascade's sinusoidal r embedding (common.py ``gen_r_embedding``): [sin | cos] of
    r * max_positions at frequencies exp(-ln(max_positions) k / (half - 1)) -- the same sinusoid as the
    UNet timestep embedding with max_period = max_positions ** (half / (half - 1)), so it runs on that
    kernel (one launch instead of the arange / exp / sin / cos / cat chain per step)."""
    half = c_r // 2
    emb = ops.timestep_embedding(r.float() * max_positions, 2 * half,
                                 max_period=float(max_positions) ** (half / (half - 1)), flip_sin_to_cos=False)
    if c_r % 2 == 1:
        emb = F.pad(emb, (0, 1))
    return emb


class _LN2d(nn.Module):
    """LayerNorm2d without affine (checkpoint index placeholder)."""

    def forward(self, x):
        return _ln(x)


class _UNetStage(nn.Module):
    """Shared down/up traversal of Stage B and Stage C (stage_b.py:176-239, stage_c.py:193-256)."""

    def _make_block(self, kind, c, nhead, c_skip, dtype, device):
        if kind == "C":
            return ResBlock(c, c_skip, kernel_size=self.kernel_size, dtype=dtype, device=device)
        if kind == "A":
            return AttnBlock(c, self.c_cond, nhead, self_attn=self.self_attn, dtype=dtype, device=device)
        if kind == "F":
            return FeedForwardBlock(c, dtype=dtype, device=device)
        if kind == "T":
            return TimestepBlock(c, self.c_r, conds=self.t_conds, dtype=dtype, device=device)
        raise ValueError(f"Block type {kind} not supported")

    def _build_levels(self, c_hidden, nhead, blocks, block_repeat, level_config, dtype, device):
        self.down_blocks = nn.ModuleList()
        self.down_repeat_mappers = nn.ModuleList()
        for i in range(len(c_hidden)):
            blk = nn.ModuleList()
            for _ in range(blocks[0][i]):
                for kind in level_config[i]:
                    blk.append(self._make_block(kind, c_hidden[i], nhead[i], 0, dtype, device))
            self.down_blocks.append(blk)
            self.down_repeat_mappers.append(nn.ModuleList(
                [Conv2d(c_hidden[i], c_hidden[i], 1, dtype=dtype, device=device) for _ in range(block_repeat[0][i] - 1)]))
        self.up_blocks = nn.ModuleList()
        self.up_repeat_mappers = nn.ModuleList()
        for i in reversed(range(len(c_hidden))):
            blk = nn.ModuleList()
            for j in range(blocks[1][::-1][i]):
                for k, kind in enumerate(level_config[i]):
                    c_skip = c_hidden[i] if i < len(c_hidden) - 1 and j == k == 0 else 0
                    blk.append(self._make_block(kind, c_hidden[i], nhead[i], c_skip, dtype, device))
            self.up_blocks.append(blk)
            self.up_repeat_mappers.append(nn.ModuleList(
                [Conv2d(c_hidden[i], c_hidden[i], 1, dtype=dtype, device=device)
                 for _ in range(block_repeat[1][::-1][i] - 1)]))

    @staticmethod
    def _add_cnet(x, cnet):
        if cnet:
            c = cnet.pop()
            if c is not None:
                c = c.to(device=x.device, dtype=x.dtype)      # NCHW projection output
                x = x + _to_nhwc(F.interpolate(c, size=x.shape[1:3], mode="bilinear", align_corners=True))
        return x

    def _attn_kv(self, clip):
        """{id(AttnBlock): [K | V] of the conditioning tokens} for every attention block, or None."""
        out = {}
        for m in self.modules():
            if isinstance(m, AttnBlock):
                kv = m.static_kv(clip)
                if kv is None:
                    return None
                out[id(m)] = kv
        return out or None

    def _static_cond(self, kwargs, srcs, compute):
        """Conditioning-only work of a sampling run -- every attention block's K/V of the clip tokens
        (kv_mapper + K/V projection, constant over the steps) and Stage B's effnet / pixel maps -- held in
        persistent buffers under the step graph's static-K/V protocol (``kv_static`` = (mode, ids of the
        plan's static cond tensors), sampling/step_graph.py; same scheme as models/attention.py
        CrossAttention.static_kv): "fill" computes and stores, "use" (the captured step) reads the
        buffers, ``refresh_static_kv`` recomputes them once per job. Returns the dict of buffers or None
        (not a static run: the caller computes inline)."""
        kvs = (kwargs.get("transformer_options") or {}).get("kv_static")
        if kvs is None:
            return None
        mode, sources = kvs
        if not all(t is None or id(t) in sources for t in srcs):
            return None
        key = tuple(id(t) for t in srcs)
        store = self.__dict__.setdefault("_kv_static", {})
        ent = store.get(key)
        fresh = ent is not None and all(a is b for a, b in zip(ent[0], srcs))
        if fresh and mode == "use":
            return ent[2]
        vals = compute()
        if vals is None or mode != "fill":
            return vals
        if fresh and ent[2].keys() == vals.keys() and all(ent[2][k].shape == v.shape for k, v in vals.items()):
            for k, v in vals.items():        # captured graphs hold these addresses: refill in place
                ent[2][k].copy_(v)
        else:
            store[key] = ent = (tuple(srcs), compute, vals)
        return ent[2]

    def refresh_static_kv(self, sources) -> int:
        n = 0
        for srcs, compute, bufs in self.__dict__.get("_kv_static", {}).values():
            if all(t is None or id(t) in sources for t in srcs):
                for k, v in compute().items():
                    bufs[k].copy_(v)
                n += 1
        return n

    def _ts_mapped(self, r_embed):
        """Every TimestepBlock's ``[a | b]`` (mapper(t0) + mapper_<cond>(t1) + ...) from ONE GEMM: the mappers
        read only r_embed = [t0 | t1 | ...], so their weights concatenated along K per block and stacked
        along N over the blocks give all of them at once (the per-block pairs were ~100 launch-bound
        skinny GEMMs per UNet call). Returns {id(block): [B, 2C] column view} or None."""
        if not (r_embed.is_cuda and r_embed.dtype in (torch.bfloat16, torch.float16) and _fuse("TSBATCH")):
            return None
        blocks = self.__dict__.get("_ts_blocks")
        if blocks is None:
            blocks = self.__dict__["_ts_blocks"] = [m for m in self.modules() if isinstance(m, TimestepBlock)]
        if not blocks or any(layers._hooked(m) for b in blocks for m in b._mappers()):
            return None
        key = (r_embed.dtype, r_embed.device, module_epoch(self), blocks[0].mapper.weight.data_ptr())
        ent = self.__dict__.get("_ts_fused")
        if ent is None or ent[0] != key:
            ws, bs, offs, off = [], [], {}, 0
            for blk in blocks:
                mods = blk._mappers()
                w = torch.cat([_cast(m.weight, r_embed) for m in mods], dim=1)
                b = torch.zeros(w.shape[0], device=r_embed.device, dtype=torch.float32)
                for m in mods:
                    if m.bias is not None:
                        b = b + m.bias.to(device=r_embed.device, dtype=torch.float32)
                ws.append(w)
                bs.append(b)
                offs[id(blk)] = (off, w.shape[0])
                off += w.shape[0]
            if len({w.shape[1] for w in ws}) != 1:          # blocks with different condition lists
                ent = (key, None, None, offs)
            else:
                ent = (key, torch.cat(ws, 0).contiguous(), torch.cat(bs).to(r_embed.dtype).contiguous(), offs)
            self.__dict__["_ts_fused"] = ent
        if ent[1] is None or ent[1].shape[1] != r_embed.shape[1]:
            return None
        ab = ops.linear(r_embed, ent[1], ent[2])
        return {k: ab[:, o:o + n] for k, (o, n) in ent[3].items()}

    def _with_ts(self, r_embed):
        pre = self._ts_mapped(r_embed)
        if pre is not None:
            r_embed = r_embed.view_as(r_embed)      # a fresh tensor object carrying the mapped coefficients
            r_embed._cgs_ts = pre
        return r_embed

    def _run_block(self, block, x, r_embed, clip, skip=None, cnet=None, nxt=None):
        if isinstance(block, ResBlock):
            x = self._add_cnet(x, cnet)
            return block(x, skip)
        if isinstance(block, AttnBlock):
            return block(x, clip)
        if isinstance(block, TimestepBlock):
            if isinstance(nxt, AttnBlock) and x.is_cuda and _fuse("AFFLN", _rows(x)):
                return block.forward_ln(x, r_embed)
            return block(x, r_embed)
        return block(x)

    def _down_encode(self, x, r_embed, clip, cnet=None):
        levels = []
        for down_block, downscaler, repmap in zip(self.down_blocks, self.down_downscalers, self.down_repeat_mappers):
            x = self._downscale(downscaler, x)
            for i in range(len(repmap) + 1):
                for bi, block in enumerate(down_block):
                    nxt = down_block[bi + 1] if bi + 1 < len(down_block) else None
                    x = self._run_block(block, x, r_embed, clip, cnet=cnet, nxt=nxt)
                if i < len(repmap):
                    x = _pw(repmap[i], x)
            levels.insert(0, x)
        return levels

    def _up_decode(self, levels, r_embed, clip, cnet=None):
        x = levels[0]
        for i, (up_block, upscaler, repmap) in enumerate(zip(self.up_blocks, self.up_upscalers, self.up_repeat_mappers)):
            for j in range(len(repmap) + 1):
                for k, block in enumerate(up_block):
                    skip = None
                    if isinstance(block, ResBlock):
                        skip = levels[i] if k == 0 and i > 0 else None
                        if skip is not None and x.shape[1:3] != skip.shape[1:3]:
                            x = _resize_nhwc(x, skip.shape[1:3])
                    nxt = up_block[k + 1] if k + 1 < len(up_block) else None
                    x = self._run_block(block, x, r_embed, clip, skip=skip, cnet=cnet, nxt=nxt)
                if j < len(repmap):
                    x = _pw(repmap[j], x)
            x = self._upscale(upscaler, x)
        return x

    def _r_embed(self, r, x_dtype, kwargs):
        e = _r_embedding(r, self.c_r).to(x_dtype)
        for c in self.t_conds:
            t_cond = kwargs.get(c, torch.zeros_like(r))
            e = torch.cat([e, _r_embedding(t_cond, self.c_r).to(x_dtype)], dim=1)
        return e

    def _embed(self, x):
        x = _to_nhwc(x)
        if self.patch_size > 1:
            B, H, W, C = x.shape
            p = self.patch_size
            # PixelUnshuffle channel order (c, i, j)
            x = x.reshape(B, H // p, p, W // p, p, C).permute(0, 1, 3, 5, 2, 4).reshape(B, H // p, W // p, C * p * p)
        return _ln(_pw(self.embedding[1], x))

    def _classify(self, x):
        x = _pw(self.clf[1], _ln(x))
        p = self.patch_size
        if p > 1:
            B, H, W, C = x.shape
            c = C // (p * p)
            x = x.reshape(B, H, W, c, p, p).permute(0, 1, 4, 2, 5, 3).reshape(B, H * p, W * p, c)
        return _to_nchw(x)


def _embedding_seq(c_in, c_hidden, patch_size, dtype, device):
    return nn.Sequential(nn.PixelUnshuffle(patch_size),
                         Conv2d(c_in * patch_size ** 2, c_hidden, 1, dtype=dtype, device=device), _LN2d())


def _clf_seq(c_hidden, c_out, patch_size, dtype, device):
    return nn.Sequential(_LN2d(), Conv2d(c_hidden, c_out * patch_size ** 2, 1, dtype=dtype, device=device),
                         nn.PixelShuffle(patch_size))


# ------------------------------------------------------------------------------------------------
# Stage C (text-conditional prior at 24x24x16)
# ------------------------------------------------------------------------------------------------
class UpDownBlock2d(nn.Module):
    def __init__(self, c_in, c_out, mode, enabled=True, dtype=None, device=None):
        super().__init__()
        self.mode = mode
        self.enabled = enabled
        mapping = Conv2d(c_in, c_out, 1, dtype=dtype, device=device)
        self.blocks = nn.ModuleList([nn.Identity(), mapping] if mode == "up" else [mapping, nn.Identity()])

    def forward(self, x):
        def interp(t):
            if not self.enabled:
                return t
            B, H, W, C = t.shape
            s = (H * 2, W * 2) if self.mode == "up" else (H // 2, W // 2)
            return _resize_nhwc(t, s)
        if self.mode == "up":
            return _pw(self.blocks[1], interp(x))
        return interp(_pw(self.blocks[0], x))


class StageC(_UNetStage):
    def __init__(self, c_in=16, c_out=16, c_r=64, patch_size=1, c_cond=2048, c_hidden=(2048, 2048), nhead=(32, 32),
                 blocks=((8, 24), (24, 8)), block_repeat=((1, 1), (1, 1)), level_config=("CTA", "CTA"),
                 c_clip_text=1280, c_clip_text_pooled=1280, c_clip_img=768, c_clip_seq=4, kernel_size=3,
                 dropout=(0.0, 0.0), self_attn=True, t_conds=("sca", "crp"), switch_level=(False,),
                 stable_cascade_stage=None, dtype=None, device=None, **_):
        super().__init__()
        self.dtype = dtype
        self.c_r, self.c_cond, self.c_clip_seq = c_r, c_cond, c_clip_seq
        self.t_conds = list(t_conds)
        self.kernel_size = kernel_size
        self.self_attn = self_attn
        self.patch_size = patch_size
        c_hidden = list(c_hidden)
        self.clip_txt_mapper = Linear(c_clip_text, c_cond, dtype=dtype, device=device)
        self.clip_txt_pooled_mapper = Linear(c_clip_text_pooled, c_cond * c_clip_seq, dtype=dtype, device=device)
        self.clip_img_mapper = Linear(c_clip_img, c_cond * c_clip_seq, dtype=dtype, device=device)
        self.embedding = _embedding_seq(c_in, c_hidden[0], patch_size, dtype, device)
        self.down_downscalers = nn.ModuleList(
            [nn.Identity()] + [nn.Sequential(_LN2d(), UpDownBlock2d(c_hidden[i - 1], c_hidden[i], "down",
                                                                   enabled=switch_level[i - 1], dtype=dtype,
                                                                   device=device))
                               for i in range(1, len(c_hidden))])
        self.up_upscalers = nn.ModuleList(
            [nn.Sequential(_LN2d(), UpDownBlock2d(c_hidden[i], c_hidden[i - 1], "up", enabled=switch_level[i - 1],
                                                  dtype=dtype, device=device))
             for i in reversed(range(1, len(c_hidden)))] + [nn.Identity()])
        self._build_levels(c_hidden, list(nhead), blocks, block_repeat, level_config, dtype, device)
        self.clf = _clf_seq(c_hidden[0], c_out, patch_size, dtype, device)

    @staticmethod
    def _downscale(mod, x):
        return x if isinstance(mod, nn.Identity) else mod[1](_ln(x))

    @staticmethod
    def _upscale(mod, x):
        return x if isinstance(mod, nn.Identity) else mod[1](_ln(x))

    def gen_c_embeddings(self, clip_txt, clip_txt_pooled, clip_img):
        clip_txt = self.clip_txt_mapper(clip_txt)
        if clip_txt_pooled.dim() == 2:
            clip_txt_pooled = clip_txt_pooled.unsqueeze(1)
        if clip_img.dim() == 2:
            clip_img = clip_img.unsqueeze(1)
        B = clip_txt_pooled.shape[0]
        pooled = self.clip_txt_pooled_mapper(clip_txt_pooled).reshape(B, clip_txt_pooled.shape[1] * self.c_clip_seq, -1)
        img = self.clip_img_mapper(clip_img).reshape(clip_img.shape[0], clip_img.shape[1] * self.c_clip_seq, -1)
        return _ln(torch.cat([clip_txt, pooled, img.to(pooled.dtype)], dim=1))

    def forward(self, x, r, clip_text, clip_text_pooled, clip_img, control=None, **kwargs):
        dt = self.clip_txt_mapper.weight.dtype
        r_embed = self._with_ts(self._r_embed(r, dt, kwargs))
        def cond():
            return self.gen_c_embeddings(clip_text.to(dt), clip_text_pooled.to(dt), clip_img.to(dt))
        clip = self._static_cond(kwargs, (clip_text, clip_text_pooled, clip_img), lambda: self._attn_kv(cond()))
        if clip is None:
            clip = cond()
        cnet = list(control.get("input")) if control is not None and control.get("input") is not None else None
        h = self._embed(x.to(dt))
        levels = self._down_encode(h, r_embed, clip, cnet)
        h = self._up_decode(levels, r_embed, clip, cnet)
        return self._classify(h)


# ------------------------------------------------------------------------------------------------
# Stage B (latent decoder conditioned on the Stage C output)
# ------------------------------------------------------------------------------------------------
class _PatchConv(Conv2d):
    """kxk / stride-k conv (no overlap) as a patchify GEMM on NHWC."""

    def forward_nhwc(self, x):
        k = self.kernel_size[0]
        B, H, W, C = x.shape
        xp = x.reshape(B, H // k, k, W // k, k, C).permute(0, 1, 3, 2, 4, 5).reshape(B, H // k, W // k, k * k * C)
        w = self._derived_get("w_patch", lambda: self.weight.permute(0, 2, 3, 1).reshape(self.out_channels, -1)
                              .contiguous())
        return ops.linear(xp, _cast(w, x), _cast(self.bias, x))


class _PatchConvTranspose(nn.Module, DerivedMixin):
    """ConvTranspose2d(k, stride=k): one GEMM to [.., k*k*Cout] + depth-to-space."""

    def __init__(self, c_in, c_out, k, dtype=None, device=None):
        super().__init__()
        self.k, self.c_out = k, c_out
        self.weight = nn.Parameter(torch.empty(c_in, c_out, k, k, dtype=dtype, device=device), requires_grad=False)
        self.bias = nn.Parameter(torch.empty(c_out, dtype=dtype, device=device), requires_grad=False)

    def forward_nhwc(self, x):
        k, co = self.k, self.c_out
        B, H, W, C = x.shape
        w = self._derived_get("w_t", lambda: self.weight.permute(2, 3, 1, 0).reshape(k * k * co, C).contiguous())
        b = self._derived_get("b_t", lambda: self.bias.repeat(k * k))
        y = ops.linear(x, _cast(w, x), _cast(b, x))
        return y.reshape(B, H, W, k, k, co).permute(0, 1, 3, 2, 4, 5).reshape(B, H * k, W * k, co)


class StageB(_UNetStage):
    def __init__(self, c_in=4, c_out=4, c_r=64, patch_size=2, c_cond=1280, c_hidden=(320, 640, 1280, 1280),
                 nhead=(-1, -1, 20, 20), blocks=((2, 6, 28, 6), (6, 28, 6, 2)), block_repeat=((1, 1, 1, 1), (3, 3, 2, 2)),
                 level_config=("CT", "CT", "CTA", "CTA"), c_clip=1280, c_clip_seq=4, c_effnet=16, c_pixels=3,
                 kernel_size=3, dropout=(0, 0, 0.0, 0.0), self_attn=True, t_conds=("sca",), stable_cascade_stage=None,
                 dtype=None, device=None, **_):
        super().__init__()
        self.dtype = dtype
        self.c_r, self.c_cond, self.c_clip_seq = c_r, c_cond, c_clip_seq
        self.t_conds = list(t_conds)
        self.kernel_size = kernel_size
        self.self_attn = self_attn
        self.patch_size = patch_size
        c_hidden = list(c_hidden)
        self.effnet_mapper = nn.Sequential(Conv2d(c_effnet, c_hidden[0] * 4, 1, dtype=dtype, device=device), nn.GELU(),
                                           Conv2d(c_hidden[0] * 4, c_hidden[0], 1, dtype=dtype, device=device), _LN2d())
        self.pixels_mapper = nn.Sequential(Conv2d(c_pixels, c_hidden[0] * 4, 1, dtype=dtype, device=device), nn.GELU(),
                                           Conv2d(c_hidden[0] * 4, c_hidden[0], 1, dtype=dtype, device=device), _LN2d())
        self.clip_mapper = Linear(c_clip, c_cond * c_clip_seq, dtype=dtype, device=device)
        self.embedding = _embedding_seq(c_in, c_hidden[0], patch_size, dtype, device)
        self.down_downscalers = nn.ModuleList(
            [nn.Identity()] + [nn.Sequential(_LN2d(), _PatchConv(c_hidden[i - 1], c_hidden[i], 2, stride=2, dtype=dtype,
                                                                 device=device))
                               for i in range(1, len(c_hidden))])
        self.up_upscalers = nn.ModuleList(
            [nn.Sequential(_LN2d(), _PatchConvTranspose(c_hidden[i], c_hidden[i - 1], 2, dtype=dtype, device=device))
             for i in reversed(range(1, len(c_hidden)))] + [nn.Identity()])
        self._build_levels(c_hidden, list(nhead), blocks, block_repeat, level_config, dtype, device)
        self.clf = _clf_seq(c_hidden[0], c_out, patch_size, dtype, device)

    @staticmethod
    def _downscale(mod, x):
        return x if isinstance(mod, nn.Identity) else mod[1].forward_nhwc(_ln(x))

    @staticmethod
    def _upscale(mod, x):
        return x if isinstance(mod, nn.Identity) else mod[1].forward_nhwc(_ln(x))

    def _mapper(self, seq, x):
        return _ln(_pw(seq[2], _pw(seq[0], x, act="gelu")))

    def gen_c_embeddings(self, clip):
        if clip.dim() == 2:
            clip = clip.unsqueeze(1)
        B, L = clip.shape[:2]
        return _ln(self.clip_mapper(clip).reshape(B, L * self.c_clip_seq, -1))

    def _cond_maps(self, effnet, pixels, size, dt):
        """effnet_mapper(effnet at the latent size) + pixels_mapper(pixels) resized (stage_b.py forward)."""
        eff = _to_nhwc(F.interpolate(effnet.to(dt), size=size, mode="bilinear", align_corners=True))
        pix = _resize_nhwc(self._mapper(self.pixels_mapper, _to_nhwc(pixels.to(dt))), size)
        return self._mapper(self.effnet_mapper, eff) + pix

    def forward(self, x, r, effnet, clip, pixels=None, **kwargs):
        dt = self.clip_mapper.weight.dtype
        pix = pixels if pixels is not None else x.new_zeros(x.shape[0], 3, 8, 8)
        r_embed = self._with_ts(self._r_embed(r, dt, kwargs))
        p = self.patch_size
        size = (x.shape[2] // p, x.shape[3] // p)

        def static():
            d = self._attn_kv(self.gen_c_embeddings(clip.to(dt)))
            if d is not None:
                d["maps"] = self._cond_maps(effnet, pix, size, dt)
            return d
        st = self._static_cond(kwargs, (effnet, clip, pixels), static)
        if st is not None:
            kv, maps = st, st["maps"]
        else:
            kv, maps = self.gen_c_embeddings(clip.to(dt)), self._cond_maps(effnet, pix, size, dt)
        h = self._embed(x.to(dt)) + maps
        levels = self._down_encode(h, r_embed, kv)
        h = self._up_decode(levels, r_embed, kv)
        return self._classify(h)


# ------------------------------------------------------------------------------------------------
# Stage A (VQGAN: 4x spatial compression, 4 latent channels)
# ------------------------------------------------------------------------------------------------
class VectorQuantize(nn.Module):
    def __init__(self, embedding_size, k):
        super().__init__()
        self.codebook = nn.Embedding(k, embedding_size)

    def forward(self, x, dim=-1):
        """Nearest codebook entry per vector (along ``dim``) -> (quantized, indices)."""
        if dim != -1:
            x = x.movedim(dim, -1)
        q, idx = ops.vq_nearest(x.reshape(-1, x.shape[-1]), self.codebook.weight)
        q = q.reshape(x.shape)
        if dim != -1:
            q = q.movedim(-1, dim)
        return q, idx.reshape(x.shape[:-1])


class ResBlockA(nn.Module):
    """Stage A ResBlock (stage_a.py:126-164): learned gammas modulate LN / depthwise / MLP branches."""

    def __init__(self, c, c_hidden, dtype=None, device=None):
        super().__init__()
        self.depthwise = nn.Sequential(nn.Identity(), DepthwiseConv2d(c, 3, replicate=True, dtype=dtype, device=device))
        self.channelwise = nn.Sequential(Linear(c, c_hidden, dtype=dtype, device=device), nn.GELU(),
                                         Linear(c_hidden, c, dtype=dtype, device=device))
        self.gammas = nn.Parameter(torch.zeros(6, dtype=dtype, device=device), requires_grad=False)

    def forward(self, x):
        g = self.gammas.float().tolist()
        xt = _ln(x) * (1 + g[0]) + g[1]
        x = x + self.depthwise[1].forward_nhwc(xt) * g[2]
        xt = _ln(x) * (1 + g[3]) + g[4]
        h = F.gelu(self.channelwise[0](xt))
        return x + self.channelwise[2](h) * g[5]


class StageA(nn.Module):
    def __init__(self, levels=2, bottleneck_blocks=12, c_hidden=384, c_latent=4, codebook_size=8192,
                 dtype=None, device=None):
        super().__init__()
        self.c_latent = c_latent
        cl = [c_hidden // (2 ** i) for i in reversed(range(levels))]
        self.in_block = nn.Sequential(nn.PixelUnshuffle(2), Conv2d(3 * 4, cl[0], 1, dtype=dtype, device=device))
        down = []
        for i in range(levels):
            if i > 0:
                down.append(nn.Conv2d(cl[i - 1], cl[i], 4, 2, 1, dtype=dtype, device=device))
            down.append(ResBlockA(cl[i], cl[i] * 4, dtype=dtype, device=device))
        down.append(nn.Sequential(Conv2d(cl[-1], c_latent, 1, bias=False, dtype=dtype, device=device),
                                  nn.BatchNorm2d(c_latent, dtype=dtype, device=device)))
        self.down_blocks = nn.Sequential(*down)
        self.codebook_size = codebook_size
        self.vquantizer = VectorQuantize(c_latent, k=codebook_size)
        up = [nn.Sequential(Conv2d(c_latent, cl[-1], 1, dtype=dtype, device=device))]
        for i in range(levels):
            for _ in range(bottleneck_blocks if i == 0 else 1):
                up.append(ResBlockA(cl[levels - 1 - i], cl[levels - 1 - i] * 4, dtype=dtype, device=device))
            if i < levels - 1:
                up.append(nn.ConvTranspose2d(cl[levels - 1 - i], cl[levels - 2 - i], 4, 2, 1, dtype=dtype,
                                             device=device))
        self.up_blocks = nn.Sequential(*up)
        self.out_block = nn.Sequential(Conv2d(cl[0], 3 * 4, 1, dtype=dtype, device=device), nn.PixelShuffle(2))

    @staticmethod
    def _torch_conv(mod, x):
        """Overlapping 4x4 stride-2 (transposed) convs: vendor conv on a channels-last view."""
        w = _cast(mod.weight, x)
        b = _cast(mod.bias, x)
        xn = x.permute(0, 3, 1, 2)
        if isinstance(mod, nn.ConvTranspose2d):
            pw = None
            if xn.is_cuda and w is mod.weight:       # phase weights cached per weight version (K09 form)
                key = (w.data_ptr(), module_epoch(mod))     # epoch: bumped on every weight patch
                ent = mod.__dict__.get("_cgs_ct_phase")
                if ent is None or ent[0] != key:
                    ent = mod.__dict__["_cgs_ct_phase"] = (key, ops.conv_transpose_phase_weights(w))
                pw = ent[1]
            y = ops.conv_transpose2d(xn, w, b, mod.stride, mod.padding, phase_weights=pw)
        elif xn.is_cuda and w is mod.weight:
            ent = mod.__dict__.get("_cgs_w_nhwc")
            key = (w.data_ptr(), module_epoch(mod))
            if ent is None or ent[0] != key:
                ent = mod.__dict__["_cgs_w_nhwc"] = (key, w.permute(0, 2, 3, 1).contiguous())
            y = ops.conv2d(xn, w, b, mod.stride, mod.padding, weight_nhwc=ent[1])
        else:
            y = F.conv2d(xn, w, b, mod.stride, mod.padding)
        return _to_nhwc(y)

    def encode(self, x, quantize=False):
        dt = self.in_block[1].weight.dtype
        h = _to_nhwc(F.pixel_unshuffle(x.to(dt), 2))
        h = _pw(self.in_block[1], h)
        for m in self.down_blocks:
            if isinstance(m, ResBlockA):
                h = m(h)
            elif isinstance(m, nn.Conv2d):
                h = self._torch_conv(m, h)
            else:
                h = _pw(m[0], h)
                bn = m[1]
                h = F.batch_norm(h.permute(0, 3, 1, 2).float(), bn.running_mean.float(), bn.running_var.float(),
                                 None if bn.weight is None else bn.weight.float(),
                                 None if bn.bias is None else bn.bias.float(), False, 0.0, bn.eps)
                h = _to_nhwc(h.to(dt))
        if quantize:
            q, idx = self.vquantizer(h, dim=-1)
            return _to_nchw(q), _to_nchw(h), idx
        return _to_nchw(h)

    def decode(self, x):
        dt = self.in_block[1].weight.dtype
        h = _to_nhwc(x.to(dt))
        for m in self.up_blocks:
            if isinstance(m, ResBlockA):
                h = m(h)
            elif isinstance(m, nn.ConvTranspose2d):
                h = self._torch_conv(m, h)
            else:
                h = _pw(m[0], h)
        h = _pw(self.out_block[0], h)
        return F.pixel_shuffle(_to_nchw(h), 2)

    def forward(self, x, quantize=False):
        if quantize:
            q, _, _ = self.encode(x, quantize=True)
            return self.decode(q)
        return self.decode(self.encode(x))


# ------------------------------------------------------------------------------------------------
# EfficientNetV2-S features (torchvision layout; torchvision itself is not available here)
# ------------------------------------------------------------------------------------------------
def _cna(c_in, c_out, k, stride=1, groups=1, act=True, padding=None):
    p = (k - 1) // 2 if padding is None else padding
    layers = [nn.Conv2d(c_in, c_out, k, stride, p, groups=groups, bias=False), nn.BatchNorm2d(c_out, eps=1e-3)]
    if act:
        layers.append(nn.SiLU())
    return nn.Sequential(*layers)


class _SqueezeExcitation(nn.Module):
    def __init__(self, c, c_sq):
        super().__init__()
        self.fc1 = nn.Conv2d(c, c_sq, 1)
        self.fc2 = nn.Conv2d(c_sq, c, 1)

    def forward(self, x):
        s = F.adaptive_avg_pool2d(x, 1)
        return x * torch.sigmoid(self.fc2(F.silu(self.fc1(s))))


class _MBConv(nn.Module):
    def __init__(self, expand, k, stride, c_in, c_out, fused):
        super().__init__()
        mid = c_in * expand
        layers = []
        if fused:
            if mid != c_in:
                layers += [_cna(c_in, mid, k, stride), _cna(mid, c_out, 1, act=False)]
            else:
                layers += [_cna(c_in, c_out, k, stride)]
        else:
            if mid != c_in:
                layers.append(_cna(c_in, mid, 1))
            layers += [_cna(mid, mid, k, stride, groups=mid), _SqueezeExcitation(mid, max(1, c_in // 4)),
                       _cna(mid, c_out, 1, act=False)]
        self.block = nn.Sequential(*layers)
        self.use_res = stride == 1 and c_in == c_out

    def forward(self, x):
        y = self.block(x)
        return y + x if self.use_res else y


_EFFNET_V2_S = [(True, 1, 3, 1, 24, 24, 2), (True, 4, 3, 2, 24, 48, 4), (True, 4, 3, 2, 48, 64, 4),
                (False, 4, 3, 2, 64, 128, 6), (False, 6, 3, 1, 128, 160, 9), (False, 6, 3, 2, 160, 256, 15)]


def efficientnet_v2_s_features(c_in=3, stem_padding=None):
    feats = [_cna(c_in, 24, 3, 2, padding=stem_padding)]
    for fused, e, k, s, ci, co, n in _EFFNET_V2_S:
        feats.append(nn.Sequential(*[_MBConv(e, k, s if i == 0 else 1, ci if i == 0 else co, co, fused)
                                     for i in range(n)]))
    feats.append(_cna(256, 1280, 1))
    return nn.Sequential(*feats)


class EfficientNetEncoder(nn.Module):
    def __init__(self, c_latent=16):
        super().__init__()
        self.backbone = efficientnet_v2_s_features()
        self.mapper = nn.Sequential(nn.Conv2d(1280, c_latent, 1, bias=False), nn.BatchNorm2d(c_latent, affine=False))
        self.mean = nn.Parameter(torch.tensor([0.485, 0.456, 0.406]), requires_grad=False)
        self.std = nn.Parameter(torch.tensor([0.229, 0.224, 0.225]), requires_grad=False)

    def forward(self, x):
        x = x * 0.5 + 0.5
        x = (x - self.mean.view(3, 1, 1).to(x)) / self.std.view(3, 1, 1).to(x)
        return self.mapper(self.backbone(x))


class Previewer(nn.Module):
    """Fast RGB decoder for Stage C latents (16x24x24 -> 3x192x192)."""

    def __init__(self, c_in=16, c_hidden=512, c_out=3):
        super().__init__()
        h = c_hidden
        spec = [("c1", c_in, h), ("c3", h, h), ("t", h, h // 2), ("c3", h // 2, h // 2), ("t", h // 2, h // 4),
                ("c3", h // 4, h // 4), ("t", h // 4, h // 4), ("c3", h // 4, h // 4)]
        layers = []
        for kind, a, b in spec:
            if kind == "c1":
                layers.append(nn.Conv2d(a, b, 1))
            elif kind == "c3":
                layers.append(nn.Conv2d(a, b, 3, padding=1))
            else:
                layers.append(nn.ConvTranspose2d(a, b, 2, stride=2))
            layers += [nn.GELU(), nn.BatchNorm2d(b)]
        layers.append(nn.Conv2d(h // 4, c_out, 1))
        self.blocks = nn.Sequential(*layers)

    def forward(self, x):
        return (self.blocks(x) - 0.5) * 2.0


class StageC_coder(nn.Module):  # noqa: N801  (checkpoint naming)
    def __init__(self):
        super().__init__()
        self.previewer = Previewer()
        self.encoder = EfficientNetEncoder()

    def encode(self, x):
        return self.encoder(x.to(self.encoder.mean.dtype))

    def decode(self, x):
        return self.previewer(x.to(self.encoder.mean.dtype))


# ------------------------------------------------------------------------------------------------
# Cascade ControlNet (controlnet.py)
# ------------------------------------------------------------------------------------------------
class _LN2dAffine(LayerNorm):
    def forward(self, x):
        return _to_nchw(super().forward(_to_nhwc(x)))


class CNetResBlock(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.blocks = nn.Sequential(_LN2dAffine(c), nn.GELU(), nn.Conv2d(c, c, 3, padding=1),
                                    _LN2dAffine(c), nn.GELU(), nn.Conv2d(c, c, 3, padding=1))

    def forward(self, x):
        return x + self.blocks(x)


class CascadeControlNet(nn.Module):
    def __init__(self, c_in=3, c_proj=2048, proj_blocks=None, bottleneck_mode=None):
        super().__init__()
        bottleneck_mode = bottleneck_mode or "effnet"
        self.proj_blocks = list(proj_blocks)
        if bottleneck_mode == "effnet":
            embd = 1280
            self.backbone = efficientnet_v2_s_features(c_in, stem_padding=None if c_in == 3 else 0)
        elif bottleneck_mode == "simple":
            embd = c_in
            self.backbone = nn.Sequential(nn.Conv2d(embd, embd * 4, 3, padding=1), nn.LeakyReLU(0.2, inplace=True),
                                          nn.Conv2d(embd * 4, embd, 3, padding=1))
        elif bottleneck_mode == "large":
            self.backbone = nn.Sequential(nn.Conv2d(c_in, 4096 * 4, 1), nn.LeakyReLU(0.2, inplace=True),
                                          nn.Conv2d(4096 * 4, 1024, 1), *[CNetResBlock(1024) for _ in range(8)],
                                          nn.Conv2d(1024, 1280, 1))
            embd = 1280
        else:
            raise ValueError(f"Unknown bottleneck mode: {bottleneck_mode}")
        self.projections = nn.ModuleList([
            nn.Sequential(nn.Conv2d(embd, embd, 1, bias=False), nn.LeakyReLU(0.2, inplace=True),
                          nn.Conv2d(embd, c_proj, 1, bias=False)) for _ in self.proj_blocks])
        self.xl = False
        self.input_channels = c_in
        self.unshuffle_amount = 8

    def forward(self, x):
        x = self.backbone(x.to(next(self.parameters()).dtype))
        out = [None] * (max(self.proj_blocks) + 1)
        for i, idx in enumerate(self.proj_blocks):
            out[idx] = self.projections[i](x)
        return out


# ------------------------------------------------------------------------------------------------
# Diffusion-model wrappers (model_base.py:512-559)
# ------------------------------------------------------------------------------------------------
def _wrappers():
    from ..runtime.model_base import BaseModel, ModelType
    from ..sampling import conds as C

    class StableCascade_C(BaseModel):  # noqa: N801
        def __init__(self, model_config, model_type=ModelType.STABLE_CASCADE, device=None):
            super().__init__(model_config, model_type, device=device, unet_model=StageC)
            self.diffusion_model.eval().requires_grad_(False)

        def get_dtype(self):
            return self.diffusion_model.clip_txt_mapper.weight.dtype

        def extra_conds(self, **kwargs):
            out = {}
            pooled = kwargs.get("pooled_output")
            if pooled is not None:
                out["clip_text_pooled"] = C.CONDRegular(pooled)
            if "unclip_conditioning" in kwargs:
                embeds = [u["clip_vision_output"].image_embeds.unsqueeze(0) * u["strength"]
                          for u in kwargs["unclip_conditioning"]]
                clip_img = torch.cat(embeds, dim=1)
            else:
                clip_img = torch.zeros((1, 1, 768))
            out["clip_img"] = C.CONDRegular(clip_img)
            out["sca"] = C.CONDRegular(torch.zeros((1,)))
            out["crp"] = C.CONDRegular(torch.zeros((1,)))
            ca = kwargs.get("cross_attn")
            if ca is not None:
                out["clip_text"] = C.CONDCrossAttn(ca)
            return out

    class StableCascade_B(BaseModel):  # noqa: N801
        def __init__(self, model_config, model_type=ModelType.STABLE_CASCADE, device=None):
            super().__init__(model_config, model_type, device=device, unet_model=StageB)
            self.diffusion_model.eval().requires_grad_(False)

        def get_dtype(self):
            return self.diffusion_model.clip_mapper.weight.dtype

        def extra_conds(self, **kwargs):
            out = {}
            noise = kwargs.get("noise")
            pooled = kwargs.get("pooled_output")
            if pooled is not None:
                out["clip"] = C.CONDRegular(pooled)
            prior = kwargs.get("stable_cascade_prior")
            if prior is None:
                prior = torch.zeros((1, 16, (noise.shape[2] * 4) // 42, (noise.shape[3] * 4) // 42),
                                    dtype=noise.dtype, device=noise.device)
            out["effnet"] = C.CONDRegular(prior)
            out["sca"] = C.CONDRegular(torch.zeros((1,)))
            return out

    return StableCascade_C, StableCascade_B


def __getattr__(name):
    if name in ("StableCascade_C", "StableCascade_B"):
        c, b = _wrappers()
        globals()["StableCascade_C"], globals()["StableCascade_B"] = c, b
        return globals()[name]
    raise AttributeError(name)
