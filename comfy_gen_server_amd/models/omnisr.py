"""Omni-SR (omni self-attention super-resolution; parity: ``comfy_extras/chainner_models/
architecture/OmniSR/{OmniSR,OSAG,OSA,esa}.py``): groups of OSA blocks — an MBConv, then a
block-window and a grid(dilated)-window pass, each made of spatial multi-head attention with a
learned relative-position bias, gated depthwise feed-forwards and channel (transposed)
attention — closed by an enhanced-spatial-attention gate, then a pixel-shuffle head.

Window regrouping is done with explicit view/permute (no einops); 1x1 convs and projections
are ``layers.Conv2d`` / ``layers.Linear`` (device GEMM kernels); depthwise convs stay on
``nn.Conv2d``. The block count per group is read from the state dict (the reference assumes 1).
"""
from __future__ import annotations

import math
import re

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from .layers import Conv2d, LayerNorm, Linear
from .swin_sr import _rel_index


class _LN2d(nn.Module):
    """Channel LayerNorm on NCHW (eps 1e-6), keys ``weight``/``bias``."""

    def __init__(self, c):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(c), requires_grad=False)
        self.bias = nn.Parameter(torch.zeros(c), requires_grad=False)

    def forward(self, x):
        xf = x.float()
        mu = xf.mean(1, keepdim=True)
        var = (xf - mu).pow(2).mean(1, keepdim=True)
        y = (xf - mu) * torch.rsqrt(var + 1e-6)
        return (y * self.weight.float().view(1, -1, 1, 1) + self.bias.float().view(1, -1, 1, 1)).to(x.dtype)


class _SE(nn.Module):
    def __init__(self, dim, rate=0.25):
        super().__init__()
        hid = int(dim * rate)
        self.gate = nn.Sequential(nn.Identity(), Linear(dim, hid, bias=False), nn.SiLU(), Linear(hid, dim, bias=False))

    def forward(self, x):
        g = torch.sigmoid(self.gate(x.mean((2, 3))))
        return x * g[:, :, None, None]


class _MBConv(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.fn = nn.Sequential(Conv2d(dim, dim, 1), nn.GELU(), nn.Conv2d(dim, dim, 3, padding=1, groups=dim),
                                nn.GELU(), _SE(dim), Conv2d(dim, dim, 1))

    def forward(self, x):
        return self.fn(x) + x


class _WinAttention(nn.Module):
    """Multi-head attention inside ``ws x ws`` token groups with a learned relative bias."""

    def __init__(self, dim, ws, heads=4):
        super().__init__()
        self.heads, self.ws = heads, ws
        self.scale = (dim // heads) ** -0.5
        self.to_qkv = Linear(dim, dim * 3, bias=False)
        self.rel_pos_bias = nn.Embedding((2 * ws - 1) ** 2, heads)
        self.rel_pos_bias.weight.requires_grad_(False)
        self.to_out = nn.Sequential(Linear(dim, dim, bias=False))
        self.register_buffer("rel_idx", _rel_index(ws), persistent=False)

    def forward(self, t):                       # t [Bw, N, C]
        Bw, N, C = t.shape
        h = self.heads
        q, k, v = self.to_qkv(t).view(Bw, N, 3, h, C // h).permute(2, 0, 3, 1, 4).unbind(0)
        bias = self.rel_pos_bias.weight.float()[self.rel_idx].permute(2, 0, 1)
        o = ops.attention_bias(q, k, v, bias, scale=self.scale).transpose(1, 2).reshape(Bw, N, C)
        return self.to_out(o)


class _PreNormAttn(nn.Module):
    def __init__(self, dim, ws, grid: bool):
        super().__init__()
        self.norm = LayerNorm(dim)
        self.fn = _WinAttention(dim, ws)
        self.grid, self.ws = grid, ws

    def forward(self, x):                       # NCHW in/out; the residual is taken in token layout
        B, C, H, W = x.shape
        w = self.ws
        X, Y = H // w, W // w
        if self.grid:    # pixel (w1 * X + x, w2 * Y + y) belongs to window (x, y)
            t = x.view(B, C, w, X, w, Y).permute(0, 3, 5, 2, 4, 1)
        else:            # pixel (x * w + w1, y * w + w2)
            t = x.view(B, C, X, w, Y, w).permute(0, 2, 4, 3, 5, 1)
        t = t.reshape(B * X * Y, w * w, C)
        t = self.fn(self.norm(t)) + t
        t = t.view(B, X, Y, w, w, C)
        if self.grid:
            return t.permute(0, 5, 3, 1, 4, 2).reshape(B, C, H, W)
        return t.permute(0, 5, 1, 3, 2, 4).reshape(B, C, H, W)


class _GatedFF(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.project_in = Conv2d(dim, dim * 2, 1, bias=False)
        self.dwconv = nn.Conv2d(dim * 2, dim * 2, 3, padding=1, groups=dim * 2, bias=False)
        self.project_out = Conv2d(dim, dim, 1, bias=False)

    def forward(self, x):
        a, g = self.dwconv(self.project_in(x)).chunk(2, 1)
        return self.project_out(F.gelu(a) * g)


class _ChannelAttn(nn.Module):
    """Transposed (d x d) attention per head, over the pixels of a window (``grid=False``) or over
    same-offset pixels across all windows (``grid=True``); cosine logits x learned temperature."""

    def __init__(self, dim, ws, grid: bool, heads=4):
        super().__init__()
        self.heads, self.ws, self.grid = heads, ws, grid
        self.temperature = nn.Parameter(torch.ones(heads, 1, 1), requires_grad=False)
        self.qkv = Conv2d(dim, dim * 3, 1, bias=False)
        self.qkv_dwconv = nn.Conv2d(dim * 3, dim * 3, 3, padding=1, groups=dim * 3, bias=False)
        self.project_out = Conv2d(dim, dim, 1, bias=False)

    def forward(self, x):
        B, C, H, W = x.shape
        p, h = self.ws, self.heads
        nh, nw = H // p, W // p
        d = C // h

        def split(t):                # -> [B, G, heads, d, T]
            t = t.reshape(B, h, d, nh, p, nw, p)
            if self.grid:
                return t.permute(0, 4, 6, 1, 2, 3, 5).reshape(B, p * p, h, d, nh * nw)
            return t.permute(0, 3, 5, 1, 2, 4, 6).reshape(B, nh * nw, h, d, p * p)

        q, k, v = (split(t) for t in self.qkv_dwconv(self.qkv(x)).chunk(3, 1))
        s = F.normalize(q.float(), dim=-1) @ F.normalize(k.float(), dim=-1).transpose(-2, -1)
        o = torch.softmax(s * self.temperature.float(), -1).to(v.dtype) @ v
        if self.grid:
            o = o.view(B, p, p, h, d, nh, nw).permute(0, 3, 4, 5, 1, 6, 2)
        else:
            o = o.view(B, nh, nw, h, d, p, p).permute(0, 3, 4, 1, 5, 2, 6)
        return self.project_out(o.reshape(B, C, H, W))


class _ConvPreNorm(nn.Module):
    def __init__(self, dim, fn):
        super().__init__()
        self.norm = _LN2d(dim)
        self.fn = fn

    def forward(self, x):
        return self.fn(self.norm(x)) + x


class OSABlock(nn.Module):
    def __init__(self, dim, ws):
        super().__init__()
        # indices match the reference Sequential (1, 3, 7, 9 are parameter-free regroupings)
        mods = [_MBConv(dim), nn.Identity(), _PreNormAttn(dim, ws, grid=False), nn.Identity(),
                _ConvPreNorm(dim, _GatedFF(dim)), _ConvPreNorm(dim, _ChannelAttn(dim, ws, grid=False)),
                _ConvPreNorm(dim, _GatedFF(dim)), nn.Identity(), _PreNormAttn(dim, ws, grid=True), nn.Identity(),
                _ConvPreNorm(dim, _GatedFF(dim)), _ConvPreNorm(dim, _ChannelAttn(dim, ws, grid=True)),
                _ConvPreNorm(dim, _GatedFF(dim))]
        self.layer = nn.Sequential(*mods)

    def forward(self, x):
        return self.layer(x)


class _ESA(nn.Module):
    def __init__(self, f, n):
        super().__init__()
        self.conv1 = Conv2d(n, f, 1)
        self.conv_f = Conv2d(f, f, 1)
        self.conv2 = Conv2d(f, f, 3, stride=2)
        self.conv3 = Conv2d(f, f, 3, padding=1)
        self.conv4 = Conv2d(f, n, 1)

    def forward(self, x):
        c1_ = self.conv1(x)
        c3 = self.conv3(F.max_pool2d(self.conv2(c1_), 7, 3))
        c3 = F.interpolate(c3, x.shape[-2:], mode="bilinear", align_corners=False)
        return x * torch.sigmoid(self.conv4(c3 + self.conv_f(c1_)))


class OSAG(nn.Module):
    def __init__(self, dim, ws, blocks):
        super().__init__()
        self.residual_layer = nn.Sequential(*[OSABlock(dim, ws) for _ in range(blocks)], Conv2d(dim, dim, 1))
        self.esa = _ESA(max(dim // 4, 16), dim)

    def forward(self, x):
        return self.esa(self.residual_layer(x) + x)


class OmniSR(nn.Module):
    def __init__(self, state_dict, strict: bool = True):
        super().__init__()
        sd = state_dict
        self.model_arch = "OmniSR"
        nf = self.num_feat = sd["input.weight"].shape[0]
        in_ch = self.in_nc = self.out_nc = sd["input.weight"].shape[1]
        self.scale = self.up_scale = int(math.sqrt(sd["up.0.weight"].shape[0] / in_ch))
        groups = 1 + max(int(k.split(".")[1]) for k in sd if k.startswith("residual_layer."))
        blocks = 1 + max([int(m.group(1)) for k in sd
                          for m in [re.match(r"^residual_layer\.0\.residual_layer\.(\d+)\.layer\.", k)] if m] or [0])
        bias_key = "residual_layer.0.residual_layer.0.layer.2.fn.rel_pos_bias.weight"
        self.window_size = int((math.sqrt(sd[bias_key].shape[0]) + 1) / 2) if bias_key in sd else 8
        self.input = Conv2d(in_ch, nf, 3, padding=1)
        self.residual_layer = nn.Sequential(*[OSAG(nf, self.window_size, blocks) for _ in range(groups)])
        self.output = Conv2d(nf, nf, 3, padding=1)
        self.up = nn.Sequential(Conv2d(nf, in_ch * self.scale ** 2, 3, padding=1), nn.PixelShuffle(self.scale))
        missing, _ = self.load_state_dict(sd, strict=False)
        if missing and strict:
            raise ValueError(f"OmniSR: missing keys {missing[:4]}")
        self.eval()

    def forward(self, x):
        H, W = x.shape[-2:]
        w = self.window_size
        x = F.pad(x, (0, (w - W % w) % w, 0, (w - H % w) % w))
        r = self.input(x)
        out = self.up(self.output(self.residual_layer(r)) + r)
        return out[:, :, :H * self.scale, :W * self.scale]
