"""DAT — Dual Aggregation Transformer super-resolution (parity: ``comfy_extras/chainner_models/
architecture/DAT.py:897-1182``). Residual groups alternate two block kinds:

* spatial blocks: the channels are split in half, each half attends inside rectangular windows
  (``split_size`` and its transpose) with a dynamic (MLP-generated) relative position bias and
  periodic half-window shifts; a depthwise-conv branch on V is mixed in through the adaptive
  interaction module (channel map from the conv branch, spatial map from the attention branch);
* channel blocks: transposed (d x d) attention per head with a learned temperature, mixed with
  the same conv branch the other way round;

each followed by the spatial-gate feed-forward (SGFN). Projections are ``layers.Linear``, dense
convs ``layers.Conv2d``; depthwise convs and BatchNorm stay on torch modules. Shift masks and
position tables are derived from the geometry (cached), not read from the file.
"""
from __future__ import annotations

import math
import re

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from .layers import Conv2d, LayerNorm, Linear
from .swin_sr import _resi_conv, _Upsample, _to_img, _to_tokens

_MASKS: dict = {}


def _rect_mask(H, W, wh, ww, sh, sw, device):
    """Shifted-window mask for ``wh x ww`` windows shifted by (sh, sw): [nW, N, N] of 0 / -100."""
    key = (H, W, wh, ww, sh, sw, str(device))
    m = _MASKS.get(key)
    if m is None:
        lab = torch.zeros(H, W)
        cnt = 0
        for hs in (slice(0, -wh), slice(-wh, -sh), slice(-sh, None)):
            for ws in (slice(0, -ww), slice(-ww, -sw), slice(-sw, None)):
                lab[hs, ws] = cnt
                cnt += 1
        win = lab.view(H // wh, wh, W // ww, ww).permute(0, 2, 1, 3).reshape(-1, wh * ww)
        d = win[:, None, :] - win[:, :, None]
        m = torch.where(d != 0, torch.tensor(-100.0), torch.tensor(0.0)).to(device)
        if len(_MASKS) > 64:
            _MASKS.clear()
        _MASKS[key] = m
    return m


class _DynPosBias(nn.Module):
    def __init__(self, dim, heads):
        super().__init__()
        p = dim // 4
        self.pos_proj = Linear(2, p)
        self.pos1 = nn.Sequential(LayerNorm(p), nn.ReLU(), Linear(p, p))
        self.pos2 = nn.Sequential(LayerNorm(p), nn.ReLU(), Linear(p, p))
        self.pos3 = nn.Sequential(LayerNorm(p), nn.ReLU(), Linear(p, heads))

    def forward(self, b):
        return self.pos3(self.pos2(self.pos1(self.pos_proj(b))))


class _RectWindowAttention(nn.Module):
    """One branch of the spatial block: attention in ``wh x ww`` windows over C/2 channels."""

    def __init__(self, dim, heads, wh, ww):
        super().__init__()
        self.heads, self.wh, self.ww = heads, wh, ww
        self.scale = (dim // heads) ** -0.5
        self.pos = _DynPosBias(dim // 4, heads)
        dh = torch.arange(1 - wh, wh)
        dw = torch.arange(1 - ww, ww)
        self.register_buffer("rpe_tab", torch.stack(torch.meshgrid(dh, dw, indexing="ij")).flatten(1).t().float(),
                             persistent=False)
        c = torch.stack(torch.meshgrid(torch.arange(wh), torch.arange(ww), indexing="ij")).flatten(1)
        r = (c[:, :, None] - c[:, None, :]).permute(1, 2, 0)
        self.register_buffer("rel_idx", (r[..., 0] + wh - 1) * (2 * ww - 1) + (r[..., 1] + ww - 1), persistent=False)

    def forward(self, q, k, v, H, W, mask):        # q/k/v [B, H, W, C] -> [B, H, W, C]
        B, _, _, C = q.shape
        wh, ww, h = self.wh, self.ww, self.heads
        N = wh * ww

        def win(t):
            t = t.reshape(B, H // wh, wh, W // ww, ww, C).permute(0, 1, 3, 2, 4, 5).reshape(-1, N, h, C // h)
            return t.transpose(1, 2)

        qw, kw, vw = win(q), win(k), win(v)
        bias = self.pos(self.rpe_tab.to(self.pos.pos_proj.weight.dtype)).float()[self.rel_idx.reshape(-1)]
        bias = bias.view(N, N, h).permute(2, 0, 1)
        o = ops.attention_bias(qw, kw, vw, bias, mask, scale=self.scale).transpose(1, 2).reshape(-1, N, C)
        return o.view(B, H // wh, W // ww, wh, ww, C).permute(0, 1, 3, 2, 4, 5).reshape(B, H, W, C)


def _aim_branches(dim):
    dw = nn.Sequential(nn.Conv2d(dim, dim, 3, padding=1, groups=dim), nn.BatchNorm2d(dim), nn.GELU())
    ci = nn.Sequential(nn.AdaptiveAvgPool2d(1), Conv2d(dim, dim // 8, 1), nn.BatchNorm2d(dim // 8), nn.GELU(),
                       Conv2d(dim // 8, dim, 1))
    si = nn.Sequential(Conv2d(dim, dim // 16, 1), nn.BatchNorm2d(dim // 16), nn.GELU(), Conv2d(dim // 16, 1, 1))
    return dw, ci, si


class AdaptiveSpatialAttention(nn.Module):
    def __init__(self, dim, heads, split, shifted: bool):
        super().__init__()
        self.split, self.shifted = split, shifted
        self.shift = [split[0] // 2, split[1] // 2]
        self.qkv = Linear(dim, dim * 3)
        self.proj = Linear(dim, dim)
        self.attns = nn.ModuleList([_RectWindowAttention(dim // 2, heads // 2, split[0], split[1]),
                                    _RectWindowAttention(dim // 2, heads // 2, split[1], split[0])])
        self.dwconv, self.channel_interaction, self.spatial_interaction = _aim_branches(dim)

    def forward(self, x, H, W):
        B, L, C = x.shape
        qkv = self.qkv(x).view(B, H, W, 3, C)
        v_img = qkv[..., 2, :].permute(0, 3, 1, 2)
        m = max(self.split)
        ph, pw = (m - H % m) % m, (m - W % m) % m
        if ph or pw:
            qkv = F.pad(qkv, (0, 0, 0, 0, 0, pw, 0, ph))
        Hp, Wp = H + ph, W + pw
        s0, s1 = self.shift
        outs = []
        for i, a in enumerate(self.attns):
            t = qkv[..., C // 2:] if i else qkv[..., :C // 2]
            shift = (s1, s0) if i else (s0, s1)
            mask = None
            if self.shifted:
                t = torch.roll(t, (-shift[0], -shift[1]), (1, 2))
                mask = _rect_mask(Hp, Wp, a.wh, a.ww, shift[0], shift[1], x.device)
            o = a(t[..., 0, :], t[..., 1, :], t[..., 2, :], Hp, Wp, mask)
            if self.shifted:
                o = torch.roll(o, shift, (1, 2))
            outs.append(o[:, :H, :W])
        att = torch.cat(outs, -1).reshape(B, L, C)
        conv = self.dwconv(v_img.contiguous())
        cmap = self.channel_interaction(conv).view(B, 1, C)
        smap = self.spatial_interaction(_to_img(att, (H, W)))
        att = att * torch.sigmoid(cmap)
        conv = (torch.sigmoid(smap) * conv).flatten(2).transpose(1, 2)
        return self.proj(att + conv)


class AdaptiveChannelAttention(nn.Module):
    def __init__(self, dim, heads):
        super().__init__()
        self.heads = heads
        self.temperature = nn.Parameter(torch.ones(heads, 1, 1), requires_grad=False)
        self.qkv = Linear(dim, dim * 3)
        self.proj = Linear(dim, dim)
        self.dwconv, self.channel_interaction, self.spatial_interaction = _aim_branches(dim)

    def forward(self, x, H, W):
        B, N, C = x.shape
        h = self.heads
        q, k, v = self.qkv(x).view(B, N, 3, h, C // h).permute(2, 0, 3, 4, 1).unbind(0)   # [B, h, d, N]
        s = F.normalize(q.float(), dim=-1) @ F.normalize(k.float(), dim=-1).transpose(-2, -1)
        att = (torch.softmax(s * self.temperature.float(), -1).to(v.dtype) @ v)      # [B, h, d, N]
        att = att.permute(0, 3, 1, 2).reshape(B, N, C)
        conv = self.dwconv(v.reshape(B, C, H, W))
        cmap = self.channel_interaction(_to_img(att, (H, W)))
        smap = self.spatial_interaction(conv).flatten(2).transpose(1, 2)             # [B, N, 1]
        att = att * torch.sigmoid(smap)
        conv = (conv * torch.sigmoid(cmap)).flatten(2).transpose(1, 2)
        return self.proj(att + conv)


class _SpatialGate(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.norm = LayerNorm(dim)
        self.conv = nn.Conv2d(dim, dim, 3, padding=1, groups=dim)

    def forward(self, x, H, W):
        a, g = x.chunk(2, -1)
        g = self.conv(_to_img(self.norm(g), (H, W)).contiguous())
        return a * _to_tokens(g)


class _SGFN(nn.Module):
    def __init__(self, dim, hidden):
        super().__init__()
        self.fc1 = Linear(dim, hidden)
        self.sg = _SpatialGate(hidden // 2)
        self.fc2 = Linear(hidden // 2, dim)

    def forward(self, x, H, W):
        return self.fc2(self.sg(F.gelu(self.fc1(x)), H, W))


def _is_shifted(rg: int, b: int) -> bool:
    """Shift pattern of the reference: blocks 2, 6, 10… in even groups; 0, 4, 8… in odd groups."""
    return (rg % 2 == 0 and b > 0 and (b - 2) % 4 == 0) or (rg % 2 != 0 and b % 4 == 0)


class DATB(nn.Module):
    def __init__(self, dim, heads, split, expansion, rg, b):
        super().__init__()
        self.norm1 = LayerNorm(dim)
        if b % 2 == 0:
            self.attn = AdaptiveSpatialAttention(dim, heads, split, _is_shifted(rg, b))
        else:
            self.attn = AdaptiveChannelAttention(dim, heads)
        self.norm2 = LayerNorm(dim)
        self.ffn = _SGFN(dim, int(dim * expansion))

    def forward(self, x, hw):
        H, W = hw
        x = x + self.attn(self.norm1(x), H, W)
        return x + self.ffn(self.norm2(x), H, W)


class ResidualGroup(nn.Module):
    def __init__(self, dim, heads, split, expansion, depth, resi, rg):
        super().__init__()
        self.blocks = nn.ModuleList([DATB(dim, heads, split, expansion, rg, b) for b in range(depth)])
        self.conv = _resi_conv(dim, resi)

    def forward(self, x, hw):
        y = x
        for blk in self.blocks:
            y = blk(y, hw)
        return _to_tokens(self.conv(_to_img(y, hw))) + x


class DAT(nn.Module):
    def __init__(self, state_dict, strict: bool = True):
        super().__init__()
        sd = state_dict
        keys = set(sd)
        self.model_arch = "DAT"
        if "conv_before_upsample.0.weight" in keys and "conv_up1.weight" not in keys:
            up = "pixelshuffle"
        elif "upsample.0.weight" in keys and "conv_before_upsample.0.weight" not in keys:
            up = "pixelshuffledirect"
        else:
            raise ValueError("DAT: only the pixelshuffle / pixelshuffledirect heads exist in the reference")
        self.upsampler = up
        in_ch = sd["conv_first.weight"].shape[1]
        dim = sd["conv_first.weight"].shape[0]
        nf = 64
        if up == "pixelshuffle":
            upscale = 1.0
            for k in keys:
                if re.match(r"^upsample\.\d+\.weight$", k):
                    upscale *= math.sqrt(sd[k].shape[0] // nf)
            upscale = int(round(upscale))
        else:
            upscale = int(math.sqrt(sd["upsample.0.bias"].shape[0] // in_ch))
        blocks = [tuple(map(int, m.groups())) for k in keys
                  for m in [re.match(r"^layers\.(\d+)\.blocks\.(\d+)\.norm1\.weight$", k)] if m]
        n_layers = 1 + max(b[0] for b in blocks)
        depth = 1 + max(b[1] for b in blocks)
        heads = sd["layers.0.blocks.1.attn.temperature"].shape[0] if "layers.0.blocks.1.attn.temperature" in keys \
            else depth
        expansion = sd["layers.0.blocks.0.ffn.fc1.weight"].shape[0] / dim
        resi = "3conv" if "layers.0.conv.4.weight" in keys else "1conv"
        split = [2, 4]
        if "layers.0.blocks.0.attn.attns.0.rpe_biases" in keys:
            split = [int(v) + 1 for v in sd["layers.0.blocks.0.attn.attns.0.rpe_biases"][-1]]
        self.in_nc = self.out_nc = in_ch
        self.scale = self.upscale = upscale
        self.embed_dim, self.split_size, self.depth, self.num_heads = dim, split, [depth] * n_layers, [heads] * n_layers
        self.img_range = 1.0
        mean = torch.tensor([0.4488, 0.4371, 0.4040]).view(1, 3, 1, 1) if in_ch == 3 else torch.zeros(1, 1, 1, 1)
        self.register_buffer("mean", mean, persistent=False)
        self.conv_first = Conv2d(in_ch, dim, 3, padding=1)
        self.before_RG = nn.Sequential(nn.Identity(), LayerNorm(dim))
        self.layers = nn.ModuleList([ResidualGroup(dim, heads, split, expansion, depth, resi, i)
                                     for i in range(n_layers)])
        self.norm = LayerNorm(dim)
        self.conv_after_body = _resi_conv(dim, resi)
        if up == "pixelshuffle":
            self.conv_before_upsample = nn.Sequential(Conv2d(dim, nf, 3, padding=1), nn.LeakyReLU(0.01))
            self.upsample = _Upsample(upscale, nf)
            self.conv_last = Conv2d(nf, in_ch, 3, padding=1)
        else:
            self.upsample = nn.Sequential(Conv2d(dim, upscale ** 2 * in_ch, 3, padding=1), nn.PixelShuffle(upscale))
        missing, _ = self.load_state_dict(sd, strict=False)
        if missing and strict:
            raise ValueError(f"DAT: missing keys {missing[:4]}")
        self.eval()

    def forward(self, x):
        mean = self.mean.to(x.dtype)
        x = (x - mean) * self.img_range
        f = self.conv_first(x)
        hw = f.shape[-2:]
        t = self.before_RG[1](_to_tokens(f))
        for layer in self.layers:
            t = layer(t, hw)
        y = self.conv_after_body(_to_img(self.norm(t), hw)) + f
        if self.upsampler == "pixelshuffle":
            y = self.conv_last(self.upsample(self.conv_before_upsample(y)))
        else:
            y = self.upsample(y)
        return y / self.img_range + mean
