"""Swin-transformer image restoration networks for ``UpscaleModelLoader``: SwinIR, Swin2SR and HAT
(parity: ``comfy_extras/chainner_models/architecture/SwinIR.py:788-1212``,
``Swin2SR.py:880-1365`` and ``HAT.py:847-1277`` — config inference from the state dict, window attention with relative
position bias / SwinV2 scaled-cosine attention with the continuous position-bias MLP, the
residual Swin transformer blocks, and every upsampler head the reference detects).

Layout: activations stay token-major ``[B, H*W, C]`` between blocks; a block rolls and
partitions the ``[B, H, W, C]`` view into ``ws x ws`` windows, runs one batched attention over
``B * nW`` windows (fp32 softmax), and reverses. Linear layers are ``layers.Linear`` (HIP GEMM
on the device), convs are ``layers.Conv2d`` (NHWC implicit-GEMM MFMA kernel). The relative
position index, the shifted-window mask and the SwinV2 coordinate table are derived from the
window geometry (cached per shape/device) instead of being read from the file.
"""
from __future__ import annotations

import math
import re

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from .layers import Conv2d, LayerNorm, Linear


def _rel_index(ws: int) -> torch.Tensor:
    c = torch.stack(torch.meshgrid(torch.arange(ws), torch.arange(ws), indexing="ij")).flatten(1)
    r = (c[:, :, None] - c[:, None, :]).permute(1, 2, 0) + (ws - 1)
    return r[..., 0] * (2 * ws - 1) + r[..., 1]          # [N, N] into the (2ws-1)^2 table


_MASKS: dict = {}


def shift_mask(H: int, W: int, ws: int, shift: int, device) -> torch.Tensor:
    """[nW, N, N] additive mask (0 / -100) separating the regions a cyclic shift glued together."""
    key = (H, W, ws, shift, str(device))
    m = _MASKS.get(key)
    if m is None:
        lab = torch.zeros(H, W)
        cnt = 0
        for hs in (slice(0, -ws), slice(-ws, -shift), slice(-shift, None)):
            for wsl in (slice(0, -ws), slice(-ws, -shift), slice(-shift, None)):
                lab[hs, wsl] = cnt
                cnt += 1
        win = lab.view(H // ws, ws, W // ws, ws).permute(0, 2, 1, 3).reshape(-1, ws * ws)
        d = win[:, None, :] - win[:, :, None]
        m = torch.where(d != 0, torch.tensor(-100.0), torch.tensor(0.0)).to(device)
        if len(_MASKS) > 64:
            _MASKS.clear()
        _MASKS[key] = m
    return m


def pad_to_multiple(x: torch.Tensor, m: int) -> torch.Tensor:
    """Reflect-pad H/W up to a multiple of ``m`` (reference ``check_image_size``); inputs smaller
    than the pad, where reflection is undefined, are edge-replicated instead."""
    H, W = x.shape[-2:]
    ph, pw = (m - H % m) % m, (m - W % m) % m
    if not ph and not pw:
        return x
    return F.pad(x, (0, pw, 0, ph), "reflect" if ph < H and pw < W else "replicate")


def _partition(x: torch.Tensor, ws: int) -> torch.Tensor:
    B, H, W, C = x.shape
    return x.view(B, H // ws, ws, W // ws, ws, C).permute(0, 1, 3, 2, 4, 5).reshape(-1, ws * ws, C)


def _reverse(w: torch.Tensor, ws: int, B: int, H: int, W: int) -> torch.Tensor:
    C = w.shape[-1]
    return w.view(B, H // ws, W // ws, ws, ws, C).permute(0, 1, 3, 2, 4, 5).reshape(B, H, W, C)


class WindowAttention(nn.Module):
    """W-MSA. ``v2``: SwinV2 scaled-cosine attention (per-head learned logit scale clamped at
    log 100) with position bias ``16 * sigmoid(cpb_mlp(log-spaced coords))`` and q/v-only bias."""

    def __init__(self, dim: int, ws: int, heads: int, v2: bool = False, qkv_bias: bool = True):
        super().__init__()
        self.dim, self.ws, self.heads, self.v2 = dim, ws, heads, v2
        self.scale = (dim // heads) ** -0.5
        if v2:
            self.logit_scale = nn.Parameter(torch.log(10 * torch.ones(heads, 1, 1)), requires_grad=False)
            self.cpb_mlp = nn.Sequential(Linear(2, 512), nn.ReLU(), Linear(512, heads, bias=False))
            self.qkv = Linear(dim, dim * 3, bias=False)
            if qkv_bias:
                self.q_bias = nn.Parameter(torch.zeros(dim), requires_grad=False)
                self.v_bias = nn.Parameter(torch.zeros(dim), requires_grad=False)
            else:
                self.q_bias = self.v_bias = None
            t = torch.arange(-(ws - 1), ws, dtype=torch.float32) / max(ws - 1, 1) * 8
            tab = torch.stack(torch.meshgrid(t, t, indexing="ij"), -1)      # [2ws-1, 2ws-1, 2]
            tab = torch.sign(tab) * torch.log2(tab.abs() + 1.0) / math.log2(8)
            self.register_buffer("coords_table", tab.reshape(-1, 2), persistent=False)
        else:
            self.relative_position_bias_table = nn.Parameter(torch.zeros((2 * ws - 1) ** 2, heads),
                                                             requires_grad=False)
            self.qkv = Linear(dim, dim * 3, bias=qkv_bias)
        self.proj = Linear(dim, dim)
        self.register_buffer("rel_index", _rel_index(ws), persistent=False)

    def position_bias(self) -> torch.Tensor:
        """[heads, N, N] additive bias (fp32)."""
        if self.v2:
            tab = self.cpb_mlp(self.coords_table.to(self.cpb_mlp[0].weight.dtype)).float()
            bias = 16 * torch.sigmoid(tab[self.rel_index.view(-1)])
        else:
            bias = self.relative_position_bias_table.float()[self.rel_index.view(-1)]
        N = self.ws * self.ws
        return bias.view(N, N, self.heads).permute(2, 0, 1)

    def forward(self, x: torch.Tensor, mask: torch.Tensor | None) -> torch.Tensor:
        Bw, N, C = x.shape
        h = self.heads
        if self.v2 and self.q_bias is not None:
            qkv = self.qkv(x) + torch.cat([self.q_bias, torch.zeros_like(self.v_bias), self.v_bias]).to(x.dtype)
        else:
            qkv = self.qkv(x)
        q, k, v = qkv.view(Bw, N, 3, h, C // h).permute(2, 0, 3, 1, 4).unbind(0)
        if self.v2:     # cosine scores: unit q / k, the per-head logit scale on the fp32 scores
            q = F.normalize(q.float(), dim=-1).to(v.dtype)
            k = F.normalize(k.float(), dim=-1).to(v.dtype)
            o = ops.attention_bias(q, k, v, self.position_bias(), mask, scale=1.0,
                                   head_scale=torch.clamp(self.logit_scale.float(), max=math.log(100.0)).exp())
        else:
            o = ops.attention_bias(q, k, v, self.position_bias(), mask, scale=self.scale)
        return self.proj(o.transpose(1, 2).reshape(Bw, N, C))


class _Mlp(nn.Module):
    def __init__(self, dim: int, hidden: int):
        super().__init__()
        self.fc1 = Linear(dim, hidden)
        self.fc2 = Linear(hidden, dim)

    def forward(self, x):
        return self.fc2(F.gelu(self.fc1(x)))


class SwinBlock(nn.Module):
    """Pre-norm (SwinIR) or res-post-norm (Swin2SR, ``v2``) shifted-window transformer block."""

    def __init__(self, dim, heads, ws, shift, mlp_ratio, img_size, v2=False):
        super().__init__()
        if img_size <= ws:                         # reference: a window never exceeds the train size
            shift, ws = 0, img_size
        self.ws, self.shift, self.v2 = ws, shift, v2
        self.norm1 = LayerNorm(dim)
        self.attn = WindowAttention(dim, ws, heads, v2=v2)
        self.norm2 = LayerNorm(dim)
        self.mlp = _Mlp(dim, int(dim * mlp_ratio))

    def _attend(self, x, hw):
        H, W = hw
        B, L, C = x.shape
        ws, sh = self.ws, self.shift
        y = x.view(B, H, W, C)
        if sh:
            y = torch.roll(y, (-sh, -sh), (1, 2))
        y = self.attn(_partition(y, ws), shift_mask(H, W, ws, sh, x.device) if sh else None)
        y = _reverse(y, ws, B, H, W)
        if sh:
            y = torch.roll(y, (sh, sh), (1, 2))
        return y.reshape(B, L, C)

    def forward(self, x, hw):
        if self.v2:
            x = x + self.norm1(self._attend(x, hw))
            return x + self.norm2(self.mlp(x))
        x = x + self._attend(self.norm1(x), hw)
        return x + self.mlp(self.norm2(x))


def _resi_conv(dim: int, kind: str) -> nn.Module:
    if kind == "1conv":
        return Conv2d(dim, dim, 3, padding=1)
    return nn.Sequential(Conv2d(dim, dim // 4, 3, padding=1), nn.LeakyReLU(0.2),
                         Conv2d(dim // 4, dim // 4, 1), nn.LeakyReLU(0.2),
                         Conv2d(dim // 4, dim, 3, padding=1))


def _to_img(x, hw):
    B, L, C = x.shape
    return x.transpose(1, 2).reshape(B, C, hw[0], hw[1])


def _to_tokens(x):
    return x.flatten(2).transpose(1, 2)


class RSTB(nn.Module):
    """Residual Swin Transformer Block: blocks -> conv on the image view -> + input."""

    def __init__(self, dim, depth, heads, ws, mlp_ratio, img_size, resi, v2=False):
        super().__init__()
        self.residual_group = nn.Module()
        self.residual_group.blocks = nn.ModuleList(
            [SwinBlock(dim, heads, ws, 0 if i % 2 == 0 else ws // 2, mlp_ratio, img_size, v2) for i in range(depth)])
        self.conv = _resi_conv(dim, resi)
        if v2:                                   # Swin2SR's patch embed is a 1x1 projection conv
            self.patch_embed = nn.Module()
            self.patch_embed.proj = Conv2d(dim, dim, 1)
        self.v2 = v2

    def forward(self, x, hw):
        y = x
        for blk in self.residual_group.blocks:
            y = blk(y, hw)
        y = self.conv(_to_img(y, hw))
        if self.v2:
            y = self.patch_embed.proj(y)
        return _to_tokens(y) + x


class _Upsample(nn.Sequential):
    """conv -> pixel-shuffle stages (2^n: x2 stages, or one x3 stage); conv keys at even indices."""

    def __init__(self, scale: int, nf: int):
        mods = []
        if scale & (scale - 1) == 0:
            for _ in range(int(math.log2(scale))):
                mods += [Conv2d(nf, 4 * nf, 3, padding=1), nn.PixelShuffle(2)]
        elif scale == 3:
            mods += [Conv2d(nf, 9 * nf, 3, padding=1), nn.PixelShuffle(3)]
        else:
            raise ValueError(f"unsupported SwinIR scale {scale}")
        super().__init__(*mods)


class SwinIR(nn.Module):
    """SwinIR (``v2=False``) / Swin2SR (``v2=True``), configured from the state dict."""

    def __init__(self, state_dict, v2: bool = False, strict: bool = True):
        super().__init__()
        sd = dict(state_dict)
        self.model_arch = "Swin2SR" if v2 else "SwinIR"
        self.start_unshuffle = 1
        if "conv_first.1.weight" in sd:                   # PixelUnshuffle stem (SwinIR only)
            sd["conv_first.weight"] = sd.pop("conv_first.1.weight")
            sd["conv_first.bias"] = sd.pop("conv_first.1.bias")
            self.start_unshuffle = round(math.sqrt(sd["conv_first.weight"].shape[1] // 3))
        keys = set(sd)
        if "conv_before_upsample.0.weight" in keys:
            if v2 and "conv_aux.weight" in keys:
                up = "pixelshuffle_aux"
            elif "conv_up1.weight" in keys:
                up = "nearest+conv"
            else:
                up = "pixelshuffle"
        elif "upsample.0.weight" in keys:
            up = "pixelshuffledirect"
        else:
            up = ""
        self.upsampler = up
        nf = sd["conv_before_upsample.0.weight"].shape[0] if "conv_before_upsample.0.weight" in keys else 64
        self.num_feat = nf
        in_ch = sd["conv_first.weight"].shape[1]
        out_ch = sd["conv_last.weight"].shape[0] if "conv_last.weight" in keys else in_ch
        if up == "nearest+conv":
            upscale = 2 ** sum(1 for k in keys if re.match(r"^conv_up\d\.weight$", k))
        elif up in ("pixelshuffle", "pixelshuffle_aux"):
            upscale = 1.0
            for k in keys:
                if re.match(r"^upsample\.\d+\.weight$", k):
                    upscale *= math.sqrt(sd[k].shape[0] // nf)
            upscale = int(round(upscale))
        elif up == "pixelshuffledirect":
            upscale = int(math.sqrt(sd["upsample.0.bias"].shape[0] // out_ch))
        else:
            upscale = 1
        blocks = [tuple(map(int, m.groups())) for k in keys
                  for m in [re.match(r"^layers\.(\d+)\.residual_group\.blocks\.(\d+)\.norm1\.weight$", k)] if m]
        n_layers = 1 + max(b[0] for b in blocks)
        depth = 1 + max(b[1] for b in blocks)
        dim = sd["conv_first.weight"].shape[0]
        b0 = "layers.0.residual_group.blocks.0."
        if v2:
            heads = sd[b0 + "attn.logit_scale"].shape[0] if b0 + "attn.logit_scale" in keys else depth
            ws = int(math.sqrt(sd[b0 + "attn.relative_position_index"].shape[0]))
        else:
            heads = sd[b0 + "attn.relative_position_bias_table"].shape[-1]
            ws = int(math.sqrt(sd[b0 + "attn.relative_position_bias_table"].shape[0])) // 2 + 1
        if b0 + "attn.relative_position_index" in keys:
            ws = int(math.sqrt(sd[b0 + "attn.relative_position_index"].shape[0]))
        mlp_ratio = sd[b0 + "mlp.fc1.bias"].shape[0] / dim
        resi = "3conv" if "layers.0.conv.4.weight" in keys else "1conv"
        img_size = 64
        if "layers.0.residual_group.blocks.1.attn_mask" in keys:
            img_size = int(math.sqrt(sd["layers.0.residual_group.blocks.1.attn_mask"].shape[0]) * ws)
        self.window_size, self.embed_dim, self.depths = ws, dim, [depth] * n_layers
        self.num_heads, self.mlp_ratio, self.resi_connection = [heads] * n_layers, mlp_ratio, resi
        self.img_range = 255.0 if ws == 7 else 1.0
        self.in_nc, self.out_nc, self.upscale = in_ch, out_ch, upscale
        self.scale = upscale // self.start_unshuffle if upscale % self.start_unshuffle == 0 \
            else upscale / self.start_unshuffle
        mean = torch.tensor([0.4488, 0.4371, 0.4040]).view(1, 3, 1, 1) if in_ch == 3 else torch.zeros(1, 1, 1, 1)
        self.register_buffer("mean", mean, persistent=False)

        self.conv_first = Conv2d(in_ch, dim, 3, padding=1)
        self.patch_embed = nn.Module()
        self.patch_embed.norm = LayerNorm(dim)
        if v2:
            self.patch_embed.proj = Conv2d(dim, dim, 1)
        self.v2 = v2
        self.layers = nn.ModuleList([RSTB(dim, depth, heads, ws, mlp_ratio, img_size, resi, v2)
                                     for _ in range(n_layers)])
        self.norm = LayerNorm(dim)
        self.conv_after_body = _resi_conv(dim, resi)
        if up in ("pixelshuffle", "pixelshuffle_aux", "nearest+conv"):
            self.conv_before_upsample = nn.Sequential(Conv2d(dim, nf, 3, padding=1), nn.LeakyReLU(0.01))
            self.conv_last = Conv2d(nf, out_ch, 3, padding=1)
        if up in ("pixelshuffle", "pixelshuffle_aux"):
            self.upsample = _Upsample(upscale, nf)
        if up == "pixelshuffle_aux":
            self.conv_bicubic = Conv2d(in_ch, nf, 3, padding=1)
            self.conv_aux = Conv2d(nf, out_ch, 3, padding=1)
            self.conv_after_aux = nn.Sequential(Conv2d(3, nf, 3, padding=1), nn.LeakyReLU(0.01))
        elif up == "pixelshuffledirect":
            self.upsample = nn.Sequential(Conv2d(dim, upscale ** 2 * out_ch, 3, padding=1), nn.PixelShuffle(upscale))
        elif up == "nearest+conv":
            self.conv_ups = [f"conv_up{i + 1}" for i in range(int(math.log2(upscale)))]
            for name in self.conv_ups:
                setattr(self, name, Conv2d(nf, nf, 3, padding=1))
            self.conv_hr = Conv2d(nf, nf, 3, padding=1)
        elif up == "":
            self.conv_last = Conv2d(dim, out_ch, 3, padding=1)
        missing, _ = self.load_state_dict(sd, strict=False)
        if missing and strict:
            raise ValueError(f"{self.model_arch}: missing keys {missing[:4]}")
        self.eval()

    def forward_features(self, x):
        hw = x.shape[-2:]
        if self.v2:
            x = self.patch_embed.proj(x)
        t = self.patch_embed.norm(_to_tokens(x))
        for layer in self.layers:
            t = layer(t, hw)
        return _to_img(self.norm(t), hw)

    def forward(self, x):
        H, W = x.shape[-2:]
        m = self.window_size * self.start_unshuffle
        x = pad_to_multiple(x, m)
        mean = self.mean.to(x.dtype)
        x = (x - mean) * self.img_range
        if self.start_unshuffle > 1:
            x = F.pixel_unshuffle(x, self.start_unshuffle)
        up = self.upsampler
        Ho, Wo = H * self.upscale, W * self.upscale
        if up == "":
            f = self.conv_first(x)
            x = x + self.conv_last(self.conv_after_body(self.forward_features(f)) + f)
        else:
            if up == "pixelshuffle_aux":
                bic = self.conv_bicubic(F.interpolate(x, size=(Ho, Wo), mode="bicubic", align_corners=False))
            f = self.conv_first(x)
            x = self.conv_after_body(self.forward_features(f)) + f
            if up == "pixelshuffledirect":
                x = self.upsample(x)
            else:
                x = self.conv_before_upsample(x)
                if up == "pixelshuffle":
                    x = self.conv_last(self.upsample(x))
                elif up == "pixelshuffle_aux":
                    x = self.upsample(self.conv_after_aux(self.conv_aux(x)))[:, :, :Ho, :Wo] + bic[:, :, :Ho, :Wo]
                    x = self.conv_last(x)
                else:
                    for name in self.conv_ups:
                        x = F.leaky_relu(getattr(self, name)(F.interpolate(x, scale_factor=2, mode="nearest")), 0.2)
                    x = self.conv_last(F.leaky_relu(self.conv_hr(x), 0.2))
        x = x / self.img_range + mean
        return x[:, :, :Ho, :Wo]


# ----------------------------------------------------------------------------------------------
# HAT (hybrid attention transformer; reference HAT.py:847-1277): window attention + a channel-
# attention conv branch per block, and one overlapping cross-attention block per group.
# ----------------------------------------------------------------------------------------------


class _CAB(nn.Module):
    def __init__(self, dim: int, mid: int, squeezed: int):
        super().__init__()
        att = nn.Sequential(nn.AdaptiveAvgPool2d(1), Conv2d(dim, squeezed, 1), nn.ReLU(), Conv2d(squeezed, dim, 1),
                            nn.Sigmoid())
        ca = nn.Module()
        ca.attention = att
        self.cab = nn.Sequential(Conv2d(dim, mid, 3, padding=1), nn.GELU(), Conv2d(mid, dim, 3, padding=1), ca)

    def forward(self, x):
        y = self.cab[2](self.cab[1](self.cab[0](x)))
        return y * self.cab[3].attention(y)


class HAB(nn.Module):
    def __init__(self, dim, heads, ws, shift, mlp_ratio, img_size, cab_mid, cab_sq, conv_scale=0.01):
        super().__init__()
        if img_size <= ws:
            shift, ws = 0, img_size
        self.ws, self.shift, self.conv_scale = ws, shift, conv_scale
        self.norm1 = LayerNorm(dim)
        self.attn = WindowAttention(dim, ws, heads)
        self.conv_block = _CAB(dim, cab_mid, cab_sq)
        self.norm2 = LayerNorm(dim)
        self.mlp = _Mlp(dim, int(dim * mlp_ratio))

    def forward(self, x, hw, mask):
        H, W = hw
        B, L, C = x.shape
        y = self.norm1(x).view(B, H, W, C)
        conv = self.conv_block(y.permute(0, 3, 1, 2)).permute(0, 2, 3, 1).reshape(B, L, C)
        ws, sh = self.ws, self.shift
        if sh:
            y = torch.roll(y, (-sh, -sh), (1, 2))
        a = _reverse(self.attn(_partition(y, ws), mask if sh else None), ws, B, H, W)
        if sh:
            a = torch.roll(a, (sh, sh), (1, 2))
        x = x + a.reshape(B, L, C) + conv * self.conv_scale
        return x + self.mlp(self.norm2(x))


def _rel_index_oca(ws: int, ows: int) -> torch.Tensor:
    def grid(n):
        return torch.stack(torch.meshgrid(torch.arange(n), torch.arange(n), indexing="ij")).flatten(1)
    r = (grid(ows)[:, None, :] - grid(ws)[:, :, None]).permute(1, 2, 0) + (ws - ows + 1)
    return r[..., 0] * (ws + ows - 1) + r[..., 1]        # [ws*ws, ows*ows]


class OCAB(nn.Module):
    """Overlapping cross-attention: queries from ``ws x ws`` windows attend to keys/values from the
    enlarged ``ows x ows`` window around them (zero padded at the border)."""

    def __init__(self, dim, heads, ws, overlap_ratio, mlp_ratio):
        super().__init__()
        self.dim, self.heads, self.ws = dim, heads, ws
        self.ows = int(ws * overlap_ratio) + ws
        self.scale = (dim // heads) ** -0.5
        self.norm1 = LayerNorm(dim)
        self.qkv = Linear(dim, dim * 3)
        self.relative_position_bias_table = nn.Parameter(torch.zeros((ws + self.ows - 1) ** 2, heads),
                                                         requires_grad=False)
        self.proj = Linear(dim, dim)
        self.norm2 = LayerNorm(dim)
        self.mlp = _Mlp(dim, int(dim * mlp_ratio))
        self.register_buffer("rel_index", _rel_index_oca(ws, self.ows), persistent=False)

    def forward(self, x, hw):
        H, W = hw
        B, L, C = x.shape
        ws, ows, h = self.ws, self.ows, self.heads
        qkv = self.qkv(self.norm1(x)).view(B, H, W, 3, C)
        q = _partition(qkv[..., 0, :], ws)                                   # [B*nW, ws*ws, C]
        kv = qkv[..., 1:, :].reshape(B, H, W, 2 * C).permute(0, 3, 1, 2)     # [B, 2C, H, W]
        kv = F.unfold(kv, ows, stride=ws, padding=(ows - ws) // 2)            # [B, 2C*ows*ows, nW]
        nW = kv.shape[-1]
        kv = kv.view(B, 2, C, ows * ows, nW).permute(1, 0, 4, 3, 2).reshape(2, B * nW, ows * ows, C)
        d = C // h
        qh = q.view(-1, ws * ws, h, d).transpose(1, 2)
        kh = kv[0].view(-1, ows * ows, h, d).transpose(1, 2)
        vh = kv[1].view(-1, ows * ows, h, d).transpose(1, 2)
        bias = self.relative_position_bias_table.float()[self.rel_index.reshape(-1)]
        bias = bias.view(ws * ws, ows * ows, h).permute(2, 0, 1)
        o = ops.attention_bias(qh, kh, vh, bias, scale=self.scale).transpose(1, 2).reshape(-1, ws * ws, C)
        x = self.proj(_reverse(o, ws, B, H, W).reshape(B, L, C)) + x
        return x + self.mlp(self.norm2(x))


class RHAG(nn.Module):
    def __init__(self, dim, depth, heads, ws, mlp_ratio, img_size, cab_mid, cab_sq, overlap_ratio, resi):
        super().__init__()
        self.residual_group = nn.Module()
        self.residual_group.blocks = nn.ModuleList(
            [HAB(dim, heads, ws, 0 if i % 2 == 0 else ws // 2, mlp_ratio, img_size, cab_mid, cab_sq)
             for i in range(depth)])
        self.residual_group.overlap_attn = OCAB(dim, heads, ws, overlap_ratio, mlp_ratio)
        self.conv = Conv2d(dim, dim, 3, padding=1) if resi == "1conv" else nn.Identity()

    def forward(self, x, hw, mask):
        y = x
        for blk in self.residual_group.blocks:
            y = blk(y, hw, mask)
        y = self.residual_group.overlap_attn(y, hw)
        return _to_tokens(self.conv(_to_img(y, hw))) + x


class HAT(nn.Module):
    """HAT (classical-SR ``pixelshuffle`` head, the one the reference runs), configured from the
    state dict; CAB compress/squeeze ratios are read from the weight shapes (HAT-S/HAT/HAT-L)."""

    def __init__(self, state_dict, strict: bool = True):
        super().__init__()
        sd = state_dict
        keys = set(sd)
        self.model_arch = "HAT"
        if "conv_before_upsample.0.weight" not in keys or "conv_up1.weight" in keys:
            raise ValueError("HAT: only the pixelshuffle reconstruction head is supported")
        self.upsampler = "pixelshuffle"
        nf = self.num_feat = sd["conv_last.weight"].shape[1]
        in_ch = sd["conv_first.weight"].shape[1]
        out_ch = sd["conv_last.weight"].shape[0]
        dim = sd["conv_first.weight"].shape[0]
        upscale = 1.0
        for k in keys:
            if re.match(r"^upsample\.\d+\.weight$", k):
                upscale *= math.sqrt(sd[k].shape[0] // nf)
        upscale = int(round(upscale))
        blocks = [tuple(map(int, m.groups())) for k in keys
                  for m in [re.match(r"^layers\.(\d+)\.residual_group\.blocks\.(\d+)\.conv_block\.cab\.0\.weight$", k)]
                  if m]
        n_layers = 1 + max(b[0] for b in blocks)
        depth = 1 + max(b[1] for b in blocks)
        b0 = "layers.0.residual_group.blocks.0."
        heads = sd[b0 + "attn.relative_position_bias_table"].shape[-1]
        if "relative_position_index_SA" in keys:
            ws = int(math.sqrt(sd["relative_position_index_SA"].shape[0]))
        else:
            ws = int(math.sqrt(sd[b0 + "attn.relative_position_bias_table"].shape[0])) // 2 + 1
        mlp_ratio = sd[b0 + "mlp.fc1.bias"].shape[0] / dim
        resi = "1conv" if "layers.0.conv.weight" in keys else "identity"
        cab_mid = sd[b0 + "conv_block.cab.0.weight"].shape[0]
        cab_sq = sd[b0 + "conv_block.cab.3.attention.1.weight"].shape[0]
        oca_table = sd["layers.0.residual_group.overlap_attn.relative_position_bias_table"].shape[0]
        ows = int(round(math.sqrt(oca_table))) - ws + 1
        overlap_ratio = (ows - ws) / ws
        img_size = 64
        if "layers.0.residual_group.blocks.1.attn_mask" in keys:
            img_size = int(math.sqrt(sd["layers.0.residual_group.blocks.1.attn_mask"].shape[0]) * ws)
        self.window_size, self.embed_dim, self.depths = ws, dim, [depth] * n_layers
        self.num_heads, self.mlp_ratio, self.resi_connection = [heads] * n_layers, mlp_ratio, resi
        self.in_nc, self.out_nc, self.upscale, self.scale = in_ch, out_ch, upscale, upscale
        self.img_range = 1.0
        mean = torch.tensor([0.4488, 0.4371, 0.4040]).view(1, 3, 1, 1) if in_ch == 3 else torch.zeros(1, 1, 1, 1)
        self.register_buffer("mean", mean, persistent=False)
        self.conv_first = Conv2d(in_ch, dim, 3, padding=1)
        self.patch_embed = nn.Module()
        self.patch_embed.norm = LayerNorm(dim)
        self.layers = nn.ModuleList([RHAG(dim, depth, heads, ws, mlp_ratio, img_size, cab_mid, cab_sq,
                                          overlap_ratio, resi) for _ in range(n_layers)])
        self.norm = LayerNorm(dim)
        self.conv_after_body = Conv2d(dim, dim, 3, padding=1) if resi == "1conv" else nn.Identity()
        self.conv_before_upsample = nn.Sequential(Conv2d(dim, nf, 3, padding=1), nn.LeakyReLU(0.01))
        self.upsample = _Upsample(upscale, nf)
        self.conv_last = Conv2d(nf, out_ch, 3, padding=1)
        missing, _ = self.load_state_dict(sd, strict=False)
        if missing and strict:
            raise ValueError(f"HAT: missing keys {missing[:4]}")
        self.eval()

    def forward(self, x):
        H, W = x.shape[-2:]
        mean = self.mean.to(x.dtype)
        x = (x - mean) * self.img_range
        ws = self.window_size
        x = pad_to_multiple(x, ws)
        f = self.conv_first(x)
        hw = f.shape[-2:]
        mask = shift_mask(hw[0], hw[1], ws, ws // 2, x.device)
        t = self.patch_embed.norm(_to_tokens(f))
        for layer in self.layers:
            t = layer(t, hw, mask)
        x = self.conv_after_body(_to_img(self.norm(t), hw)) + f
        x = self.conv_last(self.upsample(self.conv_before_upsample(x)))
        x = x / self.img_range + mean
        return x[:, :, :H * self.upscale, :W * self.upscale]


# ----------------------------------------------------------------------------------------------
# SCUNet (swin-conv UNet blind denoiser; reference SCUNet.py:274-446): 4-level UNet whose blocks
# split channels between a residual conv path and a (shifted-)window transformer path.
# ----------------------------------------------------------------------------------------------


def _scunet_mask(nh: int, nw: int, p: int, device) -> torch.Tensor:
    """[nh*nw, p*p, p*p] bool, True = blocked: after the cyclic shift only the last window row /
    column mixes pixels from opposite image borders."""
    s = p - p // 2
    m = torch.zeros(nh, nw, p, p, p, p, dtype=torch.bool)
    m[-1, :, :s, :, s:, :] = True
    m[-1, :, s:, :, :s, :] = True
    m[:, -1, :, :s, :, s:] = True
    m[:, -1, :, s:, :, :s] = True
    return m.reshape(nh * nw, p * p, p * p).to(device)


class _WMSA(nn.Module):
    def __init__(self, dim: int, head_dim: int, ws: int, shifted: bool):
        super().__init__()
        self.heads, self.hd, self.ws, self.shifted = dim // head_dim, head_dim, ws, shifted
        self.embedding_layer = Linear(dim, 3 * dim)
        self.relative_position_params = nn.Parameter(torch.zeros(self.heads, 2 * ws - 1, 2 * ws - 1),
                                                     requires_grad=False)
        self.linear = Linear(dim, dim)
        c = torch.stack(torch.meshgrid(torch.arange(ws), torch.arange(ws), indexing="ij"), -1).reshape(-1, 2)
        rel = c[:, None, :] - c[None, :, :] + ws - 1
        self.register_buffer("rel", rel, persistent=False)

    def forward(self, x):                       # x [B, H, W, C]
        B, H, W, C = x.shape
        p, h = self.ws, self.heads
        if self.shifted:
            x = torch.roll(x, (-(p // 2), -(p // 2)), (1, 2))
        win = _partition(x, p)                                          # [B*nW, N, C]
        q, k, v = self.embedding_layer(win).view(win.shape[0], p * p, 3, h, self.hd).permute(2, 0, 3, 1, 4).unbind(0)
        bias = self.relative_position_params.float()[:, self.rel[..., 0], self.rel[..., 1]]
        m = _scunet_mask(H // p, W // p, p, x.device) if self.shifted else None     # bool, True = blocked
        o = ops.attention_bias(q, k, v, bias, m, scale=self.hd ** -0.5).transpose(1, 2).reshape(-1, p * p, C)
        y = _reverse(self.linear(o), p, B, H, W)
        if self.shifted:
            y = torch.roll(y, (p // 2, p // 2), (1, 2))
        return y


class _SCUTransBlock(nn.Module):
    def __init__(self, dim, head_dim, ws, shifted):
        super().__init__()
        self.ln1 = LayerNorm(dim)
        self.msa = _WMSA(dim, head_dim, ws, shifted)
        self.ln2 = LayerNorm(dim)
        self.mlp = nn.Sequential(Linear(dim, 4 * dim), nn.GELU(), Linear(4 * dim, dim))

    def forward(self, x):
        x = x + self.msa(self.ln1(x))
        return x + self.mlp(self.ln2(x))


class ConvTransBlock(nn.Module):
    def __init__(self, conv_dim, trans_dim, head_dim, ws, shifted):
        super().__init__()
        self.conv_dim = conv_dim
        c = conv_dim + trans_dim
        self.trans_block = _SCUTransBlock(trans_dim, head_dim, ws, shifted)
        self.conv1_1 = Conv2d(c, c, 1)
        self.conv1_2 = Conv2d(c, c, 1)
        self.conv_block = nn.Sequential(Conv2d(conv_dim, conv_dim, 3, padding=1, bias=False), nn.ReLU(),
                                        Conv2d(conv_dim, conv_dim, 3, padding=1, bias=False))

    def forward(self, x):
        y = self.conv1_1(x)
        cx, tx = y[:, :self.conv_dim], y[:, self.conv_dim:]
        cx = self.conv_block(cx) + cx
        tx = self.trans_block(tx.permute(0, 2, 3, 1)).permute(0, 3, 1, 2)
        return x + self.conv1_2(torch.cat([cx, tx], 1))


class SCUNet(nn.Module):
    """SCUNet (dim 64, 4 blocks per stage, 32-wide heads, 8x8 windows — the released config)."""

    def __init__(self, state_dict, strict: bool = True):
        super().__init__()
        self.model_arch = "SCUNet"
        self.scale = 1
        dim = self.dim = state_dict["m_head.0.weight"].shape[0] if "m_head.0.weight" in state_dict else 64
        in_nc = self.in_nc = self.out_nc = state_dict["m_head.0.weight"].shape[1] if "m_head.0.weight" in state_dict else 3
        ws, hd = 8, 32
        cfg = [4] * 7
        res = 256                               # training resolution: stage-wise shift eligibility

        def stage(c, n, r):
            return [ConvTransBlock(c, c, hd, ws, bool(i % 2) and r > ws) for i in range(n)]

        self.m_head = nn.Sequential(Conv2d(in_nc, dim, 3, padding=1, bias=False))
        self.m_down1 = nn.Sequential(*stage(dim // 2, cfg[0], res), Conv2d(dim, 2 * dim, 2, stride=2, bias=False))
        self.m_down2 = nn.Sequential(*stage(dim, cfg[1], res // 2), Conv2d(2 * dim, 4 * dim, 2, stride=2, bias=False))
        self.m_down3 = nn.Sequential(*stage(2 * dim, cfg[2], res // 4),
                                     Conv2d(4 * dim, 8 * dim, 2, stride=2, bias=False))
        self.m_body = nn.Sequential(*stage(4 * dim, cfg[3], res // 8))
        self.m_up3 = nn.Sequential(nn.ConvTranspose2d(8 * dim, 4 * dim, 2, 2, bias=False), *stage(2 * dim, cfg[4], res // 4))
        self.m_up2 = nn.Sequential(nn.ConvTranspose2d(4 * dim, 2 * dim, 2, 2, bias=False), *stage(dim, cfg[5], res // 2))
        self.m_up1 = nn.Sequential(nn.ConvTranspose2d(2 * dim, dim, 2, 2, bias=False), *stage(dim // 2, cfg[6], res))
        self.m_tail = nn.Sequential(Conv2d(dim, in_nc, 3, padding=1, bias=False))
        for m in self.modules():
            if isinstance(m, nn.ConvTranspose2d):
                m.weight.requires_grad_(False)
        missing, _ = self.load_state_dict(state_dict, strict=False)
        if missing and strict:
            raise ValueError(f"SCUNet: missing keys {missing[:4]}")
        self.eval()

    def forward(self, x0):
        h, w = x0.shape[-2:]
        x0 = pad_to_multiple(x0, 64)
        x1 = self.m_head(x0)
        x2 = self.m_down1(x1)
        x3 = self.m_down2(x2)
        x4 = self.m_down3(x3)
        x = self.m_body(x4)
        x = self.m_up3(x + x4)
        x = self.m_up2(x + x3)
        x = self.m_up1(x + x2)
        return self.m_tail(x + x1)[:, :, :h, :w]
