"""KL-VAE (SD1/SD2/SDXL first stage) — Encoder / Decoder / AutoencoderKL.

Behavioural parity with ``comfy/ldm/modules/diffusionmodules/model.py:1-651`` (ResnetBlock,
asymmetric-pad Downsample, AttnBlock single-head mid attention, Encoder :451, Decoder :542) and
``comfy/ldm/models/autoencoder.py`` (quant_conv / post_quant_conv, diagonal Gaussian mode).
State-dict keys identical to ldm (``encoder.*``, ``decoder.*``, ``quant_conv``, ``post_quant_conv``).

Device path: NHWC bf16, GroupNorm+SiLU fused kernel, skip adds fused into the conv epilogue,
mid-attention (16 k tokens x d=512 at 1024²) through ``ops.attention`` with the 1x1 q/k/v convs
evaluated as one GEMM over the NHWC rows.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import ops
from .layers import Conv2d, Conv3d, GroupNorm, DerivedMixin


def _norm(c, dtype=None, device=None):
    return GroupNorm(32, c, eps=1e-6, dtype=dtype, device=device)


class ResnetBlock(nn.Module):
    def __init__(self, in_channels, out_channels=None, dtype=None, device=None, temb_channels=0):
        super().__init__()
        out_channels = out_channels or in_channels
        self.in_channels = in_channels
        self.out_channels = out_channels
        kw = dict(dtype=dtype, device=device)
        self.norm1 = _norm(in_channels, **kw)
        self.conv1 = Conv2d(in_channels, out_channels, 3, padding=1, **kw)
        self.norm2 = _norm(out_channels, **kw)
        self.conv2 = Conv2d(out_channels, out_channels, 3, padding=1, **kw)
        if in_channels != out_channels:
            self.nin_shortcut = Conv2d(in_channels, out_channels, 1, **kw)
        else:
            self.nin_shortcut = None

    def forward(self, x, temb=None):
        h = self.conv1(self.norm1(x, silu=True))
        h = self.norm2(h, silu=True)
        skip = x if self.nin_shortcut is None else self.nin_shortcut(x)
        return self.conv2(h, residual=skip)


class AttnBlock(nn.Module, DerivedMixin):
    def __init__(self, in_channels, dtype=None, device=None):
        super().__init__()
        kw = dict(dtype=dtype, device=device)
        self.in_channels = in_channels
        self.norm = _norm(in_channels, **kw)
        self.q = Conv2d(in_channels, in_channels, 1, **kw)
        self.k = Conv2d(in_channels, in_channels, 1, **kw)
        self.v = Conv2d(in_channels, in_channels, 1, **kw)
        self.proj_out = Conv2d(in_channels, in_channels, 1, **kw)

    def forward(self, x):
        b, c, h, w = x.shape
        hn = self.norm(x)
        tok = hn.permute(0, 2, 3, 1).reshape(b, h * w, c)
        if x.is_cuda and x.dtype == self.q.weight.dtype:
            wqkv = self._derived_get("w_qkv", lambda: torch.cat(
                [self.q.weight, self.k.weight, self.v.weight], 0).reshape(3 * c, c).contiguous())
            bqkv = self._derived_get("b_qkv", lambda: torch.cat([self.q.bias, self.k.bias, self.v.bias], 0))
            qkv = ops.linear(tok, wqkv, bqkv)
            q, k, v = qkv[..., :c], qkv[..., c:2 * c], qkv[..., 2 * c:]
            o = ops.attention(q, k, v, 1)
            res = x.permute(0, 2, 3, 1).reshape(b, h * w, c)
            wo = self._derived_get("w_o", lambda: self.proj_out.weight.reshape(c, c).contiguous())
            out = ops.linear(o, wo, self.proj_out.bias, residual=res if res.is_contiguous() else None)
            out = out.reshape(b, h, w, c).permute(0, 3, 1, 2)
            return out if res.is_contiguous() else out + x
        q = self.q(hn).permute(0, 2, 3, 1).reshape(b, h * w, c)
        k = self.k(hn).permute(0, 2, 3, 1).reshape(b, h * w, c)
        v = self.v(hn).permute(0, 2, 3, 1).reshape(b, h * w, c)
        o = ops.attention(q, k, v, 1)
        o = o.reshape(b, h, w, c).permute(0, 3, 1, 2)
        return self.proj_out(o, residual=x)


class Downsample(nn.Module):
    def __init__(self, c, dtype=None, device=None):
        super().__init__()
        self.conv = Conv2d(c, c, 3, stride=2, padding=0, dtype=dtype, device=device)

    def forward(self, x):
        x = torch.nn.functional.pad(x, (0, 1, 0, 1), mode="constant", value=0)
        return self.conv(x)


class Upsample(nn.Module):
    def __init__(self, c, dtype=None, device=None):
        super().__init__()
        self.conv = Conv2d(c, c, 3, padding=1, dtype=dtype, device=device)

    def forward(self, x):
        return self.conv(x, upsample2x=True)


class _Level(nn.Module):
    pass


class Encoder(nn.Module):
    def __init__(self, ch=128, ch_mult=(1, 2, 4, 4), num_res_blocks=2, in_channels=3, z_channels=4,
                 double_z=True, dtype=None, device=None, **unused):
        super().__init__()
        kw = dict(dtype=dtype, device=device)
        self.num_resolutions = len(ch_mult)
        self.num_res_blocks = num_res_blocks
        self.conv_in = Conv2d(in_channels, ch, 3, padding=1, **kw)
        in_ch_mult = (1,) + tuple(ch_mult)
        self.down = nn.ModuleList()
        block_in = ch
        for i in range(self.num_resolutions):
            lvl = _Level()
            lvl.block = nn.ModuleList()
            block_in = ch * in_ch_mult[i]
            block_out = ch * ch_mult[i]
            for _ in range(num_res_blocks):
                lvl.block.append(ResnetBlock(block_in, block_out, **kw))
                block_in = block_out
            lvl.attn = nn.ModuleList()
            if i != self.num_resolutions - 1:
                lvl.downsample = Downsample(block_in, **kw)
            self.down.append(lvl)
        self.mid = _Level()
        self.mid.block_1 = ResnetBlock(block_in, block_in, **kw)
        self.mid.attn_1 = AttnBlock(block_in, **kw)
        self.mid.block_2 = ResnetBlock(block_in, block_in, **kw)
        self.norm_out = _norm(block_in, **kw)
        self.conv_out = Conv2d(block_in, 2 * z_channels if double_z else z_channels, 3, padding=1, **kw)

    def forward(self, x):
        h = self.conv_in(x)
        for i in range(self.num_resolutions):
            for blk in self.down[i].block:
                h = blk(h)
            if i != self.num_resolutions - 1:
                h = self.down[i].downsample(h)
        h = self.mid.block_1(h)
        h = self.mid.attn_1(h)
        h = self.mid.block_2(h)
        return self.conv_out(self.norm_out(h, silu=True))


class VideoResnetBlock(ResnetBlock):
    """Temporal-VAE ResnetBlock (temporal_ae.py:25-89): spatial ResnetBlock, then a ResBlock(dims=3)
    with [3,1,1] time convs over all frames, blended as alpha * temporal + (1 - alpha) * spatial."""

    def __init__(self, in_channels, out_channels=None, dtype=None, device=None, video_kernel_size=(3, 1, 1),
                 alpha=0.0, merge_strategy="learned"):
        super().__init__(in_channels, out_channels, dtype=dtype, device=device)
        from .unet import TimeStackResBlock
        self.time_stack = TimeStackResBlock(self.out_channels, 0, video_kernel_size, skip_t_emb=True, dtype=dtype,
                                            device=device)
        self.merge_strategy = merge_strategy
        if merge_strategy == "fixed":
            self.register_buffer("mix_factor", torch.tensor([float(alpha)]))
        else:
            self.mix_factor = nn.Parameter(torch.tensor([float(alpha)]), requires_grad=False)

    def forward(self, x, temb=None, frames=None):
        x = super().forward(x)
        frames = frames or x.shape[0]
        xt = self.time_stack(x, None, frames)
        m = self.mix_factor.to(device=x.device, dtype=torch.float32)
        a = (m if self.merge_strategy == "fixed" else torch.sigmoid(m)).to(x.dtype)
        return a * xt + (1.0 - a) * x


class AE3DConv(Conv2d):
    """Decoder conv_out of the temporal VAE: 2-D conv, then a [3,1,1] time-mixing Conv3d."""

    def __init__(self, in_channels, out_channels, kernel_size=3, padding=1, video_kernel_size=(3, 1, 1),
                 dtype=None, device=None):
        super().__init__(in_channels, out_channels, kernel_size, padding=padding, dtype=dtype, device=device)
        vks = list(video_kernel_size) if isinstance(video_kernel_size, (list, tuple)) else [video_kernel_size] * 3
        self.time_mix_conv = Conv3d(out_channels, out_channels, vks, [k // 2 for k in vks], dtype=dtype,
                                    device=device)

    def forward(self, x, frames=None):
        x = super().forward(x)
        return self.time_mix_conv(x, frames or x.shape[0])


class Decoder(nn.Module):
    def __init__(self, ch=128, out_ch=3, ch_mult=(1, 2, 4, 4), num_res_blocks=2, z_channels=4,
                 dtype=None, device=None, video_kernel_size=None, alpha=0.0, merge_strategy="learned",
                 **unused):
        super().__init__()
        kw = dict(dtype=dtype, device=device)
        self.video = video_kernel_size is not None   # temporal_ae.VideoDecoder, time_mode "conv-only"
        if self.video:
            vk = dict(video_kernel_size=video_kernel_size, alpha=alpha, merge_strategy=merge_strategy)
            res = lambda a, b: VideoResnetBlock(a, b, **kw, **vk)  # noqa: E731
        else:
            res = lambda a, b: ResnetBlock(a, b, **kw)  # noqa: E731
        self.num_resolutions = len(ch_mult)
        self.num_res_blocks = num_res_blocks
        block_in = ch * ch_mult[-1]
        self.conv_in = Conv2d(z_channels, block_in, 3, padding=1, **kw)
        self.mid = _Level()
        self.mid.block_1 = res(block_in, block_in)
        self.mid.attn_1 = AttnBlock(block_in, **kw)
        self.mid.block_2 = res(block_in, block_in)
        ups = []
        for i in reversed(range(self.num_resolutions)):
            lvl = _Level()
            lvl.block = nn.ModuleList()
            lvl.attn = nn.ModuleList()
            block_out = ch * ch_mult[i]
            for _ in range(num_res_blocks + 1):
                lvl.block.append(res(block_in, block_out))
                block_in = block_out
            if i != 0:
                lvl.upsample = Upsample(block_in, **kw)
            ups.insert(0, lvl)
        self.up = nn.ModuleList(ups)
        self.norm_out = _norm(block_in, **kw)
        if self.video:
            self.conv_out = AE3DConv(block_in, out_ch, 3, padding=1, video_kernel_size=video_kernel_size, **kw)
        else:
            self.conv_out = Conv2d(block_in, out_ch, 3, padding=1, **kw)

    def forward(self, z, frames=None):
        vk = {"frames": frames or z.shape[0]} if self.video else {}
        h = self.conv_in(z)
        h = self.mid.block_1(h, **vk)
        h = self.mid.attn_1(h)
        h = self.mid.block_2(h, **vk)
        for i in reversed(range(self.num_resolutions)):
            for blk in self.up[i].block:
                h = blk(h, **vk)
            if i != 0:
                h = self.up[i].upsample(h)
        return self.conv_out(self.norm_out(h, silu=True), **vk)


class AutoencoderKL(nn.Module):
    def __init__(self, embed_dim=4, ddconfig=None, dtype=None, device=None):
        super().__init__()
        ddconfig = dict(ddconfig or {})
        ddconfig.setdefault("z_channels", embed_dim)
        kw = dict(dtype=dtype, device=device)
        self.encoder = Encoder(**{k: v for k, v in ddconfig.items()
                                  if k not in ("video_kernel_size", "alpha", "merge_strategy")}, **kw)
        self.decoder = Decoder(**ddconfig, **kw)
        zc = ddconfig["z_channels"]
        self.quant_conv = Conv2d(2 * zc, 2 * embed_dim, 1, **kw)
        self.post_quant_conv = Conv2d(embed_dim, zc, 1, **kw)
        self.embed_dim = embed_dim

    def encode(self, x, sample=False, generator=None):
        moments = self.quant_conv(self.encoder(x))
        mean, logvar = moments.float().chunk(2, dim=1)
        if sample:
            logvar = logvar.clamp(-30.0, 20.0)
            return mean + torch.exp(0.5 * logvar) * torch.randn(mean.shape, generator=generator,
                                                                   device=mean.device)
        return mean   # DiagonalGaussianRegularizer in eval mode returns the mode

    def decode(self, z):
        return self.decoder(self.post_quant_conv(z))
