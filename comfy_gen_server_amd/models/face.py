"""Face restoration networks for ``UpscaleModelLoader``: GFPGAN v1 (clean), RestoreFormer and
CodeFormer (parity: ``comfy_extras/chainner_models/architecture/face/{gfpganv1_clean_arch,
stylegan2_clean_arch,restoreformer_arch,codeformer}.py``).

GFPGAN's StyleGAN2 decoder uses *activation-side* modulation: instead of materialising one
modulated weight per sample and running a grouped conv (the reference), the input is scaled by
the per-channel style, convolved with the shared weight (one dense conv for the whole batch —
the device's MFMA implicit-GEMM kernel), and the output scaled by the per-(sample, out-channel)
demodulation factor ``rsqrt(style^2 @ sum_k W^2 + eps)``. This is the same linear map.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from .layers import Conv2d, DerivedMixin, Linear


def _lrelu(x):
    return F.leaky_relu(x, 0.2)


class ModulatedConv2d(nn.Module, DerivedMixin):
    """Keys ``weight`` [1, Cout, Cin, k, k] and ``modulation`` (Linear style -> Cin)."""

    def __init__(self, cin, cout, k, style_dim, demodulate=True, sample_mode=None, eps=1e-8):
        super().__init__()
        self.cin, self.cout, self.k = cin, cout, k
        self.demodulate, self.sample_mode, self.eps = demodulate, sample_mode, eps
        self.modulation = Linear(style_dim, cin)
        self.weight = nn.Parameter(torch.randn(1, cout, cin, k, k) / math.sqrt(cin * k * k), requires_grad=False)

    def forward(self, x, style):
        s = self.modulation(style)                                     # [b, cin]
        w = self.weight[0]
        if w.dtype != x.dtype or w.device != x.device:
            w = w.to(device=x.device, dtype=x.dtype)
        if self.sample_mode == "upsample":
            x = F.interpolate(x, scale_factor=2, mode="bilinear", align_corners=False)
        elif self.sample_mode == "downsample":
            x = F.interpolate(x, scale_factor=0.5, mode="bilinear", align_corners=False)
        xs = x * s.to(x.dtype)[:, :, None, None]
        wn = None
        if x.is_cuda and self.weight.device == x.device and self.weight.dtype == x.dtype:
            wn = self._derived_get("w_nhwc", lambda: self.weight[0].permute(0, 2, 3, 1).contiguous())
        out = ops.conv2d(xs, w, None, 1, self.k // 2, weight_nhwc=wn)
        if self.demodulate:
            wsq = self._derived_get(f"wsq_{x.device}", lambda: self.weight[0].float().pow(2).sum((2, 3)).to(x.device))
            d = torch.rsqrt(s.float().pow(2) @ wsq.t() + self.eps)       # [b, cout]
            out = out * d.to(out.dtype)[:, :, None, None]
        return out


class StyleConv(nn.Module):
    def __init__(self, cin, cout, k, style_dim, sample_mode=None):
        super().__init__()
        self.modulated_conv = ModulatedConv2d(cin, cout, k, style_dim, True, sample_mode)
        self.weight = nn.Parameter(torch.zeros(1), requires_grad=False)           # noise strength
        self.bias = nn.Parameter(torch.zeros(1, cout, 1, 1), requires_grad=False)

    def forward(self, x, style, noise=None):
        out = self.modulated_conv(x, style) * 2 ** 0.5
        if noise is None:
            noise = out.new_empty(out.shape[0], 1, *out.shape[2:]).normal_()
        out = out + self.weight.to(out.dtype) * noise.to(out.dtype) + self.bias.to(out.dtype)
        return _lrelu(out)


class ToRGB(nn.Module):
    def __init__(self, cin, style_dim, upsample=True):
        super().__init__()
        self.upsample = upsample
        self.modulated_conv = ModulatedConv2d(cin, 3, 1, style_dim, demodulate=False)
        self.bias = nn.Parameter(torch.zeros(1, 3, 1, 1), requires_grad=False)

    def forward(self, x, style, skip=None):
        out = self.modulated_conv(x, style) + self.bias.to(x.dtype)
        if skip is not None:
            if self.upsample:
                skip = F.interpolate(skip, scale_factor=2, mode="bilinear", align_corners=False)
            out = out + skip
        return out


def _stylegan_channels(mult=2, narrow=1.0):
    base = {4: 512, 8: 512, 16: 512, 32: 512, 64: 256 * mult, 128: 128 * mult, 256: 64 * mult, 512: 32 * mult,
            1024: 16 * mult}
    return {k: int(v * narrow) for k, v in base.items()}


class StyleGAN2DecoderSFT(nn.Module):
    """StyleGAN2 generator (clean) with spatial feature transforms after each upsampling conv."""

    def __init__(self, out_size=512, style_dim=512, num_mlp=8, mult=2, narrow=1.0, sft_half=True):
        super().__init__()
        self.style_dim, self.sft_half = style_dim, sft_half
        mlp = [nn.Identity()]
        for _ in range(num_mlp):
            mlp += [Linear(style_dim, style_dim), nn.LeakyReLU(0.2)]
        self.style_mlp = nn.Sequential(*mlp)
        ch = _stylegan_channels(mult, narrow)
        self.constant_input = nn.Module()
        self.constant_input.weight = nn.Parameter(torch.randn(1, ch[4], 4, 4), requires_grad=False)
        self.style_conv1 = StyleConv(ch[4], ch[4], 3, style_dim)
        self.to_rgb1 = ToRGB(ch[4], style_dim, upsample=False)
        self.log_size = int(math.log2(out_size))
        self.num_layers = (self.log_size - 2) * 2 + 1
        self.num_latent = self.log_size * 2 - 2
        self.noises = nn.Module()
        for i in range(self.num_layers):
            r = 2 ** ((i + 5) // 2)
            self.noises.register_buffer(f"noise{i}", torch.randn(1, 1, r, r))
        self.style_convs = nn.ModuleList()
        self.to_rgbs = nn.ModuleList()
        cin = ch[4]
        for i in range(3, self.log_size + 1):
            cout = ch[2 ** i]
            self.style_convs.append(StyleConv(cin, cout, 3, style_dim, "upsample"))
            self.style_convs.append(StyleConv(cout, cout, 3, style_dim))
            self.to_rgbs.append(ToRGB(cout, style_dim))
            cin = cout

    def forward(self, latent, conditions, randomize_noise=True):
        if randomize_noise:
            noise = [None] * self.num_layers
        else:
            noise = [getattr(self.noises, f"noise{i}") for i in range(self.num_layers)]
        out = self.constant_input.weight.to(latent.dtype).repeat(latent.shape[0], 1, 1, 1)
        out = self.style_conv1(out, latent[:, 0], noise[0])
        skip = self.to_rgb1(out, latent[:, 1])
        i = 1
        for c1, c2, n1, n2, rgb in zip(self.style_convs[::2], self.style_convs[1::2], noise[1::2], noise[2::2],
                                       self.to_rgbs):
            out = c1(out, latent[:, i], n1)
            if i < len(conditions):
                scale, shift = conditions[i - 1], conditions[i]
                if self.sft_half:
                    h = out.shape[1] // 2
                    out = torch.cat([out[:, :h], out[:, h:] * scale + shift], 1)
                else:
                    out = out * scale + shift
            out = c2(out, latent[:, i + 1], n2)
            skip = rgb(out, latent[:, i + 2], skip)
            i += 2
        return skip


class _BilinearResBlock(nn.Module):
    def __init__(self, cin, cout, mode):
        super().__init__()
        self.conv1 = Conv2d(cin, cin, 3, padding=1)
        self.conv2 = Conv2d(cin, cout, 3, padding=1)
        self.skip = Conv2d(cin, cout, 1, bias=False)
        self.scale = 0.5 if mode == "down" else 2

    def forward(self, x):
        out = F.interpolate(_lrelu(self.conv1(x)), scale_factor=self.scale, mode="bilinear", align_corners=False)
        out = _lrelu(self.conv2(out))
        return out + self.skip(F.interpolate(x, scale_factor=self.scale, mode="bilinear", align_corners=False))


class GFPGANv1Clean(nn.Module):
    """GFPGAN v1.3/1.4: a U-Net encoder whose bottleneck predicts the W+ latents of a StyleGAN2
    decoder, and whose decoder features drive SFT scale/shift of half the decoder channels.
    ``forward`` returns ``(image, intermediate_rgbs)`` as the reference does."""

    def __init__(self, state_dict, strict: bool = True):
        super().__init__()
        self.model_arch = "GFPGAN"
        self.sub_type = "Face SR"
        self.scale, self.in_nc, self.out_nc = 8, 3, 3
        out_size, style_dim, mult = 512, 512, 2
        self.style_dim = style_dim
        ch = {k: int(v * 0.5) for k, v in _stylegan_channels(mult).items()}      # U-Net at half width
        self.log_size = int(math.log2(out_size))
        self.conv_body_first = Conv2d(3, ch[out_size], 1)
        cin = ch[out_size]
        self.conv_body_down = nn.ModuleList()
        for i in range(self.log_size, 2, -1):
            self.conv_body_down.append(_BilinearResBlock(cin, ch[2 ** (i - 1)], "down"))
            cin = ch[2 ** (i - 1)]
        self.final_conv = Conv2d(cin, ch[4], 3, padding=1)
        cin = ch[4]
        self.conv_body_up = nn.ModuleList()
        for i in range(3, self.log_size + 1):
            self.conv_body_up.append(_BilinearResBlock(cin, ch[2 ** i], "up"))
            cin = ch[2 ** i]
        self.toRGB = nn.ModuleList([Conv2d(ch[2 ** i], 3, 1) for i in range(3, self.log_size + 1)])
        self.final_linear = Linear(ch[4] * 16, (self.log_size * 2 - 2) * style_dim)
        self.stylegan_decoder = StyleGAN2DecoderSFT(out_size, style_dim, 8, mult, 1.0, sft_half=True)
        self.condition_scale = nn.ModuleList()
        self.condition_shift = nn.ModuleList()
        for i in range(3, self.log_size + 1):
            c = ch[2 ** i]
            for lst in (self.condition_scale, self.condition_shift):
                lst.append(nn.Sequential(Conv2d(c, c, 3, padding=1), nn.LeakyReLU(0.2), Conv2d(c, c, 3, padding=1)))
        missing, _ = self.load_state_dict(state_dict, strict=False)
        if missing and strict:
            raise ValueError(f"GFPGAN: missing keys {missing[:4]}")
        self.eval()

    def forward(self, x, return_rgb=True, randomize_noise=True, **_):
        feat = _lrelu(self.conv_body_first(x))
        skips = []
        for blk in self.conv_body_down:
            feat = blk(feat)
            skips.insert(0, feat)
        feat = _lrelu(self.final_conv(feat))
        latent = self.final_linear(feat.reshape(feat.shape[0], -1)).view(feat.shape[0], -1, self.style_dim)
        conditions, rgbs = [], []
        for i, blk in enumerate(self.conv_body_up):
            feat = blk(feat + skips[i])
            conditions.append(self.condition_scale[i](feat))
            conditions.append(self.condition_shift[i](feat))
            if return_rgb:
                rgbs.append(self.toRGB[i](feat))
        image = self.stylegan_decoder(latent, conditions, randomize_noise=randomize_noise)
        return image, rgbs
