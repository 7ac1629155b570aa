"""Tiny AutoEncoder for SD / SDXL latents (parity: ``comfy/taesd/taesd.py:1-77``).

Used for live previews (runtime.preview) and as the virtual ``taesd`` / ``taesdxl`` VAEs. All convs
are 64-wide 3x3 — on the device they take the NHWC implicit-GEMM conv kernel, and each
"nearest 2x upsample + conv" pair of the decoder is one fused kernel (the input is read through the
upsample, the 4x tensor is never written). Key names match the released checkpoints
(``taesd_encoder.N.*`` / ``taesd_decoder.N.*``).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import ops
from .layers import Conv2d


def _conv(n_in, n_out, **kw):
    return Conv2d(n_in, n_out, 3, padding=1, **kw)


class Clamp(nn.Module):
    def forward(self, x):
        return torch.tanh(x / 3) * 3


class Block(nn.Module):
    def __init__(self, n_in, n_out):
        super().__init__()
        self.conv = nn.Sequential(_conv(n_in, n_out), nn.ReLU(), _conv(n_out, n_out), nn.ReLU(), _conv(n_out, n_out))
        self.skip = Conv2d(n_in, n_out, 1, bias=False) if n_in != n_out else nn.Identity()
        self.fuse = nn.ReLU()

    def forward(self, x):
        c = self.conv
        h = torch.relu(c[0](x))
        h = torch.relu(c[2](h))
        skip = x if isinstance(self.skip, nn.Identity) else self.skip(x)
        return torch.relu(c[4](h, residual=skip))      # residual add fused into the last conv


class Upsample2x(nn.Module):
    """Marker for the nearest-2x upsample; the following conv consumes it (fused)."""

    def forward(self, x):
        return ops.upsample_nearest2x(x) if x.is_cuda else torch.nn.functional.interpolate(x, scale_factor=2.0)


def Encoder(latent_channels=4):
    return nn.Sequential(
        _conv(3, 64), Block(64, 64),
        _conv(64, 64, stride=2, bias=False), Block(64, 64), Block(64, 64), Block(64, 64),
        _conv(64, 64, stride=2, bias=False), Block(64, 64), Block(64, 64), Block(64, 64),
        _conv(64, 64, stride=2, bias=False), Block(64, 64), Block(64, 64), Block(64, 64),
        _conv(64, latent_channels))


def Decoder(latent_channels=4):
    return nn.Sequential(
        Clamp(), _conv(latent_channels, 64), nn.ReLU(),
        Block(64, 64), Block(64, 64), Block(64, 64), Upsample2x(), _conv(64, 64, bias=False),
        Block(64, 64), Block(64, 64), Block(64, 64), Upsample2x(), _conv(64, 64, bias=False),
        Block(64, 64), Block(64, 64), Block(64, 64), Upsample2x(), _conv(64, 64, bias=False),
        Block(64, 64), _conv(64, 3))


def _run(seq, x):
    mods = list(seq)
    i = 0
    while i < len(mods):
        m = mods[i]
        if isinstance(m, Upsample2x) and i + 1 < len(mods) and isinstance(mods[i + 1], Conv2d):
            x = mods[i + 1](x, upsample2x=True)
            i += 2
            continue
        if isinstance(m, nn.ReLU):
            x = torch.relu(x)
        else:
            x = m(x)
        i += 1
    return x


class TAESD(nn.Module):
    latent_magnitude = 3
    latent_shift = 0.5

    def __init__(self, encoder_path=None, decoder_path=None, latent_channels=4):
        super().__init__()
        self.taesd_encoder = Encoder(latent_channels)
        self.taesd_decoder = Decoder(latent_channels)
        self.vae_scale = nn.Parameter(torch.tensor(1.0), requires_grad=False)
        if encoder_path is not None or decoder_path is not None:
            from ..runtime.checkpoint import load_state_dict
            if encoder_path is not None:
                self.taesd_encoder.load_state_dict(load_state_dict(encoder_path))
            if decoder_path is not None:
                self.taesd_decoder.load_state_dict(load_state_dict(decoder_path))

    @staticmethod
    def scale_latents(x):
        """raw latents -> [0, 1]"""
        return x.div(2 * TAESD.latent_magnitude).add(TAESD.latent_shift).clamp(0, 1)

    @staticmethod
    def unscale_latents(x):
        """[0, 1] -> raw latents"""
        return x.sub(TAESD.latent_shift).mul(2 * TAESD.latent_magnitude)

    def decode(self, x):
        if x.is_cuda:
            x = x.contiguous(memory_format=torch.channels_last)
        return _run(self.taesd_decoder, x * self.vae_scale.to(x.dtype)).sub(0.5).mul(2)

    def encode(self, x):
        if x.is_cuda:
            x = x.contiguous(memory_format=torch.channels_last)
        return _run(self.taesd_encoder, x * 0.5 + 0.5) / self.vae_scale.to(x.dtype)
