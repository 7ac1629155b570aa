"""LaMa inpainting generator (fast Fourier convolutions; parity: ``comfy_extras/chainner_models/
architecture/LaMa.py:FFCResNetGenerator/LaMa`` — the released big-lama config: 4->64 7x7 stem,
three stride-2 downsamplers, 18 FFC residual blocks at 512 channels with 3/4 of the channels on
the global (spectral) path, three transposed-conv upsamplers and a sigmoid 7x7 head).

Module indices and parameter names reproduce the reference's ``model.model.N`` layout so the
released checkpoints (``generator.model.*`` is accepted too) load unchanged. The spectral path is
rFFT2 -> 1x1 conv over the stacked (re, im) channels -> BN/ReLU -> irFFT2 in fp32 (rocFFT on
the device); the spatial convs are reflect-padded ``layers.Conv2d``.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .layers import Conv2d


class _ReflectConv(Conv2d):
    """Conv with reflect padding done explicitly (the reference uses ``padding_mode='reflect'``)."""

    def __init__(self, cin, cout, k, stride=1, padding=0):
        super().__init__(cin, cout, k, stride=stride, padding=0, bias=False)
        self.pad = padding

    def forward(self, x):
        if self.pad:
            x = F.pad(x, (self.pad,) * 4, mode="reflect")
        return super().forward(x)


class _FourierUnit(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.conv_layer = Conv2d(2 * c, 2 * c, 1, bias=False)
        self.bn = nn.BatchNorm2d(2 * c)

    def forward(self, x):
        B, C, H, W = x.shape
        f = torch.fft.rfftn(x.float(), dim=(-2, -1), norm="ortho")
        f = torch.stack((f.real, f.imag), 2).reshape(B, 2 * C, H, -1)           # channel = 2c + {re, im}
        f = F.relu(self.bn(self.conv_layer(f.to(x.dtype)))).float()
        f = f.view(B, C, 2, H, -1)
        out = torch.fft.irfftn(torch.complex(f[:, :, 0], f[:, :, 1]), s=(H, W), dim=(-2, -1), norm="ortho")
        return out.to(x.dtype)


class _SpectralTransform(nn.Module):
    def __init__(self, cin, cout):
        super().__init__()
        self.conv1 = nn.Sequential(Conv2d(cin, cout // 2, 1, bias=False), nn.BatchNorm2d(cout // 2), nn.ReLU())
        self.fu = _FourierUnit(cout // 2)
        self.conv2 = Conv2d(cout // 2, cout, 1, bias=False)

    def forward(self, x):
        x = self.conv1(x)
        return self.conv2(x + self.fu(x))


class _FFC(nn.Module):
    """Local/global split convolution: l->l, l->g, g->l spatial convs and a g->g spectral transform."""

    def __init__(self, cin, cout, k, gin, gout, stride=1, padding=0):
        super().__init__()
        self.in_g = int(cin * gin)
        in_l = cin - self.in_g
        out_g = int(cout * gout)
        out_l = cout - out_g
        self.has_l, self.has_g = gout != 1, gout != 0

        def conv(a, b):
            return _ReflectConv(a, b, k, stride, padding) if a and b else None

        self.convl2l = conv(in_l, out_l)
        self.convl2g = conv(in_l, out_g)
        self.convg2l = conv(self.in_g, out_l)
        self.convg2g = _SpectralTransform(self.in_g, out_g) if self.in_g and out_g else None

    def forward(self, xl, xg):
        ol = og = None
        if self.has_l:
            ol = self.convl2l(xl) if self.convl2l is not None else 0
            if self.convg2l is not None:
                ol = ol + self.convg2l(xg)
        if self.has_g:
            og = self.convl2g(xl) if self.convl2g is not None else 0
            if self.convg2g is not None:
                og = og + self.convg2g(xg)
        return ol, og


class FFCBnAct(nn.Module):
    def __init__(self, cin, cout, k, gin, gout, stride=1, padding=0):
        super().__init__()
        self.ffc = _FFC(cin, cout, k, gin, gout, stride, padding)
        out_g = int(cout * gout)
        self.bn_l = nn.BatchNorm2d(cout - out_g) if gout != 1 else nn.Identity()
        self.bn_g = nn.BatchNorm2d(out_g) if gout != 0 else nn.Identity()

    def forward(self, xl, xg=None):
        ol, og = self.ffc(xl, xg)
        ol = F.relu(self.bn_l(ol)) if ol is not None else None
        og = F.relu(self.bn_g(og)) if og is not None else None
        return ol, og


class FFCResBlock(nn.Module):
    def __init__(self, dim, ratio=0.75):
        super().__init__()
        self.conv1 = FFCBnAct(dim, dim, 3, ratio, ratio, padding=1)
        self.conv2 = FFCBnAct(dim, dim, 3, ratio, ratio, padding=1)

    def forward(self, xl, xg):
        yl, yg = self.conv2(*self.conv1(xl, xg))
        return xl + yl, xg + yg


class FFCResNetGenerator(nn.Module):
    def __init__(self, in_nc=4, out_nc=3, ngf=64, n_down=3, n_blocks=18, max_features=1024):
        super().__init__()
        mods: list = [nn.ReflectionPad2d(3), FFCBnAct(in_nc, ngf, 7, 0, 0)]
        for i in range(n_down):
            m = 2 ** i
            gout = 0.75 if i == n_down - 1 else 0
            mods.append(FFCBnAct(min(max_features, ngf * m), min(max_features, ngf * m * 2), 3, 0, gout, 2, 1))
        dim = min(max_features, ngf * 2 ** n_down)
        mods += [FFCResBlock(dim) for _ in range(n_blocks)]
        mods.append(nn.Identity())                                   # ConcatTupleLayer
        for i in range(n_down):
            m = 2 ** (n_down - i)
            a, b = min(max_features, ngf * m), min(max_features, ngf * m // 2)
            mods += [nn.ConvTranspose2d(a, b, 3, stride=2, padding=1, output_padding=1), nn.BatchNorm2d(b), nn.ReLU()]
        mods += [nn.ReflectionPad2d(3), Conv2d(ngf, out_nc, 7)]
        self.model = nn.Sequential(*mods)
        self.n_down, self.n_blocks = n_down, n_blocks

    def forward(self, x):
        m = self.model
        xl, xg = m[1](m[0](x))
        for i in range(2, 2 + self.n_down):
            xl, xg = m[i](xl, xg)
        i = 2 + self.n_down
        for _ in range(self.n_blocks):
            xl, xg = m[i](xl, xg)
            i += 1
        y = torch.cat([xl, xg], 1)
        for mod in m[i + 1:]:
            y = mod(y)
        return torch.sigmoid(y)


class LaMa(nn.Module):
    """Inpainting: ``forward(image, mask)`` fills the masked region and keeps the rest."""

    def __init__(self, state_dict, strict: bool = True):
        super().__init__()
        self.model_arch = "LaMa"
        self.sub_type = "Inpaint"
        self.in_nc, self.out_nc, self.scale = 4, 3, 1
        self.pad_mod = 8
        self.model = FFCResNetGenerator(self.in_nc, self.out_nc)
        for p in self.parameters():
            p.requires_grad_(False)
        sd = {k.replace("generator.model", "model.model"): v for k, v in state_dict.items()}
        missing, _ = self.load_state_dict(sd, strict=False)
        if missing and strict:
            raise ValueError(f"LaMa: missing keys {missing[:4]}")
        self.eval()

    def forward(self, img, mask):
        masked = img * (1 - mask)
        return mask * self.model(torch.cat([masked, mask], 1)) + (1 - mask) * img
