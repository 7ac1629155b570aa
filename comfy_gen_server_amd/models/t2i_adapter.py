"""T2I-Adapter and style-adapter networks (parity: ``comfy/t2i_adapter/adapter.py:1-293``).

Small conv encoders that turn a control image into per-resolution residuals for the UNet encoder
(full / light variants, SD1.x and SDXL layouts) and the CLIP-vision style adapter (tokens appended
to the text context). They run once per hint image, so plain torch modules are used; parameter
names follow the released checkpoints.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


class Downsample(nn.Module):
    """x2 downsample: strided 3x3 conv, or average pooling that pads odd sizes."""

    def __init__(self, channels, use_conv, out_channels=None, padding=1):
        super().__init__()
        self.channels = channels
        self.out_channels = out_channels or channels
        self.use_conv = use_conv
        if use_conv:
            self.op = nn.Conv2d(channels, self.out_channels, 3, stride=2, padding=padding)
        else:
            assert channels == self.out_channels
            self.op = None

    def forward(self, x):
        if self.use_conv:
            return self.op(x)
        return F.avg_pool2d(x, 2, 2, padding=(x.shape[2] % 2, x.shape[3] % 2))


class ResnetBlock(nn.Module):
    def __init__(self, in_c, out_c, down, ksize=3, sk=False, use_conv=True):
        super().__init__()
        ps = ksize // 2
        self.in_conv = nn.Conv2d(in_c, out_c, ksize, 1, ps) if (in_c != out_c or not sk) else None
        self.block1 = nn.Conv2d(out_c, out_c, 3, 1, 1)
        self.act = nn.ReLU()
        self.block2 = nn.Conv2d(out_c, out_c, ksize, 1, ps)
        self.skep = None if sk else nn.Conv2d(in_c, out_c, ksize, 1, ps)
        self.down = down
        if down:
            self.down_opt = Downsample(in_c, use_conv=use_conv)

    def forward(self, x):
        if self.down:
            x = self.down_opt(x)
        if self.in_conv is not None:
            x = self.in_conv(x)
        h = self.block2(self.act(self.block1(x)))
        return h + (self.skep(x) if self.skep is not None else x)


class Adapter(nn.Module):
    """Full adapter. SD1.x: 4 levels with downsampling at levels 1-3 (features at the 3rd, 6th, 9th
    and 12th UNet input blocks); XL (cin 256/768, 16x pixel-unshuffle): 3 spatial levels."""

    def __init__(self, channels=(320, 640, 1280, 1280), nums_rb=3, cin=64, ksize=3, sk=False, use_conv=True, xl=True):
        super().__init__()
        self.xl = xl
        self.unshuffle_amount = 16 if xl else 8
        no_down, down = ([1], [2]) if xl else ([], [3, 2, 1])
        self.input_channels = cin // (self.unshuffle_amount * self.unshuffle_amount)
        self.unshuffle = nn.PixelUnshuffle(self.unshuffle_amount)
        self.channels = list(channels)
        self.nums_rb = nums_rb
        body = []
        for i, c in enumerate(self.channels):
            for j in range(nums_rb):
                if j == 0 and i in down:
                    body.append(ResnetBlock(self.channels[i - 1], c, down=True, ksize=ksize, sk=sk, use_conv=use_conv))
                elif j == 0 and i in no_down:
                    body.append(ResnetBlock(self.channels[i - 1], c, down=False, ksize=ksize, sk=sk, use_conv=use_conv))
                else:
                    body.append(ResnetBlock(c, c, down=False, ksize=ksize, sk=sk, use_conv=use_conv))
        self.body = nn.ModuleList(body)
        self.conv_in = nn.Conv2d(cin, self.channels[0], 3, 1, 1)

    def forward(self, x):
        x = self.conv_in(self.unshuffle(x))
        feats = []
        for i in range(len(self.channels)):
            for j in range(self.nums_rb):
                x = self.body[i * self.nums_rb + j](x)
            # pad with None so the list lines up with the UNet input blocks
            if self.xl:
                feats += [None, None, None] if i == 0 else ([None, None] if i == 2 else [None])
            else:
                feats += [None, None]
            feats.append(x)
        return feats


class ResnetBlock_light(nn.Module):
    def __init__(self, in_c):
        super().__init__()
        self.block1 = nn.Conv2d(in_c, in_c, 3, 1, 1)
        self.act = nn.ReLU()
        self.block2 = nn.Conv2d(in_c, in_c, 3, 1, 1)

    def forward(self, x):
        return self.block2(self.act(self.block1(x))) + x


class extractor(nn.Module):  # noqa: N801  (checkpoint key names)
    def __init__(self, in_c, inter_c, out_c, nums_rb, down=False):
        super().__init__()
        self.in_conv = nn.Conv2d(in_c, inter_c, 1, 1, 0)
        self.body = nn.Sequential(*[ResnetBlock_light(inter_c) for _ in range(nums_rb)])
        self.out_conv = nn.Conv2d(inter_c, out_c, 1, 1, 0)
        self.down = down
        if down:
            self.down_opt = Downsample(in_c, use_conv=False)

    def forward(self, x):
        if self.down:
            x = self.down_opt(x)
        return self.out_conv(self.body(self.in_conv(x)))


class Adapter_light(nn.Module):
    def __init__(self, channels=(320, 640, 1280, 1280), nums_rb=3, cin=64):
        super().__init__()
        self.unshuffle_amount = 8
        self.unshuffle = nn.PixelUnshuffle(8)
        self.input_channels = cin // 64
        self.channels = list(channels)
        self.nums_rb = nums_rb
        self.xl = False
        self.body = nn.ModuleList([
            extractor(in_c=cin if i == 0 else self.channels[i - 1], inter_c=c // 4, out_c=c, nums_rb=nums_rb,
                      down=i > 0) for i, c in enumerate(self.channels)])

    def forward(self, x):
        x = self.unshuffle(x)
        feats = []
        for b in self.body:
            x = b(x)
            feats += [None, None, x]
        return feats


class _LN32(nn.LayerNorm):
    def forward(self, x):
        return super().forward(x.float()).to(x.dtype)


class _QuickGELU(nn.Module):
    def forward(self, x):
        return x * torch.sigmoid(1.702 * x)


class ResidualAttentionBlock(nn.Module):
    def __init__(self, d_model, n_head):
        super().__init__()
        self.attn = nn.MultiheadAttention(d_model, n_head)
        self.ln_1 = _LN32(d_model)
        self.mlp = nn.Sequential()
        self.mlp.add_module("c_fc", nn.Linear(d_model, d_model * 4))
        self.mlp.add_module("gelu", _QuickGELU())
        self.mlp.add_module("c_proj", nn.Linear(d_model * 4, d_model))
        self.ln_2 = _LN32(d_model)

    def forward(self, x):
        h = self.ln_1(x)
        x = x + self.attn(h, h, h, need_weights=False)[0]
        return x + self.mlp(self.ln_2(x))


class StyleAdapter(nn.Module):
    """CLIP-vision tokens -> ``num_token`` style tokens in the text-context width."""

    def __init__(self, width=1024, context_dim=768, num_head=8, n_layes=3, num_token=4):
        super().__init__()
        scale = width ** -0.5
        self.transformer_layes = nn.Sequential(*[ResidualAttentionBlock(width, num_head) for _ in range(n_layes)])
        self.num_token = num_token
        self.style_embedding = nn.Parameter(torch.randn(1, num_token, width) * scale)
        self.ln_post = _LN32(width)
        self.ln_pre = _LN32(width)
        self.proj = nn.Parameter(scale * torch.randn(width, context_dim))

    def forward(self, x):
        se = self.style_embedding.expand(x.shape[0], -1, -1).to(x)
        x = self.ln_pre(torch.cat([x, se], dim=1)).permute(1, 0, 2)
        x = self.transformer_layes(x).permute(1, 0, 2)
        return self.ln_post(x[:, -self.num_token:, :]) @ self.proj
