"""Image super-resolution networks for ``UpscaleModelLoader`` (parity: ``comfy_extras/chainner_models/
model_loading.py:24-99`` dispatch, ``architecture/RRDB.py`` and ``architecture/SRVGG.py``).

Supported here: ESRGAN / Real-ESRGAN (RRDBNet, old and new key layouts, x1/x2 pixel-unshuffle
variants, scale 1-8) and Real-ESRGAN compact (SRVGGNetCompact). Every 3x3 conv is a
``layers.Conv2d`` so on the device it runs as the NHWC implicit-GEMM MFMA kernel (bias fused);
the state dict is re-keyed to the old-arch ``model.N`` layout the reference uses, so any file
that loads there loads here. Other chaiNNer architectures (SwinIR/Swin2SR/HAT/DAT, OmniSR, SCUNet,
SPSR, Swift-SRGAN, LaMa, GFPGAN/CodeFormer/RestoreFormer) are detected by the same key probes and
rejected with ``UnsupportedModel`` naming the architecture.
"""
from __future__ import annotations

import math
import re

import torch
import torch.nn as nn
import torch.nn.functional as F

from .layers import Conv2d


class UnsupportedModel(Exception):
    pass


def _lrelu(x):
    return F.leaky_relu(x, 0.2)


class ResidualDenseBlock5C(nn.Module):
    def __init__(self, nf=64, gc=32):
        super().__init__()
        for i in range(5):
            cin = nf + i * gc
            cout = nf if i == 4 else gc
            setattr(self, f"conv{i + 1}", nn.Sequential(Conv2d(cin, cout, 3, padding=1)))

    def forward(self, x):
        feats = [x]
        for i in range(4):
            feats.append(_lrelu(getattr(self, f"conv{i + 1}")[0](torch.cat(feats, 1) if len(feats) > 1 else x)))
        return self.conv5[0](torch.cat(feats, 1)) * 0.2 + x


class RRDB(nn.Module):
    def __init__(self, nf, gc=32):  # gc: growth channels (32 in every released ESRGAN)
        super().__init__()
        self.RDB1 = ResidualDenseBlock5C(nf, gc)
        self.RDB2 = ResidualDenseBlock5C(nf, gc)
        self.RDB3 = ResidualDenseBlock5C(nf, gc)

    def forward(self, x):
        return self.RDB3(self.RDB2(self.RDB1(x))) * 0.2 + x


class _Trunk(nn.Module):
    """``model.1``: ShortcutBlock(sequential(RRDB x nb, conv)) -> keys model.1.sub.N"""

    def __init__(self, nf, nb, gc=32):
        super().__init__()
        self.sub = nn.ModuleList([RRDB(nf, gc) for _ in range(nb)] + [Conv2d(nf, nf, 3, padding=1)])

    def forward(self, x):
        h = x
        for m in self.sub[:-1]:
            h = m(h)
        return self.sub[-1](h, residual=x)


_NEW_ARCH = [
    (re.compile(r"^(?:RRDB_trunk|body)\.(\d+)\.(?:RDB|rdb)(\d)\.conv(\d)\.(weight|bias)$"),
     r"model.1.sub.\1.RDB\2.conv\3.0.\4"),
]


def _esrgan_old_arch(sd):
    """new-arch (conv_first / RRDB_trunk | body / upconvN / HRconv / conv_last) -> model.N keys."""
    if "conv_first.weight" not in sd:
        return sd
    nb = 1 + max(int(m.group(1)) for k in sd for m in [_NEW_ARCH[0][0].match(k)] if m)
    out = {}
    for k, v in sd.items():
        m = _NEW_ARCH[0][0].match(k)
        if m:
            out[_NEW_ARCH[0][0].sub(_NEW_ARCH[0][1], k)] = v
    for kind in ("weight", "bias"):
        out[f"model.0.{kind}"] = sd[f"conv_first.{kind}"]
        for name in ("trunk_conv", "conv_body"):
            if f"{name}.{kind}" in sd:
                out[f"model.1.sub.{nb}.{kind}"] = sd[f"{name}.{kind}"]
    max_up = 0
    for k, v in sd.items():
        m = re.match(r"^(?:upconv|conv_up)(\d)\.(weight|bias)$", k)
        if m:
            out[f"model.{int(m.group(1)) * 3}.{m.group(2)}"] = v
            max_up = max(max_up, int(m.group(1)) * 3)
    for kind in ("weight", "bias"):
        for name in ("HRconv", "conv_hr"):
            if f"{name}.{kind}" in sd:
                out[f"model.{max_up + 2}.{kind}"] = sd[f"{name}.{kind}"]
        if f"conv_last.{kind}" in sd:
            out[f"model.{max_up + 4}.{kind}"] = sd[f"conv_last.{kind}"]
    return out


class RRDBNet(nn.Module):
    """ESRGAN: conv -> trunk of RRDBs (+ long skip) -> log2(scale) x [nearest x2, conv, lrelu] ->
    HR conv, lrelu -> last conv. In-channel counts of 4x / 16x the out-channels mean a
    pixel-unshuffled input (Real-ESRGAN x2 / x1)."""

    def __init__(self, state_dict):
        super().__init__()
        sd = _esrgan_old_arch(state_dict)
        if any("conv1x1" in k for k in sd):
            raise UnsupportedModel("ESRGAN+ (conv1x1 RRDB) is not supported")
        if "model.0.weight" not in sd or "model.1.sub.0.RDB1.conv1.0.weight" not in sd:
            raise UnsupportedModel("unrecognised upscale model state dict")
        if sd["model.0.weight"].shape[-1] == 2:
            raise UnsupportedModel("ESRGAN-2c2 is not supported")
        self.model_arch = "ESRGAN"
        nums = sorted({int(k.split(".")[1]) for k in sd if re.match(r"^model\.\d+\.weight$", k)})
        last = nums[-1]
        self.num_blocks = 1 + max(int(k.split(".")[3]) for k in sd if k.startswith("model.1.sub.") and "RDB" in k)
        self.num_filters = sd["model.0.weight"].shape[0]
        self.in_nc = sd["model.0.weight"].shape[1]
        self.out_nc = sd[f"model.{last}.weight"].shape[0]
        ups = [n for n in nums if 0 < n < last - 2]     # upconv layers between the trunk and HR conv
        scale = 2 ** len(ups)
        self.shuffle_factor = None
        if self.in_nc in (self.out_nc * 4, self.out_nc * 16):
            self.shuffle_factor = int(math.sqrt(self.in_nc // self.out_nc))
        nf = self.num_filters
        gc = sd["model.1.sub.0.RDB1.conv1.0.weight"].shape[0]
        mods = {"0": Conv2d(self.in_nc, nf, 3, padding=1), "1": _Trunk(nf, self.num_blocks, gc)}
        for n in ups:
            mods[str(n)] = Conv2d(nf, nf, 3, padding=1)
        mods[str(last - 2)] = Conv2d(nf, nf, 3, padding=1)
        mods[str(last)] = Conv2d(nf, self.out_nc, 3, padding=1)
        self.model = nn.ModuleDict(mods)
        self._ups = [str(n) for n in ups]
        self._hr, self._last = str(last - 2), str(last)
        self.scale = scale
        if self.shuffle_factor:
            self.scale //= self.shuffle_factor
        missing, unexpected = self.load_state_dict({k: v for k, v in sd.items()}, strict=False)
        if missing:
            raise UnsupportedModel(f"ESRGAN: missing keys {missing[:4]}")

    def forward(self, x):
        h_in, w_in = x.shape[-2:]
        if self.shuffle_factor:
            f = self.shuffle_factor
            x = F.pad(x, (0, (f - w_in % f) % f, 0, (f - h_in % f) % f), "reflect")
            x = F.pixel_unshuffle(x, f)
        if x.is_cuda:
            x = x.contiguous(memory_format=torch.channels_last)
        m = self.model
        h = m["0"](x)
        h = m["1"](h)
        for name in self._ups:       # nearest x2 + conv: one fused kernel on the device
            h = _lrelu(m[name](h, upsample2x=True))
        h = m[self._last](_lrelu(m[self._hr](h)))
        if self.shuffle_factor:
            h = h[:, :, : h_in * self.scale, : w_in * self.scale]
        return h


class SRVGGNetCompact(nn.Module):
    """Real-ESRGAN compact: conv + PReLU, num_conv x (conv + PReLU), conv to out*s^2, pixel shuffle,
    plus the nearest-upsampled input."""

    def __init__(self, state_dict):
        super().__init__()
        self.model_arch = "RealESRGAN-Compact"
        idx = sorted({int(k.split(".")[1]) for k in state_dict if k.startswith("body.")})
        self.in_nc = state_dict["body.0.weight"].shape[1]
        self.num_feat = state_dict["body.0.weight"].shape[0]
        last = idx[-1]
        self.num_conv = (last - 2) // 2
        self.out_nc = self.in_nc
        self.scale = int(math.sqrt(state_dict[f"body.{last}.weight"].shape[0] // self.out_nc))
        prelu = state_dict["body.1.weight"].dim() == 1
        body = []
        for i in range(last + 1):
            if i % 2 == 0:
                cin = self.in_nc if i == 0 else self.num_feat
                cout = self.out_nc * self.scale ** 2 if i == last else self.num_feat
                body.append(Conv2d(cin, cout, 3, padding=1))
            else:
                body.append(nn.PReLU(num_parameters=self.num_feat) if prelu else nn.LeakyReLU(0.1))
        self.body = nn.ModuleList(body)
        self.load_state_dict(state_dict, strict=True)

    def forward(self, x):
        h = x.contiguous(memory_format=torch.channels_last) if x.is_cuda else x
        for m in self.body:
            h = m(h)
        out = F.pixel_shuffle(h, self.scale)
        return out + F.interpolate(x, scale_factor=self.scale, mode="nearest")


_UNSUPPORTED_PROBES = [
    ("SPSR", lambda k: "f_HR_conv1.0.weight" in k),
    ("HAT", lambda k: "layers.0.residual_group.blocks.0.conv_block.cab.0.weight" in k),
    ("Swin2SR", lambda k: "layers.0.residual_group.blocks.0.norm1.weight" in k and "patch_embed.proj.weight" in k),
    ("SwinIR", lambda k: "layers.0.residual_group.blocks.0.norm1.weight" in k),
    ("GFPGAN", lambda k: "toRGB.0.weight" in k and "stylegan_decoder.style_mlp.1.weight" in k),
    ("RestoreFormer", lambda k: "encoder.conv_in.weight" in k and "encoder.down.0.block.0.norm1.weight" in k),
    ("CodeFormer", lambda k: "encoder.blocks.0.weight" in k and "quantize.embedding.weight" in k),
    ("LaMa", lambda k: "model.model.1.bn_l.running_mean" in k or "generator.model.1.bn_l.running_mean" in k),
    ("OmniSR", lambda k: "residual_layer.0.residual_layer.0.layer.0.fn.0.weight" in k),
    ("SCUNet", lambda k: "m_head.0.weight" in k and "m_tail.0.weight" in k),
    ("DAT", lambda k: "layers.0.blocks.2.attn.attn_mask_0" in k),
]


def load_state_dict(state_dict) -> nn.Module:
    """Architecture dispatch by key probes, in the reference's order."""
    for wrap in ("params_ema", "params-ema", "params"):
        if wrap in state_dict and isinstance(state_dict[wrap], dict):
            state_dict = state_dict[wrap]
            break
    keys = set(state_dict.keys())
    if "body.0.weight" in keys and "body.1.weight" in keys:
        return SRVGGNetCompact(state_dict)
    if "model" in keys and isinstance(state_dict["model"], dict) and "initial.cnn.depthwise.weight" in state_dict["model"]:
        raise UnsupportedModel("Swift-SRGAN upscale models are not supported")
    for name, probe in _UNSUPPORTED_PROBES:
        if probe(keys):
            raise UnsupportedModel(f"{name} upscale models are not supported")
    try:
        return RRDBNet(state_dict)
    except UnsupportedModel:
        raise
    except Exception as e:     # anything else that is not a loadable ESRGAN
        raise UnsupportedModel(str(e)) from e
