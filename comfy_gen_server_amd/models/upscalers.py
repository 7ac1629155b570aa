"""Image super-resolution networks for ``UpscaleModelLoader`` (parity: ``comfy_extras/chainner_models/
model_loading.py:24-99`` dispatch, ``architecture/RRDB.py`` and ``architecture/SRVGG.py``).

Every architecture the reference dispatches is implemented: ESRGAN / Real-ESRGAN (RRDBNet, old and
new key layouts, x1/x2 pixel-unshuffle variants, scale 1-8), Real-ESRGAN compact
(SRVGGNetCompact), SPSR and Swift-SRGAN (here); SwinIR / Swin2SR / HAT / SCUNet (``swin_sr.py``),
Omni-SR (``omnisr.py``), DAT (``dat.py``), the LaMa inpainter (``lama.py``) and the face
restorers GFPGAN / RestoreFormer / CodeFormer (``face.py``). Every 3x3 conv is a
``layers.Conv2d`` so on the device it runs as the NHWC implicit-GEMM MFMA kernel (bias fused);
the state dict is re-keyed to the old-arch ``model.N`` layout the reference uses, so any file
that loads there loads here.
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


class _GradMag(nn.Module):
    """Per-channel gradient magnitude with [0,-1,0;0,0,0;0,1,0] / [0,0,0;-1,0,1;0,0,0] kernels
    (SPSR's gradient branch input; keys ``get_g_nopadding.weight_{h,v}``)."""

    def __init__(self):
        super().__init__()
        self.weight_h = nn.Parameter(torch.tensor([[[[0., 0., 0.], [-1., 0., 1.], [0., 0., 0.]]]]), requires_grad=False)
        self.weight_v = nn.Parameter(torch.tensor([[[[0., -1., 0.], [0., 0., 0.], [0., 1., 0.]]]]), requires_grad=False)

    def forward(self, x):
        c = x.shape[1]
        xf = x.float()
        gv = F.conv2d(xf, self.weight_v.float().expand(c, 1, 3, 3), padding=1, groups=c)
        gh = F.conv2d(xf, self.weight_h.float().expand(c, 1, 3, 3), padding=1, groups=c)
        return torch.sqrt(gv * gv + gh * gh + 1e-6).to(x.dtype)


def _seq_conv(cin, cout, k=3):
    return nn.Sequential(Conv2d(cin, cout, k, padding=k // 2))


class SPSRNet(nn.Module):
    """SPSR (structure-preserving SR): an ESRGAN trunk whose RRDB features at blocks 5/10/15/20 feed
    a gradient-map branch; both branches are fused at HR resolution (chaiNNer SPSR.py key layout:
    ``model.*``, ``b_*``, ``f_*``, ``HR_conv*_new``)."""

    def __init__(self, state_dict):
        super().__init__()
        sd = state_dict
        self.model_arch = "SPSR"
        self.in_nc = sd["model.0.weight"].shape[1]
        self.out_nc = sd["f_HR_conv1.0.bias"].shape[0]
        nf = self.num_filters = sd["model.0.weight"].shape[0]
        self.num_blocks = 1 + max(int(k.split(".")[3]) for k in sd if k.startswith("model.1.sub.") and "RDB" in k)
        ups = sorted({int(k.split(".")[1]) for k in sd if re.match(r"^model\.\d+\.weight$", k) and int(k.split(".")[1]) > 1})
        hr0 = ups[-1]                      # HR_conv0_new is the last model.N conv
        ups = ups[:-1]
        self.scale = 2 ** len(ups)
        mods = {"0": Conv2d(self.in_nc, nf, 3, padding=1), "1": _Trunk(nf, self.num_blocks)}
        for n in ups:
            mods[str(n)] = Conv2d(nf, nf, 3, padding=1)
        self.model = nn.ModuleDict(mods)
        self._ups = [str(n) for n in ups]
        self.HR_conv0_new = _seq_conv(nf, nf)
        self.HR_conv1_new = _seq_conv(nf, nf)
        self.get_g_nopadding = _GradMag()
        self.b_fea_conv = _seq_conv(self.in_nc, nf)
        for i in range(1, 5):
            setattr(self, f"b_concat_{i}", _seq_conv(2 * nf, nf))
            setattr(self, f"b_block_{i}", RRDB(2 * nf))
        self.b_LR_conv = _seq_conv(nf, nf)
        b_mods = []
        for _ in ups:
            b_mods += [nn.Upsample(scale_factor=2, mode="nearest"), Conv2d(nf, nf, 3, padding=1), nn.LeakyReLU(0.2)]
        b_mods += [Conv2d(nf, nf, 3, padding=1), nn.LeakyReLU(0.2), Conv2d(nf, nf, 3, padding=1)]
        self.b_module = nn.Sequential(*b_mods)
        self.conv_w = nn.Sequential(Conv2d(nf, self.out_nc, 1))
        self.f_concat = _seq_conv(2 * nf, nf)
        self.f_block = RRDB(2 * nf)
        self.f_HR_conv0 = _seq_conv(nf, nf)
        self.f_HR_conv1 = _seq_conv(nf, self.out_nc)
        sd = dict(sd)
        for t in ("weight", "bias"):        # HR_conv0_new is registered twice (model.N and by name)
            sd.setdefault(f"HR_conv0_new.0.{t}", sd.pop(f"model.{hr0}.{t}", None))
            sd.pop(f"model.{hr0}.{t}", None)
        missing, _ = self.load_state_dict(sd, strict=False)
        missing = [m for m in missing if not m.startswith("get_g_nopadding")]
        if missing:
            raise UnsupportedModel(f"SPSR: missing keys {missing[:4]}")

    def forward(self, x):
        if x.is_cuda:
            x = x.contiguous(memory_format=torch.channels_last)
        g = self.get_g_nopadding(x)
        m = self.model
        h = m["0"](x)
        trunk = m["1"].sub
        feats, y = [], h
        for i, blk in enumerate(trunk[:-1]):
            y = blk(y)
            if (i + 1) % 5 == 0 and len(feats) < 4:
                feats.append(y)
        while len(feats) < 4:
            feats.append(y)
        y = trunk[-1](y, residual=h)               # LR conv + long skip
        for name in self._ups:
            y = _lrelu(m[name](y, upsample2x=True))
        y = _lrelu(self.HR_conv0_new[0](y))
        y = self.HR_conv1_new[0](y)
        b_fea = self.b_fea_conv[0](g)
        xb = b_fea
        for i in range(1, 5):
            xb = getattr(self, f"b_concat_{i}")[0](getattr(self, f"b_block_{i}")(torch.cat([xb, feats[i - 1]], 1)))
        xb = self.b_LR_conv[0](xb, residual=b_fea)
        xb = self.b_module(xb)
        f = self.f_concat[0](self.f_block(torch.cat([xb, y], 1)))
        return self.f_HR_conv1[0](_lrelu(self.f_HR_conv0[0](f)))


class _SepConv(nn.Module):
    def __init__(self, cin, cout, k, padding, bias=True):
        super().__init__()
        self.depthwise = nn.Conv2d(cin, cin, k, padding=padding, groups=cin, bias=bias)
        self.pointwise = Conv2d(cin, cout, 1, bias=bias)

    def forward(self, x):
        return self.pointwise(self.depthwise(x))


class _SwiftConvBlock(nn.Module):
    def __init__(self, cin, cout, use_act=True, use_bn=True, k=3, padding=1):
        super().__init__()
        self.use_act = use_act
        self.cnn = _SepConv(cin, cout, k, padding, bias=not use_bn)
        self.bn = nn.BatchNorm2d(cout) if use_bn else nn.Identity()
        self.act = nn.PReLU(num_parameters=cout)

    def forward(self, x):
        y = self.bn(self.cnn(x))
        return self.act(y) if self.use_act else y


class SwiftSRGAN(nn.Module):
    """Swift-SRGAN generator (depthwise-separable convs, BN, PReLU, pixel-shuffle x2 stages;
    chaiNNer SwiftSRGAN.py, state dict under ``model``)."""

    def __init__(self, state_dict):
        super().__init__()
        sd = state_dict["model"] if "model" in state_dict else state_dict
        self.model_arch = "Swift-SRGAN"
        self.in_nc = sd["initial.cnn.depthwise.weight"].shape[0]
        self.out_nc = sd["final_conv.pointwise.weight"].shape[0]
        nf = self.num_filters = sd["initial.cnn.pointwise.weight"].shape[0]
        self.num_blocks = len({k.split(".")[1] for k in sd if k.startswith("residual.")})
        n_up = len({k.split(".")[1] for k in sd if k.startswith("upsampler.")})
        self.scale = 2 ** n_up
        self.initial = _SwiftConvBlock(self.in_nc, nf, use_bn=False, k=9, padding=4)
        self.residual = nn.Sequential(*[nn.Module() for _ in range(self.num_blocks)])
        for i in range(self.num_blocks):
            self.residual[i].block1 = _SwiftConvBlock(nf, nf)
            self.residual[i].block2 = _SwiftConvBlock(nf, nf, use_act=False)
        self.convblock = _SwiftConvBlock(nf, nf, use_act=False)
        self.upsampler = nn.Sequential(*[nn.Module() for _ in range(n_up)])
        for i in range(n_up):
            self.upsampler[i].conv = _SepConv(nf, nf * 4, 3, 1)
            self.upsampler[i].ps = nn.PixelShuffle(2)
            self.upsampler[i].act = nn.PReLU(num_parameters=nf)
        self.final_conv = _SepConv(nf, self.in_nc, 9, 4)
        self.load_state_dict(sd, strict=False)
        self.eval()

    def forward(self, x):
        init = self.initial(x)
        h = init
        for r in self.residual:
            h = r.block2(r.block1(h)) + h
        h = self.convblock(h) + init
        for u in self.upsampler:
            h = u.act(u.ps(u.conv(h)))
        return (torch.tanh(self.final_conv(h)) + 1) / 2


def _probe(keys: set, state_dict: dict):
    """(name, constructor) of the architecture whose signature keys are present — the
    reference's dispatch order (model_loading.py:38-95); None means "try ESRGAN"."""
    from . import dat, face, lama, omnisr, swin_sr
    if "body.0.weight" in keys and "body.1.weight" in keys:
        return "RealESRGAN-Compact", SRVGGNetCompact
    if "f_HR_conv1.0.weight" in keys:
        return "SPSR", SPSRNet
    if "model" in keys and isinstance(state_dict["model"], dict) and "initial.cnn.depthwise.weight" in state_dict["model"]:
        return "Swift-SRGAN", SwiftSRGAN
    if "layers.0.residual_group.blocks.0.norm1.weight" in keys:
        if "layers.0.residual_group.blocks.0.conv_block.cab.0.weight" in keys:
            return "HAT", swin_sr.HAT
        if "patch_embed.proj.weight" in keys:
            return "Swin2SR", lambda sd: swin_sr.SwinIR(sd, v2=True)
        return "SwinIR", swin_sr.SwinIR
    if "toRGB.0.weight" in keys and "stylegan_decoder.style_mlp.1.weight" in keys:
        return "GFPGAN", face.GFPGANv1Clean
    if "encoder.conv_in.weight" in keys and "encoder.down.0.block.0.norm1.weight" in keys:
        return "RestoreFormer", face.RestoreFormer
    if "encoder.blocks.0.weight" in keys and "quantize.embedding.weight" in keys:
        return "CodeFormer", face.CodeFormer
    if "model.model.1.bn_l.running_mean" in keys or "generator.model.1.bn_l.running_mean" in keys:
        return "LaMa", lama.LaMa
    if "residual_layer.0.residual_layer.0.layer.0.fn.0.weight" in keys:
        return "OmniSR", omnisr.OmniSR
    if "m_head.0.weight" in keys and "m_tail.0.weight" in keys:
        return "SCUNet", swin_sr.SCUNet
    if "layers.0.blocks.2.attn.attn_mask_0" in keys:
        return "DAT", dat.DAT
    return None


def load_state_dict(state_dict) -> nn.Module:
    """Architecture dispatch by key probes, in the reference's order. A recognised family whose
    file is malformed (missing / mis-shaped tensors) raises ``UnsupportedModel`` naming it."""
    for wrap in ("params_ema", "params-ema", "params"):
        if wrap in state_dict and isinstance(state_dict[wrap], dict):
            state_dict = state_dict[wrap]
            break
    keys = set(state_dict.keys())
    hit = _probe(keys, state_dict)
    if hit is not None:
        name, ctor = hit
        try:
            return ctor(state_dict)
        except (KeyError, ValueError, RuntimeError, IndexError) as e:
            raise UnsupportedModel(f"malformed {name} upscale model: {e!r}") from e
    try:
        return RRDBNet(state_dict)
    except UnsupportedModel:
        raise
    except Exception as e:     # anything else that is not a loadable ESRGAN
        raise UnsupportedModel(str(e)) from e
