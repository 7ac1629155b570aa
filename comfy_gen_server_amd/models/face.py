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
from . import vae as _vae          # ResnetBlock / Downsample / Upsample share the ldm key layout
from .layers import Conv2d, DerivedMixin, GroupNorm, LayerNorm, Linear


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


# ----------------------------------------------------------------------------------------------
# RestoreFormer (restoreformer_arch.py): VQGAN-style encoder -> 1024-entry codebook -> decoder
# whose 16x16 attention layers cross-attend from the encoder's features (multi-head, d=64).
# ----------------------------------------------------------------------------------------------



def _gn(c):
    return GroupNorm(32, c, eps=1e-6)


def _tokens(x):
    return x.flatten(2).transpose(1, 2)


def _image(t, like):
    B, C, H, W = like.shape
    return t.transpose(1, 2).reshape(B, C, H, W)


class _MHAttnBlock(nn.Module):
    """Multi-head (cross-)attention over the spatial positions: q from ``y`` (or ``x``), k/v from
    ``x``; the device runs it on the HIP flash-attention kernel."""

    def __init__(self, c, heads):
        super().__init__()
        self.heads = heads
        self.norm1, self.norm2 = _gn(c), _gn(c)
        self.q, self.k, self.v, self.proj_out = (Conv2d(c, c, 1) for _ in range(4))

    def forward(self, x, y=None):
        h = self.norm1(x)
        yq = h if y is None else self.norm2(y)
        o = ops.attention(_tokens(self.q(yq)), _tokens(self.k(h)), _tokens(self.v(h)), self.heads)
        return self.proj_out(_image(o, x), residual=x)


def _quantize(z, codebook):
    """Nearest codebook entry per position (z [B, C, H, W], codebook [n, C])."""
    B, C, H, W = z.shape
    q, _ = ops.vq_nearest(z.permute(0, 2, 3, 1).reshape(-1, C), codebook)
    return q.view(B, H, W, C).permute(0, 3, 1, 2)


class RestoreFormer(nn.Module):
    def __init__(self, state_dict, strict: bool = True):
        super().__init__()
        self.model_arch = "RestoreFormer"
        self.sub_type = "Face SR"
        self.scale, self.in_nc, self.out_nc = 8, 3, 3
        ch, mult, nrb, heads, z = 64, (1, 2, 2, 4, 4, 8), 2, 8, 256
        self.nrb = nrb
        enc = nn.Module()
        enc.conv_in = Conv2d(3, ch, 3, padding=1)
        enc.down = nn.ModuleList()
        res, cin = 512, ch
        for i, m in enumerate(mult):
            lvl = nn.Module()
            lvl.block, lvl.attn = nn.ModuleList(), nn.ModuleList()
            for _ in range(nrb):
                lvl.block.append(_vae.ResnetBlock(cin, ch * m))
                cin = ch * m
                if res == 16:
                    lvl.attn.append(_MHAttnBlock(cin, heads))
            if i != len(mult) - 1:
                lvl.downsample = _vae.Downsample(cin)
                res //= 2
            enc.down.append(lvl)
        enc.mid = nn.Module()
        enc.mid.block_1, enc.mid.attn_1, enc.mid.block_2 = (_vae.ResnetBlock(cin), _MHAttnBlock(cin, heads),
                                                            _vae.ResnetBlock(cin))
        enc.norm_out = _gn(cin)
        enc.conv_out = Conv2d(cin, z, 3, padding=1)
        self.encoder = enc
        dec = nn.Module()
        dec.conv_in = Conv2d(z, cin, 3, padding=1)
        dec.mid = nn.Module()
        dec.mid.block_1, dec.mid.attn_1, dec.mid.block_2 = (_vae.ResnetBlock(cin), _MHAttnBlock(cin, heads),
                                                            _vae.ResnetBlock(cin))
        ups = []
        res = 16
        for i in reversed(range(len(mult))):
            lvl = nn.Module()
            lvl.block, lvl.attn = nn.ModuleList(), nn.ModuleList()
            for _ in range(nrb + 1):
                lvl.block.append(_vae.ResnetBlock(cin, ch * mult[i]))
                cin = ch * mult[i]
                if res == 16:
                    lvl.attn.append(_MHAttnBlock(cin, heads))
            if i != 0:
                lvl.upsample = _vae.Upsample(cin)
                res *= 2
            ups.insert(0, lvl)
        dec.up = nn.ModuleList(ups)
        dec.norm_out = _gn(cin)
        dec.conv_out = Conv2d(cin, 3, 3, padding=1)
        self.decoder = dec
        self.quantize = nn.Module()
        self.quantize.embedding = nn.Embedding(1024, 256)
        self.quant_conv = Conv2d(z, 256, 1)
        self.post_quant_conv = Conv2d(256, z, 1)
        for p in self.parameters():
            p.requires_grad_(False)
        missing, _ = self.load_state_dict(state_dict, strict=False)
        if missing and strict:
            raise ValueError(f"RestoreFormer: missing keys {missing[:4]}")
        self.eval()

    def forward(self, x, **_):
        e, hs = self.encoder, {}
        h = e.conv_in(x)
        last = len(e.down) - 1
        for i, lvl in enumerate(e.down):
            for j in range(self.nrb):
                h = lvl.block[j](h)
                if len(lvl.attn):
                    h = lvl.attn[j](h)
            if i != last:
                h = lvl.downsample(h)
        h = e.mid.block_1(h)
        hs_block = h                                   # "block_{last}_atten"
        h = e.mid.block_2(e.mid.attn_1(h))
        hs_mid = h                                     # "mid_atten"
        h = e.conv_out(e.norm_out(h, silu=True))
        q = _quantize(self.quant_conv(h), self.quantize.embedding.weight)
        d = self.decoder
        h = d.conv_in(self.post_quant_conv(q))
        h = d.mid.block_2(d.mid.attn_1(d.mid.block_1(h), hs_mid))
        for i in reversed(range(len(d.up))):
            lvl = d.up[i]
            for j in range(self.nrb + 1):
                h = lvl.block[j](h)
                if len(lvl.attn):
                    h = lvl.attn[j](h, hs_block)
            if i != 0:
                h = lvl.upsample(h)
        return d.conv_out(d.norm_out(h, silu=True)), None


# ----------------------------------------------------------------------------------------------
# CodeFormer (codeformer.py): VQGAN encoder -> 9-layer transformer predicting codebook indices
# from the low-quality latent -> AdaIN-matched codebook features -> generator with
# controllable-fidelity SFT fusion of encoder features at 32..256 px.
# ----------------------------------------------------------------------------------------------


class _CFResBlock(nn.Module):
    def __init__(self, cin, cout=None):
        super().__init__()
        cout = cout or cin
        self.norm1, self.conv1 = _gn(cin), Conv2d(cin, cout, 3, padding=1)
        self.norm2, self.conv2 = _gn(cout), Conv2d(cout, cout, 3, padding=1)
        self.conv_out = Conv2d(cin, cout, 1) if cin != cout else None

    def forward(self, x):
        h = self.conv1(self.norm1(x, silu=True))
        skip = x if self.conv_out is None else self.conv_out(x)
        return self.conv2(self.norm2(h, silu=True), residual=skip)


class _CFAttn(nn.Module):
    """Single-head spatial self-attention (d = C = 512 at 16x16: the wide-head HIP kernel)."""

    def __init__(self, c):
        super().__init__()
        self.norm = _gn(c)
        self.q, self.k, self.v, self.proj_out = (Conv2d(c, c, 1) for _ in range(4))

    def forward(self, x):
        h = self.norm(x)
        o = ops.attention(_tokens(self.q(h)), _tokens(self.k(h)), _tokens(self.v(h)), 1)
        return self.proj_out(_image(o, x), residual=x)


def _vq_blocks(nf, mult, nrb, emb_dim, encoder: bool):
    blocks: list = []
    if encoder:
        res, cin = 512, nf
        blocks.append(Conv2d(3, nf, 3, padding=1))
        for i, m in enumerate(mult):
            for _ in range(nrb):
                blocks.append(_CFResBlock(cin, nf * m))
                cin = nf * m
                if res == 16:
                    blocks.append(_CFAttn(cin))
            if i != len(mult) - 1:
                blocks.append(_vae.Downsample(cin))
                res //= 2
        blocks += [_CFResBlock(cin), _CFAttn(cin), _CFResBlock(cin), _gn(cin), Conv2d(cin, emb_dim, 3, padding=1)]
    else:
        cin, res = nf * mult[-1], 512 // 2 ** (len(mult) - 1)
        blocks += [Conv2d(emb_dim, cin, 3, padding=1), _CFResBlock(cin), _CFAttn(cin), _CFResBlock(cin)]
        for i in reversed(range(len(mult))):
            for _ in range(nrb):
                blocks.append(_CFResBlock(cin, nf * mult[i]))
                cin = nf * mult[i]
                if res == 16:
                    blocks.append(_CFAttn(cin))
            if i != 0:
                blocks.append(_vae.Upsample(cin))
                res *= 2
        blocks += [_gn(cin), Conv2d(cin, 3, 3, padding=1)]
    m = nn.Module()
    m.blocks = nn.ModuleList(blocks)
    return m


class _SALayer(nn.Module):
    """Pre-norm transformer layer; the attention keeps ``nn.MultiheadAttention``'s packed
    ``in_proj`` weights (keys ``self_attn.in_proj_weight`` / ``out_proj``)."""

    def __init__(self, dim, heads, mlp):
        super().__init__()
        self.heads = heads
        self.self_attn = nn.Module()
        self.self_attn.in_proj_weight = nn.Parameter(torch.empty(3 * dim, dim), requires_grad=False)
        self.self_attn.in_proj_bias = nn.Parameter(torch.empty(3 * dim), requires_grad=False)
        self.self_attn.out_proj = Linear(dim, dim)
        self.linear1, self.linear2 = Linear(dim, mlp), Linear(mlp, dim)
        self.norm1, self.norm2 = LayerNorm(dim), LayerNorm(dim)

    def forward(self, t, pos):                           # t [B, S, D] (batch-first)
        D = t.shape[-1]
        w, b = self.self_attn.in_proj_weight.to(t.dtype), self.self_attn.in_proj_bias.to(t.dtype)
        h = self.norm1(t)
        qk = ops.linear(h + pos, w[:2 * D], b[:2 * D])       # q and k share their input: one GEMM
        v = ops.linear(h, w[2 * D:], b[2 * D:])
        a = ops.attention(qk[..., :D], qk[..., D:], v, self.heads)
        t = self.self_attn.out_proj(a, residual=t)
        return self.linear2(F.gelu(self.linear1(self.norm2(t))), residual=t)


def _mean_std(f, eps=1e-5):
    b, c = f.shape[:2]
    v = f.float().reshape(b, c, -1)
    return v.mean(2).view(b, c, 1, 1), (v.var(2) + eps).sqrt().view(b, c, 1, 1)


def _adain(content, style):
    cm, cs = _mean_std(content)
    sm, ss = _mean_std(style)
    return ((content.float() - cm) / cs * ss + sm).to(content.dtype)


class _FuseSFT(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.encode_enc = _CFResBlock(2 * c, c)
        self.scale = nn.Sequential(Conv2d(c, c, 3, padding=1), nn.LeakyReLU(0.2), Conv2d(c, c, 3, padding=1))
        self.shift = nn.Sequential(Conv2d(c, c, 3, padding=1), nn.LeakyReLU(0.2), Conv2d(c, c, 3, padding=1))

    def forward(self, enc, dec, w):
        e = self.encode_enc(torch.cat([enc, dec], 1))
        return dec + w * (dec * self.scale(e) + self.shift(e))


class CodeFormer(nn.Module):
    _ENC_TAP = {"512": 2, "256": 5, "128": 8, "64": 11, "32": 14, "16": 18}
    _GEN_TAP = {"16": 6, "32": 9, "64": 12, "128": 15, "256": 18, "512": 21}
    _CONNECT = ("32", "64", "128", "256")
    _CH = {"16": 512, "32": 256, "64": 256, "128": 128, "256": 128, "512": 64}

    def __init__(self, state_dict, strict: bool = True):
        super().__init__()
        sd = state_dict
        self.model_arch = "CodeFormer"
        self.sub_type = "Face SR"
        self.scale = 8
        dim = sd["position_emb"].shape[1] if "position_emb" in sd else 512
        latent = sd["position_emb"].shape[0] if "position_emb" in sd else 256
        n_layers = len({k.split(".")[1] for k in sd if k.startswith("ft_layers.")}) or 9
        n_code = sd["quantize.embedding.weight"].shape[0] if "quantize.embedding.weight" in sd else 1024
        self.in_nc = self.out_nc = sd["encoder.blocks.0.weight"].shape[1] if "encoder.blocks.0.weight" in sd else 3
        mult = (1, 2, 2, 4, 4, 8)
        self.encoder = _vq_blocks(64, mult, 2, 256, encoder=True)
        self.quantize = nn.Module()
        self.quantize.embedding = nn.Embedding(n_code, 256)
        self.generator = _vq_blocks(64, mult, 2, 256, encoder=False)
        self.position_emb = nn.Parameter(torch.zeros(latent, dim), requires_grad=False)
        self.feat_emb = Linear(256, dim)
        self.ft_layers = nn.Sequential(*[_SALayer(dim, 8, dim * 2) for _ in range(n_layers)])
        self.idx_pred_layer = nn.Sequential(LayerNorm(dim), Linear(dim, n_code, bias=False))
        self.fuse_convs_dict = nn.ModuleDict({s: _FuseSFT(self._CH[s]) for s in self._CONNECT})
        for p in self.parameters():
            p.requires_grad_(False)
        missing, _ = self.load_state_dict(sd, strict=False)
        if missing and strict:
            raise ValueError(f"CodeFormer: missing keys {missing[:4]}")
        self.eval()

    def forward(self, x, weight=0.5, **_):
        taps = {self._ENC_TAP[s] for s in self._CONNECT}
        enc = {}
        for i, blk in enumerate(self.encoder.blocks):
            x = blk(x)
            if i in taps:
                enc[str(x.shape[-1])] = x
        lq = x
        B = x.shape[0]
        t = self.feat_emb(_tokens(lq))
        pos = self.position_emb.to(t.dtype)[None]
        for layer in self.ft_layers:
            t = layer(t, pos)
        logits = self.idx_pred_layer(t)                               # [B, hw, n_code]
        idx = logits.float().argmax(-1)                               # top-1 of the softmax
        side = int(math.isqrt(t.shape[1]))
        q = self.quantize.embedding.weight[idx].to(lq.dtype).view(B, side, side, -1).permute(0, 3, 1, 2)
        x = _adain(q, lq)
        fuse_at = {self._GEN_TAP[s] for s in self._CONNECT}
        for i, blk in enumerate(self.generator.blocks):
            x = blk(x)
            if i in fuse_at and weight > 0:
                s = str(x.shape[-1])
                x = self.fuse_convs_dict[s](enc[s], x, weight)
        return x, logits
