"""GLIGEN box-grounded generation (parity: ``comfy/gligen.py:1-343``).

Grounding tokens (text embedding + Fourier-encoded box) from ``PositionNet`` are mixed into every
transformer block through gated self-attention over [visual tokens ; grounding tokens], installed
as the sampler's ``middle_patch`` (between attn1 and attn2 of each BasicTransformerBlock, indexed
by ``transformer_index``). The gated blocks reuse the UNet's CrossAttention / FeedForward modules,
so their attention and GEGLU run on the same HIP kernels.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from .attention import CrossAttention, FeedForward
from .layers import LayerNorm, Linear


class GatedCrossAttentionDense(nn.Module):
    def __init__(self, query_dim, context_dim, n_heads, d_head):
        super().__init__()
        self.attn = CrossAttention(query_dim=query_dim, context_dim=context_dim, heads=n_heads, dim_head=d_head)
        self.ff = FeedForward(query_dim, glu=True)
        self.norm1 = LayerNorm(query_dim)
        self.norm2 = LayerNorm(query_dim)
        self.alpha_attn = nn.Parameter(torch.tensor(0.0), requires_grad=False)
        self.alpha_dense = nn.Parameter(torch.tensor(0.0), requires_grad=False)
        self.scale = 1

    def forward(self, x, objs):
        x = x + self.scale * torch.tanh(self.alpha_attn) * self.attn(self.norm1(x), objs, objs)
        return x + self.scale * torch.tanh(self.alpha_dense) * self.ff(self.norm2(x))


class GatedSelfAttentionDense(nn.Module):
    def __init__(self, query_dim, context_dim, n_heads, d_head):
        super().__init__()
        self.linear = Linear(context_dim, query_dim)
        self.attn = CrossAttention(query_dim=query_dim, context_dim=query_dim, heads=n_heads, dim_head=d_head)
        self.ff = FeedForward(query_dim, glu=True)
        self.norm1 = LayerNorm(query_dim)
        self.norm2 = LayerNorm(query_dim)
        self.alpha_attn = nn.Parameter(torch.tensor(0.0), requires_grad=False)
        self.alpha_dense = nn.Parameter(torch.tensor(0.0), requires_grad=False)
        self.scale = 1

    def forward(self, x, objs):
        nv = x.shape[1]
        objs = self.linear(objs)
        a = self.attn(self.norm1(torch.cat([x, objs], dim=1)))[:, :nv, :]
        x = x + self.scale * torch.tanh(self.alpha_attn).to(x.dtype) * a
        return x + self.scale * torch.tanh(self.alpha_dense).to(x.dtype) * self.ff(self.norm2(x))


class GatedSelfAttentionDense2(GatedSelfAttentionDense):
    """Variant whose residual is the grounding-token output resized to the visual grid."""

    def forward(self, x, objs):
        B, nv, _ = x.shape
        ng = objs.shape[1]
        objs = self.linear(objs)
        sv, sg = math.isqrt(nv), math.isqrt(ng)
        assert sv * sv == nv and sg * sg == ng, "visual / grounding tokens must be square"
        out = self.attn(self.norm1(torch.cat([x, objs], dim=1)))[:, nv:, :]
        out = torch.nn.functional.interpolate(out.permute(0, 2, 1).reshape(B, -1, sg, sg), (sv, sv), mode="bicubic")
        x = x + self.scale * torch.tanh(self.alpha_attn) * out.reshape(B, -1, nv).permute(0, 2, 1)
        return x + self.scale * torch.tanh(self.alpha_dense) * self.ff(self.norm2(x))


class FourierEmbedder:
    def __init__(self, num_freqs=64, temperature=100):
        self.num_freqs = num_freqs
        self.freq_bands = temperature ** (torch.arange(num_freqs) / num_freqs)

    @torch.no_grad()
    def __call__(self, x):
        """[..., 4] -> [..., F*2*4] ordered (freq, sin|cos, coordinate)."""
        f = self.freq_bands.to(x.device, x.dtype)
        a = x[..., None] * f                                       # [..., 4, F]
        out = torch.stack([torch.sin(a), torch.cos(a)], dim=-1)    # [..., 4, F, 2]
        nd = out.ndim
        return out.permute(*range(nd - 3), nd - 2, nd - 1, nd - 3).reshape(*x.shape[:-1], -1)


class PositionNet(nn.Module):
    def __init__(self, in_dim, out_dim, fourier_freqs=8):
        super().__init__()
        self.in_dim = in_dim
        self.out_dim = out_dim
        self.fourier_embedder = FourierEmbedder(num_freqs=fourier_freqs)
        self.position_dim = fourier_freqs * 2 * 4
        self.linears = nn.Sequential(Linear(in_dim + self.position_dim, 512), nn.SiLU(), Linear(512, 512), nn.SiLU(),
                                     Linear(512, out_dim))
        self.null_positive_feature = nn.Parameter(torch.zeros([in_dim]), requires_grad=False)
        self.null_position_feature = nn.Parameter(torch.zeros([self.position_dim]), requires_grad=False)

    def forward(self, boxes, masks, positive_embeddings):
        B, N, _ = boxes.shape
        m = masks.unsqueeze(-1)
        xyxy = self.fourier_embedder(boxes)
        pnull = self.null_positive_feature.to(boxes).view(1, 1, -1)
        xnull = self.null_position_feature.to(boxes).view(1, 1, -1)
        pe = positive_embeddings * m + (1 - m) * pnull
        xyxy = xyxy * m + (1 - m) * xnull
        objs = self.linears(torch.cat([pe, xyxy], dim=-1))
        assert objs.shape == (B, N, self.out_dim)
        return objs


class Gligen(nn.Module):
    max_objs = 30

    def __init__(self, modules, position_net, key_dim):
        super().__init__()
        self.module_list = nn.ModuleList(modules)
        self.position_net = position_net
        self.key_dim = key_dim

    def _set_position(self, boxes, masks, positive_embeddings):
        objs = self.position_net(boxes, masks, positive_embeddings)

        def func(x, extra_options):
            return self.module_list[extra_options["transformer_index"]](x, objs.to(device=x.device, dtype=x.dtype))
        return func

    def set_position(self, latent_image_shape, position_params, device):
        """Memoised per (shape, boxes, phrase embeddings, device): the host-built box / mask tensors and
        the position-net output are made once (eagerly), so a captured sampler step (run_graph.py) reads
        device tensors only -- no host-to-device copy inside the capture."""
        key = (tuple(latent_image_shape), str(device),
               tuple((id(p[0]),) + tuple(float(v) for v in p[1:]) for p in position_params))
        cache = self.__dict__.setdefault("_pos_cache", {})
        hit = cache.get(key)
        if hit is not None:
            return hit[1]
        func = self._build_position(latent_image_shape, position_params, device)
        if len(cache) >= 16:
            cache.pop(next(iter(cache)))
        # the entry holds the embeddings: their ids in the key cannot be reused while it lives
        cache[key] = ([p[0] for p in position_params], func)
        return func

    def _build_position(self, latent_image_shape, position_params, device):
        batch, _, h, w = latent_image_shape
        masks = torch.zeros([self.max_objs])
        boxes, embs = [], []
        for p in position_params:                 # (embedding, height, width, y, x) in latent units
            x1, y1 = p[4] / w, p[3] / h
            x2, y2 = (p[4] + p[2]) / w, (p[3] + p[1]) / h
            masks[len(boxes)] = 1.0
            boxes.append(torch.tensor((x1, y1, x2, y2))[None])
            embs.append(p[0])
        pad = self.max_objs - len(boxes)
        if pad > 0:
            boxes.append(torch.zeros([pad, 4]))
            embs.append(torch.zeros([pad, self.key_dim]))
        box = torch.cat(boxes)[None].repeat(batch, 1, 1)
        conds = torch.cat([e.reshape(-1, self.key_dim).float().cpu() for e in embs])[None].repeat(batch, 1, 1)
        return self._set_position(box.to(device), masks[None].repeat(batch, 1).to(device), conds.to(device))

    def set_empty(self, latent_image_shape, device):
        batch = latent_image_shape[0]
        return self._set_position(torch.zeros([batch, self.max_objs, 4], device=device),
                                  torch.zeros([batch, self.max_objs], device=device),
                                  torch.zeros([batch, self.max_objs, self.key_dim], device=device))


def gligen_from_state_dict(sd):
    modules = []
    key_dim = 768
    for part in ("input_blocks", "middle_block", "output_blocks"):
        for b in range(20):
            tag = f"{part}.{b}."
            n_sd = {k.split(".fuser.")[-1]: v for k, v in sd.items() if tag in k and ".fuser." in k}
            if not n_sd:
                continue
            query_dim, key_dim = n_sd["linear.weight"].shape
            if key_dim == 768:
                n_heads, d_head = 8, query_dim // 8
            else:
                d_head = min(64, query_dim)
                n_heads = query_dim // d_head
            g = GatedSelfAttentionDense(query_dim, key_dim, n_heads, d_head)
            g.load_state_dict(n_sd, strict=False)
            modules.append(g)
    pn = None
    if "position_net.null_positive_feature" in sd:
        pn = PositionNet(sd["position_net.null_positive_feature"].shape[0], sd["position_net.linears.4.weight"].shape[0])
        pn.load_state_dict({k[len("position_net."):]: v for k, v in sd.items() if k.startswith("position_net.")},
                           strict=False)
    return Gligen(modules, pn, key_dim)


def load_gligen(path_or_sd):
    """-> ModelPatcher wrapping the Gligen module (the sampler reads ``.model``)."""
    from ..runtime import device as dm
    from ..runtime.checkpoint import load_state_dict
    from ..runtime.patcher import ModelPatcher
    sd = load_state_dict(path_or_sd) if isinstance(path_or_sd, str) else path_or_sd
    model = gligen_from_state_dict(sd)
    dtype = dm.unet_dtype()
    if dtype in (torch.float16, torch.bfloat16):
        model = model.to(dtype)
    return ModelPatcher(model.eval(), load_device=dm.get_torch_device(), offload_device=dm.unet_offload_device())
