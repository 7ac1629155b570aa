"""CLIP text (and vision) transformers.

Behavioural parity with ``comfy/clip_model.py:1-194`` (CLIPAttention/MLP/Layer/Encoder/Embeddings,
CLIPTextModel with intermediate-layer output + final-layer-norm option, pooled = hidden at the
argmax token, text_projection; CLIPVisionModelProjection). Internal keys follow the HF
transformers layout (``text_model.encoder.layers.N.self_attn.q_proj`` ...); OpenCLIP checkpoints
(SD2 / SDXL-G / Cascade) are converted at load time by ``runtime/convert.py``.

Device path: q/k/v one fused GEMM, causal flash attention kernel, residual adds fused into the
out_proj / fc2 GEMM epilogues. Latency-bound (M = 77 x prompts) — batch every prompt of a job
into one call.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import ops
from .layers import DerivedMixin, Embedding, LayerNorm, Linear, Conv2d


ACTS = {
    "quick_gelu": lambda x: x * torch.sigmoid(1.702 * x),
    "gelu": lambda x: torch.nn.functional.gelu(x),
    "gelu_pytorch_tanh": lambda x: torch.nn.functional.gelu(x, approximate="tanh"),
}


class CLIPAttention(nn.Module, DerivedMixin):
    def __init__(self, embed_dim, heads, dtype=None, device=None):
        super().__init__()
        self.heads = heads
        kw = dict(dtype=dtype, device=device)
        self.q_proj = Linear(embed_dim, embed_dim, True, **kw)
        self.k_proj = Linear(embed_dim, embed_dim, True, **kw)
        self.v_proj = Linear(embed_dim, embed_dim, True, **kw)
        self.out_proj = Linear(embed_dim, embed_dim, True, **kw)

    def forward(self, x, causal=True, mask=None, residual=None):
        C = x.shape[-1]
        if x.dtype == self.q_proj.weight.dtype and x.device == self.q_proj.weight.device:
            w = self._derived_get("w", lambda: torch.cat([self.q_proj.weight, self.k_proj.weight, self.v_proj.weight], 0))
            b = self._derived_get("b", lambda: torch.cat([self.q_proj.bias, self.k_proj.bias, self.v_proj.bias], 0))
            qkv = ops.linear(x, w, b)
            q, k, v = qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:]
        else:
            q, k, v = self.q_proj(x), self.k_proj(x), self.v_proj(x)
        o = ops.attention(q, k, v, self.heads, mask=mask, causal=causal)
        return self.out_proj(o, residual=residual)


class CLIPMLP(nn.Module):
    def __init__(self, embed_dim, intermediate, activation, dtype=None, device=None):
        super().__init__()
        self.fc1 = Linear(embed_dim, intermediate, True, dtype=dtype, device=device)
        self.act = ACTS[activation]
        self.fc2 = Linear(intermediate, embed_dim, True, dtype=dtype, device=device)

    def forward(self, x, residual=None):
        return self.fc2(self.act(self.fc1(x)), residual=residual)


class CLIPLayer(nn.Module):
    def __init__(self, embed_dim, heads, intermediate, activation, dtype=None, device=None):
        super().__init__()
        kw = dict(dtype=dtype, device=device)
        self.layer_norm1 = LayerNorm(embed_dim, **kw)
        self.self_attn = CLIPAttention(embed_dim, heads, **kw)
        self.layer_norm2 = LayerNorm(embed_dim, **kw)
        self.mlp = CLIPMLP(embed_dim, intermediate, activation, **kw)

    def forward(self, x, causal=True, mask=None):
        x = self.self_attn(self.layer_norm1(x), causal=causal, mask=mask, residual=x)
        return self.mlp(self.layer_norm2(x), residual=x)


class CLIPEncoder(nn.Module):
    def __init__(self, num_layers, embed_dim, heads, intermediate, activation, dtype=None, device=None):
        super().__init__()
        self.layers = nn.ModuleList([CLIPLayer(embed_dim, heads, intermediate, activation, dtype=dtype, device=device)
                                     for _ in range(num_layers)])

    def forward(self, x, causal=True, mask=None, intermediate_output=None):
        if intermediate_output is not None and intermediate_output < 0:
            intermediate_output = len(self.layers) + intermediate_output
        inter = None
        for i, layer in enumerate(self.layers):
            x = layer(x, causal=causal, mask=mask)
            if i == intermediate_output:
                inter = x.clone()
        return x, inter


class CLIPEmbeddings(nn.Module):
    def __init__(self, embed_dim, vocab_size=49408, num_positions=77, dtype=None, device=None):
        super().__init__()
        self.token_embedding = Embedding(vocab_size, embed_dim, dtype=dtype, device=device)
        self.position_embedding = Embedding(num_positions, embed_dim, dtype=dtype, device=device)

    def forward(self, tokens, embeds=None):
        tw, pw = self.token_embedding.weight, self.position_embedding.weight
        if embeds is None and tokens.device == tw.device and tw.dtype == pw.dtype:
            return ops.clip_embed(tokens, tw, pw)          # gather + position add, one kernel (K26)
        x = self.token_embedding(tokens) if embeds is None else embeds
        return x + pw[: x.shape[1]].to(x.dtype)


class CLIPTextModel_(nn.Module):
    def __init__(self, cfg, dtype=None, device=None):
        super().__init__()
        kw = dict(dtype=dtype, device=device)
        self.embeddings = CLIPEmbeddings(cfg["hidden_size"], cfg.get("vocab_size", 49408),
                                         cfg.get("max_position_embeddings", 77), **kw)
        self.encoder = CLIPEncoder(cfg["num_hidden_layers"], cfg["hidden_size"], cfg["num_attention_heads"],
                                   cfg["intermediate_size"], cfg["hidden_act"], **kw)
        self.final_layer_norm = LayerNorm(cfg["hidden_size"], **kw)

    def forward(self, tokens, embeds=None, intermediate_output=None, final_layer_norm_intermediate=True):
        x = self.embeddings(tokens, embeds)
        x, inter = self.encoder(x, causal=True, intermediate_output=intermediate_output)
        x = self.final_layer_norm(x)
        if inter is not None and final_layer_norm_intermediate:
            inter = self.final_layer_norm(inter)
        pooled = ops.pooled_gather(x, tokens)             # hidden state at the end-of-text token (K26)
        return x, inter, pooled


class CLIPTextModel(nn.Module):
    """HF-compatible: keys ``text_model.*`` and ``text_projection.weight``."""

    def __init__(self, cfg, dtype=None, device=None):
        super().__init__()
        self.cfg = dict(cfg)
        self.num_layers = cfg["num_hidden_layers"]
        self.text_model = CLIPTextModel_(cfg, dtype=dtype, device=device)
        pd = cfg.get("projection_dim", cfg["hidden_size"])
        self.text_projection = Linear(cfg["hidden_size"], pd, bias=False, dtype=dtype, device=device)
        self.dtype = dtype

    def get_input_embeddings(self):
        return self.text_model.embeddings.token_embedding

    def forward(self, tokens, embeds=None, intermediate_output=None, final_layer_norm_intermediate=True):
        x, inter, pooled = self.text_model(tokens, embeds, intermediate_output, final_layer_norm_intermediate)
        proj = self.text_projection(pooled)
        return x, inter, proj, pooled


# ------------------------------------------------------------------------------------------------
# Vision tower (CLIPVisionModelProjection, clip_model.py:139-194)
# ------------------------------------------------------------------------------------------------
class CLIPVisionEmbeddings(nn.Module):
    def __init__(self, embed_dim, num_channels=3, patch_size=14, image_size=224, dtype=None, device=None):
        super().__init__()
        self.class_embedding = nn.Parameter(torch.empty(embed_dim, dtype=dtype, device=device), requires_grad=False)
        self.patch_embedding = Conv2d(num_channels, embed_dim, patch_size, stride=patch_size, bias=False,
                                      dtype=dtype, device=device)
        n = (image_size // patch_size) ** 2 + 1
        self.position_embedding = Embedding(n, embed_dim, dtype=dtype, device=device)

    def forward(self, px):
        e = self.patch_embedding(px).flatten(2).transpose(1, 2)
        cls = self.class_embedding.to(e.dtype).expand(e.shape[0], 1, -1)
        return torch.cat([cls, e], dim=1) + self.position_embedding.weight.to(e.dtype)


class CLIPVision(nn.Module):
    def __init__(self, cfg, dtype=None, device=None):
        super().__init__()
        kw = dict(dtype=dtype, device=device)
        self.embeddings = CLIPVisionEmbeddings(cfg["hidden_size"], cfg.get("num_channels", 3),
                                               cfg["patch_size"], cfg["image_size"], **kw)
        self.pre_layrnorm = LayerNorm(cfg["hidden_size"], **kw)
        self.encoder = CLIPEncoder(cfg["num_hidden_layers"], cfg["hidden_size"], cfg["num_attention_heads"],
                                   cfg["intermediate_size"], cfg["hidden_act"], **kw)
        self.post_layernorm = LayerNorm(cfg["hidden_size"], **kw)

    def forward(self, px, intermediate_output=None):
        x = self.pre_layrnorm(self.embeddings(px))
        x, inter = self.encoder(x, causal=False, intermediate_output=intermediate_output)
        pooled = self.post_layernorm(x[:, 0, :])
        return x, inter, pooled


class CLIPVisionModelProjection(nn.Module):
    def __init__(self, cfg, dtype=None, device=None):
        super().__init__()
        self.vision_model = CLIPVision(cfg, dtype=dtype, device=device)
        self.visual_projection = Linear(cfg["hidden_size"], cfg["projection_dim"], bias=False, dtype=dtype, device=device)

    def forward(self, px, intermediate_output=None):
        x, inter, pooled = self.vision_model(px, intermediate_output)
        return x, inter, self.visual_projection(pooled)


CLIP_L_CONFIG = dict(hidden_size=768, intermediate_size=3072, num_attention_heads=12, num_hidden_layers=12,
                     hidden_act="quick_gelu", projection_dim=768, vocab_size=49408, max_position_embeddings=77)
CLIP_H_CONFIG = dict(hidden_size=1024, intermediate_size=4096, num_attention_heads=16, num_hidden_layers=24,
                     hidden_act="gelu", projection_dim=1024, vocab_size=49408, max_position_embeddings=77)
CLIP_G_CONFIG = dict(hidden_size=1280, intermediate_size=5120, num_attention_heads=20, num_hidden_layers=32,
                     hidden_act="gelu", projection_dim=1280, vocab_size=49408, max_position_embeddings=77)
CLIP_VISION_H = dict(hidden_size=1280, intermediate_size=5120, num_attention_heads=16, num_hidden_layers=32,
                     hidden_act="gelu", projection_dim=1024, patch_size=14, image_size=224)
CLIP_VISION_G = dict(hidden_size=1664, intermediate_size=8192, num_attention_heads=16, num_hidden_layers=48,
                     hidden_act="gelu", projection_dim=1280, patch_size=14, image_size=224)
CLIP_VISION_L = dict(hidden_size=1024, intermediate_size=4096, num_attention_heads=16, num_hidden_layers=24,
                     hidden_act="quick_gelu", projection_dim=768, patch_size=14, image_size=224)
