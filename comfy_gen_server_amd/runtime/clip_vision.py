"""CLIP vision encoder wrapper (parity: ``comfy/clip_vision.py:1-117``, ``clip_model.py:139-194``).

``encode_image`` = 224² bicubic-antialias resize + center crop + 8-bit quantise + normalise, then the
ViT tower on the device (its attention / GEMMs / LayerNorms are the HIP ops), returning an Output
with ``last_hidden_state``, ``image_embeds`` (projected pooled token) and
``penultimate_hidden_states``. Checkpoints in OpenCLIP layout (``visual.transformer.resblocks``)
are converted to the HF layout on load; the ViT size (L/H/G) is detected from the layer count.
"""
from __future__ import annotations

import logging

import torch

from ..models.clip import CLIP_VISION_G, CLIP_VISION_H, CLIP_VISION_L, CLIPVisionModelProjection
from . import device as dm
from .checkpoint import load_state_dict
from .convert import _OPENCLIP_LAYER, state_dict_prefix_replace
from .patcher import ModelPatcher

CLIP_MEAN = (0.48145466, 0.4578275, 0.40821073)
CLIP_STD = (0.26862954, 0.26130258, 0.27577711)


class Output:
    def __getitem__(self, key):
        return getattr(self, key)

    def __setitem__(self, key, item):
        setattr(self, key, item)


def clip_preprocess(image, size=224):
    """IMAGE [B,H,W,C] 0..1 -> normalised [B,3,size,size]."""
    mean = torch.tensor(CLIP_MEAN, device=image.device, dtype=image.dtype).view(3, 1, 1)
    std = torch.tensor(CLIP_STD, device=image.device, dtype=image.dtype).view(3, 1, 1)
    x = image.movedim(-1, 1)[:, :3]
    if not (x.shape[2] == size and x.shape[3] == size):
        scale = size / min(x.shape[2], x.shape[3])
        x = torch.nn.functional.interpolate(x, size=(round(scale * x.shape[2]), round(scale * x.shape[3])),
                                            mode="bicubic", antialias=True)
        h = (x.shape[2] - size) // 2
        w = (x.shape[3] - size) // 2
        x = x[:, :, h:h + size, w:w + size]
    x = torch.clip(255.0 * x, 0, 255).round() / 255.0
    return (x - mean) / std


class ClipVisionModel:
    def __init__(self, config):
        self.config = dict(config)
        self.load_device = dm.text_encoder_device()
        offload = dm.text_encoder_offload_device()
        self.dtype = dm.text_encoder_dtype(self.load_device)
        with torch.device("meta"):
            self.model = CLIPVisionModelProjection(self.config, dtype=self.dtype, device=torch.device("meta"))
        self.model.to_empty(device=offload)
        self.model.eval()
        self.patcher = ModelPatcher(self.model, load_device=self.load_device, offload_device=offload)

    def load_sd(self, sd):
        return self.model.load_state_dict(sd, strict=False, assign=False)

    def get_sd(self):
        return self.model.state_dict()

    def encode_image(self, image):
        dm.load_model_gpu(self.patcher)
        px = clip_preprocess(image.to(self.load_device).float()).to(self.dtype)
        with torch.inference_mode():
            x, inter, embeds = self.model(px, intermediate_output=-2)
        out = Output()
        dev = dm.intermediate_device()
        out["last_hidden_state"] = x.float().to(dev)
        out["image_embeds"] = embeds.float().to(dev)
        out["penultimate_hidden_states"] = inter.float().to(dev)
        return out


def convert_to_transformers(sd, prefix):
    """OpenCLIP visual tower (``{prefix}transformer.resblocks.N``) -> HF ``vision_model.*`` keys."""
    if f"{prefix}transformer.resblocks.0.attn.in_proj_weight" not in sd:
        return state_dict_prefix_replace(sd, {prefix: ""})
    ren = {f"{prefix}class_embedding": "vision_model.embeddings.class_embedding",
           f"{prefix}conv1.weight": "vision_model.embeddings.patch_embedding.weight",
           f"{prefix}positional_embedding": "vision_model.embeddings.position_embedding.weight",
           f"{prefix}ln_post.bias": "vision_model.post_layernorm.bias",
           f"{prefix}ln_post.weight": "vision_model.post_layernorm.weight",
           f"{prefix}ln_pre.bias": "vision_model.pre_layrnorm.bias",
           f"{prefix}ln_pre.weight": "vision_model.pre_layrnorm.weight"}
    for a, b in ren.items():
        if a in sd:
            sd[b] = sd.pop(a)
    if f"{prefix}proj" in sd:
        sd["visual_projection.weight"] = sd.pop(f"{prefix}proj").transpose(0, 1).contiguous()
    rb = f"{prefix}transformer.resblocks."
    n_layers = 1 + max(int(k[len(rb):].split(".")[0]) for k in sd if k.startswith(rb))
    for i in range(n_layers):
        src = f"{prefix}transformer.resblocks.{i}."
        dst = f"vision_model.encoder.layers.{i}."
        for a, b in _OPENCLIP_LAYER.items():
            for s in ("weight", "bias"):
                if f"{src}{a}.{s}" in sd:
                    sd[f"{dst}{b}.{s}"] = sd.pop(f"{src}{a}.{s}")
        for s in ("weight", "bias"):
            k = f"{src}attn.in_proj_{s}"
            if k in sd:
                w = sd.pop(k)
                n = w.shape[0] // 3
                for j, nm in enumerate(("q_proj", "k_proj", "v_proj")):
                    sd[f"{dst}self_attn.{nm}.{s}"] = w[j * n:(j + 1) * n]
    return sd


def config_for(sd):
    if "vision_model.encoder.layers.47.layer_norm1.weight" in sd:
        return CLIP_VISION_G
    if "vision_model.encoder.layers.30.layer_norm1.weight" in sd:
        return CLIP_VISION_H
    if "vision_model.encoder.layers.22.layer_norm1.weight" in sd:
        return CLIP_VISION_L
    return None


def load_clipvision_from_sd(sd, prefix="", convert_keys=False):
    if convert_keys:
        sd = convert_to_transformers(sd, prefix)
    cfg = config_for(sd)
    if cfg is None:
        return None
    cv = ClipVisionModel(cfg)
    missing, unexpected = cv.load_sd(sd)
    if missing:
        logging.warning("missing clip vision keys: %s", missing)
    used = set(cv.model.state_dict().keys())
    for k in [k for k in sd if k in used]:
        sd.pop(k)
    return cv


def load(ckpt_path):
    sd = load_state_dict(ckpt_path)
    if "visual.transformer.resblocks.0.attn.in_proj_weight" in sd:
        return load_clipvision_from_sd(sd, prefix="visual.", convert_keys=True)
    return load_clipvision_from_sd(sd)
