"""diffusers-layout loading (parity: ``comfy/diffusers_load.py``, ``comfy/diffusers_convert.py``,
``comfy/utils.py:186-250``).

``load_diffusers(dir)`` reads a diffusers pipeline folder (unet/ vae/ text_encoder[_2]/) and builds
the same (MODEL, CLIP, VAE) objects as a single-file checkpoint: the UNet config is derived from the
tensors (runtime.detection.unet_config_from_diffusers_unet) and keys are remapped to the ldm layout
the models use; VAE keys are renamed and its attention projections reshaped to 1x1 convs.
"""
from __future__ import annotations

import os
import re

import torch

from . import detection
from .checkpoint import load_state_dict
from .convert import unet_to_diffusers


def model_config_from_diffusers_unet(sd):
    return detection.model_config_from_diffusers_unet(sd)


def convert_unet_from_diffusers(sd, unet_config):
    """diffusers UNet state dict -> ldm ``diffusion_model`` keys (unprefixed)."""
    mapping = unet_to_diffusers(unet_config)
    out = {}
    for k, v in sd.items():
        if k in mapping:
            out[mapping[k]] = v
    return out


_VAE_RESNET = {"conv_shortcut": "nin_shortcut"}
_VAE_ATTN = {"group_norm": "norm", "query": "q", "key": "k", "value": "v", "proj_attn": "proj_out",
             "to_q": "q", "to_k": "k", "to_v": "v", "to_out.0": "proj_out"}


def convert_vae_state_dict(sd):
    """diffusers AutoencoderKL -> ldm (encoder.down.N.block.M / decoder.up.(L-1-N).block.M / mid.*)."""
    n_up = 1 + max((int(m.group(1)) for k in sd for m in [re.match(r"decoder\.up_blocks\.(\d+)\.", k)] if m),
                   default=-1)
    out = {}
    for k, v in sd.items():
        nk = k
        nk = re.sub(r"^encoder\.down_blocks\.(\d+)\.resnets\.(\d+)\.", r"encoder.down.\1.block.\2.", nk)
        nk = re.sub(r"^encoder\.down_blocks\.(\d+)\.downsamplers\.0\.conv\.", r"encoder.down.\1.downsample.conv.", nk)
        nk = re.sub(r"^decoder\.up_blocks\.(\d+)\.resnets\.(\d+)\.",
                    lambda m: f"decoder.up.{n_up - 1 - int(m.group(1))}.block.{m.group(2)}.", nk)
        nk = re.sub(r"^decoder\.up_blocks\.(\d+)\.upsamplers\.0\.conv\.",
                    lambda m: f"decoder.up.{n_up - 1 - int(m.group(1))}.upsample.conv.", nk)
        nk = re.sub(r"^(encoder|decoder)\.mid_block\.resnets\.(\d+)\.",
                    lambda m: f"{m.group(1)}.mid.block_{int(m.group(2)) + 1}.", nk)
        nk = re.sub(r"^(encoder|decoder)\.mid_block\.attentions\.0\.", r"\1.mid.attn_1.", nk)
        nk = nk.replace("conv_norm_out", "norm_out")
        for a, b in _VAE_RESNET.items():
            nk = nk.replace(f".{a}.", f".{b}.")
        if ".mid.attn_1." in nk:
            head, tail = nk.split(".mid.attn_1.", 1)
            for a, b in _VAE_ATTN.items():
                if tail.startswith(a + "."):
                    tail = b + tail[len(a):]
                    break
            nk = f"{head}.mid.attn_1.{tail}"
            if tail.split(".")[0] in ("q", "k", "v", "proj_out") and tail.endswith("weight") and v.ndim == 2:
                v = v.reshape(v.shape[0], v.shape[1], 1, 1)
        out[nk] = v
    return out


def _first_file(path, names):
    for n in names:
        p = os.path.join(path, n)
        if os.path.exists(p):
            return p
    return None


def load_diffusers(model_path, output_vae=True, output_clip=True, embedding_directory=None):
    from . import sd as sdl
    weights = ["diffusion_pytorch_model.fp16.safetensors", "diffusion_pytorch_model.safetensors",
               "diffusion_pytorch_model.fp16.bin", "diffusion_pytorch_model.bin"]
    te_names = ["model.fp16.safetensors", "model.safetensors", "pytorch_model.fp16.bin", "pytorch_model.bin"]
    unet_path = _first_file(os.path.join(model_path, "unet"), weights)
    vae_path = _first_file(os.path.join(model_path, "vae"), weights)
    te_paths = [p for p in (_first_file(os.path.join(model_path, "text_encoder"), te_names),
                            _first_file(os.path.join(model_path, "text_encoder_2"), te_names)) if p is not None]
    unet = sdl.load_unet(unet_path)
    clip = sdl.load_clip(te_paths, embedding_directory=embedding_directory) if output_clip and te_paths else None
    vae = sdl.VAE(sd=load_state_dict(vae_path)) if output_vae and vae_path else None
    return unet, clip, vae
