"""State-dict key utilities and format conversions.

Parity with ``comfy/utils.py:45-250`` (state_dict_prefix_replace, state_dict_key_replace,
transformers_convert / clip_text_transformers_convert for OpenCLIP -> HF CLIP keys,
unet_to_diffusers map) and the text-encoder part of ``comfy/diffusers_convert.py``
(HF -> OpenCLIP for saving).
"""
from __future__ import annotations

import torch


def state_dict_prefix_replace(sd, replace_prefix, filter_keys=False):
    out = {} if filter_keys else sd
    for rp, new in replace_prefix.items():
        for k in [k for k in list(sd.keys()) if k.startswith(rp)]:
            out[new + k[len(rp):]] = sd.pop(k)
    return out


def state_dict_key_replace(sd, keys_to_replace):
    for k, v in keys_to_replace.items():
        if k in sd:
            sd[v] = sd.pop(k)
    return sd


_OPENCLIP_LAYER = {
    "ln_1": "layer_norm1",
    "ln_2": "layer_norm2",
    "mlp.c_fc": "mlp.fc1",
    "mlp.c_proj": "mlp.fc2",
    "attn.out_proj": "self_attn.out_proj",
}


def openclip_to_hf(sd, prefix_from, prefix_to, num_layers=None):
    """Convert an OpenCLIP text tower (``{pf}transformer.resblocks.N...``) to HF CLIPTextModel keys
    under ``{pt}text_model...``. Operates in place on ``sd``; returns sd."""
    pf = prefix_from
    tm = prefix_to + "text_model."
    if num_layers is None:
        num_layers = 0
        while f"{pf}transformer.resblocks.{num_layers}.ln_1.weight" in sd:
            num_layers += 1
    for i in range(num_layers):
        src = f"{pf}transformer.resblocks.{i}."
        dst = f"{tm}encoder.layers.{i}."
        for a, b in _OPENCLIP_LAYER.items():
            for s in ("weight", "bias"):
                k = f"{src}{a}.{s}"
                if k in sd:
                    sd[f"{dst}{b}.{s}"] = sd.pop(k)
        for s in ("weight", "bias"):
            k = f"{src}attn.in_proj_{s}"
            if k in sd:
                w = sd.pop(k)
                n = w.shape[0] // 3
                for j, nm in enumerate(("q_proj", "k_proj", "v_proj")):
                    sd[f"{dst}self_attn.{nm}.{s}"] = w[j * n:(j + 1) * n]
    ren = {
        f"{pf}token_embedding.weight": f"{tm}embeddings.token_embedding.weight",
        f"{pf}positional_embedding": f"{tm}embeddings.position_embedding.weight",
        f"{pf}ln_final.weight": f"{tm}final_layer_norm.weight",
        f"{pf}ln_final.bias": f"{tm}final_layer_norm.bias",
    }
    for a, b in ren.items():
        if a in sd:
            sd[b] = sd.pop(a)
    if f"{pf}text_projection" in sd:
        sd[f"{prefix_to}text_projection.weight"] = sd.pop(f"{pf}text_projection").transpose(0, 1).contiguous()
    sd.pop(f"{pf}logit_scale", None)
    return sd


def hf_to_openclip(sd, prefix_from, prefix_to):
    """Inverse of ``openclip_to_hf`` (used by CheckpointSave for SDXL / SD2 G/H towers)."""
    out = {}
    tm = prefix_from + "transformer.text_model."
    inv = {v: k for k, v in _OPENCLIP_LAYER.items()}
    i = 0
    while f"{tm}encoder.layers.{i}.layer_norm1.weight" in sd:
        src = f"{tm}encoder.layers.{i}."
        dst = f"{prefix_to}transformer.resblocks.{i}."
        for b, a in inv.items():
            for s in ("weight", "bias"):
                k = f"{src}{b}.{s}"
                if k in sd:
                    out[f"{dst}{a}.{s}"] = sd[k]
        for s in ("weight", "bias"):
            parts = [sd.get(f"{src}self_attn.{n}.{s}") for n in ("q_proj", "k_proj", "v_proj")]
            if all(p is not None for p in parts):
                out[f"{dst}attn.in_proj_{s}"] = torch.cat(parts, 0)
        i += 1
    ren = {
        f"{tm}embeddings.token_embedding.weight": f"{prefix_to}token_embedding.weight",
        f"{tm}embeddings.position_embedding.weight": f"{prefix_to}positional_embedding",
        f"{tm}final_layer_norm.weight": f"{prefix_to}ln_final.weight",
        f"{tm}final_layer_norm.bias": f"{prefix_to}ln_final.bias",
    }
    for a, b in ren.items():
        if a in sd:
            out[b] = sd[a]
    tp = f"{prefix_from}transformer.text_projection.weight"
    if tp in sd:
        out[f"{prefix_to}text_projection"] = sd[tp].transpose(0, 1).contiguous()
    return out


def convert_sd_to(sd, dtype):
    return {k: (v.to(dtype) if torch.is_tensor(v) and v.is_floating_point() else v) for k, v in sd.items()}


# ------------------------------------------------------------------------------------------------
# UNet ldm <-> diffusers key map (utils.py:186-250) — used by LoRA key maps and diffusers loading
# ------------------------------------------------------------------------------------------------
UNET_MAP_ATTENTIONS = {"proj_in.weight", "proj_in.bias", "proj_out.weight", "proj_out.bias",
                       "norm.weight", "norm.bias"}
TRANSFORMER_BLOCKS = {"norm1.weight", "norm1.bias", "norm2.weight", "norm2.bias", "norm3.weight", "norm3.bias",
                      "attn1.to_q.weight", "attn1.to_k.weight", "attn1.to_v.weight", "attn1.to_out.0.weight",
                      "attn1.to_out.0.bias", "attn2.to_q.weight", "attn2.to_k.weight", "attn2.to_v.weight",
                      "attn2.to_out.0.weight", "attn2.to_out.0.bias", "ff.net.0.proj.weight", "ff.net.0.proj.bias",
                      "ff.net.2.weight", "ff.net.2.bias"}
UNET_MAP_RESNET = {"in_layers.2.weight": "conv1.weight", "in_layers.2.bias": "conv1.bias",
                   "emb_layers.1.weight": "time_emb_proj.weight", "emb_layers.1.bias": "time_emb_proj.bias",
                   "out_layers.3.weight": "conv2.weight", "out_layers.3.bias": "conv2.bias",
                   "skip_connection.weight": "conv_shortcut.weight", "skip_connection.bias": "conv_shortcut.bias",
                   "in_layers.0.weight": "norm1.weight", "in_layers.0.bias": "norm1.bias",
                   "out_layers.0.weight": "norm2.weight", "out_layers.0.bias": "norm2.bias"}
UNET_MAP_BASIC = {("label_emb.0.0.weight", "class_embedding.linear_1.weight"),
                  ("label_emb.0.0.bias", "class_embedding.linear_1.bias"),
                  ("label_emb.0.2.weight", "class_embedding.linear_2.weight"),
                  ("label_emb.0.2.bias", "class_embedding.linear_2.bias"),
                  ("label_emb.0.0.weight", "add_embedding.linear_1.weight"),
                  ("label_emb.0.0.bias", "add_embedding.linear_1.bias"),
                  ("label_emb.0.2.weight", "add_embedding.linear_2.weight"),
                  ("label_emb.0.2.bias", "add_embedding.linear_2.bias"),
                  ("input_blocks.0.0.weight", "conv_in.weight"), ("input_blocks.0.0.bias", "conv_in.bias"),
                  ("out.0.weight", "conv_norm_out.weight"), ("out.0.bias", "conv_norm_out.bias"),
                  ("out.2.weight", "conv_out.weight"), ("out.2.bias", "conv_out.bias"),
                  ("time_embed.0.weight", "time_embedding.linear_1.weight"),
                  ("time_embed.0.bias", "time_embedding.linear_1.bias"),
                  ("time_embed.2.weight", "time_embedding.linear_2.weight"),
                  ("time_embed.2.bias", "time_embedding.linear_2.bias")}


def unet_to_diffusers(unet_config):
    """diffusers key -> ldm key map for a UNet config (utils.unet_to_diffusers semantics)."""
    if "num_res_blocks" not in unet_config:
        return {}
    nrb = unet_config["num_res_blocks"]
    cm = unet_config["channel_mult"]
    td = list(unet_config["transformer_depth"])
    tdo = list(unet_config["transformer_depth_output"])
    nb = len(cm)
    tpl = lambda l: l if isinstance(l, list) else [l] * nb  # noqa: E731
    nrb = tpl(nrb)
    out = {}
    for x in range(nb):
        n = 1 + (nrb[x] + 1) * x
        for i in range(nrb[x]):
            for b in UNET_MAP_RESNET:
                out[f"down_blocks.{x}.resnets.{i}.{UNET_MAP_RESNET[b]}"] = f"input_blocks.{n}.0.{b}"
            num_t = td.pop(0) if td else 0
            if num_t > 0:
                for b in UNET_MAP_ATTENTIONS:
                    out[f"down_blocks.{x}.attentions.{i}.{b}"] = f"input_blocks.{n}.1.{b}"
                for t in range(num_t):
                    for b in TRANSFORMER_BLOCKS:
                        out[f"down_blocks.{x}.attentions.{i}.transformer_blocks.{t}.{b}"] = \
                            f"input_blocks.{n}.1.transformer_blocks.{t}.{b}"
            n += 1
        for k in ["weight", "bias"]:
            out[f"down_blocks.{x}.downsamplers.0.conv.{k}"] = f"input_blocks.{n}.0.op.{k}"
    i = 0
    for b in UNET_MAP_ATTENTIONS:
        out[f"mid_block.attentions.{i}.{b}"] = f"middle_block.1.{b}"
    for t in range(unet_config.get("transformer_depth_middle", 0) or 0):
        for b in TRANSFORMER_BLOCKS:
            out[f"mid_block.attentions.{i}.transformer_blocks.{t}.{b}"] = f"middle_block.1.transformer_blocks.{t}.{b}"
    for i, n in enumerate([0, 2]):
        for b in UNET_MAP_RESNET:
            out[f"mid_block.resnets.{i}.{UNET_MAP_RESNET[b]}"] = f"middle_block.{n}.{b}"
    nrb_r = list(reversed(nrb))
    for x in range(nb):
        n = (nrb_r[x] + 1) * x
        length = nrb_r[x] + 1
        for i in range(length):
            c = 0
            for b in UNET_MAP_RESNET:
                out[f"up_blocks.{x}.resnets.{i}.{UNET_MAP_RESNET[b]}"] = f"output_blocks.{n}.0.{b}"
            c += 1
            num_t = tdo.pop() if tdo else 0
            if num_t > 0:
                c += 1
                for b in UNET_MAP_ATTENTIONS:
                    out[f"up_blocks.{x}.attentions.{i}.{b}"] = f"output_blocks.{n}.1.{b}"
                for t in range(num_t):
                    for b in TRANSFORMER_BLOCKS:
                        out[f"up_blocks.{x}.attentions.{i}.transformer_blocks.{t}.{b}"] = \
                            f"output_blocks.{n}.1.transformer_blocks.{t}.{b}"
            if i == length - 1:
                for k in ["weight", "bias"]:
                    out[f"up_blocks.{x}.upsamplers.0.conv.{k}"] = f"output_blocks.{n}.{c}.conv.{k}"
            n += 1
    for a, b in UNET_MAP_BASIC:
        out[b] = a
    return out
