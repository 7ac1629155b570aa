"""LoRA / LyCORIS file parsing and key maps (parity: ``comfy/lora.py:1-241``).

Supported adapter families (each -> one patch tuple per target weight):
  lora   (kohya ``.lora_up/.lora_down[/.lora_mid]``, diffusers ``_lora.up/down``,
          transformers ``.lora_linear_layer.up/down``) + ``alpha`` + DoRA ``dora_scale``
  loha   (``hada_w1_a/b, hada_w2_a/b[, hada_t1/t2]``)
  lokr   (``lokr_w1[_a/_b], lokr_w2[_a/_b][, lokr_t2]``)
  glora  (``a1/a2/b1/b2``)
  diff   (``.diff``, ``.diff_b``, ``.w_norm``/``.b_norm``)
Key maps cover ldm names, kohya ``lora_unet_*`` / ``lora_te{,1,2}_*`` / Cascade ``lora_prior_*``,
and diffusers/PEFT names derived from ``convert.unet_to_diffusers``.
"""
from __future__ import annotations

import logging

from .convert import unet_to_diffusers

LORA_CLIP_MAP = {
    "mlp.fc1": "mlp_fc1",
    "mlp.fc2": "mlp_fc2",
    "self_attn.k_proj": "self_attn_k_proj",
    "self_attn.q_proj": "self_attn_q_proj",
    "self_attn.v_proj": "self_attn_v_proj",
    "self_attn.out_proj": "self_attn_out_proj",
}

# (up, down, mid) name templates for the three LoRA spellings
_LORA_FORMS = (
    ("{}.lora_up.weight", "{}.lora_down.weight", "{}.lora_mid.weight"),
    ("{}_lora.up.weight", "{}_lora.down.weight", None),
    ("{}.lora_linear_layer.up.weight", "{}.lora_linear_layer.down.weight", None),
)


def load_lora(lora: dict, to_load: dict) -> dict:
    """lora: adapter state dict; to_load: adapter key prefix -> model weight key. -> patch dict."""
    patches = {}
    used = set()

    def take(name):
        if name is not None and name in lora:
            used.add(name)
            return lora[name]
        return None

    for x, target in to_load.items():
        alpha_t = take(f"{x}.alpha")
        alpha = alpha_t.item() if alpha_t is not None else None
        dora = take(f"{x}.dora_scale")
        for up_n, down_n, mid_n in _LORA_FORMS:
            up_k = up_n.format(x)
            if up_k in lora:
                up = take(up_k)
                down = take(down_n.format(x))
                mid = take(mid_n.format(x)) if mid_n else None
                patches[target] = ("lora", (up, down, alpha, mid, dora))
                break
        w1a = take(f"{x}.hada_w1_a")
        if w1a is not None:
            t1 = take(f"{x}.hada_t1")
            t2 = take(f"{x}.hada_t2")
            patches[target] = ("loha", (w1a, take(f"{x}.hada_w1_b"), alpha, take(f"{x}.hada_w2_a"),
                                        take(f"{x}.hada_w2_b"), t1, t2, dora))
        lk = {n: take(f"{x}.lokr_{n}") for n in ("w1", "w2", "w1_a", "w1_b", "w2_a", "w2_b", "t2")}
        if any(lk[n] is not None for n in ("w1", "w2", "w1_a", "w2_a")):
            patches[target] = ("lokr", (lk["w1"], lk["w2"], alpha, lk["w1_a"], lk["w1_b"], lk["w2_a"],
                                        lk["w2_b"], lk["t2"], dora))
        a1 = take(f"{x}.a1.weight")
        if a1 is not None:
            patches[target] = ("glora", (a1, take(f"{x}.a2.weight"), take(f"{x}.b1.weight"),
                                         take(f"{x}.b2.weight"), alpha, dora))
        bias_target = target[: -len(".weight")] + ".bias" if target.endswith(".weight") else None
        wn = take(f"{x}.w_norm")
        if wn is not None:
            patches[target] = ("diff", (wn,))
            bn = take(f"{x}.b_norm")
            if bn is not None and bias_target:
                patches[bias_target] = ("diff", (bn,))
        d = take(f"{x}.diff")
        if d is not None:
            patches[target] = ("diff", (d,))
        db = take(f"{x}.diff_b")
        if db is not None and bias_target:
            patches[bias_target] = ("diff", (db,))
    for k in lora:
        if k not in used:
            logging.warning("lora key not loaded: %s", k)
    return patches


def model_lora_keys_clip(model, key_map=None):
    key_map = {} if key_map is None else key_map
    sdk = set(model.state_dict().keys())
    clip_l_present = False
    for b in range(48):
        for c, short in LORA_CLIP_MAP.items():
            kh = f"clip_h.transformer.text_model.encoder.layers.{b}.{c}.weight"
            if kh in sdk:
                key_map[f"lora_te_text_model_encoder_layers_{b}_{short}"] = kh
                key_map[f"lora_te1_text_model_encoder_layers_{b}_{short}"] = kh
                key_map[f"text_encoder.text_model.encoder.layers.{b}.{c}"] = kh
            kl = f"clip_l.transformer.text_model.encoder.layers.{b}.{c}.weight"
            if kl in sdk:
                key_map[f"lora_te_text_model_encoder_layers_{b}_{short}"] = kl
                key_map[f"lora_te1_text_model_encoder_layers_{b}_{short}"] = kl
                key_map[f"text_encoder.text_model.encoder.layers.{b}.{c}"] = kl
                clip_l_present = True
            kg = f"clip_g.transformer.text_model.encoder.layers.{b}.{c}.weight"
            if kg in sdk:
                if clip_l_present:
                    key_map[f"lora_te2_text_model_encoder_layers_{b}_{short}"] = kg
                    key_map[f"text_encoder_2.text_model.encoder.layers.{b}.{c}"] = kg
                else:
                    key_map[f"lora_te_text_model_encoder_layers_{b}_{short}"] = kg
                    key_map[f"text_encoder.text_model.encoder.layers.{b}.{c}"] = kg
                    key_map[f"lora_prior_te_text_model_encoder_layers_{b}_{short}"] = kg
    if "clip_g.transformer.text_projection.weight" in sdk:
        key_map["lora_prior_te_text_projection"] = "clip_g.transformer.text_projection.weight"
    return key_map


def model_lora_keys_unet(model, key_map=None):
    key_map = {} if key_map is None else key_map
    for k in model.state_dict().keys():
        if k.startswith("diffusion_model.") and k.endswith(".weight"):
            kl = k[len("diffusion_model."):-len(".weight")].replace(".", "_")
            key_map[f"lora_unet_{kl}"] = k
            key_map[f"lora_prior_unet_{kl}"] = k
    dk = unet_to_diffusers(model.model_config.unet_config)
    for k, v in dk.items():
        if not k.endswith(".weight"):
            continue
        unet_key = f"diffusion_model.{v}"
        key_map["lora_unet_" + k[:-len(".weight")].replace(".", "_")] = unet_key
        for p in ("", "unet."):
            dl = p + k[:-len(".weight")].replace(".to_", ".processor.to_")
            if dl.endswith(".to_out.0"):
                dl = dl[:-2]
            key_map[dl] = unet_key
    return key_map
