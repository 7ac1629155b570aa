"""State-dict -> UNet architecture inference (parity: ``comfy/model_detection.py:1-199``).

Infers channels, per-level res-block counts, transformer depths (in/out/middle), context dim,
linear-vs-conv proj, ADM channels and video/Cascade stage purely from key names and shapes, then
matches the first family in ``families.MODELS`` (``supported_models.py:479-481`` order).
"""
from __future__ import annotations

import logging


def count_blocks(keys, fmt):
    n = 0
    while any(k.startswith(fmt.format(n)) for k in keys):
        n += 1
    return n


def _transformer_depth(prefix, keys, sd):
    tp = prefix + "1.transformer_blocks."
    if not any(k.startswith(tp) for k in keys):
        return None
    depth = count_blocks(keys, tp + "{}")
    context_dim = sd[f"{tp}0.attn2.to_k.weight"].shape[1]
    use_linear = len(sd[f"{prefix}1.proj_in.weight"].shape) == 2
    time_stack = (f"{prefix}1.time_stack.0.attn1.to_q.weight" in sd or
                  f"{prefix}1.time_mix_blocks.0.attn1.to_q.weight" in sd)
    return depth, context_dim, use_linear, time_stack


def detect_unet_config(sd, key_prefix=""):
    keys = list(sd.keys())
    if f"{key_prefix}clf.1.weight" in sd:   # Stable Cascade
        cfg = {}
        tm = f"{key_prefix}clip_txt_mapper.weight"
        if tm in sd:
            cfg["stable_cascade_stage"] = "c"
            w = sd[tm]
            if w.shape[0] == 1536:
                cfg.update(c_cond=1536, c_hidden=[1536, 1536], nhead=[24, 24], blocks=[[4, 12], [12, 4]])
            elif w.shape[0] == 2048:
                cfg["c_cond"] = 2048
        elif f"{key_prefix}clip_mapper.weight" in sd:
            cfg["stable_cascade_stage"] = "b"
            w = sd[f"{key_prefix}down_blocks.1.0.channelwise.0.weight"]
            if w.shape[-1] == 640:
                cfg.update(c_hidden=[320, 640, 1280, 1280], nhead=[-1, -1, 20, 20],
                           blocks=[[2, 6, 28, 6], [6, 28, 6, 2]], block_repeat=[[1, 1, 1, 1], [3, 3, 2, 2]])
            elif w.shape[-1] == 576:
                cfg.update(c_hidden=[320, 576, 1152, 1152], nhead=[-1, 9, 18, 18],
                           blocks=[[2, 4, 14, 4], [4, 14, 4, 2]], block_repeat=[[1, 1, 1, 1], [2, 2, 2, 2]])
        return cfg

    cfg = {"use_checkpoint": False, "image_size": 32, "use_spatial_transformer": True, "legacy": False}
    y = f"{key_prefix}label_emb.0.0.weight"
    if y in sd:
        cfg["num_classes"] = "sequential"
        cfg["adm_in_channels"] = sd[y].shape[1]
    else:
        cfg["adm_in_channels"] = None
    w0 = sd[f"{key_prefix}input_blocks.0.0.weight"]
    model_channels, in_channels = w0.shape[0], w0.shape[1]
    out_channels = sd[f"{key_prefix}out.2.weight"].shape[0] if f"{key_prefix}out.2.weight" in sd else 4

    num_res_blocks, channel_mult = [], []
    transformer_depth, transformer_depth_output = [], []
    context_dim, use_linear, video = None, False, False
    last_rb, last_cm = 0, 0
    nin = count_blocks(keys, f"{key_prefix}input_blocks" + ".{}.")
    for c in range(nin):
        prefix = f"{key_prefix}input_blocks.{c}."
        prefix_out = f"{key_prefix}output_blocks.{nin - c - 1}."
        bk = [k for k in keys if k.startswith(prefix)]
        if not bk:
            break
        bko = [k for k in keys if k.startswith(prefix_out)]
        if f"{prefix}0.op.weight" in bk:
            num_res_blocks.append(last_rb)
            channel_mult.append(last_cm)
            last_rb, last_cm = 0, 0
            o = _transformer_depth(prefix_out, keys, sd)
            transformer_depth_output.append(o[0] if o else 0)
        else:
            if f"{prefix}0.in_layers.0.weight" in bk:
                last_rb += 1
                last_cm = sd[f"{prefix}0.out_layers.3.weight"].shape[0] // model_channels
                o = _transformer_depth(prefix, keys, sd)
                if o is not None:
                    transformer_depth.append(o[0])
                    if context_dim is None:
                        context_dim, use_linear, video = o[1], o[2], o[3]
                else:
                    transformer_depth.append(0)
            if f"{prefix_out}0.in_layers.0.weight" in bko:
                o = _transformer_depth(prefix_out, keys, sd)
                transformer_depth_output.append(o[0] if o else 0)
    num_res_blocks.append(last_rb)
    channel_mult.append(last_cm)
    if f"{key_prefix}middle_block.1.proj_in.weight" in sd:
        tdm = count_blocks(keys, f"{key_prefix}middle_block.1.transformer_blocks." + "{}")
    elif f"{key_prefix}middle_block.0.in_layers.0.weight" in sd:
        tdm = -1
    else:
        tdm = -2
    cfg.update(in_channels=in_channels, out_channels=out_channels, model_channels=model_channels,
               num_res_blocks=num_res_blocks, transformer_depth=transformer_depth,
               transformer_depth_output=transformer_depth_output, channel_mult=channel_mult,
               transformer_depth_middle=tdm, use_linear_in_transformer=use_linear, context_dim=context_dim,
               use_temporal_resblock=video, use_temporal_attention=video)
    if video:
        cfg.update(extra_ff_mix_layer=True, use_spatial_context=True, merge_strategy="learned_with_images",
                   merge_factor=0.0, video_kernel_size=[3, 1, 1])
    return cfg


def model_config_from_unet_config(unet_config, sd=None):
    from .families import MODELS
    for fam in MODELS:
        if fam.matches(unet_config, sd):
            return fam(unet_config)
    logging.error("no match %s", unet_config)
    return None


def model_config_from_unet(sd, unet_key_prefix, use_base_if_no_match=False):
    from .families import BASE
    cfg = detect_unet_config(sd, unet_key_prefix)
    mc = model_config_from_unet_config(cfg, sd)
    if mc is None and use_base_if_no_match:
        return BASE(cfg)
    return mc


def convert_config(unet_config):
    """Expand ``attention_resolutions`` configs (yaml/diffusers) to per-block depth lists."""
    cfg = dict(unet_config)
    nrb = cfg.get("num_res_blocks")
    cm = cfg.get("channel_mult")
    if isinstance(nrb, int):
        nrb = [nrb] * len(cm)
    if "attention_resolutions" in cfg:
        ar = cfg.pop("attention_resolutions")
        td = cfg.get("transformer_depth")
        tdm = cfg.get("transformer_depth_middle")
        if isinstance(td, int):
            td = [td] * len(cm)
        if tdm is None:
            tdm = td[-1]
        t_in, t_out, s = [], [], 1
        for i in range(len(nrb)):
            d = td[i] if s in ar else 0
            t_in += [d] * nrb[i]
            t_out += [d] * (nrb[i] + 1)
            s *= 2
        cfg.update(transformer_depth=t_in, transformer_depth_output=t_out, transformer_depth_middle=tdm)
    cfg["num_res_blocks"] = nrb
    return cfg


# ------------------------------------------------------------------------------------------------
# diffusers layout (parity: model_detection.py:240-377 — the reference matches 16 fixed templates;
# here the same config is derived from the tensors, and heads follow the ldm rule: SD1.x (context
# 768) uses 8 heads, everything else 64-wide heads)
# ------------------------------------------------------------------------------------------------
def unet_config_from_diffusers_unet(sd, dtype=None):
    keys = set(sd.keys())
    w_in = sd["conv_in.weight"]
    model_channels, in_channels = w_in.shape[0], w_in.shape[1]
    levels = count_blocks(keys, "down_blocks.{}.")
    num_res_blocks, channel_mult, transformer_depth = [], [], []
    context_dim, use_linear = None, False
    for i in range(levels):
        nrb = count_blocks(keys, f"down_blocks.{i}.resnets." + "{}.")
        num_res_blocks.append(nrb)
        channel_mult.append(sd[f"down_blocks.{i}.resnets.0.conv2.weight"].shape[0] // model_channels)
        for j in range(nrb):
            d = count_blocks(keys, f"down_blocks.{i}.attentions.{j}.transformer_blocks." + "{}.")
            transformer_depth.append(d)
            if d and context_dim is None:
                context_dim = sd[f"down_blocks.{i}.attentions.{j}.transformer_blocks.0.attn2.to_k.weight"].shape[1]
                use_linear = sd[f"down_blocks.{i}.attentions.{j}.proj_in.weight"].ndim == 2
    tdm = count_blocks(keys, "mid_block.attentions.0.transformer_blocks.{}.")
    if tdm == 0 and "mid_block.resnets.0.conv1.weight" in keys and "mid_block.attentions.0.proj_in.weight" not in keys:
        tdm = -1
    if context_dim is None and "mid_block.attentions.0.transformer_blocks.0.attn2.to_k.weight" in keys:
        context_dim = sd["mid_block.attentions.0.transformer_blocks.0.attn2.to_k.weight"].shape[1]
    transformer_depth_output = []
    for i in range(count_blocks(keys, "up_blocks.{}.")):
        for j in range(count_blocks(keys, f"up_blocks.{i}.resnets." + "{}.")):
            transformer_depth_output.append(count_blocks(keys, f"up_blocks.{i}.attentions.{j}.transformer_blocks." + "{}."))
    transformer_depth_output = transformer_depth_output[::-1] if transformer_depth_output else None
    cfg = {"use_checkpoint": False, "image_size": 32, "use_spatial_transformer": True, "legacy": False,
           "in_channels": in_channels, "model_channels": model_channels,
           "out_channels": sd["conv_out.weight"].shape[0] if "conv_out.weight" in keys else 4,
           "num_res_blocks": num_res_blocks, "channel_mult": channel_mult, "transformer_depth": transformer_depth,
           "transformer_depth_middle": tdm, "context_dim": context_dim, "use_linear_in_transformer": use_linear,
           "use_temporal_resblock": False, "use_temporal_attention": False}
    if transformer_depth_output is not None:
        cfg["transformer_depth_output"] = transformer_depth_output
    if "add_embedding.linear_1.weight" in keys:
        cfg["num_classes"] = "sequential"
        cfg["adm_in_channels"] = sd["add_embedding.linear_1.weight"].shape[1]
    elif "class_embedding.linear_1.weight" in keys:
        cfg["num_classes"] = "sequential"
        cfg["adm_in_channels"] = sd["class_embedding.linear_1.weight"].shape[1]
    else:
        cfg["adm_in_channels"] = None
    if context_dim == 768:
        cfg.update(num_heads=8, num_head_channels=-1)
    else:
        cfg.update(num_heads=-1, num_head_channels=64)
    return cfg


def model_config_from_diffusers_unet(state_dict):
    cfg = unet_config_from_diffusers_unet(state_dict)
    return model_config_from_unet_config(cfg) if cfg is not None else None
