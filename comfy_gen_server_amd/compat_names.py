"""Reference-named adapters for the custom-node import surface (``compat.install()``).

``compat`` maps ``comfy.*`` / ``nodes`` / ``execution`` / ... onto this package's modules. The names
below are the public top-level names of the reference modules that have no same-named object in the
module an alias points at: each is either our implementation under its reference name, a thin
adapter with the reference signature, or (``ALLOWED_MISSING``) deliberately absent with a reason.
``tests/test_custom_nodes_compat.py`` parses the reference modules and checks that every public name
resolves or is listed.

Nothing here copies reference code: helpers re-state the documented behaviour of the reference
functions (cited per name) on top of our kernels and modules.
"""
from __future__ import annotations

import math
import os
import threading

import torch

# ------------------------------------------------------------------------------------------------
# names a custom node cannot get from us, and why
# ------------------------------------------------------------------------------------------------
ALLOWED_MISSING = {
    "comfy.ldm.cascade.stage_a": {
        "Discriminator": "Stage A GAN discriminator: training only (SURVEY C55), never on an inference path",
    },
    "comfy.ldm.modules.diffusionmodules.model": {
        "Model": "the original LDM DDPM network of model.py; no ComfyUI code path instantiates it "
                 "(the VAE uses Encoder / Decoder, which we provide)",
    },
    "comfy.diffusers_convert": {
        n: "string-rewrite table of the reference's diffusers converter; our converter is config-driven "
           "(runtime/convert.unet_to_diffusers) and the public convert_* functions are provided"
        for n in ("unet_conversion_map", "unet_conversion_map_resnet", "unet_conversion_map_layer",
                  "hf_mid_atn_prefix", "sd_mid_atn_prefix", "vae_conversion_map", "vae_conversion_map_attn",
                  "textenc_conversion_lst", "protected", "textenc_pattern", "code2idx")
    },
    "comfy.extra_samplers.uni_pc": {
        n: "internal class / function of the reference's UniPC solver; the public entry points "
           "sample_unipc / sample_unipc_bh2 are provided (sampling/uni_pc.py, k-diffusion sigma form)"
        for n in ("NoiseScheduleVP", "model_wrapper", "UniPC", "SigmaConvert", "predict_eps_sigma")
    },
    "execution": {
        n: "internal step of the reference's recursive executor; ours is a different (iterative, "
           "demand-driven) executor behind the same PromptExecutor / validate_prompt / PromptQueue API"
        for n in ("InputData", "MapNodeOverListInput", "GetOutputDataInput", "ValidateInputsInput",
                  "recursive_execute", "recursive_will_execute", "recursive_output_delete_if_changed")
    },
}


def _ref_attention(q, k, v, heads, mask=None, attn_precision=None, skip_reshape=False, **_):
    """``attention_basic`` / ``optimized_attention`` signature (``comfy/ldm/modules/attention.py:88``,
    ``:352-383``): q/k/v [B, S, heads*D] (or [B, heads, S, D] with ``skip_reshape``) -> [B, Sq, heads*D],
    on the HIP flash kernel (fp32 softmax)."""
    from . import ops
    if skip_reshape:
        b, h, sq, d = q.shape
        q, k, v = (t.transpose(1, 2).reshape(b, t.shape[2], h * d) for t in (q, k, v))
    if mask is not None and mask.dtype == torch.bool:
        mask = torch.zeros(mask.shape, dtype=q.dtype, device=q.device).masked_fill_(~mask, -torch.finfo(q.dtype).max)
    if mask is not None and mask.dim() == 2:
        mask = mask.unsqueeze(0)
    return ops.attention(q, k, v, heads, mask=mask)


def _vae_attention(q, k, v):
    """Single-head spatial attention of the VAE mid block (``model.py:188-279``): q/k/v [B, C, H, W]."""
    from . import ops
    b, c, h, w = q.shape
    flat = [t.reshape(b, c, h * w).transpose(1, 2) for t in (q, k, v)]
    o = ops.attention(flat[0], flat[1], flat[2], 1)
    return o.transpose(1, 2).reshape(b, c, h, w)


def _set_attr(obj, attr, value):
    parts = attr.split(".")
    for a in parts[:-1]:
        obj = getattr(obj, a)
    prev = getattr(obj, parts[-1])
    setattr(obj, parts[-1], value)
    return prev


def _get_attr(obj, attr):
    for a in attr.split("."):
        obj = getattr(obj, a)
    return obj


def _parse_parentheses(string):
    from .models.text_encoders import split_parentheses
    return split_parentheses(string)


def _token_weights(string, current_weight):
    from .models.text_encoders import weighted_segments
    return weighted_segments(string, current_weight)


def _lcm(a, b):
    return abs(a * b) // math.gcd(a, b) if a and b else 0


def _expand_dims(v, dims):
    return v[(...,) + (None,) * (dims - 1)]


def _interpolate_fn(x, xp, yp):
    """Piecewise-linear f(x) through (xp, yp) per row, extrapolating linearly (``uni_pc.py:interpolate_fn``):
    x [N, C], xp / yp [C, K]."""
    n, k = x.shape[0], xp.shape[1]
    all_x = torch.cat([x.unsqueeze(2), xp.unsqueeze(0).repeat((n, 1, 1))], dim=2)
    sorted_x, idx = torch.sort(all_x, dim=2)
    x_idx = torch.argmin(idx, dim=2)
    cand = x_idx - 1
    start = torch.where(x_idx == 0, torch.tensor(1, device=x.device),
                        torch.where(x_idx == k, torch.tensor(k - 2, device=x.device), cand))
    end = torch.where(start == cand, start + 2, start + 1)
    sx = torch.gather(sorted_x, 2, start.unsqueeze(2)).squeeze(2)
    ex = torch.gather(sorted_x, 2, end.unsqueeze(2)).squeeze(2)
    start2 = torch.where(x_idx == 0, torch.tensor(0, device=x.device),
                         torch.where(x_idx == k, torch.tensor(k - 2, device=x.device), cand))
    yexp = yp.unsqueeze(0).expand(n, -1, -1)
    sy = torch.gather(yexp, 2, start2.unsqueeze(2)).squeeze(2)
    ey = torch.gather(yexp, 2, (start2 + 1).unsqueeze(2)).squeeze(2)
    return sy + (x - sx) * (ey - sy) / (ex - sx)


def _first_file(path, filenames):
    for f in filenames:
        p = os.path.join(path, f)
        if os.path.exists(p):
            return p
    return None


def _get_timestep_embedding(timesteps, embedding_dim):
    """Sinusoidal embedding [sin | cos] of ``model.py:get_timestep_embedding`` (DDPM order)."""
    half = embedding_dim // 2
    freqs = torch.exp(-math.log(10000) * torch.arange(half, dtype=torch.float32, device=timesteps.device) / (half - 1))
    emb = timesteps.float()[:, None] * freqs[None, :]
    emb = torch.cat([torch.sin(emb), torch.cos(emb)], dim=1)
    if embedding_dim % 2 == 1:
        emb = torch.nn.functional.pad(emb, (0, 1, 0, 0))
    return emb


def _vector_quantize(x, codebook):
    """Nearest-codebook quantisation (``stage_a.py:vector_quantize``): x [N, D], codebook [K, D] ->
    (codebook rows [N, D], indices [N]) on the HIP VQ kernel (K31)."""
    from . import ops
    q, idx = ops.vq_nearest(x, codebook)
    return q, idx


def extra_names(alias: str) -> dict:
    """Reference-named objects for ``alias`` (built on first import of the alias)."""
    fn = _BUILDERS.get(alias)
    return fn() if fn is not None else {}


# ------------------------------------------------------------------------------------------------
# per-alias builders
# ------------------------------------------------------------------------------------------------
def _b_attention():
    from .models import unet
    from .models.layers import GroupNorm
    return {
        "exists": lambda val: val is not None,
        "uniq": lambda arr: {el: True for el in arr}.keys(),
        "default": lambda val, d: val if val is not None else d,
        "max_neg_value": lambda t: -torch.finfo(t.dtype).max,
        "init_": lambda t: t.uniform_(-1 / math.sqrt(t.shape[-1]), 1 / math.sqrt(t.shape[-1])),
        "Normalize": lambda in_channels, dtype=None, device=None: GroupNorm(32, in_channels, eps=1e-6, dtype=dtype,
                                                                             device=device),
        "attention_basic": _ref_attention, "attention_sub_quad": _ref_attention, "attention_split": _ref_attention,
        "attention_xformers": _ref_attention, "attention_pytorch": _ref_attention,
        "optimized_attention": _ref_attention, "optimized_attention_masked": _ref_attention,
        "optimized_attention_for_device": lambda device, mask=False, small_input=False: _ref_attention,
        "BROKEN_XFORMERS": False,
        "SpatialVideoTransformer": unet.SpatialVideoTransformer,
    }


def _b_vae_model():
    from .models import vae
    from .models.layers import GroupNorm

    def make_attn(in_channels, attn_type="vanilla", attn_kwargs=None):
        return vae.AttnBlock(in_channels)
    return {
        "get_timestep_embedding": _get_timestep_embedding,
        "nonlinearity": lambda x: x * torch.sigmoid(x),
        "Normalize": lambda in_channels, num_groups=32: GroupNorm(num_groups, in_channels, eps=1e-6),
        "slice_attention": lambda q, k, v: _vae_attention(q, k, v),
        "normal_attention": _vae_attention, "xformers_attention": _vae_attention,
        "pytorch_attention": _vae_attention, "make_attn": make_attn,
    }


def _b_openaimodel():
    from .models import unet

    class TimestepBlock(torch.nn.Module):
        """Marker base of modules whose forward takes (x, emb) (``openaimodel.py:21``)."""

        def forward(self, x, emb):  # pragma: no cover - abstract
            raise NotImplementedError

    class Timestep(torch.nn.Module):
        def __init__(self, dim):
            super().__init__()
            self.dim = dim

        def forward(self, t):
            from . import ops
            return ops.timestep_embedding(t, self.dim)

    def forward_timestep_embed(ts, x, emb, context=None, transformer_options=None, output_shape=None,
                               time_context=None, num_video_frames=None, image_only_indicator=None):
        """Run one ``TimestepEmbedSequential`` block (``openaimodel.py:33``)."""
        transformer_options = transformer_options if transformer_options is not None else {}
        kw = {}
        if output_shape is not None:
            kw["output_shape"] = output_shape
        if isinstance(ts, unet.TimestepEmbedSequential):
            # our ResBlocks take SiLU(emb) (computed once per forward instead of once per block)
            emb_silu = None if emb is None else torch.nn.functional.silu(emb)
            return ts(x, emb_silu, context, transformer_options, time_context=time_context,
                      num_video_frames=num_video_frames, image_only_indicator=image_only_indicator, **kw)
        return ts(x)
    return {"TimestepBlock": TimestepBlock, "Timestep": Timestep,
            "forward_timestep_embed": forward_timestep_embed,
            "apply_control": lambda h, control, name: unet._apply_control(h, control, name)}


def _b_model_management():
    from .runtime import device as dm
    from .cli_args import args
    free = dm.get_total_memory(dm.get_torch_device()) if dm.cpu_state == dm.CPUState.GPU else 0

    def is_device_type(device, type):
        return getattr(device, "type", None) == type

    def supports_dtype(device, dtype):
        return dtype in (torch.float32, torch.float16, torch.bfloat16) if getattr(device, "type", "") == "cuda" \
            else dtype in (torch.float32, torch.bfloat16)

    def should_use_fp16(device=None, model_params=0, prioritize_performance=True, manual_cast=False):
        return dm._fp16_on_device("unet") if hasattr(dm, "_fp16_on_device") else False

    def should_use_bf16(device=None, model_params=0, prioritize_performance=True, manual_cast=False):
        return device is None or getattr(device, "type", "cuda") == "cuda"

    def unload_model_clones(model, unload_weights_only=True, force_unload=True):
        """Drop resident models sharing ``model``'s weights (``model_management.py:324``)."""
        same = [m for m in dm.loaded_models() if getattr(m, "model", None) is getattr(model, "model", object())
                and m is not model]
        for m in same:
            dm.free_memory(0, dm.get_torch_device(), keep_loaded=[model])
        return True if same else None

    def resolve_lowvram_weight(weight, model, key):
        return weight
    return {
        "set_vram_to": dm.vram_state, "total_vram": free / (1024 * 1024), "lowvram_available": True,
        "xpu_available": False, "directml_enabled": False, "is_intel_xpu": lambda: False,
        "total_ram": _total_ram_mb(), "XFORMERS_VERSION": "", "XFORMERS_ENABLED_VAE": False,
        "is_nvidia": lambda: False, "ENABLE_PYTORCH_ATTENTION": False,
        "VAE_DTYPE": torch.bfloat16 if dm.cpu_state == dm.CPUState.GPU else torch.float32,
        "FORCE_FP32": bool(getattr(args, "force_fp32", False)), "FORCE_FP16": bool(getattr(args, "force_fp16", False)),
        "DISABLE_SMART_MEMORY": bool(getattr(args, "disable_smart_memory", False)),
        "minimum_inference_memory": lambda: 1024 * 1024 * 1024,
        "unload_model_clones": unload_model_clones,
        "get_autocast_device": lambda dev: getattr(dev, "type", "cuda"),
        "supports_dtype": supports_dtype,
        "device_supports_non_blocking": lambda device: getattr(device, "type", "") == "cuda",
        "xformers_enabled": lambda: False, "xformers_enabled_vae": lambda: False,
        "pytorch_attention_enabled": lambda: False, "pytorch_attention_flash_attention": lambda: False,
        "cpu_mode": lambda: dm.cpu_state == dm.CPUState.CPU, "mps_mode": lambda: False,
        "is_device_type": is_device_type, "is_device_cpu": lambda d: is_device_type(d, "cpu"),
        "is_device_mps": lambda d: is_device_type(d, "mps"),
        "should_use_fp16": should_use_fp16, "should_use_bf16": should_use_bf16,
        "resolve_lowvram_weight": resolve_lowvram_weight,
    }


def _total_ram_mb():
    try:
        import psutil
        return psutil.virtual_memory().total / (1024 * 1024)
    except Exception:  # pragma: no cover
        return 0.0


def _b_sd1_clip():
    from .models import text_encoders as te

    class ClipTokenWeightEncoder:
        """Mixin: ``encode_token_weights`` over ``self.encode`` (``sd1_clip.py:25``), the weighted
        interpolation against the empty-prompt encoding included."""

        def encode_token_weights(self, token_weight_pairs):
            return te.SDClipModel.encode_token_weights(self, token_weight_pairs)

    class SD1Tokenizer(te.ClipStackTokenizer):
        def __init__(self, embedding_directory=None, clip_name="l", tokenizer=None):
            super().__init__(te.SD1ClipModel, embedding_directory=embedding_directory)
            self.clip_name = clip_name
            self.clip = "clip_{}".format(clip_name)

    def load_embed(embedding_name, embedding_directory, embedding_size, embed_key=None):
        return te.load_embedding(embedding_name, embedding_directory, embedding_size, embed_key)

    def expand_directory_list(directories):
        dirs = set()
        for x in directories:
            dirs.add(x)
            for root, subdir, _ in os.walk(x, followlinks=True):
                dirs.add(root)
        return list(dirs)

    def safe_load_embed_zip(embed_path):
        raise RuntimeError("pickled (.pt zip) embeddings are not loaded: use .safetensors (no code execution)")
    def gen_empty_tokens(special_tokens, length):
        """[start?, end?, pad...] of ``length`` (``sd1_clip.py:13``)."""
        out = [t for t in (special_tokens.get("start"), special_tokens.get("end")) if t is not None]
        return out + [special_tokens.get("pad")] * (length - len(out))
    return {"gen_empty_tokens": gen_empty_tokens,
            "ClipTokenWeightEncoder": ClipTokenWeightEncoder, "SD1Tokenizer": SD1Tokenizer,
            "parse_parentheses": _parse_parentheses, "token_weights": _token_weights, "load_embed": load_embed,
            "expand_directory_list": expand_directory_list, "safe_load_embed_zip": safe_load_embed_zip}


def _b_sdxl_clip():
    from .models import text_encoders as te
    from .models.clip import CLIP_G_CONFIG

    class SDXLClipG(te.SDClipModel):
        def __init__(self, device="cpu", max_length=77, freeze=True, layer="penultimate", layer_idx=None,
                     dtype=None):
            if layer == "penultimate":
                layer, layer_idx = "hidden", -2
            super().__init__(CLIP_G_CONFIG, layer=layer, layer_idx=layer_idx, layer_norm_hidden_state=False,
                             special_tokens={"start": 49406, "end": 49407, "pad": 0}, dtype=dtype, device=device)

    class StableCascadeClipG(te.SDClipModel):
        def __init__(self, device="cpu", max_length=77, freeze=True, layer="hidden", layer_idx=-1, dtype=None):
            super().__init__(CLIP_G_CONFIG, layer=layer, layer_idx=layer_idx, layer_norm_hidden_state=False,
                             special_tokens={"start": 49406, "end": 49407, "pad": 49407},
                             enable_attention_masks=True, dtype=dtype, device=device)

    def _tok(pad_with_end):
        class _T(te.SDTokenizer):
            def __init__(self, tokenizer_path=None, embedding_directory=None):
                super().__init__(pad_with_end=pad_with_end, embedding_directory=embedding_directory,
                                 embedding_size=1280, embedding_key="clip_g")
        return _T

    class SDXLTokenizer(te.ClipStackTokenizer):
        def __init__(self, embedding_directory=None):
            super().__init__(te.SDXLClipModel, embedding_directory=embedding_directory)

    class StableCascadeTokenizer(te.ClipStackTokenizer):
        def __init__(self, embedding_directory=None):
            super().__init__(te.StableCascadeClipModel, embedding_directory=embedding_directory)
    return {"SDXLClipG": SDXLClipG, "SDXLClipGTokenizer": _tok(False), "SDXLTokenizer": SDXLTokenizer,
            "StableCascadeClipGTokenizer": _tok(True), "StableCascadeTokenizer": StableCascadeTokenizer,
            "StableCascadeClipG": StableCascadeClipG}


def _b_utils():
    from .runtime import convert

    def set_attr_param(obj, attr, value):
        return _set_attr(obj, attr, torch.nn.Parameter(value, requires_grad=False))

    def copy_to_param(obj, attr, value):
        _get_attr(obj, attr).data.copy_(value)

    def transformers_convert(sd, prefix_from, prefix_to, number):
        return convert.openclip_to_hf(sd, prefix_from, prefix_to, number)

    def clip_text_transformers_convert(sd, prefix_from, prefix_to):
        return convert.openclip_to_hf(sd, prefix_from, prefix_to)
    return {"set_attr": _set_attr, "set_attr_param": set_attr_param, "copy_to_param": copy_to_param,
            "get_attr": _get_attr, "transformers_convert": transformers_convert,
            "clip_text_transformers_convert": clip_text_transformers_convert}


def _b_ops():
    from .models import layers
    return {"cast_bias_weight": layers.cast_bias_weight, "CastWeightBiasOp": layers.CastWeightBiasOp}


def _b_sd():
    from .runtime import sd as rsd
    from .models.gligen import load_gligen as _lg

    def load_model_weights(model, sd):
        m, u = model.load_state_dict(sd, strict=False)
        return model

    def load_clip_weights(model, sd):
        return load_model_weights(model, sd)

    def load_gligen(ckpt_path):
        from .runtime.patcher import ModelPatcher
        from .runtime import device as dm
        g = _lg(ckpt_path)
        return ModelPatcher(g, load_device=dm.get_torch_device(), offload_device=dm.unet_offload_device())

    def load_checkpoint(config_path=None, ckpt_path=None, output_vae=True, output_clip=True,
                        embedding_directory=None, state_dict=None, config=None):
        """yaml-config checkpoint load (``sd.py:416``): the architecture is detected from the weights."""
        if state_dict is not None:
            return rsd.load_state_dict_guess_config(state_dict, output_vae=output_vae, output_clip=output_clip,
                                                    embedding_directory=embedding_directory)[:3]
        return rsd.load_checkpoint_guess_config(ckpt_path, output_vae=output_vae, output_clip=output_clip,
                                                embedding_directory=embedding_directory)[:3]
    return {"load_model_weights": load_model_weights, "load_clip_weights": load_clip_weights,
            "load_gligen": load_gligen, "load_checkpoint": load_checkpoint}


def _b_diffusers_convert():
    from .runtime import convert, detection, diffusers

    def convert_unet_state_dict(unet_state_dict):
        cfg = detection.unet_config_from_diffusers_unet(unet_state_dict)
        return diffusers.convert_unet_from_diffusers(unet_state_dict, cfg)

    def reshape_weight_for_sd(w):
        return w.reshape(*w.shape, 1, 1)

    def cat_tensors(tensors):
        return torch.cat(tensors)

    def convert_text_enc_state_dict_v20(text_enc_dict, prefix=""):
        return convert.hf_to_openclip(text_enc_dict, prefix, prefix)
    return {"convert_unet_state_dict": convert_unet_state_dict,
            "convert_vae_state_dict": diffusers.convert_vae_state_dict,
            "reshape_weight_for_sd": reshape_weight_for_sd, "cat_tensors": cat_tensors,
            "convert_text_enc_state_dict_v20": convert_text_enc_state_dict_v20,
            "convert_text_enc_state_dict": lambda text_enc_dict: text_enc_dict}


def _b_k_sampling():
    from .sampling import brownian, schedulers
    return {"append_zero": schedulers.append_zero, "get_sigmas_karras": schedulers.get_sigmas_karras,
            "get_sigmas_exponential": schedulers.get_sigmas_exponential,
            "get_sigmas_polyexponential": schedulers.get_sigmas_polyexponential,
            "get_sigmas_vp": schedulers.get_sigmas_vp,
            "BatchedBrownianTree": getattr(brownian, "BatchedBrownianTree", brownian.BrownianTreeNoiseSampler)}


_BUILDERS = {
    "comfy.ldm.modules.attention": _b_attention,
    "comfy.ldm.modules.diffusionmodules.model": _b_vae_model,
    "comfy.ldm.modules.diffusionmodules.openaimodel": _b_openaimodel,
    "comfy.model_management": _b_model_management,
    "comfy.sd1_clip": _b_sd1_clip,
    "comfy.sdxl_clip": _b_sdxl_clip,
    "comfy.utils": _b_utils,
    "comfy.ops": _b_ops,
    "comfy.sd": _b_sd,
    "comfy.diffusers_convert": _b_diffusers_convert,
    "comfy.k_diffusion.sampling": _b_k_sampling,
    "comfy.cldm.cldm": lambda: {"ControlledUnetModel": _lazy("models.unet", "UNetModel")},
    "comfy.clip_model": lambda: {"ACTIVATIONS": _lazy("models.clip", "ACTS")},
    "comfy.conds": lambda: {"lcm": _lcm},
    "comfy.controlnet": lambda: {"ControlLoraOps": _lazy("runtime.controlnet", "ControlLoraOps")},
    "comfy.diffusers_load": lambda: {"first_file": _first_file},
    "comfy.extra_samplers.uni_pc": lambda: {"interpolate_fn": _interpolate_fn, "expand_dims": _expand_dims},
    "comfy.gligen": lambda: {"ops": _lazy_module("models.layers"), "exists": lambda v: v is not None,
                             "uniq": lambda arr: {el: True for el in arr}.keys(),
                             "default": lambda v, d: v if v is not None else d,
                             "GEGLU": _lazy("models.attention", "GEGLU")},
    "comfy.ldm.cascade.stage_a": lambda: {"vector_quantize": _vector_quantize},
    "comfy.model_base": lambda: {"sdxl_pooled": _lazy("runtime.model_base", "_pooled"),
                                 "StableCascade_C": _lazy("models.cascade", "StableCascade_C"),
                                 "StableCascade_B": _lazy("models.cascade", "StableCascade_B")},
    "comfy.model_detection": lambda: {"calculate_transformer_depth": _lazy("runtime.detection", "_transformer_depth")},
    "comfy.model_patcher": lambda: {"apply_weight_decompose": _lazy("runtime.patcher", "weight_decompose")},
    "comfy.sample": lambda: {"prepare_sampling": _lazy("sampling.sampler_helpers", "prepare_sampling"),
                             "cleanup_additional_models": _lazy("sampling.sampler_helpers",
                                                                "cleanup_additional_models")},
    "comfy.samplers": lambda: {"simple_scheduler": _lazy("sampling.schedulers", "simple_scheduler"),
                               "ddim_scheduler": _lazy("sampling.schedulers", "ddim_scheduler"),
                               "normal_scheduler": _lazy("sampling.schedulers", "normal_scheduler")},
    "comfy.supported_models": lambda: {"models": _lazy("runtime.families", "MODELS")},
    "comfy.t2i_adapter.adapter": lambda: _t2i_names(),
    "comfy.taesd.taesd": lambda: {"conv": _lazy("models.taesd", "_conv")},
    "latent_preview": lambda: {"prepare_callback": _lazy("nodes.helpers", "prepare_callback")},
    "execution": lambda: _execution_names(),
    "nodes": lambda: _nodes_names(),
    "server": lambda: {"send_socket_catch_exception": _send_socket_catch_exception},
    "comfy.cli_args": lambda: _cli_names(),
}


def _lazy(mod, name):
    import importlib
    return getattr(importlib.import_module(f"comfy_gen_server_amd.{mod}"), name)


def _lazy_module(mod):
    import importlib
    return importlib.import_module(f"comfy_gen_server_amd.{mod}")


def _t2i_names():
    from .models import t2i_adapter as t2i

    def conv_nd(dims, *args, **kwargs):
        return {1: torch.nn.Conv1d, 2: torch.nn.Conv2d, 3: torch.nn.Conv3d}[dims](*args, **kwargs)

    def avg_pool_nd(dims, *args, **kwargs):
        return {1: torch.nn.AvgPool1d, 2: torch.nn.AvgPool2d, 3: torch.nn.AvgPool3d}[dims](*args, **kwargs)
    return {"conv_nd": conv_nd, "avg_pool_nd": avg_pool_nd, "LayerNorm": t2i._LN32, "QuickGELU": t2i._QuickGELU}


def _execution_names():
    from .graph import queue, validation
    return {"validate_inputs": validation.validate_inputs, "validate_prompt": validation.validate_prompt,
            "PromptQueue": queue.PromptQueue, "MAXIMUM_HISTORY_SIZE": getattr(queue, "MAXIMUM_HISTORY_SIZE", 10000)}


def _nodes_names():
    from .graph import registry
    from .nodes import core, extras_misc
    out = {n: getattr(extras_misc, n) for n in ("SDAPI", "SDAPISaveImage", "SDAPIPreviewImage",
                                                "SaveAndPreviewImage")}
    out["save_image_to_respective_path"] = core.save_image_to_respective_path
    out["init_custom_nodes"] = lambda: registry.init_nodes(custom_nodes=True)
    return out


async def _send_socket_catch_exception(function, message):
    """Send on a websocket, swallowing connection errors (``server.py:send_socket_catch_exception``)."""
    try:
        await function(message)
    except Exception as err:  # aiohttp ClientError / ConnectionResetError / closed transport
        import logging
        logging.warning("send error: %s", err)


def _cli_names():
    from . import cli_args
    out = dict(cli_args.GROUPS)     # the reference's mutually-exclusive group names, by name
    out["parser"] = cli_args.parser
    import logging
    out["logging_level"] = logging.DEBUG if getattr(cli_args.args, "verbose", False) else logging.INFO
    return out


_inject_lock = threading.Lock()


def inject(alias: str, module) -> None:
    """Set every missing reference name of ``alias`` on ``module`` (our module object: custom nodes
    that monkeypatch ``comfy.x.f`` then patch the function our code calls)."""
    with _inject_lock:
        if getattr(module, "__cgs_compat_injected__", set()) and alias in module.__cgs_compat_injected__:
            return
        for name, obj in extra_names(alias).items():
            if not hasattr(module, name):
                setattr(module, name, obj)
        done = set(getattr(module, "__cgs_compat_injected__", set()))
        done.add(alias)
        module.__cgs_compat_injected__ = done
