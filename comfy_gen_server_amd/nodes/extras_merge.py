"""Model merging / saving / hypernetwork nodes (parity: ``comfy_extras/nodes_model_merging.py``,
``nodes_model_merging_model_specific.py``, ``nodes_hypernetwork.py``, ``nodes_video_model.py``
ImageOnlyCheckpointSave; SURVEY §2.2 'Model patches / advanced').

Merges are lazy weight patches on a cloned ModelPatcher/CLIP (``get_key_patches`` of the second
model, strengths (1-r, r)); they are folded into the weights on the device when the model is
loaded (runtime.patcher.calculate_weight), so a merge costs one fused pass over the weights on
MI355X, not a host round trip. Checkpoints are written with the native safetensors writer.
"""
from __future__ import annotations

import json
import logging
import os

import torch

from ..runtime import device as dm
from ..runtime import model_base as MB
from ..runtime import sd as sdl
from ..runtime.checkpoint import load_state_dict, save_state_dict
from ..runtime.convert import state_dict_prefix_replace
from ..sampling import model_sampling as MS
from ..utils import folder_paths
from . import helpers as NH

_RATIO = ("FLOAT", {"default": 1.0, "min": 0.0, "max": 1.0, "step": 0.01})
_SKIP_CLIP_KEYS = (".position_ids", ".logit_scale")


def _merge_models(model1, model2, strength_patch, strength_model):
    m = model1.clone()
    kp = model2.get_key_patches("diffusion_model.")
    for k, v in kp.items():
        m.add_patches({k: v}, strength_patch, strength_model)
    return m


class ModelMergeSimple:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"model1": ("MODEL",), "model2": ("MODEL",), "ratio": _RATIO}}
    RETURN_TYPES = ("MODEL",)
    FUNCTION = "merge"
    CATEGORY = "advanced/model_merging"

    def merge(self, model1, model2, ratio):
        return (_merge_models(model1, model2, 1.0 - ratio, ratio),)


class ModelMergeSubtract:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"model1": ("MODEL",), "model2": ("MODEL",),
                             "multiplier": ("FLOAT", {"default": 1.0, "min": -10.0, "max": 10.0, "step": 0.01})}}
    RETURN_TYPES = ("MODEL",)
    FUNCTION = "merge"
    CATEGORY = "advanced/model_merging"

    def merge(self, model1, model2, multiplier):
        return (_merge_models(model1, model2, -multiplier, multiplier),)


class ModelMergeAdd:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"model1": ("MODEL",), "model2": ("MODEL",)}}
    RETURN_TYPES = ("MODEL",)
    FUNCTION = "merge"
    CATEGORY = "advanced/model_merging"

    def merge(self, model1, model2):
        return (_merge_models(model1, model2, 1.0, 1.0),)


class ModelMergeBlocks:
    """Per-block ratio: the longest matching key prefix among the node's float inputs wins."""

    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"model1": ("MODEL",), "model2": ("MODEL",), "input": _RATIO, "middle": _RATIO,
                             "out": _RATIO}}
    RETURN_TYPES = ("MODEL",)
    FUNCTION = "merge"
    CATEGORY = "advanced/model_merging"

    def merge(self, model1, model2, **kwargs):
        m = model1.clone()
        kp = model2.get_key_patches("diffusion_model.")
        default = next(iter(kwargs.values()))
        for k, v in kp.items():
            ku = k[len("diffusion_model."):]
            ratio, best = default, 0
            for prefix, r in kwargs.items():
                if ku.startswith(prefix) and len(prefix) > best:
                    ratio, best = r, len(prefix)
            m.add_patches({k: v}, 1.0 - ratio, ratio)
        return (m,)


class ModelMergeSD1(ModelMergeBlocks):
    CATEGORY = "advanced/model_merging/model_specific"

    @classmethod
    def INPUT_TYPES(s):
        d = {"model1": ("MODEL",), "model2": ("MODEL",), "time_embed.": _RATIO, "label_emb.": _RATIO}
        d.update({f"input_blocks.{i}.": _RATIO for i in range(12)})
        d.update({f"middle_block.{i}.": _RATIO for i in range(3)})
        d.update({f"output_blocks.{i}.": _RATIO for i in range(12)})
        d["out."] = _RATIO
        return {"required": d}


class ModelMergeSDXL(ModelMergeBlocks):
    CATEGORY = "advanced/model_merging/model_specific"

    @classmethod
    def INPUT_TYPES(s):
        d = {"model1": ("MODEL",), "model2": ("MODEL",), "time_embed.": _RATIO, "label_emb.": _RATIO}
        d.update({f"input_blocks.{i}": _RATIO for i in range(9)})
        d.update({f"middle_block.{i}": _RATIO for i in range(3)})
        d.update({f"output_blocks.{i}": _RATIO for i in range(9)})
        d["out."] = _RATIO
        return {"required": d}


def _merge_clips(clip1, clip2, strength_patch, strength_model):
    m = clip1.clone()
    for k, v in clip2.get_key_patches().items():
        if k.endswith(_SKIP_CLIP_KEYS):
            continue
        m.add_patches({k: v}, strength_patch, strength_model)
    return m


class CLIPMergeSimple:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"clip1": ("CLIP",), "clip2": ("CLIP",), "ratio": _RATIO}}
    RETURN_TYPES = ("CLIP",)
    FUNCTION = "merge"
    CATEGORY = "advanced/model_merging"

    def merge(self, clip1, clip2, ratio):
        return (_merge_clips(clip1, clip2, 1.0 - ratio, ratio),)


class CLIPMergeSubtract:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"clip1": ("CLIP",), "clip2": ("CLIP",),
                             "multiplier": ("FLOAT", {"default": 1.0, "min": -10.0, "max": 10.0, "step": 0.01})}}
    RETURN_TYPES = ("CLIP",)
    FUNCTION = "merge"
    CATEGORY = "advanced/model_merging"

    def merge(self, clip1, clip2, multiplier):
        return (_merge_clips(clip1, clip2, -multiplier, multiplier),)


class CLIPMergeAdd:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"clip1": ("CLIP",), "clip2": ("CLIP",)}}
    RETURN_TYPES = ("CLIP",)
    FUNCTION = "merge"
    CATEGORY = "advanced/model_merging"

    def merge(self, clip1, clip2):
        return (_merge_clips(clip1, clip2, 1.0, 1.0),)


# ---------------------------------------------------------------- saving
def _metadata(prompt, extra_pnginfo):
    md = {}
    if not NH.args_disable_metadata():
        md["prompt"] = json.dumps(prompt) if prompt is not None else ""
        for k, v in (extra_pnginfo or {}).items():
            md[k] = json.dumps(v)
    return md


def save_checkpoint(model, clip=None, vae=None, clip_vision=None, filename_prefix=None, output_dir=None, prompt=None,
                    extra_pnginfo=None):
    folder, filename, counter, _, _ = folder_paths.get_save_image_path(filename_prefix, output_dir)
    metadata = {}
    arch = None
    if isinstance(model.model, MB.SDXLRefiner):
        arch = "stable-diffusion-xl-v1-refiner"
    elif isinstance(model.model, MB.SDXL):
        arch = "stable-diffusion-xl-v1-base"
    if arch is not None:
        metadata.update({"modelspec.architecture": arch, "modelspec.sai_model_spec": "1.0.0",
                         "modelspec.implementation": "sgm", "modelspec.title": f"{filename} {counter}"})
    extra_keys = {}
    ms = model.get_model_object("model_sampling")
    if isinstance(ms, MS.ModelSamplingContinuousEDM) and isinstance(ms, MS.V_PREDICTION):
        extra_keys["edm_vpred.sigma_max"] = torch.tensor(float(ms.sigma_max)).float()
        extra_keys["edm_vpred.sigma_min"] = torch.tensor(float(ms.sigma_min)).float()
    if model.model.model_type == MB.ModelType.EPS:
        metadata["modelspec.predict_key"] = "epsilon"
    elif model.model.model_type == MB.ModelType.V_PREDICTION:
        metadata["modelspec.predict_key"] = "v"
    metadata.update(_metadata(prompt, extra_pnginfo))
    path = os.path.join(folder, f"{filename}_{counter:05}_.safetensors")
    sdl.save_checkpoint(path, model, clip, vae, clip_vision, metadata=metadata, extra_keys=extra_keys)
    return path


class CheckpointSave:
    def __init__(self):
        self.output_dir = folder_paths.get_output_directory()

    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"model": ("MODEL",), "clip": ("CLIP",), "vae": ("VAE",),
                             "filename_prefix": ("STRING", {"default": "checkpoints/ComfyUI"})},
                "hidden": {"prompt": "PROMPT", "extra_pnginfo": "EXTRA_PNGINFO"}}
    RETURN_TYPES = ()
    FUNCTION = "save"
    OUTPUT_NODE = True
    CATEGORY = "advanced/model_merging"

    def save(self, model, clip, vae, filename_prefix, prompt=None, extra_pnginfo=None):
        save_checkpoint(model, clip=clip, vae=vae, filename_prefix=filename_prefix,
                        output_dir=folder_paths.get_output_directory(), prompt=prompt, extra_pnginfo=extra_pnginfo)
        return {}


class ImageOnlyCheckpointSave(CheckpointSave):
    CATEGORY = "_for_testing"

    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"model": ("MODEL",), "clip_vision": ("CLIP_VISION",), "vae": ("VAE",),
                             "filename_prefix": ("STRING", {"default": "checkpoints/ComfyUI"})},
                "hidden": {"prompt": "PROMPT", "extra_pnginfo": "EXTRA_PNGINFO"}}

    def save(self, model, clip_vision, vae, filename_prefix, prompt=None, extra_pnginfo=None):
        save_checkpoint(model, clip_vision=clip_vision, vae=vae, filename_prefix=filename_prefix,
                        output_dir=folder_paths.get_output_directory(), prompt=prompt, extra_pnginfo=extra_pnginfo)
        return {}


class CLIPSave:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"clip": ("CLIP",), "filename_prefix": ("STRING", {"default": "clip/ComfyUI"})},
                "hidden": {"prompt": "PROMPT", "extra_pnginfo": "EXTRA_PNGINFO"}}
    RETURN_TYPES = ()
    FUNCTION = "save"
    OUTPUT_NODE = True
    CATEGORY = "advanced/model_merging"

    def save(self, clip, filename_prefix, prompt=None, extra_pnginfo=None):
        metadata = _metadata(prompt, extra_pnginfo)
        dm.load_models_gpu([clip.load_model()])
        clip_sd = clip.get_sd()
        out_dir = folder_paths.get_output_directory()
        for prefix in ("clip_l.", "clip_g.", ""):
            part = {k: clip_sd.pop(k) for k in [k for k in clip_sd if k.startswith(prefix)]}
            if not part:
                continue
            fp = filename_prefix
            repl = {"transformer.": ""}
            if prefix:
                fp = f"{filename_prefix}_{prefix[:-1]}"
                repl[prefix] = ""
            folder, filename, counter, _, _ = folder_paths.get_save_image_path(fp, out_dir)
            part = state_dict_prefix_replace(part, repl)
            save_state_dict(part, os.path.join(folder, f"{filename}_{counter:05}_.safetensors"), metadata=metadata)
        return {}


class VAESave:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"vae": ("VAE",), "filename_prefix": ("STRING", {"default": "vae/ComfyUI_vae"})},
                "hidden": {"prompt": "PROMPT", "extra_pnginfo": "EXTRA_PNGINFO"}}
    RETURN_TYPES = ()
    FUNCTION = "save"
    OUTPUT_NODE = True
    CATEGORY = "advanced/model_merging"

    def save(self, vae, filename_prefix, prompt=None, extra_pnginfo=None):
        folder, filename, counter, _, _ = folder_paths.get_save_image_path(filename_prefix,
                                                                           folder_paths.get_output_directory())
        save_state_dict(vae.get_sd(), os.path.join(folder, f"{filename}_{counter:05}_.safetensors"),
                        metadata=_metadata(prompt, extra_pnginfo))
        return {}


# ---------------------------------------------------------------- hypernetworks
_ACTIVATIONS = {"linear": torch.nn.Identity, "relu": torch.nn.ReLU, "leakyrelu": torch.nn.LeakyReLU,
                "elu": torch.nn.ELU, "swish": torch.nn.Hardswish, "tanh": torch.nn.Tanh,
                "sigmoid": torch.nn.Sigmoid, "softsign": torch.nn.Softsign, "mish": torch.nn.Mish}


class HypernetworkPatch:
    """attn1/attn2 patch: k += hn_k(k) * s, v += hn_v(v) * s for the matching context width."""

    def __init__(self, nets, strength):
        self.hypernet = nets
        self.strength = strength

    def __call__(self, q, k, v, extra_options):
        hn = self.hypernet.get(k.shape[-1])
        if hn is not None:
            k = k + hn[0](k.to(hn[0][0].weight.dtype)).to(k.dtype) * self.strength
            v = v + hn[1](v.to(hn[1][0].weight.dtype)).to(v.dtype) * self.strength
        return q, k, v

    def to(self, device):
        for d in list(self.hypernet):
            self.hypernet[d] = self.hypernet[d].to(device)
        return self


def load_hypernetwork_patch(path, strength):
    """Build the per-width MLP pairs of an A1111 hypernetwork file (loaded without unpickling code)."""
    sd = load_state_dict(path)
    act = sd.get("activation_func", "linear")
    is_ln = sd.get("is_layer_norm", False)
    use_dropout = sd.get("use_dropout", False)
    activate_output = sd.get("activate_output", False)
    last_layer_dropout = sd.get("last_layer_dropout", False)
    if act not in _ACTIVATIONS:
        logging.error("Unsupported hypernetwork format %s: activation %s", path, act)
        return None
    nets = {}
    for key in sd:
        try:
            dim = int(key)
        except (TypeError, ValueError):
            continue
        pair = []
        for idx in (0, 1):
            w = sd[key][idx]
            names = [n[:-len(".weight")] for n in w if n.endswith(".weight")]
            layers = []
            i = 0
            while i < len(names):
                last = i == len(names) - 1
                penult = i == len(names) - 2
                lw, lb = w[f"{names[i]}.weight"], w[f"{names[i]}.bias"]
                lin = torch.nn.Linear(lw.shape[1], lw.shape[0])
                lin.load_state_dict({"weight": lw, "bias": lb})
                layers.append(lin)
                if act != "linear" and (not last or activate_output):
                    layers.append(_ACTIVATIONS[act]())
                if is_ln:
                    i += 1
                    lnw, lnb = w[f"{names[i]}.weight"], w[f"{names[i]}.bias"]
                    ln = torch.nn.LayerNorm(lnw.shape[0])
                    ln.load_state_dict({"weight": lnw, "bias": lnb})
                    layers.append(ln)
                if use_dropout and not last and (not penult or last_layer_dropout):
                    layers.append(torch.nn.Dropout(p=0.3))
                i += 1
            pair.append(torch.nn.Sequential(*layers).eval())
        nets[dim] = torch.nn.ModuleList(pair)
    return HypernetworkPatch(nets, strength)


class HypernetworkLoader:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"model": ("MODEL",),
                             "hypernetwork_name": (folder_paths.get_filename_list("hypernetworks"),),
                             "strength": ("FLOAT", {"default": 1.0, "min": -10.0, "max": 10.0, "step": 0.01})}}
    RETURN_TYPES = ("MODEL",)
    FUNCTION = "load_hypernetwork"
    CATEGORY = "loaders"

    def load_hypernetwork(self, model, hypernetwork_name, strength):
        m = model.clone()
        patch = load_hypernetwork_patch(folder_paths.get_full_path("hypernetworks", hypernetwork_name), strength)
        if patch is not None:
            m.set_model_attn1_patch(patch)
            m.set_model_attn2_patch(patch)
        return (m,)


NODE_CLASS_MAPPINGS = {
    "ModelMergeSimple": ModelMergeSimple, "ModelMergeBlocks": ModelMergeBlocks,
    "ModelMergeSubtract": ModelMergeSubtract, "ModelMergeAdd": ModelMergeAdd, "CheckpointSave": CheckpointSave,
    "CLIPMergeSimple": CLIPMergeSimple, "CLIPMergeSubtract": CLIPMergeSubtract, "CLIPMergeAdd": CLIPMergeAdd,
    "CLIPSave": CLIPSave, "VAESave": VAESave, "ModelMergeSD1": ModelMergeSD1, "ModelMergeSD2": ModelMergeSD1,
    "ModelMergeSDXL": ModelMergeSDXL, "ImageOnlyCheckpointSave": ImageOnlyCheckpointSave,
    "HypernetworkLoader": HypernetworkLoader,
}
