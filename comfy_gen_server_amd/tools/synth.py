"""Synthetic random-init models and checkpoints with exact ldm key names.

The reference ships no synthetic checkpoints; there is no network here, so
every test and benchmark runs on random weights of the real architectures:

* ``unet_config(family)`` — the detected-style UNet config of SD1.5 / SD2.1 / SDXL / SDXL-refiner
  (``comfy/model_detection.py:270-304`` values).
* ``build_pipeline(family, device, dtype)`` — (ModelPatcher, CLIP, VAE) built directly on the device
  (meta -> empty -> random), no disk I/O — used by ``bench.py``.
* ``write_checkpoint(family, path)`` — a full single-file ``.safetensors`` checkpoint in the
  original ldm / sgm layout (``model.diffusion_model.*``, ``first_stage_model.*``,
  ``cond_stage_model.*`` / ``conditioner.embedders.*`` with OpenCLIP keys) so the loader,
  detection and key conversions are exercised end to end.
* tiny variants (``tiny=True``) register a test family with small channels for fast CPU tests.
"""
from __future__ import annotations

import copy

import torch

from ..models.layers import init_random_, init_random_fast_
from ..runtime import families

SDXL_UNET = dict(use_checkpoint=False, image_size=32, out_channels=4, use_spatial_transformer=True, legacy=False,
                 num_classes="sequential", adm_in_channels=2816, in_channels=4, model_channels=320,
                 num_res_blocks=[2, 2, 2], transformer_depth=[0, 0, 2, 2, 10, 10], channel_mult=[1, 2, 4],
                 transformer_depth_middle=10, use_linear_in_transformer=True, context_dim=2048,
                 transformer_depth_output=[0, 0, 0, 2, 2, 2, 10, 10, 10], use_temporal_resblock=False,
                 use_temporal_attention=False)
SDXL_REFINER_UNET = dict(use_checkpoint=False, image_size=32, out_channels=4, use_spatial_transformer=True,
                         legacy=False, num_classes="sequential", adm_in_channels=2560, in_channels=4,
                         model_channels=384, num_res_blocks=[2, 2, 2, 2], transformer_depth=[0, 0, 4, 4, 4, 4, 0, 0],
                         channel_mult=[1, 2, 4, 4], transformer_depth_middle=4, use_linear_in_transformer=True,
                         context_dim=1280, transformer_depth_output=[0, 0, 0, 4, 4, 4, 4, 4, 4, 0, 0, 0],
                         use_temporal_resblock=False, use_temporal_attention=False)
SD15_UNET = dict(use_checkpoint=False, image_size=32, out_channels=4, use_spatial_transformer=True, legacy=False,
                 adm_in_channels=None, in_channels=4, model_channels=320, num_res_blocks=[2, 2, 2, 2],
                 transformer_depth=[1, 1, 1, 1, 1, 1, 0, 0], channel_mult=[1, 2, 4, 4], transformer_depth_middle=1,
                 use_linear_in_transformer=False, context_dim=768,
                 transformer_depth_output=[1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0], use_temporal_resblock=False,
                 use_temporal_attention=False)
SD21_UNET = dict(SD15_UNET, use_linear_in_transformer=True, context_dim=1024)

FAMILY_UNET = {"sdxl": (families.SDXL, SDXL_UNET), "sdxl_refiner": (families.SDXLRefiner, SDXL_REFINER_UNET),
               "sd15": (families.SD15, SD15_UNET), "sd21": (families.SD20, SD21_UNET)}


# ------------------------------------------------------------------------------------------------
# tiny test family (registered on demand)
# ------------------------------------------------------------------------------------------------
TINY_CLIP = dict(hidden_size=64, intermediate_size=128, num_attention_heads=2, num_hidden_layers=2,
                 hidden_act="quick_gelu", projection_dim=64, vocab_size=49408, max_position_embeddings=77)
TINY_UNET = dict(use_checkpoint=False, image_size=32, out_channels=4, use_spatial_transformer=True, legacy=False,
                 adm_in_channels=None, in_channels=4, model_channels=32, num_res_blocks=[1, 1], channel_mult=[1, 2],
                 transformer_depth=[1, 1], transformer_depth_output=[1, 1, 1, 1], transformer_depth_middle=1,
                 use_linear_in_transformer=False, context_dim=64, use_temporal_resblock=False,
                 use_temporal_attention=False)


def _tiny_stack():
    from ..models import text_encoders as te

    class TinyClipModel(te._Stack):
        tokenizer_specs = {"l": dict(embedding_size=64, embedding_key="clip_l")}

        def __init__(self, dtype=None, device=None):
            super().__init__()
            self.clip_l = te.SDClipModel(TINY_CLIP, layer="last", dtype=dtype, device=device)

        def encode_token_weights(self, tw):
            return self.clip_l.encode_token_weights(tw["l"])
    return TinyClipModel


class TinySD(families.SD15):
    unet_config = {"context_dim": 64, "model_channels": 32, "use_linear_in_transformer": False,
                   "adm_in_channels": None}
    unet_extra_config = {"num_heads": 2, "num_head_channels": -1}

    def clip_target(self):
        return families.ClipTarget(_tiny_stack())


def register_tiny_family():
    if TinySD not in families.MODELS:
        families.MODELS.insert(0, TinySD)
    FAMILY_UNET["tiny"] = (TinySD, TINY_UNET)


TINY_VAE = dict(double_z=True, z_channels=4, in_channels=3, out_ch=3, ch=32, ch_mult=[1, 2, 2, 2], num_res_blocks=1)


# ------------------------------------------------------------------------------------------------
def build_pipeline(family="sdxl", device=None, dtype=torch.bfloat16, seed=0, with_clip=True, with_vae=True):
    """Random-init (ModelPatcher, CLIP, VAE) of a family directly on ``device``."""
    from ..runtime import device as dm
    from ..runtime.patcher import ModelPatcher
    from ..runtime.sd import CLIP, VAE
    from ..models.vae import AutoencoderKL
    if family == "tiny":
        register_tiny_family()
    device = device or dm.get_torch_device()
    fam_cls, ucfg = FAMILY_UNET[family]
    mc = fam_cls(copy.deepcopy(ucfg))
    mc.set_inference_dtype(dtype, None)
    with torch.device("meta"):
        model = mc.get_model({}, "", device=torch.device("meta"))
    model.to_empty(device=device)
    model.model_sampling = model.model_sampling.__class__(mc)
    model.model_sampling.to(device)
    init = init_random_fast_ if device.type == "cuda" else init_random_
    init(model.diffusion_model, seed=seed)
    patcher = ModelPatcher(model, load_device=device, offload_device=device)
    clip = vae = None
    if with_clip:
        ct = mc.clip_target()
        clip = CLIP(ct, dtype=dtype if device.type == "cuda" else torch.float32, device=device)
        clip.cond_stage_model.to(device)
        init(clip.cond_stage_model, seed=seed + 1)
        clip.patcher.offload_device = device
    if with_vae:
        vae = VAE(sd=None, device=device, dtype=dtype if device.type == "cuda" else torch.float32)
        if family == "tiny":
            from ..runtime.patcher import ModelPatcher as _MP
            vae.first_stage_model = AutoencoderKL(4, TINY_VAE).to(vae.vae_dtype)
            vae.patcher = _MP(vae.first_stage_model, load_device=device, offload_device=device)
        vae.first_stage_model.to(device)
        init(vae.first_stage_model, seed=seed + 2)
        vae.patcher.offload_device = device
    return patcher, clip, vae


def random_state_dict(family="sdxl", seed=0, dtype=torch.float16, tiny_vae=False):
    """Full ldm-layout checkpoint state dict with random weights (CPU)."""
    from ..models import text_encoders as te
    from ..models.vae import AutoencoderKL
    from ..runtime.convert import hf_to_openclip
    if family == "tiny":
        register_tiny_family()
    fam_cls, ucfg = FAMILY_UNET[family]
    mc = fam_cls(copy.deepcopy(ucfg))
    mc.set_inference_dtype(torch.float32, None)
    model = mc.get_model({}, "")
    init_random_(model.diffusion_model, seed=seed)
    sd = {f"model.diffusion_model.{k}": v.to(dtype) for k, v in model.diffusion_model.state_dict().items()}
    del model
    if family == "tiny" or tiny_vae:
        vae = AutoencoderKL(4, TINY_VAE)
    else:
        vae = AutoencoderKL(4, dict(ch=128, ch_mult=[1, 2, 4, 4], num_res_blocks=2, z_channels=4))
    init_random_(vae, seed=seed + 2)
    sd.update({f"first_stage_model.{k}": v.to(dtype) for k, v in vae.state_dict().items()})
    stack = mc.clip_target().stack()
    init_random_(stack, seed=seed + 1)
    csd = stack.state_dict()
    if family in ("sd15", "tiny"):
        for k, v in csd.items():
            if "text_projection" in k:
                continue
            sd["cond_stage_model." + k[len("clip_l."):]] = v.to(dtype)
    elif family == "sd21":
        sd.update({k: v.to(dtype) for k, v in hf_to_openclip(csd, "clip_h.", "cond_stage_model.model.").items()})
    elif family == "sdxl":
        for k, v in csd.items():
            if k.startswith("clip_l.") and "text_projection" not in k:
                sd["conditioner.embedders.0." + k[len("clip_l."):]] = v.to(dtype)
        sd.update({k: v.to(dtype) for k, v in hf_to_openclip(csd, "clip_g.", "conditioner.embedders.1.model.").items()})
    elif family == "sdxl_refiner":
        sd.update({k: v.to(dtype) for k, v in hf_to_openclip(csd, "clip_g.", "conditioner.embedders.0.model.").items()})
    return sd


def write_checkpoint(family, path, seed=0, dtype=torch.float16):
    from ..runtime.checkpoint import save_state_dict
    sd = random_state_dict(family, seed=seed, dtype=dtype)
    save_state_dict(sd, path, metadata={"synthetic": "random-init", "family": family})
    return path


def random_lora(model_patcher, rank=4, seed=0, prefix_filter=("attn1.to_q", "attn2.to_k", "ff.net.2")):
    """A kohya-format LoRA over a subset of UNet linear layers of ``model_patcher``."""
    g = torch.Generator().manual_seed(seed)
    sd = {}
    for k, v in model_patcher.model.diffusion_model.state_dict().items():
        if not k.endswith(".weight") or v.dim() != 2 or not any(p in k for p in prefix_filter):
            continue
        name = "lora_unet_" + k[:-len(".weight")].replace(".", "_")
        out_f, in_f = v.shape
        sd[f"{name}.lora_up.weight"] = torch.randn((out_f, rank), generator=g) * 0.01
        sd[f"{name}.lora_down.weight"] = torch.randn((rank, in_f), generator=g) * 0.01
        sd[f"{name}.alpha"] = torch.tensor(float(rank))
    return sd


_PIPELINES: dict = {}


class SyntheticCheckpointLoader:
    """Workflow node: random-init (MODEL, CLIP, VAE) of a family's exact architecture, built once per
    (family, seed) on the device -- the product workflow path (bench.py --via-executor, tests) without
    a checkpoint file. Registered on demand (``register_node``), never by default."""

    @classmethod
    def INPUT_TYPES(cls):
        return {"required": {"family": (sorted(FAMILY_UNET),), "seed": ("INT", {"default": 0, "min": 0})}}

    RETURN_TYPES = ("MODEL", "CLIP", "VAE")
    FUNCTION = "load"
    CATEGORY = "loaders/testing"

    def load(self, family, seed):
        key = (family, int(seed))
        if key not in _PIPELINES:
            from ..runtime import device as dm
            dev = dm.get_torch_device()
            dtype = torch.bfloat16 if dev.type == "cuda" else torch.float32
            with torch.inference_mode():
                _PIPELINES[key] = build_pipeline(family, device=dev, dtype=dtype, seed=int(seed))
        return _PIPELINES[key]


def register_node():
    from ..graph import registry
    registry.NODE_CLASS_MAPPINGS["CGSSyntheticCheckpoint"] = SyntheticCheckpointLoader
    registry.NODE_DISPLAY_NAME_MAPPINGS["CGSSyntheticCheckpoint"] = "Synthetic checkpoint (random init)"


def text_to_image_workflow(family="sdxl", seed=0, text="a photo", negative="blurry", width=1024, height=1024,
                           batch=1, steps=20, cfg=8.0, sampler="euler_ancestral", scheduler="normal",
                           model_seed=1234, save_prefix="bench"):
    """The reference's default text-to-image graph (script_examples/basic_api_example.py shape) on the
    synthetic loader."""
    enc = "CLIPTextEncode"
    return {
        "4": {"class_type": "CGSSyntheticCheckpoint", "inputs": {"family": family, "seed": model_seed}},
        "5": {"class_type": "EmptyLatentImage", "inputs": {"width": width, "height": height, "batch_size": batch}},
        "6": {"class_type": enc, "inputs": {"text": text, "clip": ["4", 1]}},
        "7": {"class_type": enc, "inputs": {"text": negative, "clip": ["4", 1]}},
        "3": {"class_type": "KSampler", "inputs": {"seed": seed, "steps": steps, "cfg": cfg, "sampler_name": sampler,
                                                  "scheduler": scheduler, "denoise": 1.0, "model": ["4", 0],
                                                  "positive": ["6", 0], "negative": ["7", 0],
                                                  "latent_image": ["5", 0]}},
        "8": {"class_type": "VAEDecode", "inputs": {"samples": ["3", 0], "vae": ["4", 2]}},
        "9": {"class_type": "SaveImage", "inputs": {"filename_prefix": save_prefix, "images": ["8", 0]}},
    }
