"""Diffusion-model wrappers: c_in scaling -> UNet -> denoised, plus per-family extra conds.

Parity with ``comfy/model_base.py:1-559``: ModelType, BaseModel.apply_model (:74-98),
extra_conds (c_concat for inpaint/IP2P, ADM ``y``, c_crossattn), SDXL / SDXL-refiner ADM size
embeddings (pooled 1280 + 6x256 Timestep embeds = 2816, :317-334), SD21UNCLIP, IP2P, SD_X4,
StableCascade_C/B (wired in ``models/cascade.py``), inpaint setup, memory estimate, saving.
"""
from __future__ import annotations

import enum
import logging
import math

import torch

from .. import ops
from ..sampling import conds as C
from ..sampling.model_sampling import model_sampling


class ModelType(enum.Enum):
    EPS = 1
    V_PREDICTION = 2
    V_PREDICTION_EDM = 3
    STABLE_CASCADE = 4
    EDM = 5
    X0 = 6


def timestep_embed_256(values, dim=256):
    """``Timestep(256)`` of the reference (util.timestep_embedding, cos first)."""
    t = torch.tensor(values, dtype=torch.float32)
    return ops.core.timestep_embedding(t, dim)   # CPU tensor -> reference path


def common_upscale(samples, width, height, method="bilinear", crop="disabled"):
    from ..utils.image import common_upscale as cu
    return cu(samples, width, height, method, crop)


class BaseModel(torch.nn.Module):
    def __init__(self, model_config, model_type=ModelType.EPS, device=None, unet_model=None):
        super().__init__()
        from ..models.unet import UNetModel
        unet_model = unet_model or UNetModel
        unet_config = dict(model_config.unet_config)
        self.latent_format = model_config.latent_format
        self.model_config = model_config
        self.manual_cast_dtype = getattr(model_config, "manual_cast_dtype", None)
        if not unet_config.get("disable_unet_model_creation", False):
            dtype = unet_config.pop("dtype", torch.float32)
            self.diffusion_model = unet_model(**unet_config, dtype=dtype, device=device)
        self.model_type = model_type
        self.model_sampling = model_sampling(model_config, model_type)
        self.adm_channels = unet_config.get("adm_in_channels", None) or 0
        self.concat_keys = ()
        self.inpaint_model = False

    # ------------------------------------------------------------------------------------------
    def get_dtype(self):
        return self.diffusion_model.dtype

    def apply_model(self, x, t, c_concat=None, c_crossattn=None, control=None, transformer_options=None, **kwargs):
        sigma = t
        xc = self.model_sampling.calculate_input(sigma, x)
        if c_concat is not None:
            xc = torch.cat([xc, c_concat.to(xc)], dim=1)
        dtype = self.manual_cast_dtype or self.get_dtype()
        xc = xc.to(dtype)
        ts = self.model_sampling.timestep(t).float()
        context = c_crossattn.to(dtype) if c_crossattn is not None else None
        extra = {}
        for k, v in kwargs.items():
            if hasattr(v, "dtype") and v.dtype not in (torch.int, torch.long):
                v = v.to(dtype)
            extra[k] = v
        out = self.denoiser_forward()(xc, ts, context=context, control=control,
                                      transformer_options=transformer_options if transformer_options is not None else {},
                                      **extra).float()
        return self.model_sampling.calculate_denoised(sigma, out, x)

    def denoiser_forward(self):
        """The diffusion model's forward, replayed from per-plan hipGraphs on the device
        (``runtime/graphs.py``); eager on the CPU or whenever hooks make the forward dynamic."""
        r = self.__dict__.get("_graph_runner")
        if r is None or r.module is not self.diffusion_model:
            from .graphs import GraphedForward
            r = GraphedForward(self.diffusion_model)
            self.__dict__["_graph_runner"] = r
        return r

    def is_adm(self):
        return self.adm_channels > 0

    def encode_adm(self, **kwargs):
        return None

    def extra_conds(self, **kwargs):
        out = {}
        if self.concat_keys:
            noise = kwargs["noise"]
            device = kwargs["device"]
            mask = kwargs.get("concat_mask", kwargs.get("denoise_mask"))
            cli = kwargs.get("concat_latent_image")
            if cli is None:
                cli = kwargs.get("latent_image")
            else:
                cli = self.process_latent_in(cli)
            if cli.shape[1:] != noise.shape[1:]:
                cli = common_upscale(cli, noise.shape[-1], noise.shape[-2], "bilinear", "center")
            cli = C.repeat_to_batch_size(cli, noise.shape[0])
            if mask is not None:
                if mask.ndim == noise.ndim:
                    mask = mask[:, :1]
                mask = mask.reshape((-1, 1, mask.shape[-2], mask.shape[-1]))
                if mask.shape[-2:] != noise.shape[-2:]:
                    mask = common_upscale(mask, noise.shape[-1], noise.shape[-2], "bilinear", "center")
                mask = C.repeat_to_batch_size(mask.round(), noise.shape[0])
            parts = []
            for ck in self.concat_keys:
                if mask is not None:
                    if ck == "mask":
                        parts.append(mask.to(device))
                    elif ck == "masked_image":
                        parts.append(cli.to(device))
                else:
                    if ck == "mask":
                        parts.append(torch.ones_like(noise)[:, :1])
                    elif ck == "masked_image":
                        parts.append(self.blank_inpaint_image_like(noise))
            out["c_concat"] = C.CONDNoiseShape(torch.cat(parts, dim=1))
        adm = self.encode_adm(**kwargs)
        if adm is not None:
            out["y"] = C.CONDRegular(adm)
        ca = kwargs.get("cross_attn")
        if ca is not None:
            out["c_crossattn"] = C.CONDCrossAttn(ca)
        cac = kwargs.get("cross_attn_controlnet")
        if cac is not None:
            out["crossattn_controlnet"] = C.CONDCrossAttn(cac)
        return out

    def load_model_weights(self, sd, unet_prefix=""):
        to_load = {k[len(unet_prefix):]: sd.pop(k) for k in list(sd.keys()) if k.startswith(unet_prefix)}
        to_load = self.model_config.process_unet_state_dict(to_load)
        m, u = self.diffusion_model.load_state_dict(to_load, strict=False, assign=False)
        if m:
            logging.warning("unet missing: %s", m[:20])
        if u:
            logging.warning("unet unexpected: %s", u[:20])
        return self

    def process_latent_in(self, latent):
        return self.latent_format.process_in(latent)

    def process_latent_out(self, latent):
        return self.latent_format.process_out(latent)

    def set_inpaint(self):
        self.concat_keys = ("mask", "masked_image")
        self.inpaint_model = True

    @staticmethod
    def blank_inpaint_image_like(latent):
        b = torch.ones_like(latent)
        for i, v in enumerate((0.8223, -0.6876, 0.6364, 0.1380)):
            b[:, i] *= v
        return b

    def memory_required(self, input_shape):
        """Activation budget estimate in bytes (model_base.py:227-238, flash-attention branch)."""
        area = input_shape[0] * input_shape[2] * input_shape[3]
        return (area * 2 / 50) * (1024 * 1024)

    def state_dict_for_saving(self, clip_state_dict=None, vae_state_dict=None, clip_vision_state_dict=None):
        extra = []
        mc = self.model_config
        if clip_state_dict is not None:
            extra.append(mc.process_clip_state_dict_for_saving(clip_state_dict))
        if vae_state_dict is not None:
            extra.append(mc.process_vae_state_dict_for_saving(vae_state_dict))
        if clip_vision_state_dict is not None:
            extra.append(mc.process_clip_vision_state_dict_for_saving(clip_vision_state_dict))
        sd = mc.process_unet_state_dict_for_saving(self.diffusion_model.state_dict())
        if self.model_type == ModelType.V_PREDICTION:
            sd["v_pred"] = torch.tensor([])
        for e in extra:
            sd.update(e)
        return sd


# ------------------------------------------------------------------------------------------------
def _pooled(args, noise_augmentor=None):
    if args.get("unclip_conditioning") is not None and noise_augmentor is not None:
        return unclip_adm(args["unclip_conditioning"], args["device"], noise_augmentor,
                          seed=args.get("seed", 0) - 10)[:, :1280]
    return args["pooled_output"]


def unclip_adm(unclip_conditioning, device, noise_augmentor, noise_augment_merge=0.0, seed=None):
    adm_inputs = []
    weights = []
    noise_aug = []
    for u in unclip_conditioning:
        for a in u["clip_vision_output"].image_embeds:
            w = u["strength"]
            na = u["noise_augmentation"]
            level = round((noise_augmentor.max_noise_level - 1) * na)
            c_adm, noise_level_emb = noise_augmentor(a.to(device), noise_level=torch.tensor([level], device=device), seed=seed)
            adm_out = torch.cat((c_adm, noise_level_emb), 1) * w
            weights.append(w)
            noise_aug.append(na)
            adm_inputs.append(adm_out)
    if len(noise_aug) > 1:
        adm_out = torch.stack(adm_inputs).sum(0)
        na = noise_augment_merge
        level = round((noise_augmentor.max_noise_level - 1) * na)
        c_adm, noise_level_emb = noise_augmentor(adm_out[:, :noise_augmentor.time_embed.dim], noise_level=torch.tensor([level], device=device))
        adm_out = torch.cat((c_adm, noise_level_emb), 1)
    return adm_out


class SDXLRefiner(BaseModel):
    def encode_adm(self, **kw):
        pooled = _pooled(kw)
        w, h = kw.get("width", 768), kw.get("height", 768)
        aest = kw.get("aesthetic_score", 2.5 if kw.get("prompt_type", "") == "negative" else 6)
        vals = [h, w, kw.get("crop_h", 0), kw.get("crop_w", 0), aest]
        flat = timestep_embed_256(vals).flatten().unsqueeze(0).repeat(pooled.shape[0], 1)
        return torch.cat((pooled.to(flat.device), flat), dim=1)


class SDXL(BaseModel):
    def encode_adm(self, **kw):
        pooled = _pooled(kw)
        w, h = kw.get("width", 768), kw.get("height", 768)
        vals = [h, w, kw.get("crop_h", 0), kw.get("crop_w", 0), kw.get("target_height", h), kw.get("target_width", w)]
        flat = timestep_embed_256(vals).flatten().unsqueeze(0).repeat(pooled.shape[0], 1)
        return torch.cat((pooled.to(flat.device), flat), dim=1)


class SD21UNCLIP(BaseModel):
    def __init__(self, model_config, noise_aug_config=None, model_type=ModelType.V_PREDICTION, device=None):
        super().__init__(model_config, model_type, device=device)
        from ..models.noise_aug import CLIPEmbeddingNoiseAugmentation
        self.noise_augmentor = CLIPEmbeddingNoiseAugmentation(**(noise_aug_config or {}))

    def encode_adm(self, **kw):
        uc = kw.get("unclip_conditioning")
        device = kw["device"]
        if uc is None:
            return torch.zeros((1, self.adm_channels))
        return unclip_adm(uc, device, self.noise_augmentor, kw.get("unclip_noise_augment_merge", 0.05), kw.get("seed", 0) - 10)


class IP2P:
    def extra_conds(self, **kwargs):
        out = {}
        image = kwargs.get("concat_latent_image")
        noise = kwargs.get("noise")
        device = kwargs["device"]
        if image is None:
            image = torch.zeros_like(noise)
        if image.shape[1:] != noise.shape[1:]:
            image = common_upscale(image.to(device), noise.shape[-1], noise.shape[-2], "bilinear", "center")
        image = C.repeat_to_batch_size(image, noise.shape[0])
        out["c_concat"] = C.CONDNoiseShape(self.process_ip2p_image_in(image))
        adm = self.encode_adm(**kwargs)
        if adm is not None:
            out["y"] = C.CONDRegular(adm)
        ca = kwargs.get("cross_attn")
        if ca is not None:
            out["c_crossattn"] = C.CONDCrossAttn(ca)
        return out


class SD15_instructpix2pix(IP2P, BaseModel):
    def process_ip2p_image_in(self, image):
        return image


class SDXL_instructpix2pix(IP2P, SDXL):
    def process_ip2p_image_in(self, image):
        return self.latent_format.process_in(image)


class SD_X4Upscaler(BaseModel):
    def __init__(self, model_config, model_type=ModelType.V_PREDICTION, device=None):
        super().__init__(model_config, model_type, device=device)
        from ..models.noise_aug import ImageConcatWithNoiseAugmentation
        self.noise_augmentor = ImageConcatWithNoiseAugmentation(
            noise_schedule_config={"linear_start": 0.0001, "linear_end": 0.02}, max_noise_level=350)

    def extra_conds(self, **kwargs):
        out = {}
        image = kwargs.get("concat_image")
        noise = kwargs.get("noise")
        noise_augment = kwargs.get("noise_augmentation", 0.0)
        device = kwargs["device"]
        seed = kwargs["seed"] - 10
        level = round(self.noise_augmentor.max_noise_level * noise_augment)
        if image is None:
            image = torch.zeros_like(noise)[:, :3]
        if image.shape[1:] != noise.shape[1:]:
            image = common_upscale(image.to(device), noise.shape[-1], noise.shape[-2], "bilinear", "center")
        nl = torch.tensor([level], device=device)
        if noise_augment > 0:
            image, nl = self.noise_augmentor(image.to(device), noise_level=nl, seed=seed)
        image = C.repeat_to_batch_size(image, noise.shape[0])
        out["c_concat"] = C.CONDNoiseShape(image)
        out["y"] = C.CONDRegular(nl)
        ca = kwargs.get("cross_attn")
        if ca is not None:
            out["c_crossattn"] = C.CONDCrossAttn(ca)
        return out


# ------------------------------------------------------------------------------------------------
# Video / novel-view families (model_base.py:336-442): SVD img2vid, SV3D (u / p), Stable Zero123
# ------------------------------------------------------------------------------------------------
def _concat_latent(kwargs, noise):
    from ..utils.image import resize_to_batch_size
    latent_image = kwargs.get("concat_latent_image")
    if latent_image is None:
        latent_image = torch.zeros_like(noise)
    if latent_image.shape[1:] != noise.shape[1:]:
        latent_image = common_upscale(latent_image, noise.shape[-1], noise.shape[-2], "bilinear", "center")
    return resize_to_batch_size(latent_image, noise.shape[0])


class SVD_img2vid(BaseModel):
    """Video UNet (VideoResBlock / SpatialVideoTransformer) conditioned on the CLIP-vision embedding
    (c_crossattn), the start-frame latent (c_concat) and fps / motion bucket / augmentation ADM."""

    def __init__(self, model_config, model_type=ModelType.V_PREDICTION_EDM, device=None):
        super().__init__(model_config, model_type, device=device)

    def encode_adm(self, **kwargs):
        vals = [kwargs.get("fps", 6) - 1, kwargs.get("motion_bucket_id", 127), kwargs.get("augmentation_level", 0)]
        return timestep_embed_256(vals).flatten().unsqueeze(0)

    def extra_conds(self, **kwargs):
        out = {}
        adm = self.encode_adm(**kwargs)
        if adm is not None:
            out["y"] = C.CONDRegular(adm)
        noise = kwargs.get("noise")
        out["c_concat"] = C.CONDNoiseShape(_concat_latent(kwargs, noise))
        ca = kwargs.get("cross_attn")
        if ca is not None:
            out["c_crossattn"] = C.CONDCrossAttn(ca)
        if "time_conditioning" in kwargs:
            out["time_context"] = C.CONDCrossAttn(kwargs["time_conditioning"])
        out["num_video_frames"] = C.CONDConstant(noise.shape[0])
        return out


class SV3D_u(SVD_img2vid):
    def encode_adm(self, **kwargs):
        return timestep_embed_256([kwargs.get("augmentation_level", 0)]).flatten().unsqueeze(0)


class SV3D_p(SVD_img2vid):
    def encode_adm(self, **kwargs):
        from ..utils.image import resize_to_batch_size
        noise = kwargs.get("noise")
        aug = timestep_embed_256([kwargs.get("augmentation_level", 0)])
        elev = torch.deg2rad(torch.fmod(torch.tensor([90.0 - float(v) for v in _as_list(kwargs.get("elevation", 0))]),
                                        360.0))
        azim = torch.deg2rad(torch.fmod(torch.tensor([float(v) for v in _as_list(kwargs.get("azimuth", 0))]), 360.0))
        parts = [aug, ops.core.timestep_embedding(elev, 512), ops.core.timestep_embedding(azim, 512)]
        parts = [resize_to_batch_size(p, noise.shape[0]) for p in parts]
        return torch.cat(parts, dim=1)


def _as_list(v):
    if isinstance(v, torch.Tensor):
        return v.flatten().tolist()
    return list(v) if isinstance(v, (list, tuple)) else [v]


class Stable_Zero123(BaseModel):
    """SD1.5-shaped UNet with 8 input channels: noise ‖ start-image latent, and a ``cc_projection``
    (768+4 -> 768) applied to the CLIP-vision + camera embedding (model_base.py:414-442)."""

    def __init__(self, model_config, model_type=ModelType.EPS, device=None, cc_in=772, cc_out=768):
        super().__init__(model_config, model_type, device=device)
        from ..models.layers import Linear
        self.cc_projection = Linear(cc_in, cc_out, dtype=self.get_dtype(), device=device)

    def load_model_weights(self, sd, unet_prefix=""):
        for name in ("weight", "bias"):
            k = f"cc_projection.{name}"
            if k in sd:
                getattr(self.cc_projection, name).data = sd.pop(k).to(self.get_dtype())
        return super().load_model_weights(sd, unet_prefix)

    def extra_conds(self, **kwargs):
        out = {}
        noise = kwargs.get("noise")
        out["c_concat"] = C.CONDNoiseShape(_concat_latent(kwargs, noise))
        ca = kwargs.get("cross_attn")
        if ca is not None:
            if ca.shape[-1] != 768:
                w = self.cc_projection.weight
                ca = self.cc_projection(ca.to(device=w.device, dtype=w.dtype))
            out["c_crossattn"] = C.CONDCrossAttn(ca)
        return out
