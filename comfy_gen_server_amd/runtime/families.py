"""Model-family registry (parity: ``comfy/supported_models.py:1-481`` and
``supported_models_base.py:1-95``).

Each family: UNet-config match keys, extra config, latent format, sampling settings, CLIP stack,
state-dict prefix remaps for load and save, model-type detection (eps / v / EDM / v-EDM).
"""
from __future__ import annotations

import torch

from . import latent_formats
from . import model_base
from .convert import state_dict_prefix_replace, openclip_to_hf, hf_to_openclip


class ClipTarget:
    def __init__(self, stack_cls):
        self.stack = stack_cls
        self.params = {}


class BASE:
    unet_config = {}
    unet_extra_config = {"num_heads": -1, "num_head_channels": 64}
    required_keys = {}
    clip_prefix = []
    clip_vision_prefix = None
    noise_aug_config = None
    sampling_settings = {}
    latent_format = latent_formats.LatentFormat
    vae_key_prefix = ["first_stage_model."]
    text_encoder_key_prefix = ["cond_stage_model."]
    supported_inference_dtypes = [torch.bfloat16, torch.float16, torch.float32]
    manual_cast_dtype = None

    @classmethod
    def matches(cls, unet_config, sd=None):
        for k, v in cls.unet_config.items():
            if k not in unet_config or unet_config[k] != v:
                return False
        if sd is not None:
            for k in cls.required_keys:
                if k not in sd:
                    return False
        return True

    def __init__(self, unet_config):
        self.unet_config = dict(unet_config)
        self.sampling_settings = dict(self.sampling_settings)
        self.latent_format = self.latent_format()
        self.unet_config.update(self.unet_extra_config)

    def model_type(self, sd, prefix=""):
        return model_base.ModelType.EPS

    def inpaint_model(self):
        return self.unet_config.get("in_channels", 4) > 4

    def get_model(self, sd, prefix="", device=None):
        if self.noise_aug_config is not None:
            out = model_base.SD21UNCLIP(self, self.noise_aug_config, model_type=self.model_type(sd, prefix), device=device)
        else:
            out = model_base.BaseModel(self, model_type=self.model_type(sd, prefix), device=device)
        if self.inpaint_model():
            out.set_inpaint()
        return out

    def clip_target(self):
        return None

    def process_clip_state_dict(self, sd):
        return state_dict_prefix_replace(sd, {k: "" for k in self.text_encoder_key_prefix}, filter_keys=True)

    def process_unet_state_dict(self, sd):
        return sd

    def process_vae_state_dict(self, sd):
        return sd

    def process_clip_state_dict_for_saving(self, sd):
        return state_dict_prefix_replace(dict(sd), {"": self.text_encoder_key_prefix[0]})

    def process_clip_vision_state_dict_for_saving(self, sd):
        rp = {"": self.clip_vision_prefix} if self.clip_vision_prefix is not None else {}
        return state_dict_prefix_replace(dict(sd), rp)

    def process_unet_state_dict_for_saving(self, sd):
        return state_dict_prefix_replace(dict(sd), {"": "model.diffusion_model."})

    def process_vae_state_dict_for_saving(self, sd):
        return state_dict_prefix_replace(dict(sd), {"": self.vae_key_prefix[0]})

    def set_inference_dtype(self, dtype, manual_cast_dtype=None):
        self.unet_config["dtype"] = dtype
        self.manual_cast_dtype = manual_cast_dtype


def _text_encoders():
    from ..models import text_encoders as te
    return te


class SD15(BASE):
    unet_config = {"context_dim": 768, "model_channels": 320, "use_linear_in_transformer": False,
                   "adm_in_channels": None, "use_temporal_attention": False}
    unet_extra_config = {"num_heads": 8, "num_head_channels": -1}
    latent_format = latent_formats.SD15

    def process_clip_state_dict(self, sd):
        for k in list(sd.keys()):
            if k.startswith("cond_stage_model.transformer.") and not k.startswith("cond_stage_model.transformer.text_model."):
                sd[k.replace("cond_stage_model.transformer.", "cond_stage_model.transformer.text_model.")] = sd.pop(k)
        sd.pop("cond_stage_model.transformer.text_model.embeddings.position_ids", None)
        return state_dict_prefix_replace(sd, {"cond_stage_model.": "clip_l."}, filter_keys=True)

    def process_clip_state_dict_for_saving(self, sd):
        sd = dict(sd)
        for p in ("clip_l.transformer.text_projection.weight", "clip_l.logit_scale"):
            sd.pop(p, None)
        return state_dict_prefix_replace(sd, {"clip_l.": "cond_stage_model."})

    def clip_target(self):
        return ClipTarget(_text_encoders().SD1ClipModel)


class SD20(BASE):
    unet_config = {"context_dim": 1024, "model_channels": 320, "use_linear_in_transformer": True,
                   "adm_in_channels": None, "use_temporal_attention": False}
    latent_format = latent_formats.SD15

    def model_type(self, sd, prefix=""):
        if self.unet_config["in_channels"] == 4:
            k = f"{prefix}output_blocks.11.1.transformer_blocks.0.norm1.bias"
            out = sd.get(k)
            if out is not None and torch.std(out.float(), unbiased=False) > 0.09:
                return model_base.ModelType.V_PREDICTION
        return model_base.ModelType.EPS

    def process_clip_state_dict(self, sd):
        sd = state_dict_prefix_replace(sd, {"conditioner.embedders.0.model.": "clip_h.",
                                            "cond_stage_model.model.": "clip_h."}, filter_keys=True)
        return openclip_to_hf(sd, "clip_h.", "clip_h.transformer.")

    def process_clip_state_dict_for_saving(self, sd):
        out = hf_to_openclip(sd, "clip_h.", "")
        return state_dict_prefix_replace(out, {"": "cond_stage_model.model."})

    def clip_target(self):
        return ClipTarget(_text_encoders().SD2ClipModel)


class SD21UnclipL(SD20):
    unet_config = {"context_dim": 1024, "model_channels": 320, "use_linear_in_transformer": True,
                   "adm_in_channels": 1536, "use_temporal_attention": False}
    clip_vision_prefix = "embedder.model.visual."
    noise_aug_config = {"noise_schedule_config": {"timesteps": 1000, "beta_schedule": "squaredcos_cap_v2"},
                        "timestep_dim": 768}


class SD21UnclipH(SD20):
    unet_config = {"context_dim": 1024, "model_channels": 320, "use_linear_in_transformer": True,
                   "adm_in_channels": 2048, "use_temporal_attention": False}
    clip_vision_prefix = "embedder.model.visual."
    noise_aug_config = {"noise_schedule_config": {"timesteps": 1000, "beta_schedule": "squaredcos_cap_v2"},
                        "timestep_dim": 1024}


class SDXLRefiner(BASE):
    unet_config = {"model_channels": 384, "use_linear_in_transformer": True, "context_dim": 1280,
                   "adm_in_channels": 2560, "transformer_depth": [0, 0, 4, 4, 4, 4, 0, 0],
                   "use_temporal_attention": False}
    latent_format = latent_formats.SDXL

    def get_model(self, sd, prefix="", device=None):
        return model_base.SDXLRefiner(self, device=device)

    def process_clip_state_dict(self, sd):
        sd = state_dict_prefix_replace(sd, {"conditioner.embedders.0.model.": "clip_g."}, filter_keys=True)
        return openclip_to_hf(sd, "clip_g.", "clip_g.transformer.")

    def process_clip_state_dict_for_saving(self, sd):
        out = hf_to_openclip(sd, "clip_g.", "")
        return state_dict_prefix_replace(out, {"": "conditioner.embedders.0.model."})

    def clip_target(self):
        return ClipTarget(_text_encoders().SDXLRefinerClipModel)


class SDXL(BASE):
    unet_config = {"model_channels": 320, "use_linear_in_transformer": True,
                   "transformer_depth": [0, 0, 2, 2, 10, 10], "context_dim": 2048, "adm_in_channels": 2816,
                   "use_temporal_attention": False}
    latent_format = latent_formats.SDXL

    def model_type(self, sd, prefix=""):
        if "edm_mean" in sd and "edm_std" in sd:   # Playground 2.5
            self.latent_format = latent_formats.SDXL_Playground_2_5()
            self.sampling_settings.update(sigma_data=0.5, sigma_max=80.0, sigma_min=0.002)
            return model_base.ModelType.EDM
        if "edm_vpred.sigma_max" in sd:
            self.sampling_settings["sigma_max"] = float(sd["edm_vpred.sigma_max"].item())
            if "edm_vpred.sigma_min" in sd:
                self.sampling_settings["sigma_min"] = float(sd["edm_vpred.sigma_min"].item())
            return model_base.ModelType.V_PREDICTION_EDM
        if "v_pred" in sd:
            return model_base.ModelType.V_PREDICTION
        return model_base.ModelType.EPS

    def get_model(self, sd, prefix="", device=None):
        out = model_base.SDXL(self, model_type=self.model_type(sd, prefix), device=device)
        if self.inpaint_model():
            out.set_inpaint()
        return out

    def process_clip_state_dict(self, sd):
        sd = state_dict_prefix_replace(sd, {"conditioner.embedders.0.transformer.text_model": "clip_l.transformer.text_model",
                                            "conditioner.embedders.1.model.": "clip_g."}, filter_keys=True)
        sd.pop("clip_l.transformer.text_model.embeddings.position_ids", None)
        return openclip_to_hf(sd, "clip_g.", "clip_g.transformer.")

    def process_clip_state_dict_for_saving(self, sd):
        out = hf_to_openclip(sd, "clip_g.", "conditioner.embedders.1.model.")
        for k, v in sd.items():
            if k.startswith("clip_l.") and "text_projection" not in k and "logit_scale" not in k:
                out["conditioner.embedders.0." + k[len("clip_l."):]] = v
        out["conditioner.embedders.0.transformer.text_model.embeddings.position_ids"] = torch.arange(77).expand((1, -1))
        return out

    def clip_target(self):
        return ClipTarget(_text_encoders().SDXLClipModel)


class SSD1B(SDXL):
    unet_config = {"model_channels": 320, "use_linear_in_transformer": True, "transformer_depth": [0, 0, 2, 2, 4, 4],
                   "context_dim": 2048, "adm_in_channels": 2816, "use_temporal_attention": False}


class Segmind_Vega(SDXL):
    unet_config = {"model_channels": 320, "use_linear_in_transformer": True, "transformer_depth": [0, 0, 1, 1, 2, 2],
                   "context_dim": 2048, "adm_in_channels": 2816, "use_temporal_attention": False}


class KOALA_700M(SDXL):
    unet_config = {"model_channels": 320, "use_linear_in_transformer": True, "transformer_depth": [0, 2, 5],
                   "context_dim": 2048, "adm_in_channels": 2816, "use_temporal_attention": False}


class KOALA_1B(SDXL):
    unet_config = {"model_channels": 320, "use_linear_in_transformer": True, "transformer_depth": [0, 2, 6],
                   "context_dim": 2048, "adm_in_channels": 2816, "use_temporal_attention": False}


class SD_X4Upscaler(SD20):
    unet_config = {"context_dim": 1024, "model_channels": 256, "in_channels": 7, "use_linear_in_transformer": True,
                   "adm_in_channels": None, "use_temporal_attention": False}
    unet_extra_config = {"disable_self_attentions": [True, True, True, False], "num_classes": 1000,
                         "num_heads": 8, "num_head_channels": -1}
    latent_format = latent_formats.SD_X4
    sampling_settings = {"linear_start": 0.0001, "linear_end": 0.02}

    def get_model(self, sd, prefix="", device=None):
        return model_base.SD_X4Upscaler(self, device=device)


class SD15_instructpix2pix(SD15):
    unet_config = dict(SD15.unet_config, in_channels=8)

    def get_model(self, sd, prefix="", device=None):
        return model_base.SD15_instructpix2pix(self, device=device)


class SDXL_instructpix2pix(SDXL):
    unet_config = dict(SDXL.unet_config, in_channels=8)

    def get_model(self, sd, prefix="", device=None):
        return model_base.SDXL_instructpix2pix(self, model_type=self.model_type(sd, prefix), device=device)


class Stable_Zero123(BASE):
    unet_config = {"context_dim": 768, "model_channels": 320, "use_linear_in_transformer": False,
                   "adm_in_channels": None, "use_temporal_attention": False, "in_channels": 8}
    unet_extra_config = {"num_heads": 8, "num_head_channels": -1}
    required_keys = {"cc_projection.weight": None, "cc_projection.bias": None}
    clip_vision_prefix = "cond_stage_model.model.visual."
    latent_format = latent_formats.SD15

    def get_model(self, sd, prefix="", device=None):
        w = sd.get("cc_projection.weight") if sd else None
        shape = tuple(w.shape) if w is not None else (768, 772)
        return model_base.Stable_Zero123(self, device=device, cc_in=shape[1], cc_out=shape[0])


class SVD_img2vid(BASE):
    """Stable Video Diffusion img2vid (supported_models.py:267-290)."""
    unet_config = {"model_channels": 320, "in_channels": 8, "use_linear_in_transformer": True,
                   "transformer_depth": [1, 1, 1, 1, 1, 1, 0, 0], "context_dim": 1024, "adm_in_channels": 768,
                   "use_temporal_attention": True, "use_temporal_resblock": True}
    unet_extra_config = {"num_heads": -1, "num_head_channels": 64}
    clip_vision_prefix = "conditioner.embedders.0.open_clip.model.visual."
    latent_format = latent_formats.SD15
    sampling_settings = {"sigma_max": 700.0, "sigma_min": 0.002}

    def model_type(self, sd, prefix=""):
        return model_base.ModelType.V_PREDICTION_EDM

    def get_model(self, sd, prefix="", device=None):
        return model_base.SVD_img2vid(self, device=device)


class SV3D_u(SVD_img2vid):
    unet_config = dict(SVD_img2vid.unet_config, adm_in_channels=256)
    vae_key_prefix = ["conditioner.embedders.1.encoder."]

    def get_model(self, sd, prefix="", device=None):
        return model_base.SV3D_u(self, device=device)


class SV3D_p(SV3D_u):
    unet_config = dict(SVD_img2vid.unet_config, adm_in_channels=1280)

    def get_model(self, sd, prefix="", device=None):
        return model_base.SV3D_p(self, device=device)


class Stable_Cascade_C(BASE):
    unet_config = {"stable_cascade_stage": "c"}
    unet_extra_config = {}
    latent_format = latent_formats.SC_Prior
    supported_inference_dtypes = [torch.bfloat16, torch.float32]
    sampling_settings = {"shift": 2.0}
    vae_key_prefix = ["vae."]
    text_encoder_key_prefix = ["text_encoder."]
    clip_vision_prefix = "clip_l_vision."

    def model_type(self, sd, prefix=""):
        return model_base.ModelType.STABLE_CASCADE

    def process_unet_state_dict(self, sd):
        for k in [k for k in list(sd.keys()) if k.endswith("in_proj_weight") or k.endswith("in_proj_bias")]:
            w = sd.pop(k)
            suffix = k.rsplit(".", 1)[1].replace("in_proj_", "")
            prefix = k[: -(len("in_proj_") + len(suffix) + 1)]
            n = w.shape[0] // 3
            for i, nm in enumerate(("to_q", "to_k", "to_v")):
                sd[f"{prefix}.{nm}.{suffix}"] = w[i * n:(i + 1) * n]
        return sd

    def process_clip_state_dict(self, sd):
        sd = state_dict_prefix_replace(sd, {k: "" for k in self.text_encoder_key_prefix}, filter_keys=True)
        if "clip_g.text_projection" in sd:
            sd["clip_g.transformer.text_projection.weight"] = sd.pop("clip_g.text_projection").transpose(0, 1)
        return sd

    def get_model(self, sd, prefix="", device=None):
        from ..models.cascade import StableCascade_C
        return StableCascade_C(self, device=device)

    def clip_target(self):
        return ClipTarget(_text_encoders().StableCascadeClipModel)


class Stable_Cascade_B(Stable_Cascade_C):
    unet_config = {"stable_cascade_stage": "b"}
    latent_format = latent_formats.SC_B
    supported_inference_dtypes = [torch.float16, torch.bfloat16, torch.float32]
    sampling_settings = {"shift": 1.0}
    clip_vision_prefix = None

    def get_model(self, sd, prefix="", device=None):
        from ..models.cascade import StableCascade_B
        return StableCascade_B(self, device=device)


MODELS = [Stable_Zero123, SD15_instructpix2pix, SD15, SD20, SD21UnclipL, SD21UnclipH, SDXL_instructpix2pix,
          SDXLRefiner, SDXL, SSD1B, KOALA_700M, KOALA_1B, Segmind_Vega, SD_X4Upscaler, Stable_Cascade_C,
          Stable_Cascade_B, SV3D_u, SV3D_p, SVD_img2vid]
