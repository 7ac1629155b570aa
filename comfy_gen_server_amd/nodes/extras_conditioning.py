"""Conditioning extras (parity: ``comfy_extras/nodes_clip_sdxl.py``, ``nodes_cond.py``, ``nodes_ip2p.py``,
``nodes_sdupscale.py``, ``nodes_stable3d.py``, ``nodes_photomaker.py``, ``nodes_video_model.py``
(image-only loader + SVD conditioning); SURVEY §2.2 'Conditioning').
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ..models.clip import CLIPVisionModelProjection
from ..models.layers import LayerNorm, Linear
from ..runtime import device as dm
from ..runtime import sd as sdl
from ..runtime.checkpoint import load_state_dict
from ..runtime.clip_vision import clip_preprocess
from ..utils import folder_paths
from ..utils import image as U

MAX_RESOLUTION = 16384


class CLIPTextEncodeSDXLRefiner:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"ascore": ("FLOAT", {"default": 6.0, "min": 0.0, "max": 1000.0, "step": 0.01}),
                             "width": ("INT", {"default": 1024.0, "min": 0, "max": MAX_RESOLUTION}),
                             "height": ("INT", {"default": 1024.0, "min": 0, "max": MAX_RESOLUTION}),
                             "text": ("STRING", {"multiline": True, "dynamicPrompts": True}), "clip": ("CLIP",)}}
    RETURN_TYPES = ("CONDITIONING",)
    FUNCTION = "encode"
    CATEGORY = "advanced/conditioning"

    def encode(self, clip, ascore, width, height, text):
        cond, pooled = clip.encode_from_tokens(clip.tokenize(text), return_pooled=True)
        return ([[cond, {"pooled_output": pooled, "aesthetic_score": ascore, "width": width, "height": height}]],)


class CLIPTextEncodeSDXL:
    @classmethod
    def INPUT_TYPES(s):
        i = lambda d: ("INT", {"default": d, "min": 0, "max": MAX_RESOLUTION})  # noqa: E731
        return {"required": {"width": i(1024.0), "height": i(1024.0), "crop_w": i(0), "crop_h": i(0),
                             "target_width": i(1024.0), "target_height": i(1024.0),
                             "text_g": ("STRING", {"multiline": True, "dynamicPrompts": True}), "clip": ("CLIP",),
                             "text_l": ("STRING", {"multiline": True, "dynamicPrompts": True})}}
    RETURN_TYPES = ("CONDITIONING",)
    FUNCTION = "encode"
    CATEGORY = "advanced/conditioning"

    def encode(self, clip, width, height, crop_w, crop_h, target_width, target_height, text_g, text_l):
        tokens = clip.tokenize(text_g)
        tokens["l"] = clip.tokenize(text_l)["l"]
        if len(tokens["l"]) != len(tokens["g"]):      # pad the shorter stream with empty 77-chunks
            empty = clip.tokenize("")
            while len(tokens["l"]) < len(tokens["g"]):
                tokens["l"] += empty["l"]
            while len(tokens["l"]) > len(tokens["g"]):
                tokens["g"] += empty["g"]
        cond, pooled = clip.encode_from_tokens(tokens, return_pooled=True)
        return ([[cond, {"pooled_output": pooled, "width": width, "height": height, "crop_w": crop_w,
                         "crop_h": crop_h, "target_width": target_width, "target_height": target_height}]],)


class CLIPTextEncodeControlnet:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"clip": ("CLIP",), "conditioning": ("CONDITIONING",),
                             "text": ("STRING", {"multiline": True, "dynamicPrompts": True})}}
    RETURN_TYPES = ("CONDITIONING",)
    FUNCTION = "encode"
    CATEGORY = "_for_testing/conditioning"

    def encode(self, clip, conditioning, text):
        cond, pooled = clip.encode_from_tokens(clip.tokenize(text), return_pooled=True)
        out = []
        for t in conditioning:
            d = t[1].copy()
            d["cross_attn_controlnet"] = cond
            d["pooled_output_controlnet"] = pooled
            out.append([t[0], d])
        return (out,)


def _with(conditioning, **values):
    out = []
    for t in conditioning:
        d = t[1].copy()
        d.update(values)
        out.append([t[0], d])
    return out


class InstructPixToPixConditioning:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"positive": ("CONDITIONING",), "negative": ("CONDITIONING",), "vae": ("VAE",),
                             "pixels": ("IMAGE",)}}
    RETURN_TYPES = ("CONDITIONING", "CONDITIONING", "LATENT")
    RETURN_NAMES = ("positive", "negative", "latent")
    FUNCTION = "encode"
    CATEGORY = "conditioning/instructpix2pix"

    def encode(self, positive, negative, pixels, vae):
        x = (pixels.shape[1] // 8) * 8
        y = (pixels.shape[2] // 8) * 8
        if pixels.shape[1] != x or pixels.shape[2] != y:
            xo = (pixels.shape[1] % 8) // 2
            yo = (pixels.shape[2] % 8) // 2
            pixels = pixels[:, xo:x + xo, yo:y + yo, :]
        concat = vae.encode(pixels)
        return (_with(positive, concat_latent_image=concat), _with(negative, concat_latent_image=concat),
                {"samples": torch.zeros_like(concat)})


class SD_4XUpscale_Conditioning:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"images": ("IMAGE",), "positive": ("CONDITIONING",), "negative": ("CONDITIONING",),
                             "scale_ratio": ("FLOAT", {"default": 4.0, "min": 0.0, "max": 10.0, "step": 0.01}),
                             "noise_augmentation": ("FLOAT", {"default": 0.0, "min": 0.0, "max": 1.0, "step": 0.001})}}
    RETURN_TYPES = ("CONDITIONING", "CONDITIONING", "LATENT")
    RETURN_NAMES = ("positive", "negative", "latent")
    FUNCTION = "encode"
    CATEGORY = "conditioning/upscale_diffusion"

    def encode(self, images, positive, negative, scale_ratio, noise_augmentation):
        w = max(1, round(images.shape[-2] * scale_ratio))
        h = max(1, round(images.shape[-3] * scale_ratio))
        px = U.common_upscale(images.movedim(-1, 1) * 2.0 - 1.0, w // 4, h // 4, "bilinear", "center")
        kw = {"concat_image": px, "noise_augmentation": noise_augmentation}
        return (_with(positive, **kw), _with(negative, **kw),
                {"samples": torch.zeros([images.shape[0], 4, h // 4, w // 4])})


# ---------------------------------------------------------------- image-conditioned (3D / video)
def camera_embeddings(elevation, azimuth):
    """Zero123 camera embedding [1,1,4]: (polar offset, sin az, cos az, 90 deg) in radians."""
    el = torch.as_tensor([elevation])
    az = torch.as_tensor([azimuth])
    return torch.stack([torch.deg2rad((90 - el) - 90), torch.sin(torch.deg2rad(az)),
                        torch.cos(torch.deg2rad(az)), torch.deg2rad(90 - torch.full_like(el, 0))], dim=-1)[:, None]


def _encode_init(clip_vision, init_image, vae, width, height):
    out = clip_vision.encode_image(init_image)
    pooled = out.image_embeds.unsqueeze(0)
    px = U.common_upscale(init_image.movedim(-1, 1), width, height, "bilinear", "center").movedim(1, -1)
    return pooled, px[:, :, :, :3], vae


class StableZero123_Conditioning:
    @classmethod
    def INPUT_TYPES(s):
        f = lambda: ("FLOAT", {"default": 0.0, "min": -180.0, "max": 180.0, "step": 0.1, "round": False})  # noqa: E731
        return {"required": {"clip_vision": ("CLIP_VISION",), "init_image": ("IMAGE",), "vae": ("VAE",),
                             "width": ("INT", {"default": 256, "min": 16, "max": MAX_RESOLUTION, "step": 8}),
                             "height": ("INT", {"default": 256, "min": 16, "max": MAX_RESOLUTION, "step": 8}),
                             "batch_size": ("INT", {"default": 1, "min": 1, "max": 4096}),
                             "elevation": f(), "azimuth": f()}}
    RETURN_TYPES = ("CONDITIONING", "CONDITIONING", "LATENT")
    RETURN_NAMES = ("positive", "negative", "latent")
    FUNCTION = "encode"
    CATEGORY = "conditioning/3d_models"

    def encode(self, clip_vision, init_image, vae, width, height, batch_size, elevation, azimuth):
        pooled, px, _ = _encode_init(clip_vision, init_image, vae, width, height)
        t = vae.encode(px)
        cam = camera_embeddings(elevation, azimuth).to(pooled.device).repeat(pooled.shape[0], 1, 1)
        cond = torch.cat([pooled, cam], dim=-1)
        return ([[cond, {"concat_latent_image": t}]],
                [[torch.zeros_like(pooled), {"concat_latent_image": torch.zeros_like(t)}]],
                {"samples": torch.zeros([batch_size, 4, height // 8, width // 8])})


class StableZero123_Conditioning_Batched(StableZero123_Conditioning):
    @classmethod
    def INPUT_TYPES(s):
        d = StableZero123_Conditioning.INPUT_TYPES()
        f = ("FLOAT", {"default": 0.0, "min": -180.0, "max": 180.0, "step": 0.1, "round": False})
        d["required"]["elevation_batch_increment"] = f
        d["required"]["azimuth_batch_increment"] = f
        return d

    def encode(self, clip_vision, init_image, vae, width, height, batch_size, elevation, azimuth,
               elevation_batch_increment=0.0, azimuth_batch_increment=0.0):
        pooled, px, _ = _encode_init(clip_vision, init_image, vae, width, height)
        t = vae.encode(px)
        cams = []
        for _ in range(batch_size):
            cams.append(camera_embeddings(elevation, azimuth))
            elevation += elevation_batch_increment
            azimuth += azimuth_batch_increment
        cond = torch.cat([U.repeat_to_batch_size(pooled, batch_size), torch.cat(cams, 0).to(pooled.device)], -1)
        return ([[cond, {"concat_latent_image": t}]],
                [[torch.zeros_like(pooled), {"concat_latent_image": torch.zeros_like(t)}]],
                {"samples": torch.zeros([batch_size, 4, height // 8, width // 8]), "batch_index": [0] * batch_size})


class SV3D_Conditioning:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"clip_vision": ("CLIP_VISION",), "init_image": ("IMAGE",), "vae": ("VAE",),
                             "width": ("INT", {"default": 576, "min": 16, "max": MAX_RESOLUTION, "step": 8}),
                             "height": ("INT", {"default": 576, "min": 16, "max": MAX_RESOLUTION, "step": 8}),
                             "video_frames": ("INT", {"default": 21, "min": 1, "max": 4096}),
                             "elevation": ("FLOAT", {"default": 0.0, "min": -90.0, "max": 90.0, "step": 0.1,
                                                     "round": False})}}
    RETURN_TYPES = ("CONDITIONING", "CONDITIONING", "LATENT")
    RETURN_NAMES = ("positive", "negative", "latent")
    FUNCTION = "encode"
    CATEGORY = "conditioning/3d_models"

    def encode(self, clip_vision, init_image, vae, width, height, video_frames, elevation):
        pooled, px, _ = _encode_init(clip_vision, init_image, vae, width, height)
        t = vae.encode(px)
        inc = 360 / (max(video_frames, 2) - 1)
        elevations = [elevation] * video_frames
        azimuths = [i * inc for i in range(video_frames)]
        extra = {"elevation": elevations, "azimuth": azimuths}
        return ([[pooled, dict(concat_latent_image=t, **extra)]],
                [[torch.zeros_like(pooled), dict(concat_latent_image=torch.zeros_like(t), **extra)]],
                {"samples": torch.zeros([video_frames, 4, height // 8, width // 8])})


class ImageOnlyCheckpointLoader:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"ckpt_name": (folder_paths.get_filename_list("checkpoints"),)}}
    RETURN_TYPES = ("MODEL", "CLIP_VISION", "VAE")
    FUNCTION = "load_checkpoint"
    CATEGORY = "loaders/video_models"

    def load_checkpoint(self, ckpt_name, output_vae=True, output_clip=True):
        out = sdl.load_checkpoint_guess_config(folder_paths.get_full_path("checkpoints", ckpt_name), output_vae=True,
                                               output_clip=False, output_clipvision=True,
                                               embedding_directory=folder_paths.get_folder_paths("embeddings"))
        return (out[0], out[3], out[2])


class SVD_img2vid_Conditioning:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"clip_vision": ("CLIP_VISION",), "init_image": ("IMAGE",), "vae": ("VAE",),
                             "width": ("INT", {"default": 1024, "min": 16, "max": MAX_RESOLUTION, "step": 8}),
                             "height": ("INT", {"default": 576, "min": 16, "max": MAX_RESOLUTION, "step": 8}),
                             "video_frames": ("INT", {"default": 14, "min": 1, "max": 4096}),
                             "motion_bucket_id": ("INT", {"default": 127, "min": 1, "max": 1023}),
                             "fps": ("INT", {"default": 6, "min": 1, "max": 1024}),
                             "augmentation_level": ("FLOAT", {"default": 0.0, "min": 0.0, "max": 10.0, "step": 0.01})}}
    RETURN_TYPES = ("CONDITIONING", "CONDITIONING", "LATENT")
    RETURN_NAMES = ("positive", "negative", "latent")
    FUNCTION = "encode"
    CATEGORY = "conditioning/video_models"

    def encode(self, clip_vision, init_image, vae, width, height, video_frames, motion_bucket_id, fps,
               augmentation_level):
        pooled, px, _ = _encode_init(clip_vision, init_image, vae, width, height)
        if augmentation_level > 0:
            px = px + torch.randn_like(px) * augmentation_level
        t = vae.encode(px)
        kw = {"motion_bucket_id": motion_bucket_id, "fps": fps, "augmentation_level": augmentation_level}
        return ([[pooled, dict(concat_latent_image=t, **kw)]],
                [[torch.zeros_like(pooled), dict(concat_latent_image=torch.zeros_like(t), **kw)]],
                {"samples": torch.zeros([video_frames, 4, height // 8, width // 8])})


# ---------------------------------------------------------------- PhotoMaker
PHOTOMAKER_VISION = dict(hidden_size=1024, image_size=224, intermediate_size=4096, num_attention_heads=16,
                         num_channels=3, num_hidden_layers=24, patch_size=14, projection_dim=768,
                         hidden_act="quick_gelu")


class _MLP(nn.Module):
    def __init__(self, in_dim, out_dim, hidden_dim, use_residual=True, dtype=None, device=None):
        super().__init__()
        assert not use_residual or in_dim == out_dim
        self.layernorm = LayerNorm(in_dim, dtype=dtype, device=device)
        self.fc1 = Linear(in_dim, hidden_dim, dtype=dtype, device=device)
        self.fc2 = Linear(hidden_dim, out_dim, dtype=dtype, device=device)
        self.use_residual = use_residual

    def forward(self, x):
        y = self.fc2(torch.nn.functional.gelu(self.fc1(self.layernorm(x))))
        return y + x if self.use_residual else y


class FuseModule(nn.Module):
    """Fuse the ID embedding into the class-token embeddings of the prompt."""

    def __init__(self, embed_dim, dtype=None, device=None):
        super().__init__()
        self.mlp1 = _MLP(embed_dim * 2, embed_dim, embed_dim, use_residual=False, dtype=dtype, device=device)
        self.mlp2 = _MLP(embed_dim, embed_dim, embed_dim, use_residual=True, dtype=dtype, device=device)
        self.layer_norm = LayerNorm(embed_dim, dtype=dtype, device=device)

    def fuse_fn(self, prompt_embeds, id_embeds):
        s = self.mlp1(torch.cat([prompt_embeds, id_embeds], dim=-1)) + prompt_embeds
        return self.layer_norm(self.mlp2(s))

    def forward(self, prompt_embeds, id_embeds, class_tokens_mask):
        id_embeds = id_embeds.to(prompt_embeds.dtype)
        num_inputs = class_tokens_mask.sum().unsqueeze(0)
        b, max_inputs = id_embeds.shape[:2]
        seq = prompt_embeds.shape[1]
        flat = id_embeds.view(-1, id_embeds.shape[-2], id_embeds.shape[-1])
        valid = torch.arange(max_inputs, device=flat.device)[None, :] < num_inputs[:, None]
        valid_ids = flat[valid.flatten()].view(-1, flat.shape[-1])
        pe = prompt_embeds.reshape(-1, prompt_embeds.shape[-1]).clone()
        mask = class_tokens_mask.view(-1)
        fused = self.fuse_fn(pe[mask], valid_ids)
        assert int(mask.sum()) == fused.shape[0]
        pe.masked_scatter_(mask[:, None], fused.to(pe.dtype))
        return pe.view(b, seq, -1)


class PhotoMakerIDEncoder(CLIPVisionModelProjection):
    def __init__(self):
        self.load_device = dm.text_encoder_device()
        dtype = dm.text_encoder_dtype(self.load_device)
        super().__init__(PHOTOMAKER_VISION, dtype=dtype, device=self.load_device)
        self.visual_projection_2 = Linear(1024, 1280, bias=False, dtype=dtype, device=self.load_device)
        self.fuse_module = FuseModule(2048, dtype=dtype, device=self.load_device)

    def forward(self, id_pixel_values, prompt_embeds, class_tokens_mask):
        b, n, c, h, w = id_pixel_values.shape
        _, _, shared = self.vision_model(id_pixel_values.view(b * n, c, h, w))
        e1 = self.visual_projection(shared).view(b, n, 1, -1)
        e2 = self.visual_projection_2(shared).view(b, n, 1, -1)
        return self.fuse_module(prompt_embeds, torch.cat((e1, e2), dim=-1), class_tokens_mask)


class PhotoMakerLoader:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"photomaker_model_name": (folder_paths.get_filename_list("photomaker"),)}}
    RETURN_TYPES = ("PHOTOMAKER",)
    FUNCTION = "load_photomaker_model"
    CATEGORY = "_for_testing/photomaker"

    def load_photomaker_model(self, photomaker_model_name):
        m = PhotoMakerIDEncoder()
        data = load_state_dict(folder_paths.get_full_path("photomaker", photomaker_model_name))
        if "id_encoder" in data:
            data = data["id_encoder"]
        m.load_state_dict(data)
        return (m,)


class PhotoMakerEncode:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"photomaker": ("PHOTOMAKER",), "image": ("IMAGE",), "clip": ("CLIP",),
                             "text": ("STRING", {"multiline": True, "dynamicPrompts": True,
                                                 "default": "photograph of photomaker"})}}
    RETURN_TYPES = ("CONDITIONING",)
    FUNCTION = "apply_photomaker"
    CATEGORY = "_for_testing/photomaker"

    def apply_photomaker(self, photomaker, image, clip, text):
        dev = photomaker.load_device
        px = clip_preprocess(image.to(dev).float()).to(next(photomaker.parameters()).dtype)
        try:
            index = text.split(" ").index("photomaker") + 1
        except ValueError:
            index = -1
        tokens = clip.tokenize(text, return_word_ids=True)
        out_tokens = {}
        for k, chunks in tokens.items():        # drop the trigger word's tokens, pad with the last token
            out_tokens[k] = []
            for t in chunks:
                f = [x for x in t if x[2] != index]
                f += [t[-1]] * (len(t) - len(f))
                out_tokens[k].append(f)
        cond, pooled = clip.encode_from_tokens(out_tokens, return_pooled=True)
        if index > 0:
            mask = torch.tensor([index - 1 <= i < index for i in range(77)], dtype=torch.bool, device=dev)[None]
            out = photomaker(id_pixel_values=px.unsqueeze(0), prompt_embeds=cond.to(dev, px.dtype),
                             class_tokens_mask=mask).to(cond.dtype).to(cond.device)
        else:
            out = cond
        return ([[out, {"pooled_output": pooled}]],)


NODE_CLASS_MAPPINGS = {
    "CLIPTextEncodeSDXLRefiner": CLIPTextEncodeSDXLRefiner, "CLIPTextEncodeSDXL": CLIPTextEncodeSDXL,
    "CLIPTextEncodeControlnet": CLIPTextEncodeControlnet,
    "InstructPixToPixConditioning": InstructPixToPixConditioning,
    "SD_4XUpscale_Conditioning": SD_4XUpscale_Conditioning, "StableZero123_Conditioning": StableZero123_Conditioning,
    "StableZero123_Conditioning_Batched": StableZero123_Conditioning_Batched, "SV3D_Conditioning": SV3D_Conditioning,
    "ImageOnlyCheckpointLoader": ImageOnlyCheckpointLoader, "SVD_img2vid_Conditioning": SVD_img2vid_Conditioning,
    "PhotoMakerLoader": PhotoMakerLoader, "PhotoMakerEncode": PhotoMakerEncode,
}
NODE_DISPLAY_NAME_MAPPINGS = {"ImageOnlyCheckpointLoader": "Image Only Checkpoint Loader (img2vid model)"}
