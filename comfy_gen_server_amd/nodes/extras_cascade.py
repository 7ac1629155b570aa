"""Stable Cascade helper nodes (parity: ``comfy_extras/nodes_stable_cascade.py``).

Stage C works on 16-channel latents at 1/42 (``compression``) of the image, Stage B on 4-channel
latents at 1/4; Stage B is conditioned on the Stage C result through ``stable_cascade_prior``.
"""
from __future__ import annotations

import torch

from ..utils import image as U
from .core import MAX_RESOLUTION


class StableCascade_EmptyLatentImage:
    RETURN_TYPES = ("LATENT", "LATENT")
    RETURN_NAMES = ("stage_c", "stage_b")
    FUNCTION = "generate"
    CATEGORY = "latent/stable_cascade"

    @classmethod
    def INPUT_TYPES(s):
        return {"required": {
            "width": ("INT", {"default": 1024, "min": 256, "max": MAX_RESOLUTION, "step": 8}),
            "height": ("INT", {"default": 1024, "min": 256, "max": MAX_RESOLUTION, "step": 8}),
            "compression": ("INT", {"default": 42, "min": 4, "max": 128, "step": 1}),
            "batch_size": ("INT", {"default": 1, "min": 1, "max": 4096})}}

    def generate(self, width, height, compression, batch_size=1):
        c = torch.zeros([batch_size, 16, height // compression, width // compression])
        b = torch.zeros([batch_size, 4, height // 4, width // 4])
        return ({"samples": c}, {"samples": b})


class StableCascade_StageC_VAEEncode:
    RETURN_TYPES = ("LATENT", "LATENT")
    RETURN_NAMES = ("stage_c", "stage_b")
    FUNCTION = "generate"
    CATEGORY = "latent/stable_cascade"

    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"image": ("IMAGE",), "vae": ("VAE",),
                             "compression": ("INT", {"default": 42, "min": 4, "max": 128, "step": 1})}}

    def generate(self, image, vae, compression):
        """Resize so the effnet encoder (32x down) lands on the 1/compression grid, then encode."""
        h, w = image.shape[-3], image.shape[-2]
        ow, oh = (w // compression) * vae.downscale_ratio, (h // compression) * vae.downscale_ratio
        s = U.common_upscale(image.movedim(-1, 1), ow, oh, "bicubic", "center").movedim(1, -1)
        c = vae.encode(s[:, :, :, :3])
        b = torch.zeros([c.shape[0], 4, (h // 8) * 2, (w // 8) * 2])
        return ({"samples": c}, {"samples": b})


class StableCascade_StageB_Conditioning:
    RETURN_TYPES = ("CONDITIONING",)
    FUNCTION = "set_prior"
    CATEGORY = "conditioning/stable_cascade"

    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"conditioning": ("CONDITIONING",), "stage_c": ("LATENT",)}}

    def set_prior(self, conditioning, stage_c):
        out = []
        for t in conditioning:
            d = t[1].copy()
            d["stable_cascade_prior"] = stage_c["samples"]
            out.append([t[0], d])
        return (out,)


class StableCascade_SuperResolutionControlnet:
    RETURN_TYPES = ("IMAGE", "LATENT", "LATENT")
    RETURN_NAMES = ("controlnet_input", "stage_c", "stage_b")
    FUNCTION = "generate"
    CATEGORY = "_for_testing/stable_cascade"

    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"image": ("IMAGE",), "vae": ("VAE",)}}

    def generate(self, image, vae):
        h, w, n = image.shape[-3], image.shape[-2], image.shape[0]
        cn_in = vae.encode(image[:, :, :, :3]).movedim(1, -1)
        c = torch.zeros([n, 16, h // 16, w // 16])
        b = torch.zeros([n, 4, h // 2, w // 2])
        return (cn_in, {"samples": c}, {"samples": b})


NODE_CLASS_MAPPINGS = {
    "StableCascade_EmptyLatentImage": StableCascade_EmptyLatentImage,
    "StableCascade_StageB_Conditioning": StableCascade_StageB_Conditioning,
    "StableCascade_StageC_VAEEncode": StableCascade_StageC_VAEEncode,
    "StableCascade_SuperResolutionControlnet": StableCascade_SuperResolutionControlnet,
}
