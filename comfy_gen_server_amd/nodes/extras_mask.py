"""Mask nodes + masked compositing (parity: ``comfy_extras/nodes_mask.py``; SURVEY §2.2 'Image / mask').

MASK = float [B,H,W] (or [H,W]) in 0..1 on the host; IMAGE = float [B,H,W,C] in 0..1.
Deliberate fix: ``FeatherMask`` feathers the LAST ``right``/``bottom`` columns/rows (the reference
indexes ``-x`` from x = 0, which hits column 0 first, nodes_mask.py:287-297). ``ImageColorToMask``
keeps the reference's 255 for a match (nodes_mask.py:149) for workflow compatibility.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ..utils import image as U

MAX_RESOLUTION = 16384


def composite(destination, source, x, y, mask=None, multiplier=8, resize_source=False):
    """Paste ``source`` into ``destination`` (NCHW) at pixel (x, y) (/multiplier for latents), blended by
    ``mask``; out-of-bounds parts are clipped (nodes_mask.py:8-40)."""
    source = source.to(destination.device)
    if resize_source:
        source = F.interpolate(source, size=destination.shape[2:], mode="bilinear")
    source = U.repeat_to_batch_size(source, destination.shape[0])
    x = max(-source.shape[3] * multiplier, min(x, destination.shape[3] * multiplier))
    y = max(-source.shape[2] * multiplier, min(y, destination.shape[2] * multiplier))
    left, top = x // multiplier, y // multiplier
    right, bottom = left + source.shape[3], top + source.shape[2]
    if mask is None:
        mask = torch.ones_like(source)
    else:
        mask = F.interpolate(mask.to(destination.device).reshape(-1, 1, mask.shape[-2], mask.shape[-1]).float(),
                             size=source.shape[2:], mode="bilinear")
        mask = U.repeat_to_batch_size(mask, source.shape[0])
    vis_w = destination.shape[3] - left + min(0, x)
    vis_h = destination.shape[2] - top + min(0, y)
    mask = mask[:, :, :vis_h, :vis_w]
    src = source[:, :, :vis_h, :vis_w]
    t0, l0 = max(top, 0), max(left, 0)
    dst = destination[:, :, t0:bottom, l0:right]
    # negative offsets: crop the source/mask from the other side
    src = src[:, :, t0 - top:t0 - top + dst.shape[2], l0 - left:l0 - left + dst.shape[3]]
    mask = mask[:, :, t0 - top:t0 - top + dst.shape[2], l0 - left:l0 - left + dst.shape[3]]
    destination[:, :, t0:t0 + dst.shape[2], l0:l0 + dst.shape[3]] = mask * src + (1.0 - mask) * dst
    return destination


class LatentCompositeMasked:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"destination": ("LATENT",), "source": ("LATENT",),
                             "x": ("INT", {"default": 0, "min": 0, "max": MAX_RESOLUTION, "step": 8}),
                             "y": ("INT", {"default": 0, "min": 0, "max": MAX_RESOLUTION, "step": 8}),
                             "resize_source": ("BOOLEAN", {"default": False})},
                "optional": {"mask": ("MASK",)}}
    RETURN_TYPES = ("LATENT",)
    FUNCTION = "composite"
    CATEGORY = "latent"

    def composite(self, destination, source, x, y, resize_source, mask=None):
        out = destination.copy()
        out["samples"] = composite(destination["samples"].clone(), source["samples"], x, y, mask, 8, resize_source)
        return (out,)


class ImageCompositeMasked:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"destination": ("IMAGE",), "source": ("IMAGE",),
                             "x": ("INT", {"default": 0, "min": 0, "max": MAX_RESOLUTION, "step": 1}),
                             "y": ("INT", {"default": 0, "min": 0, "max": MAX_RESOLUTION, "step": 1}),
                             "resize_source": ("BOOLEAN", {"default": False})},
                "optional": {"mask": ("MASK",)}}
    RETURN_TYPES = ("IMAGE",)
    FUNCTION = "composite"
    CATEGORY = "image"

    def composite(self, destination, source, x, y, resize_source, mask=None):
        out = composite(destination.clone().movedim(-1, 1), source.movedim(-1, 1), x, y, mask, 1, resize_source)
        return (out.movedim(1, -1),)


class MaskToImage:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"mask": ("MASK",)}}
    CATEGORY = "mask"
    RETURN_TYPES = ("IMAGE",)
    FUNCTION = "mask_to_image"

    def mask_to_image(self, mask):
        return (mask.reshape(-1, 1, mask.shape[-2], mask.shape[-1]).movedim(1, -1).expand(-1, -1, -1, 3),)


class ImageToMask:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"image": ("IMAGE",), "channel": (["red", "green", "blue", "alpha"],)}}
    CATEGORY = "mask"
    RETURN_TYPES = ("MASK",)
    FUNCTION = "image_to_mask"

    def image_to_mask(self, image, channel):
        return (image[:, :, :, ["red", "green", "blue", "alpha"].index(channel)],)


class ImageColorToMask:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"image": ("IMAGE",),
                             "color": ("INT", {"default": 0, "min": 0, "max": 0xFFFFFF, "step": 1, "display": "color"})}}
    CATEGORY = "mask"
    RETURN_TYPES = ("MASK",)
    FUNCTION = "image_to_mask"

    def image_to_mask(self, image, color):
        q = (image.clamp(0, 1) * 255.0).round().to(torch.int64)
        packed = (q[..., 0] << 16) + (q[..., 1] << 8) + q[..., 2]
        return (torch.where(packed == color, 255, 0).float(),)


class SolidMask:
    @classmethod
    def INPUT_TYPES(cls):
        return {"required": {"value": ("FLOAT", {"default": 1.0, "min": 0.0, "max": 1.0, "step": 0.01}),
                             "width": ("INT", {"default": 512, "min": 1, "max": MAX_RESOLUTION, "step": 1}),
                             "height": ("INT", {"default": 512, "min": 1, "max": MAX_RESOLUTION, "step": 1})}}
    CATEGORY = "mask"
    RETURN_TYPES = ("MASK",)
    FUNCTION = "solid"

    def solid(self, value, width, height):
        return (torch.full((1, height, width), value, dtype=torch.float32),)


class InvertMask:
    @classmethod
    def INPUT_TYPES(cls):
        return {"required": {"mask": ("MASK",)}}
    CATEGORY = "mask"
    RETURN_TYPES = ("MASK",)
    FUNCTION = "invert"

    def invert(self, mask):
        return (1.0 - mask,)


class CropMask:
    @classmethod
    def INPUT_TYPES(cls):
        return {"required": {"mask": ("MASK",),
                             "x": ("INT", {"default": 0, "min": 0, "max": MAX_RESOLUTION, "step": 1}),
                             "y": ("INT", {"default": 0, "min": 0, "max": MAX_RESOLUTION, "step": 1}),
                             "width": ("INT", {"default": 512, "min": 1, "max": MAX_RESOLUTION, "step": 1}),
                             "height": ("INT", {"default": 512, "min": 1, "max": MAX_RESOLUTION, "step": 1})}}
    CATEGORY = "mask"
    RETURN_TYPES = ("MASK",)
    FUNCTION = "crop"

    def crop(self, mask, x, y, width, height):
        m = mask.reshape(-1, mask.shape[-2], mask.shape[-1])
        return (m[:, y:y + height, x:x + width],)


class MaskComposite:
    OPS = ["multiply", "add", "subtract", "and", "or", "xor"]

    @classmethod
    def INPUT_TYPES(cls):
        return {"required": {"destination": ("MASK",), "source": ("MASK",),
                             "x": ("INT", {"default": 0, "min": 0, "max": MAX_RESOLUTION, "step": 1}),
                             "y": ("INT", {"default": 0, "min": 0, "max": MAX_RESOLUTION, "step": 1}),
                             "operation": (cls.OPS,)}}
    CATEGORY = "mask"
    RETURN_TYPES = ("MASK",)
    FUNCTION = "combine"

    def combine(self, destination, source, x, y, operation):
        out = destination.reshape(-1, destination.shape[-2], destination.shape[-1]).clone()
        src = source.reshape(-1, source.shape[-2], source.shape[-1])
        r = min(x + src.shape[-1], out.shape[-1])
        b = min(y + src.shape[-2], out.shape[-2])
        s = src[:, :b - y, :r - x]
        d = out[:, y:b, x:r]
        if operation == "multiply":
            v = d * s
        elif operation == "add":
            v = d + s
        elif operation == "subtract":
            v = d - s
        else:
            fn = {"and": torch.logical_and, "or": torch.logical_or, "xor": torch.logical_xor}[operation]
            v = fn(d.round().bool(), s.round().bool()).float()
        out[:, y:b, x:r] = v
        return (out.clamp(0.0, 1.0),)


class FeatherMask:
    @classmethod
    def INPUT_TYPES(cls):
        e = ("INT", {"default": 0, "min": 0, "max": MAX_RESOLUTION, "step": 1})
        return {"required": {"mask": ("MASK",), "left": e, "top": e, "right": e, "bottom": e}}
    CATEGORY = "mask"
    RETURN_TYPES = ("MASK",)
    FUNCTION = "feather"

    def feather(self, mask, left, top, right, bottom):
        out = mask.reshape(-1, mask.shape[-2], mask.shape[-1]).clone()
        H, W = out.shape[-2:]
        left, right, top, bottom = min(left, W), min(right, W), min(top, H), min(bottom, H)
        cols = torch.ones(W)
        rows = torch.ones(H)
        if left:
            cols[:left] *= (torch.arange(left) + 1.0) / left
        if right:
            cols[W - right:] *= torch.flip((torch.arange(right) + 1.0) / right, (0,))
        if top:
            rows[:top] *= (torch.arange(top) + 1.0) / top
        if bottom:
            rows[H - bottom:] *= torch.flip((torch.arange(bottom) + 1.0) / bottom, (0,))
        return (out * rows[:, None] * cols[None, :],)


def _dilate(m, tapered):
    """One 3x3 grey dilation (scipy 'reflect' boundary == replicate for a 1-pixel border)."""
    p = F.pad(m[:, None], (1, 1, 1, 1), mode="replicate")[:, 0]
    c = p[:, 1:-1, 1:-1]
    out = torch.maximum(torch.maximum(c, p[:, :-2, 1:-1]), torch.maximum(p[:, 2:, 1:-1], p[:, 1:-1, :-2]))
    out = torch.maximum(out, p[:, 1:-1, 2:])
    if not tapered:
        out = torch.maximum(torch.maximum(out, p[:, :-2, :-2]), torch.maximum(p[:, :-2, 2:], p[:, 2:, :-2]))
        out = torch.maximum(out, p[:, 2:, 2:])
    return out


class GrowMask:
    @classmethod
    def INPUT_TYPES(cls):
        return {"required": {"mask": ("MASK",),
                             "expand": ("INT", {"default": 0, "min": -MAX_RESOLUTION, "max": MAX_RESOLUTION, "step": 1}),
                             "tapered_corners": ("BOOLEAN", {"default": True})}}
    CATEGORY = "mask"
    RETURN_TYPES = ("MASK",)
    FUNCTION = "expand_mask"

    def expand_mask(self, mask, expand, tapered_corners):
        m = mask.reshape(-1, mask.shape[-2], mask.shape[-1]).float()
        for _ in range(abs(expand)):
            m = _dilate(m, tapered_corners) if expand > 0 else -_dilate(-m, tapered_corners)
        return (m,)


class ThresholdMask:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"mask": ("MASK",),
                             "value": ("FLOAT", {"default": 0.5, "min": 0.0, "max": 1.0, "step": 0.01})}}
    CATEGORY = "mask"
    RETURN_TYPES = ("MASK",)
    FUNCTION = "image_to_mask"

    def image_to_mask(self, mask, value):
        return ((mask > value).float(),)


NODE_CLASS_MAPPINGS = {
    "LatentCompositeMasked": LatentCompositeMasked, "ImageCompositeMasked": ImageCompositeMasked,
    "MaskToImage": MaskToImage, "ImageToMask": ImageToMask, "ImageColorToMask": ImageColorToMask,
    "SolidMask": SolidMask, "InvertMask": InvertMask, "CropMask": CropMask, "MaskComposite": MaskComposite,
    "FeatherMask": FeatherMask, "GrowMask": GrowMask, "ThresholdMask": ThresholdMask,
}
NODE_DISPLAY_NAME_MAPPINGS = {"ImageToMask": "Convert Image to Mask", "MaskToImage": "Convert Mask to Image"}
