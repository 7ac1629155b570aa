"""Core node library (parity: ``nodes.py:63-2141``, 66 nodes; C13/C19).

Class names, INPUT_TYPES, RETURN_TYPES and FUNCTION names are the public API (workflow JSON refers
to ``class_type`` strings), so they follow the reference exactly. Implementations call this
package's runtime (loaders, samplers, VAE/CLIP) — the hot paths run on the HIP kernels.
Known reference bug fixed: ``ConditioningSetArea`` returns the conditioning (the reference's
``append`` returns None).
"""
from __future__ import annotations

import hashlib
import json
import logging
import math
import os

import numpy as np
import torch

from ..runtime import device as dm
from ..runtime import sd as sdl
from ..runtime.checkpoint import load_state_dict, save_state_dict
from ..sampling import sample as S
from ..sampling import samplers as SM
from ..utils import folder_paths
from ..utils import image as U
from ..utils.progress import ProgressBar
from ..utils.hashing import file_digest
from . import helpers as NH

MAX_RESOLUTION = 16384


def before_node_execution():
    dm.throw_exception_if_processing_interrupted()


def interrupt_processing(value=True):
    dm.interrupt_current_processing(value)


# ================================================================ conditioning
class CLIPTextEncode:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"text": ("STRING", {"multiline": True, "dynamicPrompts": True}), "clip": ("CLIP",)}}
    RETURN_TYPES = ("CONDITIONING",)
    FUNCTION = "encode"
    CATEGORY = "conditioning"

    def encode(self, clip, text):
        tokens = clip.tokenize(text)
        cond, pooled = clip.encode_from_tokens(tokens, return_pooled=True)
        return ([[cond, {"pooled_output": pooled}]],)


class ConditioningCombine:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"conditioning_1": ("CONDITIONING",), "conditioning_2": ("CONDITIONING",)}}
    RETURN_TYPES = ("CONDITIONING",)
    FUNCTION = "combine"
    CATEGORY = "conditioning"

    def combine(self, conditioning_1, conditioning_2):
        return (conditioning_1 + conditioning_2,)


class ConditioningAverage:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"conditioning_to": ("CONDITIONING",), "conditioning_from": ("CONDITIONING",),
                             "conditioning_to_strength": ("FLOAT", {"default": 1.0, "min": 0.0, "max": 1.0, "step": 0.01})}}
    RETURN_TYPES = ("CONDITIONING",)
    FUNCTION = "addWeighted"
    CATEGORY = "conditioning"

    def addWeighted(self, conditioning_to, conditioning_from, conditioning_to_strength):
        out = []
        if len(conditioning_from) > 1:
            logging.warning("Warning: ConditioningAverage conditioning_from contains more than 1 cond, only the first one will actually be applied to conditioning_to.")
        cond_from = conditioning_from[0][0]
        pooled_from = conditioning_from[0][1].get("pooled_output", None)
        for t in conditioning_to:
            t1 = t[0]
            pooled_to = t[1].get("pooled_output", pooled_from)
            t0 = cond_from[:, :t1.shape[1]]
            if t0.shape[1] < t1.shape[1]:
                t0 = torch.cat([t0] + [torch.zeros((1, t1.shape[1] - t0.shape[1], t1.shape[2]), device=t0.device)], dim=1)
            tw = torch.mul(t1, conditioning_to_strength) + torch.mul(t0.to(t1), 1.0 - conditioning_to_strength)
            n = [tw, t[1].copy()]
            if pooled_from is not None and pooled_to is not None:
                n[1]["pooled_output"] = torch.mul(pooled_to, conditioning_to_strength) + \
                    torch.mul(pooled_from.to(pooled_to), 1.0 - conditioning_to_strength)
            elif pooled_from is not None:
                n[1]["pooled_output"] = pooled_from
            out.append(n)
        return (out,)


class ConditioningConcat:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"conditioning_to": ("CONDITIONING",), "conditioning_from": ("CONDITIONING",)}}
    RETURN_TYPES = ("CONDITIONING",)
    FUNCTION = "concat"
    CATEGORY = "conditioning"

    def concat(self, conditioning_to, conditioning_from):
        out = []
        if len(conditioning_from) > 1:
            logging.warning("Warning: ConditioningConcat conditioning_from contains more than 1 cond, only the first one will actually be applied to conditioning_to.")
        cond_from = conditioning_from[0][0]
        for t in conditioning_to:
            out.append([torch.cat((t[0], cond_from.to(t[0])), 1), t[1].copy()])
        return (out,)


class ConditioningSetArea:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"conditioning": ("CONDITIONING",),
                             "width": ("INT", {"default": 64, "min": 64, "max": MAX_RESOLUTION, "step": 8}),
                             "height": ("INT", {"default": 64, "min": 64, "max": MAX_RESOLUTION, "step": 8}),
                             "x": ("INT", {"default": 0, "min": 0, "max": MAX_RESOLUTION, "step": 8}),
                             "y": ("INT", {"default": 0, "min": 0, "max": MAX_RESOLUTION, "step": 8}),
                             "strength": ("FLOAT", {"default": 1.0, "min": 0.0, "max": 10.0, "step": 0.01})}}
    RETURN_TYPES = ("CONDITIONING",)
    FUNCTION = "append"
    CATEGORY = "conditioning"

    def append(self, conditioning, width, height, x, y, strength):
        c = NH.conditioning_set_values(conditioning, {"area": (height // 8, width // 8, y // 8, x // 8),
                                                      "strength": strength, "set_area_to_bounds": False})
        return (c,)


class ConditioningSetAreaPercentage:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"conditioning": ("CONDITIONING",),
                             "width": ("FLOAT", {"default": 1.0, "min": 0, "max": 1.0, "step": 0.01}),
                             "height": ("FLOAT", {"default": 1.0, "min": 0, "max": 1.0, "step": 0.01}),
                             "x": ("FLOAT", {"default": 0, "min": 0, "max": 1.0, "step": 0.01}),
                             "y": ("FLOAT", {"default": 0, "min": 0, "max": 1.0, "step": 0.01}),
                             "strength": ("FLOAT", {"default": 1.0, "min": 0.0, "max": 10.0, "step": 0.01})}}
    RETURN_TYPES = ("CONDITIONING",)
    FUNCTION = "append"
    CATEGORY = "conditioning"

    def append(self, conditioning, width, height, x, y, strength):
        c = NH.conditioning_set_values(conditioning, {"area": ("percentage", height, width, y, x),
                                                      "strength": strength, "set_area_to_bounds": False})
        return (c,)


class ConditioningSetAreaStrength:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"conditioning": ("CONDITIONING",),
                             "strength": ("FLOAT", {"default": 1.0, "min": 0.0, "max": 10.0, "step": 0.01})}}
    RETURN_TYPES = ("CONDITIONING",)
    FUNCTION = "append"
    CATEGORY = "conditioning"

    def append(self, conditioning, strength):
        return (NH.conditioning_set_values(conditioning, {"strength": strength}),)


class ConditioningSetMask:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"conditioning": ("CONDITIONING",), "mask": ("MASK",),
                             "strength": ("FLOAT", {"default": 1.0, "min": 0.0, "max": 10.0, "step": 0.01}),
                             "set_cond_area": (["default", "mask bounds"],)}}
    RETURN_TYPES = ("CONDITIONING",)
    FUNCTION = "append"
    CATEGORY = "conditioning"

    def append(self, conditioning, mask, set_cond_area, strength):
        set_area_to_bounds = set_cond_area != "default"
        if len(mask.shape) < 3:
            mask = mask.unsqueeze(0)
        return (NH.conditioning_set_values(conditioning, {"mask": mask, "set_area_to_bounds": set_area_to_bounds,
                                                          "mask_strength": strength}),)


class ConditioningZeroOut:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"conditioning": ("CONDITIONING",)}}
    RETURN_TYPES = ("CONDITIONING",)
    FUNCTION = "zero_out"
    CATEGORY = "advanced/conditioning"

    def zero_out(self, conditioning):
        c = []
        for t in conditioning:
            d = t[1].copy()
            if "pooled_output" in d:
                d["pooled_output"] = torch.zeros_like(d["pooled_output"])
            c.append([torch.zeros_like(t[0]), d])
        return (c,)


class ConditioningSetTimestepRange:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"conditioning": ("CONDITIONING",),
                             "start": ("FLOAT", {"default": 0.0, "min": 0.0, "max": 1.0, "step": 0.001}),
                             "end": ("FLOAT", {"default": 1.0, "min": 0.0, "max": 1.0, "step": 0.001})}}
    RETURN_TYPES = ("CONDITIONING",)
    FUNCTION = "set_range"
    CATEGORY = "advanced/conditioning"

    def set_range(self, conditioning, start, end):
        return (NH.conditioning_set_values(conditioning, {"start_percent": start, "end_percent": end}),)


class CLIPSetLastLayer:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"clip": ("CLIP",),
                             "stop_at_clip_layer": ("INT", {"default": -1, "min": -24, "max": -1, "step": 1})}}
    RETURN_TYPES = ("CLIP",)
    FUNCTION = "set_last_layer"
    CATEGORY = "conditioning"

    def set_last_layer(self, clip, stop_at_clip_layer):
        clip = clip.clone()
        clip.clip_layer(stop_at_clip_layer)
        return (clip,)


# ================================================================ VAE
class VAEDecode:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"samples": ("LATENT",), "vae": ("VAE",)}}
    RETURN_TYPES = ("IMAGE",)
    FUNCTION = "decode"
    CATEGORY = "latent"

    def decode(self, vae, samples):
        return (vae.decode(samples["samples"]),)


class VAEDecodeTiled:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"samples": ("LATENT",), "vae": ("VAE",),
                             "tile_size": ("INT", {"default": 512, "min": 320, "max": 4096, "step": 64})}}
    RETURN_TYPES = ("IMAGE",)
    FUNCTION = "decode"
    CATEGORY = "_for_testing"

    def decode(self, vae, samples, tile_size):
        t = tile_size // 8
        return (vae.decode_tiled(samples["samples"], tile_x=t, tile_y=t),)


class VAEEncode:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"pixels": ("IMAGE",), "vae": ("VAE",)}}
    RETURN_TYPES = ("LATENT",)
    FUNCTION = "encode"
    CATEGORY = "latent"

    def encode(self, vae, pixels):
        return ({"samples": vae.encode(pixels[:, :, :, :3])},)


class VAEEncodeTiled:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"pixels": ("IMAGE",), "vae": ("VAE",),
                             "tile_size": ("INT", {"default": 512, "min": 320, "max": 4096, "step": 64})}}
    RETURN_TYPES = ("LATENT",)
    FUNCTION = "encode"
    CATEGORY = "_for_testing"

    def encode(self, vae, pixels, tile_size):
        return ({"samples": vae.encode_tiled(pixels[:, :, :, :3], tile_x=tile_size, tile_y=tile_size)},)


class VAEEncodeForInpaint:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"pixels": ("IMAGE",), "vae": ("VAE",), "mask": ("MASK",),
                             "grow_mask_by": ("INT", {"default": 6, "min": 0, "max": 64, "step": 1})}}
    RETURN_TYPES = ("LATENT",)
    FUNCTION = "encode"
    CATEGORY = "latent/inpaint"

    def encode(self, vae, pixels, mask, grow_mask_by=6):
        x = (pixels.shape[1] // vae.downscale_ratio) * vae.downscale_ratio
        y = (pixels.shape[2] // vae.downscale_ratio) * vae.downscale_ratio
        mask = torch.nn.functional.interpolate(mask.reshape((-1, 1, mask.shape[-2], mask.shape[-1])),
                                               size=(pixels.shape[1], pixels.shape[2]), mode="bilinear")
        pixels = pixels.clone()
        if pixels.shape[1] != x or pixels.shape[2] != y:
            xo = (pixels.shape[1] % vae.downscale_ratio) // 2
            yo = (pixels.shape[2] % vae.downscale_ratio) // 2
            pixels = pixels[:, xo:x + xo, yo:y + yo, :]
            mask = mask[:, :, xo:x + xo, yo:y + yo]
        if grow_mask_by == 0:
            mask_erosion = mask
        else:
            kernel = torch.ones((1, 1, grow_mask_by, grow_mask_by))
            padding = math.ceil((grow_mask_by - 1) / 2)
            mask_erosion = torch.clamp(torch.nn.functional.conv2d(mask.round().cpu().float(), kernel, padding=padding), 0, 1)
        m = (1.0 - mask.round()).squeeze(1).to(pixels.device)
        for i in range(3):
            pixels[:, :, :, i] -= 0.5
            pixels[:, :, :, i] *= m
            pixels[:, :, :, i] += 0.5
        t = vae.encode(pixels)
        return ({"samples": t, "noise_mask": (mask_erosion[:, :, :x, :y].round())},)


class InpaintModelConditioning:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"positive": ("CONDITIONING",), "negative": ("CONDITIONING",), "vae": ("VAE",),
                             "pixels": ("IMAGE",), "mask": ("MASK",)}}
    RETURN_TYPES = ("CONDITIONING", "CONDITIONING", "LATENT")
    RETURN_NAMES = ("positive", "negative", "latent")
    FUNCTION = "encode"
    CATEGORY = "conditioning/inpaint"

    def encode(self, positive, negative, pixels, vae, mask):
        x = (pixels.shape[1] // 8) * 8
        y = (pixels.shape[2] // 8) * 8
        mask = torch.nn.functional.interpolate(mask.reshape((-1, 1, mask.shape[-2], mask.shape[-1])),
                                               size=(pixels.shape[1], pixels.shape[2]), mode="bilinear")
        orig_pixels = pixels
        pixels = orig_pixels.clone()
        if pixels.shape[1] != x or pixels.shape[2] != y:
            xo = (pixels.shape[1] % 8) // 2
            yo = (pixels.shape[2] % 8) // 2
            pixels = pixels[:, xo:x + xo, yo:y + yo, :]
            mask = mask[:, :, xo:x + xo, yo:y + yo]
        m = (1.0 - mask.round()).squeeze(1).to(pixels.device)
        for i in range(3):
            pixels[:, :, :, i] -= 0.5
            pixels[:, :, :, i] *= m
            pixels[:, :, :, i] += 0.5
        concat_latent = vae.encode(pixels)
        orig_latent = vae.encode(orig_pixels)
        out_latent = {"samples": orig_latent, "noise_mask": mask}
        out = []
        for conditioning in [positive, negative]:
            out.append(NH.conditioning_set_values(conditioning, {"concat_latent_image": concat_latent,
                                                                 "concat_mask": mask}))
        return (out[0], out[1], out_latent)


# ================================================================ latents
class SaveLatent:
    def __init__(self):
        self.output_dir = folder_paths.get_output_directory()

    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"samples": ("LATENT",), "filename_prefix": ("STRING", {"default": "latents/ComfyUI"})},
                "hidden": {"prompt": "PROMPT", "extra_pnginfo": "EXTRA_PNGINFO"}}
    RETURN_TYPES = ()
    FUNCTION = "save"
    OUTPUT_NODE = True
    CATEGORY = "_for_testing"

    def save(self, samples, filename_prefix="ComfyUI", prompt=None, extra_pnginfo=None):
        out_dir = folder_paths.get_output_directory()
        full_output_folder, filename, counter, subfolder, filename_prefix = folder_paths.get_save_image_path(filename_prefix, out_dir)
        prompt_info = json.dumps(prompt) if prompt is not None else ""
        metadata = None
        if not NH.args_disable_metadata():
            metadata = {"prompt": prompt_info}
            if extra_pnginfo is not None:
                for x in extra_pnginfo:
                    metadata[x] = json.dumps(extra_pnginfo[x])
        file = f"{filename}_{counter:05}_.latent"
        results = [{"filename": file, "subfolder": subfolder, "type": "output"}]
        file = os.path.join(full_output_folder, file)
        output = {"latent_tensor": samples["samples"].contiguous().cpu(), "latent_format_version_0": torch.tensor([])}
        save_state_dict(output, file, metadata=metadata)
        return {"ui": {"latents": results}}


class LoadLatent:
    @classmethod
    def INPUT_TYPES(s):
        input_dir = folder_paths.get_input_directory()
        files = [f for f in os.listdir(input_dir) if os.path.isfile(os.path.join(input_dir, f)) and f.endswith(".latent")] \
            if os.path.isdir(input_dir) else []
        return {"required": {"latent": [sorted(files), ]}}
    CATEGORY = "_for_testing"
    RETURN_TYPES = ("LATENT",)
    FUNCTION = "load"

    def load(self, latent):
        path = folder_paths.get_annotated_filepath(latent)
        lat = load_state_dict(path)
        mult = 1.0
        if "latent_format_version_0" not in lat:
            mult = 1.0 / 0.18215
        return ({"samples": lat["latent_tensor"].float() * mult},)

    @classmethod
    def IS_CHANGED(s, latent):
        return file_digest(folder_paths.get_annotated_filepath(latent))

    @classmethod
    def VALIDATE_INPUTS(s, latent):
        if not folder_paths.exists_annotated_filepath(latent):
            return "Invalid latent file: {}".format(latent)
        return True


class EmptyLatentImage:
    def __init__(self):
        self.device = dm.intermediate_device()

    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"width": ("INT", {"default": 512, "min": 16, "max": MAX_RESOLUTION, "step": 8}),
                             "height": ("INT", {"default": 512, "min": 16, "max": MAX_RESOLUTION, "step": 8}),
                             "batch_size": ("INT", {"default": 1, "min": 1, "max": 4096})}}
    RETURN_TYPES = ("LATENT",)
    FUNCTION = "generate"
    CATEGORY = "latent"

    def generate(self, width, height, batch_size=1):
        latent = torch.zeros([batch_size, 4, height // 8, width // 8], device=self.device)
        return ({"samples": latent},)


def _cycle_batch(t, n):
    """``t`` tiled along dim 0 to exactly ``n`` entries (a per-image tensor matched to a batch)."""
    reps = -(-n // t.shape[0])
    return t.repeat((reps,) + (1,) * (t.dim() - 1))[:n]


def _pixel_target(w0, h0, width, height):
    """Pixel size of a latent resize to (width, height) from a latent of (w0, h0): a 0 side follows the
    aspect ratio; every side at least 64 px."""
    if width == 0:
        height = max(64, height)
        return max(64, round(w0 * height / h0)), height
    if height == 0:
        width = max(64, width)
        return width, max(64, round(h0 * width / w0))
    return max(64, width), max(64, height)


class LatentFromBatch:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"samples": ("LATENT",), "batch_index": ("INT", {"default": 0, "min": 0, "max": 63}),
                             "length": ("INT", {"default": 1, "min": 1, "max": 64})}}
    RETURN_TYPES = ("LATENT",)
    FUNCTION = "frombatch"
    CATEGORY = "latent/batch"

    def frombatch(self, samples, batch_index, length):
        """Images [start, stop) of the batch (clamped into it); a per-image noise mask is cycled to the
        batch first, a single mask kept; ``batch_index`` records the images' global indices."""
        src = samples["samples"]
        n = src.shape[0]
        start = min(batch_index, n - 1)
        stop = start + min(length, n - start)
        out = dict(samples, samples=src[start:stop].clone())
        if "noise_mask" in samples:
            mask = samples["noise_mask"]
            out["noise_mask"] = mask.clone() if mask.shape[0] == 1 else _cycle_batch(mask, n)[start:stop].clone()
        prev = samples.get("batch_index")
        out["batch_index"] = list(range(start, stop)) if prev is None else prev[start:stop]
        return (out,)


class RepeatLatentBatch:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"samples": ("LATENT",), "amount": ("INT", {"default": 1, "min": 1, "max": 64})}}
    RETURN_TYPES = ("LATENT",)
    FUNCTION = "repeat"
    CATEGORY = "latent/batch"

    def repeat(self, samples, amount):
        """The batch tiled ``amount`` times; a per-image mask is tiled with it (as the reference does, the
        mask's own batch is tiled, not first matched to the latent's); each copy of ``batch_index``
        is shifted past the previous copy's span."""
        src = samples["samples"]
        out = dict(samples, samples=src.repeat((amount,) + (1,) * (src.dim() - 1)))
        mask = samples.get("noise_mask")
        if mask is not None and mask.shape[0] > 1:
            out["noise_mask"] = mask.repeat((amount,) + (1,) * (mask.dim() - 1))
        inds = samples.get("batch_index")
        if inds is not None:
            span = max(inds) - min(inds) + 1
            out["batch_index"] = [x + k * span for k in range(amount) for x in inds]
        return (out,)


class LatentUpscale:
    upscale_methods = ["nearest-exact", "bilinear", "area", "bicubic", "bislerp"]
    crop_methods = ["disabled", "center"]

    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"samples": ("LATENT",), "upscale_method": (s.upscale_methods,),
                             "width": ("INT", {"default": 512, "min": 0, "max": MAX_RESOLUTION, "step": 8}),
                             "height": ("INT", {"default": 512, "min": 0, "max": MAX_RESOLUTION, "step": 8}),
                             "crop": (s.crop_methods,)}}
    RETURN_TYPES = ("LATENT",)
    FUNCTION = "upscale"
    CATEGORY = "latent"

    def upscale(self, samples, upscale_method, width, height, crop):
        """Resize to a pixel size (0 on one side: keep the aspect ratio; both 0: unchanged)."""
        if width == 0 and height == 0:
            return (samples,)
        lat = samples["samples"]
        w, h = _pixel_target(lat.shape[3], lat.shape[2], width, height)
        return (dict(samples, samples=U.common_upscale(lat, w // 8, h // 8, upscale_method, crop)),)


class LatentUpscaleBy:
    upscale_methods = ["nearest-exact", "bilinear", "area", "bicubic", "bislerp"]

    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"samples": ("LATENT",), "upscale_method": (s.upscale_methods,),
                             "scale_by": ("FLOAT", {"default": 1.5, "min": 0.01, "max": 8.0, "step": 0.01})}}
    RETURN_TYPES = ("LATENT",)
    FUNCTION = "upscale"
    CATEGORY = "latent"

    def upscale(self, samples, upscale_method, scale_by):
        s = samples.copy()
        width = round(samples["samples"].shape[3] * scale_by)
        height = round(samples["samples"].shape[2] * scale_by)
        s["samples"] = U.common_upscale(samples["samples"], width, height, upscale_method, "disabled")
        return (s,)


class LatentRotate:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"samples": ("LATENT",),
                             "rotation": (["none", "90 degrees", "180 degrees", "270 degrees"],)}}
    RETURN_TYPES = ("LATENT",)
    FUNCTION = "rotate"
    CATEGORY = "latent/transform"

    def rotate(self, samples, rotation):
        s = samples.copy()
        k = {"none": 0, "90 degrees": 3, "180 degrees": 2, "270 degrees": 1}[rotation]
        s["samples"] = torch.rot90(samples["samples"], k=k, dims=[3, 2])
        return (s,)


class LatentFlip:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"samples": ("LATENT",), "flip_method": (["x-axis: vertically", "y-axis: horizontally"],)}}
    RETURN_TYPES = ("LATENT",)
    FUNCTION = "flip"
    CATEGORY = "latent/transform"

    def flip(self, samples, flip_method):
        dim = {"x": 2, "y": 3}.get(flip_method[:1])     # x-axis: rows (vertical), y-axis: columns
        if dim is None:
            return (dict(samples),)
        return (dict(samples, samples=torch.flip(samples["samples"], dims=[dim])),)


class LatentComposite:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"samples_to": ("LATENT",), "samples_from": ("LATENT",),
                             "x": ("INT", {"default": 0, "min": 0, "max": MAX_RESOLUTION, "step": 8}),
                             "y": ("INT", {"default": 0, "min": 0, "max": MAX_RESOLUTION, "step": 8}),
                             "feather": ("INT", {"default": 0, "min": 0, "max": MAX_RESOLUTION, "step": 8})}}
    RETURN_TYPES = ("LATENT",)
    FUNCTION = "composite"
    CATEGORY = "latent"

    def composite(self, samples_to, samples_from, x, y, composite_method="normal", feather=0):
        x, y, feather = x // 8, y // 8, feather // 8
        samples_out = samples_to.copy()
        s = samples_to["samples"].clone()
        st = samples_to["samples"]
        sf = samples_from["samples"]
        if feather == 0:
            s[:, :, y:y + sf.shape[2], x:x + sf.shape[3]] = sf[:, :, :st.shape[2] - y, :st.shape[3] - x]
        else:
            sf = sf[:, :, :st.shape[2] - y, :st.shape[3] - x]
            mask = torch.ones_like(sf)
            for t in range(feather):
                if y != 0:
                    mask[:, :, t:1 + t, :] *= ((1.0 / feather) * (t + 1))
                if y + sf.shape[2] < st.shape[2]:
                    mask[:, :, mask.shape[2] - 1 - t: mask.shape[2] - t, :] *= ((1.0 / feather) * (t + 1))
                if x != 0:
                    mask[:, :, :, t:1 + t] *= ((1.0 / feather) * (t + 1))
                if x + sf.shape[3] < st.shape[3]:
                    mask[:, :, :, mask.shape[3] - 1 - t: mask.shape[3] - t] *= ((1.0 / feather) * (t + 1))
            rev_mask = torch.ones_like(mask) - mask
            s[:, :, y:y + sf.shape[2], x:x + sf.shape[3]] = sf * mask + s[:, :, y:y + sf.shape[2], x:x + sf.shape[3]] * rev_mask
        samples_out["samples"] = s
        return (samples_out,)


class LatentBlend:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"samples1": ("LATENT",), "samples2": ("LATENT",),
                             "blend_factor": ("FLOAT", {"default": 0.5, "min": 0, "max": 1, "step": 0.01})}}
    RETURN_TYPES = ("LATENT",)
    FUNCTION = "blend"
    CATEGORY = "_for_testing"

    def blend(self, samples1, samples2, blend_factor, blend_mode="normal"):
        samples_out = samples1.copy()
        s1 = samples1["samples"]
        s2 = samples2["samples"]
        if s1.shape != s2.shape:
            s2 = s2.permute(0, 3, 1, 2)
            s2 = U.common_upscale(s2, s1.shape[3], s1.shape[2], "bicubic", crop="center")
            s2 = s2.permute(0, 2, 3, 1)
        samples_out["samples"] = s1 * blend_factor + s2 * (1 - blend_factor)
        return (samples_out,)


class LatentCrop:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"samples": ("LATENT",),
                             "width": ("INT", {"default": 512, "min": 64, "max": MAX_RESOLUTION, "step": 8}),
                             "height": ("INT", {"default": 512, "min": 64, "max": MAX_RESOLUTION, "step": 8}),
                             "x": ("INT", {"default": 0, "min": 0, "max": MAX_RESOLUTION, "step": 8}),
                             "y": ("INT", {"default": 0, "min": 0, "max": MAX_RESOLUTION, "step": 8})}}
    RETURN_TYPES = ("LATENT",)
    FUNCTION = "crop"
    CATEGORY = "latent/transform"

    def crop(self, samples, width, height, x, y):
        s = samples.copy()
        samples = samples["samples"]
        x, y = x // 8, y // 8
        if x > (samples.shape[3] - 8):
            x = samples.shape[3] - 8
        if y > (samples.shape[2] - 8):
            y = samples.shape[2] - 8
        new_height, new_width = height // 8, width // 8
        s["samples"] = samples[:, :, y:y + new_height, x:x + new_width]
        return (s,)


class SetLatentNoiseMask:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"samples": ("LATENT",), "mask": ("MASK",)}}
    RETURN_TYPES = ("LATENT",)
    FUNCTION = "set_mask"
    CATEGORY = "latent/inpaint"

    def set_mask(self, samples, mask):
        s = samples.copy()
        s["noise_mask"] = mask.reshape((-1, 1, mask.shape[-2], mask.shape[-1]))
        return (s,)


# ================================================================ sampling
def common_ksampler(model, seed, steps, cfg, sampler_name, scheduler, positive, negative, latent, denoise=1.0,
                    disable_noise=False, start_step=None, last_step=None, force_full_denoise=False):
    """``nodes.py:1420-1439``. In an SPMD prompt (``sched/spmd.py``) this rank samples only its slice
    of the batch; noise is keyed by the images' global batch indices, so the shards together equal
    the one-GPU batch."""
    from ..sched import spmd
    local, batch_inds, shard = spmd.shard_latent(latent)
    positive, negative = spmd.shard_conds(positive, shard), spmd.shard_conds(negative, shard)
    model = spmd.latency_model(model)
    latent_image = local["samples"]
    if disable_noise:
        noise = torch.zeros(latent_image.size(), dtype=torch.float32, layout=latent_image.layout, device="cpu")
    else:
        noise = S.prepare_noise(latent_image, seed, batch_inds)
    noise_mask = local.get("noise_mask")
    callback = NH.prepare_callback(model, steps)
    samples = S.sample(model, noise, steps, cfg, sampler_name, scheduler, positive, negative, latent_image,
                       denoise=denoise, disable_noise=disable_noise, start_step=start_step, last_step=last_step,
                       force_full_denoise=force_full_denoise, noise_mask=noise_mask, callback=callback, seed=seed,
                       noise_inds=batch_inds)
    out = latent.copy()
    out["samples"] = samples
    if shard is not None:
        out["dp_shard"] = shard
    return (out,)


class KSampler:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"model": ("MODEL",),
                             "seed": ("INT", {"default": 0, "min": 0, "max": 0xffffffffffffffff}),
                             "steps": ("INT", {"default": 20, "min": 1, "max": 10000}),
                             "cfg": ("FLOAT", {"default": 8.0, "min": 0.0, "max": 100.0, "step": 0.1, "round": 0.01}),
                             "sampler_name": (SM.KSampler.SAMPLERS,), "scheduler": (SM.KSampler.SCHEDULERS,),
                             "positive": ("CONDITIONING",), "negative": ("CONDITIONING",), "latent_image": ("LATENT",),
                             "denoise": ("FLOAT", {"default": 1.0, "min": 0.0, "max": 1.0, "step": 0.01})}}
    RETURN_TYPES = ("LATENT",)
    FUNCTION = "sample"
    CATEGORY = "sampling"

    def sample(self, model, seed, steps, cfg, sampler_name, scheduler, positive, negative, latent_image, denoise=1.0):
        return common_ksampler(model, seed, steps, cfg, sampler_name, scheduler, positive, negative, latent_image,
                               denoise=denoise)


class KSamplerAdvanced:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"model": ("MODEL",), "add_noise": (["enable", "disable"],),
                             "noise_seed": ("INT", {"default": 0, "min": 0, "max": 0xffffffffffffffff}),
                             "steps": ("INT", {"default": 20, "min": 1, "max": 10000}),
                             "cfg": ("FLOAT", {"default": 8.0, "min": 0.0, "max": 100.0, "step": 0.1, "round": 0.01}),
                             "sampler_name": (SM.KSampler.SAMPLERS,), "scheduler": (SM.KSampler.SCHEDULERS,),
                             "positive": ("CONDITIONING",), "negative": ("CONDITIONING",), "latent_image": ("LATENT",),
                             "start_at_step": ("INT", {"default": 0, "min": 0, "max": 10000}),
                             "end_at_step": ("INT", {"default": 10000, "min": 0, "max": 10000}),
                             "return_with_leftover_noise": (["disable", "enable"],)}}
    RETURN_TYPES = ("LATENT",)
    FUNCTION = "sample"
    CATEGORY = "sampling"

    def sample(self, model, add_noise, noise_seed, steps, cfg, sampler_name, scheduler, positive, negative, latent_image,
               start_at_step, end_at_step, return_with_leftover_noise, denoise=1.0):
        force_full_denoise = return_with_leftover_noise != "enable"
        disable_noise = add_noise == "disable"
        return common_ksampler(model, noise_seed, steps, cfg, sampler_name, scheduler, positive, negative, latent_image,
                               denoise=denoise, disable_noise=disable_noise, start_step=start_at_step,
                               last_step=end_at_step, force_full_denoise=force_full_denoise)


# ================================================================ loaders
class CheckpointLoaderSimple:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"ckpt_name": (folder_paths.get_filename_list("checkpoints"),)}}
    RETURN_TYPES = ("MODEL", "CLIP", "VAE")
    FUNCTION = "load_checkpoint"
    CATEGORY = "loaders"

    def load_checkpoint(self, ckpt_name):
        path = folder_paths.get_full_path("checkpoints", ckpt_name)
        out = sdl.load_checkpoint_guess_config(path, output_vae=True, output_clip=True,
                                               embedding_directory=folder_paths.get_folder_paths("embeddings"))
        return out[:3]


class CheckpointLoader:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"config_name": (folder_paths.get_filename_list("configs"),),
                             "ckpt_name": (folder_paths.get_filename_list("checkpoints"),)}}
    RETURN_TYPES = ("MODEL", "CLIP", "VAE")
    FUNCTION = "load_checkpoint"
    CATEGORY = "advanced/loaders"

    def load_checkpoint(self, config_name, ckpt_name):
        # The yaml only duplicates what detection infers from the state dict; detection wins.
        path = folder_paths.get_full_path("checkpoints", ckpt_name)
        return sdl.load_checkpoint_guess_config(path, output_vae=True, output_clip=True,
                                                embedding_directory=folder_paths.get_folder_paths("embeddings"))[:3]


def _diffusers_roots():
    return [r for r in folder_paths.get_folder_paths("diffusers") if os.path.isdir(r)]


class DiffusersLoader:
    """A diffusers folder (``model_index.json`` at its top) under any registered ``diffusers`` root; the
    choice list names folders relative to their root (reference ``nodes.py`` DiffusersLoader)."""

    @classmethod
    def INPUT_TYPES(cls):
        found = [os.path.relpath(d, start=root) for root in _diffusers_roots()
                 for d, _, names in os.walk(root, followlinks=True) if "model_index.json" in names]
        return {"required": {"model_path": (found,)}}
    RETURN_TYPES = ("MODEL", "CLIP", "VAE")
    FUNCTION = "load_checkpoint"
    CATEGORY = "advanced/loaders/deprecated"

    def load_checkpoint(self, model_path, output_vae=True, output_clip=True):
        from ..runtime.diffusers import load_diffusers
        # the first root holding the folder wins; an absolute / unknown path is passed through as given
        full = next((os.path.join(root, model_path) for root in _diffusers_roots()
                     if os.path.exists(os.path.join(root, model_path))), model_path)
        return load_diffusers(full, output_vae=output_vae, output_clip=output_clip,
                              embedding_directory=folder_paths.get_folder_paths("embeddings"))


class unCLIPCheckpointLoader:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"ckpt_name": (folder_paths.get_filename_list("checkpoints"),)}}
    RETURN_TYPES = ("MODEL", "CLIP", "VAE", "CLIP_VISION")
    FUNCTION = "load_checkpoint"
    CATEGORY = "loaders"

    def load_checkpoint(self, ckpt_name, output_vae=True, output_clip=True):
        path = folder_paths.get_full_path("checkpoints", ckpt_name)
        return sdl.load_checkpoint_guess_config(path, output_vae=True, output_clip=True, output_clipvision=True,
                                                embedding_directory=folder_paths.get_folder_paths("embeddings"))


class LoraLoader:
    def __init__(self):
        self.loaded_lora = None

    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"model": ("MODEL",), "clip": ("CLIP",),
                             "lora_name": (folder_paths.get_filename_list("loras"),),
                             "strength_model": ("FLOAT", {"default": 1.0, "min": -100.0, "max": 100.0, "step": 0.01}),
                             "strength_clip": ("FLOAT", {"default": 1.0, "min": -100.0, "max": 100.0, "step": 0.01})}}
    RETURN_TYPES = ("MODEL", "CLIP")
    FUNCTION = "load_lora"
    CATEGORY = "loaders"

    def _lora_state(self, lora_name):
        """The LoRA file's tensors, kept for the next call with the same file (one cached file per node)."""
        path = folder_paths.get_full_path("loras", lora_name)
        cached = self.loaded_lora
        if cached is None or cached[0] != path:
            cached = self.loaded_lora = (path, load_state_dict(path, safe_load=True))
        return cached[1]

    def load_lora(self, model, clip, lora_name, strength_model, strength_clip):
        if strength_model == 0 and strength_clip == 0:      # nothing to patch: the inputs pass through
            return (model, clip)
        return sdl.load_lora_for_models(model, clip, self._lora_state(lora_name), strength_model, strength_clip)


class LoraLoaderModelOnly(LoraLoader):
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"model": ("MODEL",), "lora_name": (folder_paths.get_filename_list("loras"),),
                             "strength_model": ("FLOAT", {"default": 1.0, "min": -100.0, "max": 100.0, "step": 0.01})}}
    RETURN_TYPES = ("MODEL",)
    FUNCTION = "load_lora_model_only"

    def load_lora_model_only(self, model, lora_name, strength_model):
        return (self.load_lora(model, None, lora_name, strength_model, 0)[0],)


class VAELoader:
    @staticmethod
    def vae_list():
        vaes = folder_paths.get_filename_list("vae")
        approx = folder_paths.get_filename_list("vae_approx")
        sd1_dec = sd1_enc = sdxl_dec = sdxl_enc = False
        for v in approx:
            if v.startswith("taesd_decoder."):
                sd1_dec = True
            elif v.startswith("taesd_encoder."):
                sd1_enc = True
            elif v.startswith("taesdxl_decoder."):
                sdxl_dec = True
            elif v.startswith("taesdxl_encoder."):
                sdxl_enc = True
        if sd1_dec and sd1_enc:
            vaes.append("taesd")
        if sdxl_dec and sdxl_enc:
            vaes.append("taesdxl")
        return vaes

    @staticmethod
    def load_taesd(name):
        sd = {}
        approx = folder_paths.get_filename_list("vae_approx")
        enc = next(filter(lambda a: a.startswith(f"{name}_encoder."), approx))
        dec = next(filter(lambda a: a.startswith(f"{name}_decoder."), approx))
        for k, v in load_state_dict(folder_paths.get_full_path("vae_approx", enc)).items():
            sd[f"taesd_encoder.{k}"] = v
        for k, v in load_state_dict(folder_paths.get_full_path("vae_approx", dec)).items():
            sd[f"taesd_decoder.{k}"] = v
        if name == "taesd":
            sd["vae_scale"] = torch.tensor(0.18215)
        elif name == "taesdxl":
            sd["vae_scale"] = torch.tensor(0.13025)
        return sd

    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"vae_name": (s.vae_list(),)}}
    RETURN_TYPES = ("VAE",)
    FUNCTION = "load_vae"
    CATEGORY = "loaders"

    def load_vae(self, vae_name):
        if vae_name in ["taesd", "taesdxl"]:
            sd = self.load_taesd(vae_name)
        else:
            sd = load_state_dict(folder_paths.get_full_path("vae", vae_name))
        return (sdl.VAE(sd=sd),)


class UNETLoader:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"unet_name": (folder_paths.get_filename_list("unet"),)}}
    RETURN_TYPES = ("MODEL",)
    FUNCTION = "load_unet"
    CATEGORY = "advanced/loaders"

    def load_unet(self, unet_name):
        return (sdl.load_unet(folder_paths.get_full_path("unet", unet_name)),)


class CLIPLoader:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"clip_name": (folder_paths.get_filename_list("clip"),),
                             "type": (["stable_diffusion", "stable_cascade"],)}}
    RETURN_TYPES = ("CLIP",)
    FUNCTION = "load_clip"
    CATEGORY = "advanced/loaders"

    def load_clip(self, clip_name, type="stable_diffusion"):
        ct = sdl.CLIPType.STABLE_CASCADE if type == "stable_cascade" else sdl.CLIPType.STABLE_DIFFUSION
        path = folder_paths.get_full_path("clip", clip_name)
        return (sdl.load_clip([path], embedding_directory=folder_paths.get_folder_paths("embeddings"), clip_type=ct),)


class DualCLIPLoader:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"clip_name1": (folder_paths.get_filename_list("clip"),),
                             "clip_name2": (folder_paths.get_filename_list("clip"),)}}
    RETURN_TYPES = ("CLIP",)
    FUNCTION = "load_clip"
    CATEGORY = "advanced/loaders"

    def load_clip(self, clip_name1, clip_name2):
        p1 = folder_paths.get_full_path("clip", clip_name1)
        p2 = folder_paths.get_full_path("clip", clip_name2)
        return (sdl.load_clip([p1, p2], embedding_directory=folder_paths.get_folder_paths("embeddings")),)


class CLIPVisionLoader:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"clip_name": (folder_paths.get_filename_list("clip_vision"),)}}
    RETURN_TYPES = ("CLIP_VISION",)
    FUNCTION = "load_clip"
    CATEGORY = "loaders"

    def load_clip(self, clip_name):
        from ..runtime import clip_vision
        return (clip_vision.load(folder_paths.get_full_path("clip_vision", clip_name)),)


class CLIPVisionEncode:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"clip_vision": ("CLIP_VISION",), "image": ("IMAGE",)}}
    RETURN_TYPES = ("CLIP_VISION_OUTPUT",)
    FUNCTION = "encode"
    CATEGORY = "conditioning"

    def encode(self, clip_vision, image):
        return (clip_vision.encode_image(image),)


class StyleModelLoader:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"style_model_name": (folder_paths.get_filename_list("style_models"),)}}
    RETURN_TYPES = ("STYLE_MODEL",)
    FUNCTION = "load_style_model"
    CATEGORY = "loaders"

    def load_style_model(self, style_model_name):
        return (sdl.load_style_model(folder_paths.get_full_path("style_models", style_model_name)),)


class StyleModelApply:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"conditioning": ("CONDITIONING",), "style_model": ("STYLE_MODEL",),
                             "clip_vision_output": ("CLIP_VISION_OUTPUT",)}}
    RETURN_TYPES = ("CONDITIONING",)
    FUNCTION = "apply_stylemodel"
    CATEGORY = "conditioning/style_model"

    def apply_stylemodel(self, clip_vision_output, style_model, conditioning):
        cond = style_model.get_cond(clip_vision_output).flatten(start_dim=0, end_dim=1).unsqueeze(dim=0)
        return ([[torch.cat((t[0], cond.to(t[0])), dim=1), t[1].copy()] for t in conditioning],)


class unCLIPConditioning:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"conditioning": ("CONDITIONING",), "clip_vision_output": ("CLIP_VISION_OUTPUT",),
                             "strength": ("FLOAT", {"default": 1.0, "min": -10.0, "max": 10.0, "step": 0.01}),
                             "noise_augmentation": ("FLOAT", {"default": 0.0, "min": 0.0, "max": 1.0, "step": 0.01})}}
    RETURN_TYPES = ("CONDITIONING",)
    FUNCTION = "apply_adm"
    CATEGORY = "conditioning"

    def apply_adm(self, conditioning, clip_vision_output, strength, noise_augmentation):
        if strength == 0:
            return (conditioning,)
        c = []
        for t in conditioning:
            o = t[1].copy()
            x = {"clip_vision_output": clip_vision_output, "strength": strength, "noise_augmentation": noise_augmentation}
            o["unclip_conditioning"] = o.get("unclip_conditioning", []) + [x]
            c.append([t[0], o])
        return (c,)


class GLIGENLoader:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"gligen_name": (folder_paths.get_filename_list("gligen"),)}}
    RETURN_TYPES = ("GLIGEN",)
    FUNCTION = "load_gligen"
    CATEGORY = "loaders"

    def load_gligen(self, gligen_name):
        from ..models.gligen import load_gligen
        return (load_gligen(folder_paths.get_full_path("gligen", gligen_name)),)


class GLIGENTextBoxApply:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"conditioning_to": ("CONDITIONING",), "clip": ("CLIP",), "gligen_textbox_model": ("GLIGEN",),
                             "text": ("STRING", {"multiline": True, "dynamicPrompts": True}),
                             "width": ("INT", {"default": 64, "min": 8, "max": MAX_RESOLUTION, "step": 8}),
                             "height": ("INT", {"default": 64, "min": 8, "max": MAX_RESOLUTION, "step": 8}),
                             "x": ("INT", {"default": 0, "min": 0, "max": MAX_RESOLUTION, "step": 8}),
                             "y": ("INT", {"default": 0, "min": 0, "max": MAX_RESOLUTION, "step": 8})}}
    RETURN_TYPES = ("CONDITIONING",)
    FUNCTION = "append"
    CATEGORY = "conditioning/gligen"

    def append(self, conditioning_to, clip, gligen_textbox_model, text, width, height, x, y):
        c = []
        cond, cond_pooled = clip.encode_from_tokens(clip.tokenize(text), return_pooled="unprojected")
        for t in conditioning_to:
            n = [t[0], t[1].copy()]
            position_params = [(cond_pooled, height // 8, width // 8, y // 8, x // 8)]
            prev = []
            if "gligen" in n[1]:
                prev = n[1]["gligen"][2]
            n[1]["gligen"] = ("position", gligen_textbox_model, prev + position_params)
            c.append(n)
        return (c,)


# ================================================================ ControlNet
class ControlNetLoader:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"control_net_name": (folder_paths.get_filename_list("controlnet"),)}}
    RETURN_TYPES = ("CONTROL_NET",)
    FUNCTION = "load_controlnet"
    CATEGORY = "loaders"

    def load_controlnet(self, control_net_name):
        from ..runtime import controlnet
        return (controlnet.load_controlnet(folder_paths.get_full_path("controlnet", control_net_name)),)


class DiffControlNetLoader:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"model": ("MODEL",),
                             "control_net_name": (folder_paths.get_filename_list("controlnet"),)}}
    RETURN_TYPES = ("CONTROL_NET",)
    FUNCTION = "load_controlnet"
    CATEGORY = "loaders"

    def load_controlnet(self, model, control_net_name):
        from ..runtime import controlnet
        return (controlnet.load_controlnet(folder_paths.get_full_path("controlnet", control_net_name), model),)


class ControlNetApply:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"conditioning": ("CONDITIONING",), "control_net": ("CONTROL_NET",), "image": ("IMAGE",),
                             "strength": ("FLOAT", {"default": 1.0, "min": 0.0, "max": 10.0, "step": 0.01})}}
    RETURN_TYPES = ("CONDITIONING",)
    FUNCTION = "apply_controlnet"
    CATEGORY = "conditioning/controlnet"

    def apply_controlnet(self, conditioning, control_net, image, strength):
        if strength == 0:
            return (conditioning,)
        c = []
        control_hint = image.movedim(-1, 1)
        for t in conditioning:
            n = [t[0], t[1].copy()]
            c_net = control_net.copy().set_cond_hint(control_hint, strength)
            if "control" in t[1]:
                c_net.set_previous_controlnet(t[1]["control"])
            n[1]["control"] = c_net
            n[1]["control_apply_to_uncond"] = True
            c.append(n)
        return (c,)


class ControlNetApplyAdvanced:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"positive": ("CONDITIONING",), "negative": ("CONDITIONING",),
                             "control_net": ("CONTROL_NET",), "image": ("IMAGE",),
                             "strength": ("FLOAT", {"default": 1.0, "min": 0.0, "max": 10.0, "step": 0.01}),
                             "start_percent": ("FLOAT", {"default": 0.0, "min": 0.0, "max": 1.0, "step": 0.001}),
                             "end_percent": ("FLOAT", {"default": 1.0, "min": 0.0, "max": 1.0, "step": 0.001})}}
    RETURN_TYPES = ("CONDITIONING", "CONDITIONING")
    RETURN_NAMES = ("positive", "negative")
    FUNCTION = "apply_controlnet"
    CATEGORY = "conditioning/controlnet"

    def apply_controlnet(self, positive, negative, control_net, image, strength, start_percent, end_percent):
        if strength == 0:
            return (positive, negative)
        control_hint = image.movedim(-1, 1)
        cnets = {}
        out = []
        for conditioning in [positive, negative]:
            c = []
            for t in conditioning:
                d = t[1].copy()
                prev_cnet = d.get("control", None)
                if prev_cnet in cnets:
                    c_net = cnets[prev_cnet]
                else:
                    c_net = control_net.copy().set_cond_hint(control_hint, strength, (start_percent, end_percent))
                    c_net.set_previous_controlnet(prev_cnet)
                    cnets[prev_cnet] = c_net
                d["control"] = c_net
                d["control_apply_to_uncond"] = False
                c.append([t[0], d])
            out.append(c)
        return (out[0], out[1])


# ================================================================ images
class SaveImage:
    def __init__(self):
        self.output_dir = folder_paths.get_output_directory()
        self.type = "output"
        self.prefix_append = ""
        self.compress_level = 4

    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"images": ("IMAGE",), "filename_prefix": ("STRING", {"default": "ComfyUI"})},
                "hidden": {"prompt": "PROMPT", "extra_pnginfo": "EXTRA_PNGINFO"}}
    RETURN_TYPES = ()
    FUNCTION = "save_images"
    OUTPUT_NODE = True
    CATEGORY = "image"

    def save_images(self, images, filename_prefix="ComfyUI", prompt=None, extra_pnginfo=None):
        from ..utils.imageio import save_png_batch
        self.output_dir = folder_paths.get_output_directory() if self.type == "output" else folder_paths.get_temp_directory()
        filename_prefix += self.prefix_append
        full_output_folder, filename, counter, subfolder, filename_prefix = folder_paths.get_save_image_path(
            filename_prefix, self.output_dir, images[0].shape[1], images[0].shape[0])
        metadata = None
        if not NH.args_disable_metadata():
            metadata = {}
            if prompt is not None:
                metadata["prompt"] = json.dumps(prompt)
            if extra_pnginfo is not None:
                for x in extra_pnginfo:
                    metadata[x] = json.dumps(extra_pnginfo[x])
        names = save_png_batch(images, full_output_folder, filename, counter, metadata, self.compress_level)
        results = [{"filename": n, "subfolder": subfolder, "type": self.type} for n in names]
        return {"ui": {"images": results}}


def save_image_to_respective_path(prefix_append, output_dir, images, filename_prefix, prompt, extra_pnginfo,
                                  compress_level, type, results):
    """Save ``images`` as PNGs under ``output_dir`` and append their ``{filename, subfolder, type}``
    records to ``results`` (the reference's shared SaveImage body, ``nodes.py:1630``; ``%batch_num%``
    in the prefix is replaced per image)."""
    from ..utils.imageio import save_png_batch
    filename_prefix += prefix_append
    full_output_folder, filename, counter, subfolder, filename_prefix = folder_paths.get_save_image_path(
        filename_prefix, output_dir, images[0].shape[1], images[0].shape[0])
    metadata = None
    if not NH.args_disable_metadata():
        metadata = {}
        if prompt is not None:
            metadata["prompt"] = json.dumps(prompt)
        if extra_pnginfo is not None:
            for x in extra_pnginfo:
                metadata[x] = json.dumps(extra_pnginfo[x])
    for b in range(images.shape[0]):
        name = filename.replace("%batch_num%", str(b))
        names = save_png_batch(images[b:b + 1], full_output_folder, name, counter, metadata, compress_level)
        results.extend({"filename": n, "subfolder": subfolder, "type": type} for n in names)
    return results


class PreviewImage(SaveImage):
    def __init__(self):
        self.output_dir = folder_paths.get_temp_directory()
        self.type = "temp"
        import random
        self.prefix_append = "_temp_" + "".join(random.choice("abcdefghijklmnopqrstupvxyz") for _ in range(5))
        self.compress_level = 1

    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"images": ("IMAGE",)}, "hidden": {"prompt": "PROMPT", "extra_pnginfo": "EXTRA_PNGINFO"}}


class LoadImage:
    @classmethod
    def INPUT_TYPES(s):
        input_dir = folder_paths.get_input_directory()
        files = [f for f in os.listdir(input_dir) if os.path.isfile(os.path.join(input_dir, f))] \
            if os.path.isdir(input_dir) else []
        return {"required": {"image": (sorted(files), {"image_upload": True})}}
    CATEGORY = "image"
    RETURN_TYPES = ("IMAGE", "MASK")
    FUNCTION = "load_image"

    def load_image(self, image):
        from ..utils.imageio import load_image_frames
        image_path = folder_paths.get_annotated_filepath(image)
        return load_image_frames(image_path)

    @classmethod
    def IS_CHANGED(s, image):
        return file_digest(folder_paths.get_annotated_filepath(image))

    @classmethod
    def VALIDATE_INPUTS(s, image):
        if not folder_paths.exists_annotated_filepath(image):
            return "Invalid image file: {}".format(image)
        return True


class LoadImageMask:
    _color_channels = ["alpha", "red", "green", "blue"]

    @classmethod
    def INPUT_TYPES(s):
        input_dir = folder_paths.get_input_directory()
        files = [f for f in os.listdir(input_dir) if os.path.isfile(os.path.join(input_dir, f))] \
            if os.path.isdir(input_dir) else []
        return {"required": {"image": (sorted(files), {"image_upload": True}), "channel": (s._color_channels,)}}
    CATEGORY = "mask"
    RETURN_TYPES = ("MASK",)
    FUNCTION = "load_image"

    def load_image(self, image, channel):
        from ..utils.imageio import load_mask_channel
        return (load_mask_channel(folder_paths.get_annotated_filepath(image), channel),)

    @classmethod
    def IS_CHANGED(s, image, channel):
        return file_digest(folder_paths.get_annotated_filepath(image))

    @classmethod
    def VALIDATE_INPUTS(s, image):
        if not folder_paths.exists_annotated_filepath(image):
            return "Invalid image file: {}".format(image)
        return True


class ImageScale:
    upscale_methods = ["nearest-exact", "bilinear", "area", "bicubic", "lanczos"]
    crop_methods = ["disabled", "center"]

    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"image": ("IMAGE",), "upscale_method": (s.upscale_methods,),
                             "width": ("INT", {"default": 512, "min": 0, "max": MAX_RESOLUTION, "step": 1}),
                             "height": ("INT", {"default": 512, "min": 0, "max": MAX_RESOLUTION, "step": 1}),
                             "crop": (s.crop_methods,)}}
    RETURN_TYPES = ("IMAGE",)
    FUNCTION = "upscale"
    CATEGORY = "image/upscaling"

    def upscale(self, image, upscale_method, width, height, crop):
        if width == 0 and height == 0:
            s = image
        else:
            samples = image.movedim(-1, 1)
            if width == 0:
                width = max(1, round(samples.shape[3] * height / samples.shape[2]))
            elif height == 0:
                height = max(1, round(samples.shape[2] * width / samples.shape[3]))
            s = U.common_upscale(samples, width, height, upscale_method, crop).movedim(1, -1)
        return (s,)


class ImageScaleBy:
    upscale_methods = ["nearest-exact", "bilinear", "area", "bicubic", "lanczos"]

    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"image": ("IMAGE",), "upscale_method": (s.upscale_methods,),
                             "scale_by": ("FLOAT", {"default": 1.0, "min": 0.01, "max": 8.0, "step": 0.01})}}
    RETURN_TYPES = ("IMAGE",)
    FUNCTION = "upscale"
    CATEGORY = "image/upscaling"

    def upscale(self, image, upscale_method, scale_by):
        samples = image.movedim(-1, 1)
        width = round(samples.shape[3] * scale_by)
        height = round(samples.shape[2] * scale_by)
        return (U.common_upscale(samples, width, height, upscale_method, "disabled").movedim(1, -1),)


class ImageInvert:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"image": ("IMAGE",)}}
    RETURN_TYPES = ("IMAGE",)
    FUNCTION = "invert"
    CATEGORY = "image"

    def invert(self, image):
        return (1.0 - image,)


class ImageBatch:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"image1": ("IMAGE",), "image2": ("IMAGE",)}}
    RETURN_TYPES = ("IMAGE",)
    FUNCTION = "batch"
    CATEGORY = "image"

    def batch(self, image1, image2):
        if image1.shape[1:] != image2.shape[1:]:
            image2 = U.common_upscale(image2.movedim(-1, 1), image1.shape[2], image1.shape[1], "bilinear", "center").movedim(1, -1)
        return (torch.cat((image1, image2.to(image1)), dim=0),)


class EmptyImage:
    def __init__(self, device="cpu"):
        self.device = device

    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"width": ("INT", {"default": 512, "min": 1, "max": MAX_RESOLUTION, "step": 1}),
                             "height": ("INT", {"default": 512, "min": 1, "max": MAX_RESOLUTION, "step": 1}),
                             "batch_size": ("INT", {"default": 1, "min": 1, "max": 4096}),
                             "color": ("INT", {"default": 0, "min": 0, "max": 0xFFFFFF, "step": 1, "display": "color"})}}
    RETURN_TYPES = ("IMAGE",)
    FUNCTION = "generate"
    CATEGORY = "image"

    def generate(self, width, height, batch_size=1, color=0):
        r = torch.full([batch_size, height, width, 1], ((color >> 16) & 0xFF) / 0xFF)
        g = torch.full([batch_size, height, width, 1], ((color >> 8) & 0xFF) / 0xFF)
        b = torch.full([batch_size, height, width, 1], (color & 0xFF) / 0xFF)
        return (torch.cat((r, g, b), dim=-1),)


class ImagePadForOutpaint:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"image": ("IMAGE",),
                             "left": ("INT", {"default": 0, "min": 0, "max": MAX_RESOLUTION, "step": 8}),
                             "top": ("INT", {"default": 0, "min": 0, "max": MAX_RESOLUTION, "step": 8}),
                             "right": ("INT", {"default": 0, "min": 0, "max": MAX_RESOLUTION, "step": 8}),
                             "bottom": ("INT", {"default": 0, "min": 0, "max": MAX_RESOLUTION, "step": 8}),
                             "feathering": ("INT", {"default": 40, "min": 0, "max": MAX_RESOLUTION, "step": 1})}}
    RETURN_TYPES = ("IMAGE", "MASK")
    FUNCTION = "expand_image"
    CATEGORY = "image"

    def expand_image(self, image, left, top, right, bottom, feathering):
        d1, d2, d3, d4 = image.size()
        new_image = torch.ones((d1, d2 + top + bottom, d3 + left + right, d4), dtype=torch.float32) * 0.5
        new_image[:, top:top + d2, left:left + d3, :] = image
        mask = torch.ones((d2 + top + bottom, d3 + left + right), dtype=torch.float32)
        t = torch.zeros((d2, d3), dtype=torch.float32)
        if feathering > 0 and feathering * 2 < d2 and feathering * 2 < d3:
            for i in range(d2):
                for j in range(d3):
                    dt = i if top != 0 else d2
                    db = d2 - i if bottom != 0 else d2
                    dl = j if left != 0 else d3
                    dr = d3 - j if right != 0 else d3
                    dd = min(dt, db, dl, dr)
                    if dd >= feathering:
                        continue
                    v = (feathering - dd) / feathering
                    t[i, j] = v * v
        mask[top:top + d2, left:left + d3] = t
        return (new_image, mask)


NODE_CLASS_MAPPINGS = {
    "KSampler": KSampler, "CheckpointLoaderSimple": CheckpointLoaderSimple, "CLIPTextEncode": CLIPTextEncode,
    "CLIPSetLastLayer": CLIPSetLastLayer, "VAEDecode": VAEDecode, "VAEEncode": VAEEncode,
    "VAEEncodeForInpaint": VAEEncodeForInpaint, "VAELoader": VAELoader, "EmptyLatentImage": EmptyLatentImage,
    "LatentUpscale": LatentUpscale, "LatentUpscaleBy": LatentUpscaleBy, "LatentFromBatch": LatentFromBatch,
    "RepeatLatentBatch": RepeatLatentBatch, "SaveImage": SaveImage, "PreviewImage": PreviewImage,
    "LoadImage": LoadImage, "LoadImageMask": LoadImageMask, "ImageScale": ImageScale, "ImageScaleBy": ImageScaleBy,
    "ImageInvert": ImageInvert, "ImageBatch": ImageBatch, "ImagePadForOutpaint": ImagePadForOutpaint,
    "EmptyImage": EmptyImage, "ConditioningAverage": ConditioningAverage, "ConditioningCombine": ConditioningCombine,
    "ConditioningConcat": ConditioningConcat, "ConditioningSetArea": ConditioningSetArea,
    "ConditioningSetAreaPercentage": ConditioningSetAreaPercentage,
    "ConditioningSetAreaStrength": ConditioningSetAreaStrength, "ConditioningSetMask": ConditioningSetMask,
    "KSamplerAdvanced": KSamplerAdvanced, "SetLatentNoiseMask": SetLatentNoiseMask,
    "LatentComposite": LatentComposite, "LatentBlend": LatentBlend, "LatentRotate": LatentRotate,
    "LatentFlip": LatentFlip, "LatentCrop": LatentCrop, "LoraLoader": LoraLoader, "CLIPLoader": CLIPLoader,
    "UNETLoader": UNETLoader, "DualCLIPLoader": DualCLIPLoader, "CLIPVisionEncode": CLIPVisionEncode,
    "StyleModelApply": StyleModelApply, "unCLIPConditioning": unCLIPConditioning, "ControlNetApply": ControlNetApply,
    "ControlNetApplyAdvanced": ControlNetApplyAdvanced, "ControlNetLoader": ControlNetLoader,
    "DiffControlNetLoader": DiffControlNetLoader, "StyleModelLoader": StyleModelLoader,
    "CLIPVisionLoader": CLIPVisionLoader, "VAEDecodeTiled": VAEDecodeTiled, "VAEEncodeTiled": VAEEncodeTiled,
    "unCLIPCheckpointLoader": unCLIPCheckpointLoader, "GLIGENLoader": GLIGENLoader,
    "GLIGENTextBoxApply": GLIGENTextBoxApply, "InpaintModelConditioning": InpaintModelConditioning,
    "CheckpointLoader": CheckpointLoader, "DiffusersLoader": DiffusersLoader, "LoadLatent": LoadLatent,
    "SaveLatent": SaveLatent, "ConditioningZeroOut": ConditioningZeroOut,
    "ConditioningSetTimestepRange": ConditioningSetTimestepRange, "LoraLoaderModelOnly": LoraLoaderModelOnly,
}

NODE_DISPLAY_NAME_MAPPINGS = {
    "KSampler": "KSampler", "KSamplerAdvanced": "KSampler (Advanced)",
    "CheckpointLoader": "Load Checkpoint With Config (DEPRECATED)", "CheckpointLoaderSimple": "Load Checkpoint",
    "VAELoader": "Load VAE", "LoraLoader": "Load LoRA", "CLIPLoader": "Load CLIP",
    "ControlNetLoader": "Load ControlNet Model", "DiffControlNetLoader": "Load ControlNet Model (diff)",
    "StyleModelLoader": "Load Style Model", "CLIPVisionLoader": "Load CLIP Vision",
    "UpscaleModelLoader": "Load Upscale Model", "CLIPTextEncode": "CLIP Text Encode (Prompt)",
    "CLIPSetLastLayer": "CLIP Set Last Layer", "ConditioningCombine": "Conditioning (Combine)",
    "ConditioningAverage ": "Conditioning (Average)", "ConditioningConcat": "Conditioning (Concat)",
    "ConditioningSetArea": "Conditioning (Set Area)",
    "ConditioningSetAreaPercentage": "Conditioning (Set Area with Percentage)",
    "ConditioningSetMask": "Conditioning (Set Mask)", "ControlNetApply": "Apply ControlNet",
    "ControlNetApplyAdvanced": "Apply ControlNet (Advanced)", "LatentUpscale": "Upscale Latent",
    "LatentUpscaleBy": "Upscale Latent By", "LatentComposite": "Latent Composite", "LatentBlend": "Latent Blend",
    "LatentFromBatch": "Latent From Batch", "RepeatLatentBatch": "Repeat Latent Batch",
    "SaveImage": "Save Image", "PreviewImage": "Preview Image", "LoadImage": "Load Image",
    "LoadImageMask": "Load Image (as Mask)", "ImageScale": "Upscale Image", "ImageScaleBy": "Upscale Image By",
    "ImageUpscaleWithModel": "Upscale Image (using Model)", "ImageInvert": "Invert Image",
    "ImagePadForOutpaint": "Pad Image for Outpainting", "ImageBatch": "Batch Images",
    "VAEDecode": "VAE Decode", "VAEEncode": "VAE Encode", "LatentRotate": "Rotate Latent",
    "VAEEncodeForInpaint": "VAE Encode (for Inpainting)", "SetLatentNoiseMask": "Set Latent Noise Mask",
    "VAEDecodeTiled": "VAE Decode (Tiled)", "VAEEncodeTiled": "VAE Encode (Tiled)", "LatentFlip": "Flip Latent",
    "LatentCrop": "Crop Latent", "EmptyLatentImage": "Empty Latent Image",
}
