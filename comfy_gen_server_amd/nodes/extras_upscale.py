"""Model-based image upscaling nodes (parity: ``comfy_extras/nodes_upscale_model.py``).

``ImageUpscaleWithModel`` runs the network tile by tile (512 px tiles, 32 px overlap, feathered
blend) and halves the tile on device OOM down to 128 px, like the reference.
"""
from __future__ import annotations

import torch

from ..models import upscalers
from ..runtime import device as dm
from ..runtime.checkpoint import load_state_dict
from ..runtime.convert import state_dict_prefix_replace
from ..utils import folder_paths
from ..utils import image as U
from ..utils.progress import ProgressBar


class UpscaleModelLoader:
    RETURN_TYPES = ("UPSCALE_MODEL",)
    FUNCTION = "load_model"
    CATEGORY = "loaders"

    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"model_name": (folder_paths.get_filename_list("upscale_models"),)}}

    def load_model(self, model_name):
        sd = load_state_dict(folder_paths.get_full_path("upscale_models", model_name))
        if "module.layers.0.residual_group.blocks.0.norm1.weight" in sd:
            sd = state_dict_prefix_replace(sd, {"module.": ""})
        return (upscalers.load_state_dict(sd).eval(),)


def _first(out):
    """Face-restoration nets return (image, aux...) like the reference architectures."""
    return out[0] if isinstance(out, (tuple, list)) else out


class ImageUpscaleWithModel:
    RETURN_TYPES = ("IMAGE",)
    FUNCTION = "upscale"
    CATEGORY = "image/upscaling"

    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"upscale_model": ("UPSCALE_MODEL",), "image": ("IMAGE",)}}

    def upscale(self, upscale_model, image):
        device = dm.get_torch_device()
        dtype = torch.bfloat16 if device.type == "cuda" else torch.float32
        upscale_model.to(device=device, dtype=dtype)
        x = image.movedim(-1, -3).to(device=device, dtype=dtype)
        tile, overlap = 512, 32
        while True:
            try:
                steps = x.shape[0] * U.get_tiled_scale_steps(x.shape[3], x.shape[2], tile, tile, overlap)
                pbar = ProgressBar(steps)
                with torch.inference_mode():
                    s = U.tiled_scale(x, lambda a: _first(upscale_model(a)).float(), tile_x=tile, tile_y=tile,
                                      overlap=overlap, upscale_amount=upscale_model.scale, pbar=pbar,
                                      output_device=dm.intermediate_device())
                break
            except torch.cuda.OutOfMemoryError:
                tile //= 2
                if tile < 128:
                    raise
        upscale_model.to("cpu")
        return (torch.clamp(s.movedim(-3, -1), 0.0, 1.0),)


NODE_CLASS_MAPPINGS = {"UpscaleModelLoader": UpscaleModelLoader, "ImageUpscaleWithModel": ImageUpscaleWithModel}
