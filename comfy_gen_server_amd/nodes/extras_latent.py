"""Latent arithmetic / batching nodes (parity: ``comfy_extras/nodes_latent.py``, ``nodes_rebatch.py``).

LATENT = {"samples": [B,C,H,W] (host), optional "noise_mask", "batch_index" (per-image noise
replay indices, see sampling.sample.prepare_noise)}.
"""
from __future__ import annotations

import torch

from ..utils import image as U


def reshape_latent_to(target_shape, latent):
    """Resize (bilinear, center crop) + repeat to the target batch (nodes_latent.py:4-7)."""
    if latent.shape[1:] != target_shape[1:]:
        latent = U.common_upscale(latent, target_shape[3], target_shape[2], "bilinear", "center")
    return U.repeat_to_batch_size(latent, target_shape[0])


class _Binary:
    RETURN_TYPES = ("LATENT",)
    FUNCTION = "op"
    CATEGORY = "latent/advanced"

    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"samples1": ("LATENT",), "samples2": ("LATENT",)}}

    def combine(self, a, b):
        raise NotImplementedError

    def op(self, samples1, samples2):
        out = samples1.copy()
        s1 = samples1["samples"]
        out["samples"] = self.combine(s1, reshape_latent_to(s1.shape, samples2["samples"]))
        return (out,)


class LatentAdd(_Binary):
    def combine(self, a, b):
        return a + b


class LatentSubtract(_Binary):
    def combine(self, a, b):
        return a - b


class LatentMultiply:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"samples": ("LATENT",),
                             "multiplier": ("FLOAT", {"default": 1.0, "min": -10.0, "max": 10.0, "step": 0.01})}}
    RETURN_TYPES = ("LATENT",)
    FUNCTION = "op"
    CATEGORY = "latent/advanced"

    def op(self, samples, multiplier):
        out = samples.copy()
        out["samples"] = samples["samples"] * multiplier
        return (out,)


class LatentInterpolate:
    """Interpolate directions (per-pixel channel vectors) and magnitudes separately."""

    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"samples1": ("LATENT",), "samples2": ("LATENT",),
                             "ratio": ("FLOAT", {"default": 1.0, "min": 0.0, "max": 1.0, "step": 0.01})}}
    RETURN_TYPES = ("LATENT",)
    FUNCTION = "op"
    CATEGORY = "latent/advanced"

    def op(self, samples1, samples2, ratio):
        out = samples1.copy()
        a = samples1["samples"]
        b = reshape_latent_to(a.shape, samples2["samples"])
        na = torch.linalg.vector_norm(a, dim=1, keepdim=True)
        nb = torch.linalg.vector_norm(b, dim=1, keepdim=True)
        mix = torch.nan_to_num(a / na) * ratio + torch.nan_to_num(b / nb) * (1.0 - ratio)
        direction = torch.nan_to_num(mix / torch.linalg.vector_norm(mix, dim=1, keepdim=True))
        out["samples"] = direction * (na * ratio + nb * (1.0 - ratio))
        return (out,)


class LatentBatch:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"samples1": ("LATENT",), "samples2": ("LATENT",)}}
    RETURN_TYPES = ("LATENT",)
    FUNCTION = "batch"
    CATEGORY = "latent/batch"

    def batch(self, samples1, samples2):
        out = samples1.copy()
        a, b = samples1["samples"], samples2["samples"]
        if a.shape[1:] != b.shape[1:]:
            b = U.common_upscale(b, a.shape[3], a.shape[2], "bilinear", "center")
        out["samples"] = torch.cat((a, b), dim=0)
        out["batch_index"] = (samples1.get("batch_index", list(range(a.shape[0]))) +
                              samples2.get("batch_index", list(range(b.shape[0]))))
        return (out,)


class LatentBatchSeedBehavior:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"samples": ("LATENT",),
                             "seed_behavior": (["random", "fixed"], {"default": "fixed"})}}
    RETURN_TYPES = ("LATENT",)
    FUNCTION = "op"
    CATEGORY = "latent/advanced"

    def op(self, samples, seed_behavior):
        out = samples.copy()
        if seed_behavior == "random":
            out.pop("batch_index", None)
        else:
            first = out.get("batch_index", [0])[0]
            out["batch_index"] = [first] * samples["samples"].shape[0]
        return (out,)


# ---------------------------------------------------------------- rebatching
def _expand_mask(mask, samples):
    """noise_mask -> one [1,1,H,W]-per-sample list matching ``samples``."""
    if mask is None:
        return [None] * samples.shape[0]
    m = mask
    if m.ndim == 2:
        m = m[None, None]
    elif m.ndim == 3:
        m = m[:, None]
    if m.shape[-2:] != samples.shape[-2:]:
        m = torch.nn.functional.interpolate(m.float(), size=samples.shape[-2:], mode="bilinear")
    m = U.repeat_to_batch_size(m, samples.shape[0])
    return [m[i:i + 1] for i in range(samples.shape[0])]


class RebatchLatents:
    """Regroup a list of latents into batches of ``batch_size`` (shape changes start a new group)."""

    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"latents": ("LATENT",),
                             "batch_size": ("INT", {"default": 1, "min": 1, "max": 4096})}}
    RETURN_TYPES = ("LATENT",)
    INPUT_IS_LIST = True
    OUTPUT_IS_LIST = (True,)
    FUNCTION = "rebatch"
    CATEGORY = "latent/batch"

    def rebatch(self, latents, batch_size):
        batch_size = batch_size[0]
        items = []   # (sample [1,C,H,W], mask or None, batch index)
        for lat in latents:
            s = lat["samples"]
            masks = _expand_mask(lat.get("noise_mask"), s)
            idx = lat.get("batch_index", list(range(s.shape[0])))
            for i in range(s.shape[0]):
                items.append((s[i:i + 1], masks[i], idx[i] if i < len(idx) else i))
        out, cur = [], []

        def flush():
            if not cur:
                return
            d = {"samples": torch.cat([c[0] for c in cur]), "batch_index": [c[2] for c in cur]}
            if any(c[1] is not None for c in cur):
                d["noise_mask"] = torch.cat([c[1] if c[1] is not None else torch.ones_like(c[0][:, :1])
                                             for c in cur])
            out.append(d)
            cur.clear()

        for it in items:
            if cur and (it[0].shape[1:] != cur[0][0].shape[1:] or len(cur) >= batch_size):
                flush()
            cur.append(it)
        flush()
        return (out,)


class RebatchImages:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"images": ("IMAGE",),
                             "batch_size": ("INT", {"default": 1, "min": 1, "max": 4096})}}
    RETURN_TYPES = ("IMAGE",)
    INPUT_IS_LIST = True
    OUTPUT_IS_LIST = (True,)
    FUNCTION = "rebatch"
    CATEGORY = "image/batch"

    def rebatch(self, images, batch_size):
        batch_size = batch_size[0]
        frames = [img[i:i + 1] for img in images for i in range(img.shape[0])]
        out, cur = [], []
        for f in frames:
            if cur and (f.shape[1:] != cur[0].shape[1:] or len(cur) >= batch_size):
                out.append(torch.cat(cur))
                cur = []
            cur.append(f)
        if cur:
            out.append(torch.cat(cur))
        return (out,)


NODE_CLASS_MAPPINGS = {
    "LatentAdd": LatentAdd, "LatentSubtract": LatentSubtract, "LatentMultiply": LatentMultiply,
    "LatentInterpolate": LatentInterpolate, "LatentBatch": LatentBatch,
    "LatentBatchSeedBehavior": LatentBatchSeedBehavior, "RebatchLatents": RebatchLatents,
    "RebatchImages": RebatchImages,
}
NODE_DISPLAY_NAME_MAPPINGS = {"RebatchLatents": "Rebatch Latents", "RebatchImages": "Rebatch Images"}
