"""Image / latent resizing and tiling utilities (parity: ``comfy/utils.py:318-454``; K24/K25).

common_upscale: nearest-exact / bilinear / area / bicubic / lanczos (PIL) / bislerp, optional
center crop. tiled_scale: feather-blended tiled application of a function (VAE / upscalers).
"""
from __future__ import annotations

import itertools
import math

import numpy as np
import torch
import torch.nn.functional as F


def bislerp(samples, width, height):
    """Spherical-linear bilinear resize of latents (channel vectors slerped)."""
    def slerp(b1, b2, r):
        c = b1.shape[-1]
        n1 = torch.norm(b1, dim=-1, keepdim=True)
        n2 = torch.norm(b2, dim=-1, keepdim=True)
        b1n = b1 / n1
        b2n = b2 / n2
        b1n[n1.expand(-1, c) == 0.0] = 0.0
        b2n[n2.expand(-1, c) == 0.0] = 0.0
        dot = (b1n * b2n).sum(1)
        omega = torch.acos(dot)
        so = torch.sin(omega)
        res = (torch.sin((1.0 - r.squeeze(1)) * omega) / so).unsqueeze(1) * b1n + \
              (torch.sin(r.squeeze(1) * omega) / so).unsqueeze(1) * b2n
        res *= (n1 * (1.0 - r) + n2 * r).expand(-1, c)
        res[dot > 1 - 1e-5] = b1[dot > 1 - 1e-5]
        res[dot < 1e-5 - 1] = (b1 * (1.0 - r) + b2 * r)[dot < 1e-5 - 1]
        return res

    def coords(l_in, l_out):
        ramp = torch.arange(l_out, dtype=torch.float32) * (l_in / l_out)
        c1 = ramp.floor().long()
        ratios = ramp - c1
        c2 = (c1 + 1).clamp(max=l_in - 1)
        return c1, c2, ratios

    orig_dtype = samples.dtype
    samples = samples.float()
    n, c, h, w = samples.shape
    h_new, w_new = height, width
    c1, c2, r = coords(w, w_new)
    c1 = c1.view(1, 1, 1, -1).expand((n, c, h, w_new)).to(samples.device)
    c2 = c2.view(1, 1, 1, -1).expand((n, c, h, w_new)).to(samples.device)
    r = r.view(1, 1, 1, -1).expand((n, 1, h, w_new)).to(samples.device)
    p1 = samples.gather(-1, c1).movedim(1, -1).reshape((-1, c))
    p2 = samples.gather(-1, c2).movedim(1, -1).reshape((-1, c))
    r = r.movedim(1, -1).reshape((-1, 1))
    result = slerp(p1, p2, r).reshape(n, h, w_new, c).movedim(-1, 1)
    c1, c2, r = coords(h, h_new)
    c1 = c1.view(1, 1, -1, 1).expand((n, c, h_new, w_new)).to(samples.device)
    c2 = c2.view(1, 1, -1, 1).expand((n, c, h_new, w_new)).to(samples.device)
    r = r.view(1, 1, -1, 1).expand((n, 1, h_new, w_new)).to(samples.device)
    p1 = result.gather(-2, c1).movedim(1, -1).reshape((-1, c))
    p2 = result.gather(-2, c2).movedim(1, -1).reshape((-1, c))
    r = r.movedim(1, -1).reshape((-1, 1))
    result = slerp(p1, p2, r).reshape(n, h_new, w_new, c).movedim(-1, 1)
    return result.to(orig_dtype)


def lanczos(samples, width, height):
    from PIL import Image
    imgs = [Image.fromarray(np.clip(255.0 * im.movedim(0, -1).cpu().numpy(), 0, 255).astype(np.uint8)) for im in samples]
    imgs = [im.resize((width, height), resample=Image.Resampling.LANCZOS) for im in imgs]
    imgs = [torch.from_numpy(np.array(im).astype(np.float32) / 255.0).movedim(-1, 0) for im in imgs]
    return torch.stack(imgs).to(samples.device, samples.dtype)


def common_upscale(samples, width, height, upscale_method, crop):
    if crop == "center":
        old_w, old_h = samples.shape[3], samples.shape[2]
        old_aspect = old_w / old_h
        new_aspect = width / height
        x = y = 0
        if old_aspect > new_aspect:
            x = round((old_w - old_w * (new_aspect / old_aspect)) / 2)
        elif old_aspect < new_aspect:
            y = round((old_h - old_h * (old_aspect / new_aspect)) / 2)
        s = samples[:, :, y:old_h - y, x:old_w - x]
    else:
        s = samples
    if upscale_method == "bislerp":
        return bislerp(s, width, height)
    if upscale_method == "lanczos":
        return lanczos(s, width, height)
    from .. import ops
    return ops.interpolate(s, (height, width), upscale_method)


def get_tiled_scale_steps(width, height, tile_x, tile_y, overlap):
    return math.ceil(height / (tile_y - overlap)) * math.ceil(width / (tile_x - overlap))


@torch.inference_mode()
def tiled_scale(samples, function, tile_x=64, tile_y=64, overlap=8, upscale_amount=4, out_channels=3,
                output_device="cpu", pbar=None):
    from .. import ops
    out_full = torch.empty((samples.shape[0], out_channels, round(samples.shape[2] * upscale_amount),
                            round(samples.shape[3] * upscale_amount)), device=output_device)
    for b in range(samples.shape[0]):
        s = samples[b:b + 1]
        out = torch.zeros((1, out_channels, round(s.shape[2] * upscale_amount), round(s.shape[3] * upscale_amount)),
                          device=output_device)
        div = torch.zeros_like(out)
        for y in range(0, s.shape[2], tile_y - overlap):
            for x in range(0, s.shape[3], tile_x - overlap):
                x0 = max(0, min(s.shape[-1] - overlap, x))
                y0 = max(0, min(s.shape[-2] - overlap, y))
                piece = s[:, :, y0:y0 + tile_y, x0:x0 + tile_x]
                ps = function(piece).to(output_device)
                feather = round(overlap * upscale_amount)
                oy, ox = round(y0 * upscale_amount), round(x0 * upscale_amount)
                # out += piece * ramp ; div += ramp (separable feather ramp; one HIP kernel, K24)
                ops.region_accumulate(out, div, ps, oy, ox, feather=feather)
                if pbar is not None:
                    pbar.update(1)
        out_full[b:b + 1] = ops.region_normalize(out, div)
    return out_full


def resize_to_batch_size(tensor, batch_size):
    in_bs = tensor.shape[0]
    if in_bs == batch_size:
        return tensor
    if batch_size <= 1:
        return tensor[:batch_size]
    out = torch.empty([batch_size] + list(tensor.shape)[1:], dtype=tensor.dtype, device=tensor.device)
    if batch_size < in_bs:
        scale = (in_bs - 1) / (batch_size - 1)
        for i in range(batch_size):
            out[i] = tensor[min(round(i * scale), in_bs - 1)]
    else:
        scale = in_bs / batch_size
        for i in range(batch_size):
            out[i] = tensor[min(math.floor((i + 0.5) * scale), in_bs - 1)]
    return out


def pil_to_tensor(img):
    arr = np.array(img).astype(np.float32) / 255.0
    return torch.from_numpy(arr)[None]


def tensor_to_pil(t):
    from PIL import Image
    arr = np.clip(255.0 * t.detach().float().cpu().numpy(), 0, 255).astype(np.uint8)
    return Image.fromarray(arr)


def repeat_to_batch_size(tensor, batch_size, dim=0):
    """Tile (then truncate) along ``dim`` to ``batch_size`` (comfy/utils.py repeat_to_batch_size)."""
    n = tensor.shape[dim]
    if n > batch_size:
        return tensor.narrow(dim, 0, batch_size)
    if n < batch_size:
        reps = [1] * tensor.ndim
        reps[dim] = math.ceil(batch_size / n)
        return tensor.repeat(reps).narrow(dim, 0, batch_size)
    return tensor
