"""Image <-> bytes conversion decorator for nodes that talk to external services
(parity: ``helper_decorators.py:12-145``).

``convert_image_format`` inspects the wrapped function's annotations and converts arguments on the
fly: ``torch.Tensor`` parameters accept encoded image bytes (decoded, all frames), ``bytes`` /
``BinaryIO`` parameters accept an IMAGE tensor (PNG-encoded, batch of 1).
"""
from __future__ import annotations

import functools
import inspect
import io
from typing import BinaryIO

import numpy as np
import torch


def bytes_to_tensor(data: bytes) -> torch.Tensor:
    """Encoded image (any PIL format, multi-frame ok) -> [F, H, W, 3] float in [0, 1]."""
    from PIL import Image, ImageOps, ImageSequence
    img = Image.open(io.BytesIO(data))
    frames = []
    for f in ImageSequence.Iterator(img):
        f = ImageOps.exif_transpose(f)
        if f.mode == "I":
            f = f.point(lambda v: v * (1 / 255))
        arr = np.asarray(f.convert("RGB"), dtype=np.float32) / 255.0
        frames.append(torch.from_numpy(arr)[None])
    return torch.cat(frames, 0) if len(frames) > 1 else frames[0]


def _png(tensor: torch.Tensor) -> io.BytesIO:
    from PIL import Image
    if tensor.ndim == 4:
        if tensor.shape[0] != 1:
            raise ValueError("The input tensor should have a batch size of 1 or no batch dimension.")
        tensor = tensor[0]
    arr = np.clip(255.0 * tensor.detach().float().cpu().numpy(), 0, 255).astype(np.uint8)
    bio = io.BytesIO()
    Image.fromarray(arr).save(bio, format="PNG")
    bio.seek(0)
    return bio


def tensor_to_bytes(tensor: torch.Tensor) -> bytes:
    return _png(tensor).getvalue()


def tensor_to_binaryio(tensor: torch.Tensor) -> BinaryIO:
    return _png(tensor)


def convert_image_format(func):
    sig = inspect.signature(func)
    ann = {n: p.annotation for n, p in sig.parameters.items() if p.annotation is not inspect.Parameter.empty}

    @functools.wraps(func)
    def wrapper(*args, **kwargs):
        bound = sig.bind(*args, **kwargs)
        bound.apply_defaults()
        for name, value in list(bound.arguments.items()):
            want = ann.get(name)
            if want in (torch.Tensor, "torch.Tensor") and isinstance(value, (bytes, bytearray)):
                bound.arguments[name] = bytes_to_tensor(bytes(value))
            elif want in (bytes, "bytes") and isinstance(value, torch.Tensor):
                bound.arguments[name] = tensor_to_bytes(value)
            elif want in (BinaryIO, "BinaryIO") and isinstance(value, torch.Tensor):
                bound.arguments[name] = tensor_to_binaryio(value)
        return func(*bound.args, **bound.kwargs)

    return wrapper
