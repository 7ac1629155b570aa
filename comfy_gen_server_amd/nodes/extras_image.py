"""Image nodes (parity: ``comfy_extras/nodes_images.py``, ``nodes_post_processing.py``, ``nodes_compositing.py``,
``nodes_morphology.py``, ``nodes_canny.py``).

IMAGE = float [B,H,W,C] in 0..1 (host). Filters run on the compute device when one is present.
The reference's morphology and Canny come from kornia, which is not in this image: both are
re-implemented here in plain torch (grey morphology with a flat square kernel; Canny = 5x5
Gaussian (sigma 1) -> Sobel -> non-maximum suppression -> double threshold -> hysteresis), so
their outputs are "parity unpinned" against kornia (tests check the defining properties instead).
"""
from __future__ import annotations

import enum
import json
import math
import os

import numpy as np
import torch
import torch.nn.functional as F

from ..runtime import device as dm
from ..utils import folder_paths
from ..utils import image as U
from . import helpers as NH

MAX_RESOLUTION = 16384


# ---------------------------------------------------------------- batch / crop
class ImageCrop:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"image": ("IMAGE",),
                             "width": ("INT", {"default": 512, "min": 1, "max": MAX_RESOLUTION, "step": 1}),
                             "height": ("INT", {"default": 512, "min": 1, "max": MAX_RESOLUTION, "step": 1}),
                             "x": ("INT", {"default": 0, "min": 0, "max": MAX_RESOLUTION, "step": 1}),
                             "y": ("INT", {"default": 0, "min": 0, "max": MAX_RESOLUTION, "step": 1})}}
    RETURN_TYPES = ("IMAGE",)
    FUNCTION = "crop"
    CATEGORY = "image/transform"

    def crop(self, image, width, height, x, y):
        x = min(x, image.shape[2] - 1)
        y = min(y, image.shape[1] - 1)
        return (image[:, y:y + height, x:x + width, :],)


class RepeatImageBatch:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"image": ("IMAGE",), "amount": ("INT", {"default": 1, "min": 1, "max": 4096})}}
    RETURN_TYPES = ("IMAGE",)
    FUNCTION = "repeat"
    CATEGORY = "image/batch"

    def repeat(self, image, amount):
        return (image.repeat((amount, 1, 1, 1)),)


class ImageFromBatch:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"image": ("IMAGE",), "batch_index": ("INT", {"default": 0, "min": 0, "max": 4095}),
                             "length": ("INT", {"default": 1, "min": 1, "max": 4096})}}
    RETURN_TYPES = ("IMAGE",)
    FUNCTION = "frombatch"
    CATEGORY = "image/batch"

    def frombatch(self, image, batch_index, length):
        batch_index = min(image.shape[0] - 1, batch_index)
        length = min(image.shape[0] - batch_index, length)
        return (image[batch_index:batch_index + length].clone(),)


def _pil_frames(images):
    from PIL import Image
    arr = np.clip(images.detach().float().cpu().numpy() * 255.0, 0, 255).astype(np.uint8)
    return [Image.fromarray(a) for a in arr]


class SaveAnimatedWEBP:
    methods = {"default": 4, "fastest": 0, "slowest": 6}

    def __init__(self):
        self.output_dir = folder_paths.get_output_directory()
        self.type = "output"
        self.prefix_append = ""

    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"images": ("IMAGE",), "filename_prefix": ("STRING", {"default": "ComfyUI"}),
                             "fps": ("FLOAT", {"default": 6.0, "min": 0.01, "max": 1000.0, "step": 0.01}),
                             "lossless": ("BOOLEAN", {"default": True}),
                             "quality": ("INT", {"default": 80, "min": 0, "max": 100}),
                             "method": (list(s.methods.keys()),)},
                "hidden": {"prompt": "PROMPT", "extra_pnginfo": "EXTRA_PNGINFO"}}
    RETURN_TYPES = ()
    FUNCTION = "save_images"
    OUTPUT_NODE = True
    CATEGORY = "image/animation"

    def save_images(self, images, fps, filename_prefix, lossless, quality, method, num_frames=0, prompt=None,
                    extra_pnginfo=None):
        self.output_dir = folder_paths.get_output_directory()
        folder, filename, counter, subfolder, _ = folder_paths.get_save_image_path(
            filename_prefix + self.prefix_append, self.output_dir, images[0].shape[1], images[0].shape[0])
        frames = _pil_frames(images)
        exif = frames[0].getexif()
        if not NH.args_disable_metadata():
            if prompt is not None:
                exif[0x0110] = "prompt:{}".format(json.dumps(prompt))
            if extra_pnginfo is not None:
                tag = 0x010F
                for k in extra_pnginfo:
                    exif[tag] = "{}:{}".format(k, json.dumps(extra_pnginfo[k]))
                    tag -= 1
        num_frames = num_frames or len(frames)
        results = []
        for i in range(0, len(frames), num_frames):
            file = f"{filename}_{counter:05}_.webp"
            frames[i].save(os.path.join(folder, file), save_all=True, duration=int(1000.0 / fps),
                           append_images=frames[i + 1:i + num_frames], exif=exif, lossless=lossless,
                           quality=quality, method=self.methods.get(method))
            results.append({"filename": file, "subfolder": subfolder, "type": self.type})
            counter += 1
        return {"ui": {"images": results, "animated": (num_frames != 1,)}}


class SaveAnimatedPNG:
    def __init__(self):
        self.output_dir = folder_paths.get_output_directory()
        self.type = "output"
        self.prefix_append = ""

    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"images": ("IMAGE",), "filename_prefix": ("STRING", {"default": "ComfyUI"}),
                             "fps": ("FLOAT", {"default": 6.0, "min": 0.01, "max": 1000.0, "step": 0.01}),
                             "compress_level": ("INT", {"default": 4, "min": 0, "max": 9})},
                "hidden": {"prompt": "PROMPT", "extra_pnginfo": "EXTRA_PNGINFO"}}
    RETURN_TYPES = ()
    FUNCTION = "save_images"
    OUTPUT_NODE = True
    CATEGORY = "image/animation"

    def save_images(self, images, fps, compress_level, filename_prefix="ComfyUI", prompt=None, extra_pnginfo=None):
        from PIL.PngImagePlugin import PngInfo
        self.output_dir = folder_paths.get_output_directory()
        folder, filename, counter, subfolder, _ = folder_paths.get_save_image_path(
            filename_prefix + self.prefix_append, self.output_dir, images[0].shape[1], images[0].shape[0])
        frames = _pil_frames(images)
        meta = None
        if not NH.args_disable_metadata():
            meta = PngInfo()
            if prompt is not None:
                meta.add(b"comf", b"prompt\0" + json.dumps(prompt).encode("latin-1", "strict"), after_idat=True)
            if extra_pnginfo is not None:
                for k in extra_pnginfo:
                    meta.add(b"comf", k.encode("latin-1", "strict") + b"\0" +
                             json.dumps(extra_pnginfo[k]).encode("latin-1", "strict"), after_idat=True)
        file = f"{filename}_{counter:05}_.png"
        frames[0].save(os.path.join(folder, file), pnginfo=meta, compress_level=compress_level, save_all=True,
                       duration=int(1000.0 / fps), append_images=frames[1:])
        return {"ui": {"images": [{"filename": file, "subfolder": subfolder, "type": self.type}],
                       "animated": (True,)}}


# ---------------------------------------------------------------- post-processing
def _dev():
    return dm.get_torch_device()


class ImageBlend:
    MODES = ["normal", "multiply", "screen", "overlay", "soft_light", "difference"]

    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"image1": ("IMAGE",), "image2": ("IMAGE",),
                             "blend_factor": ("FLOAT", {"default": 0.5, "min": 0.0, "max": 1.0, "step": 0.01}),
                             "blend_mode": (s.MODES,)}}
    RETURN_TYPES = ("IMAGE",)
    FUNCTION = "blend_images"
    CATEGORY = "image/postprocessing"

    @staticmethod
    def _mode(a, b, mode):
        if mode == "normal":
            return b
        if mode == "multiply":
            return a * b
        if mode == "screen":
            return 1 - (1 - a) * (1 - b)
        if mode == "overlay":
            return torch.where(a <= 0.5, 2 * a * b, 1 - 2 * (1 - a) * (1 - b))
        if mode == "soft_light":
            g = torch.where(a <= 0.25, ((16 * a - 12) * a + 4) * a, torch.sqrt(a))
            return torch.where(b <= 0.5, a - (1 - 2 * b) * a * (1 - a), a + (2 * b - 1) * (g - a))
        if mode == "difference":
            return a - b
        raise ValueError(f"Unsupported blend mode: {mode}")

    def blend_images(self, image1, image2, blend_factor, blend_mode):
        image2 = image2.to(image1.device)
        if image1.shape != image2.shape:
            image2 = U.common_upscale(image2.movedim(-1, 1), image1.shape[2], image1.shape[1], "bicubic",
                                      "center").movedim(1, -1)
        out = image1 * (1 - blend_factor) + self._mode(image1, image2, blend_mode) * blend_factor
        return (out.clamp(0, 1),)


def gaussian_kernel(kernel_size: int, sigma: float, device=None):
    lin = torch.linspace(-1, 1, kernel_size, device=device)
    y, x = torch.meshgrid(lin, lin, indexing="ij")
    g = torch.exp(-(x * x + y * y) / (2.0 * sigma * sigma))
    return g / g.sum()


def _depthwise(image_bhwc, kernel, radius):
    c = image_bhwc.shape[-1]
    x = image_bhwc.movedim(-1, 1)
    x = F.pad(x, (radius, radius, radius, radius), mode="reflect")
    k = kernel.to(x.dtype).expand(c, 1, *kernel.shape)
    y = F.conv2d(x, k, groups=c)
    return y.movedim(1, -1)


class ImageBlur:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"image": ("IMAGE",), "blur_radius": ("INT", {"default": 1, "min": 1, "max": 31, "step": 1}),
                             "sigma": ("FLOAT", {"default": 1.0, "min": 0.1, "max": 10.0, "step": 0.1})}}
    RETURN_TYPES = ("IMAGE",)
    FUNCTION = "blur"
    CATEGORY = "image/postprocessing"

    def blur(self, image, blur_radius, sigma):
        if blur_radius == 0:
            return (image,)
        x = image.to(_dev())
        k = gaussian_kernel(2 * blur_radius + 1, sigma, device=x.device)
        return (_depthwise(x, k, blur_radius).to(dm.intermediate_device()),)


class ImageSharpen:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"image": ("IMAGE",),
                             "sharpen_radius": ("INT", {"default": 1, "min": 1, "max": 31, "step": 1}),
                             "sigma": ("FLOAT", {"default": 1.0, "min": 0.1, "max": 10.0, "step": 0.01}),
                             "alpha": ("FLOAT", {"default": 1.0, "min": 0.0, "max": 5.0, "step": 0.01})}}
    RETURN_TYPES = ("IMAGE",)
    FUNCTION = "sharpen"
    CATEGORY = "image/postprocessing"

    def sharpen(self, image, sharpen_radius, sigma, alpha):
        if sharpen_radius == 0:
            return (image,)
        ks = 2 * sharpen_radius + 1
        k = gaussian_kernel(ks, sigma, device=image.device) * -(alpha * 10)
        c = ks // 2
        k[c, c] = k[c, c] - k.sum() + 1.0          # unsharp mask: identity - scaled blur, sums to 1
        return (_depthwise(image, k, sharpen_radius).clamp(0, 1),)


class ImageQuantize:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"image": ("IMAGE",), "colors": ("INT", {"default": 256, "min": 1, "max": 256, "step": 1}),
                             "dither": (["none", "floyd-steinberg", "bayer-2", "bayer-4", "bayer-8", "bayer-16"],)}}
    RETURN_TYPES = ("IMAGE",)
    FUNCTION = "quantize"
    CATEGORY = "image/postprocessing"

    @staticmethod
    def _bayer(n):
        """Normalised n-level recursive Bayer threshold matrix (values in roughly [-0.5, 0.5))."""
        if n == 0:
            return np.zeros((1, 1), np.float32)
        q = 4 ** n
        m = q * ImageQuantize._bayer(n - 1)
        return np.block([[m - 1.5, m + 0.5], [m + 1.5, m - 0.5]]) / q

    def quantize(self, image, colors, dither):
        from PIL import Image
        out = torch.zeros_like(image)
        for b in range(image.shape[0]):
            im = Image.fromarray((image[b].clamp(0, 1) * 255).to(torch.uint8).numpy(), mode="RGB")
            pal = im.quantize(colors=colors)
            if dither == "none":
                q = im.quantize(palette=pal, dither=Image.Dither.NONE)
            elif dither == "floyd-steinberg":
                q = im.quantize(palette=pal, dither=Image.Dither.FLOYDSTEINBERG)
            else:
                order = int(dither.split("-")[-1])
                spread = 2 * 256 / (len(pal.getpalette()) // 3)
                mat = spread * self._bayer(int(math.log2(order))) + 0.5
                arr = np.asarray(im).astype(np.float32)
                tiled = np.tile(mat, (math.ceil(arr.shape[0] / order), math.ceil(arr.shape[1] / order)))
                arr = np.clip(arr + tiled[:arr.shape[0], :arr.shape[1], None], 0, 255).astype(np.uint8)
                q = Image.fromarray(arr).quantize(palette=pal, dither=Image.Dither.NONE)
            out[b] = torch.from_numpy(np.asarray(q.convert("RGB")).astype(np.float32) / 255.0)
        return (out,)


class ImageScaleToTotalPixels:
    upscale_methods = ["nearest-exact", "bilinear", "area", "bicubic", "lanczos"]

    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"image": ("IMAGE",), "upscale_method": (s.upscale_methods,),
                             "megapixels": ("FLOAT", {"default": 1.0, "min": 0.01, "max": 16.0, "step": 0.01})}}
    RETURN_TYPES = ("IMAGE",)
    FUNCTION = "upscale"
    CATEGORY = "image/upscaling"

    def upscale(self, image, upscale_method, megapixels):
        s = image.movedim(-1, 1)
        scale = math.sqrt(int(megapixels * 1024 * 1024) / (s.shape[3] * s.shape[2]))
        w, h = round(s.shape[3] * scale), round(s.shape[2] * scale)
        return (U.common_upscale(s, w, h, upscale_method, "disabled").movedim(1, -1),)


# ---------------------------------------------------------------- compositing
class PorterDuffMode(enum.Enum):
    ADD = 0
    CLEAR = 1
    DARKEN = 2
    DST = 3
    DST_ATOP = 4
    DST_IN = 5
    DST_OUT = 6
    DST_OVER = 7
    LIGHTEN = 8
    MULTIPLY = 9
    OVERLAY = 10
    SCREEN = 11
    SRC = 12
    SRC_ATOP = 13
    SRC_IN = 14
    SRC_OUT = 15
    SRC_OVER = 16
    XOR = 17


def porter_duff_composite(s, sa, d, da, mode: PorterDuffMode):
    """Premultiplied Porter-Duff operators (+ the separable darken/lighten/multiply/overlay/screen)."""
    union = sa + da - sa * da
    M = PorterDuffMode
    table = {
        M.ADD: lambda: ((s + d).clamp(0, 1), (sa + da).clamp(0, 1)),
        M.CLEAR: lambda: (torch.zeros_like(d), torch.zeros_like(da)),
        M.DARKEN: lambda: ((1 - da) * s + (1 - sa) * d + torch.minimum(s, d), union),
        M.DST: lambda: (d, da),
        M.DST_ATOP: lambda: (sa * d + (1 - da) * s, sa),
        M.DST_IN: lambda: (d * sa, sa * da),
        M.DST_OUT: lambda: ((1 - sa) * d, (1 - sa) * da),
        M.DST_OVER: lambda: (d + (1 - da) * s, da + (1 - da) * sa),
        M.LIGHTEN: lambda: ((1 - da) * s + (1 - sa) * d + torch.maximum(s, d), union),
        M.MULTIPLY: lambda: (s * d, sa * da),
        M.OVERLAY: lambda: (torch.where(2 * d < da, 2 * s * d, sa * da - 2 * (da - s) * (sa - d)), union),
        M.SCREEN: lambda: (s + d - s * d, union),
        M.SRC: lambda: (s, sa),
        M.SRC_ATOP: lambda: (da * s + (1 - sa) * d, da),
        M.SRC_IN: lambda: (s * da, sa * da),
        M.SRC_OUT: lambda: ((1 - da) * s, (1 - da) * sa),
        M.SRC_OVER: lambda: (s + (1 - sa) * d, sa + (1 - sa) * da),
        M.XOR: lambda: ((1 - da) * s + (1 - sa) * d, (1 - da) * sa + (1 - sa) * da),
    }
    return table[mode]()


def _fit(x_hwc, H, W):
    if x_hwc.shape[:2] == (H, W):
        return x_hwc
    return U.common_upscale(x_hwc[None].movedim(-1, 1), W, H, "bicubic", "center").movedim(1, -1)[0]


class PorterDuffImageComposite:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"source": ("IMAGE",), "source_alpha": ("MASK",), "destination": ("IMAGE",),
                             "destination_alpha": ("MASK",),
                             "mode": ([m.name for m in PorterDuffMode], {"default": PorterDuffMode.DST.name})}}
    RETURN_TYPES = ("IMAGE", "MASK")
    FUNCTION = "composite"
    CATEGORY = "mask/compositing"

    def composite(self, source, source_alpha, destination, destination_alpha, mode):
        n = min(len(source), len(source_alpha), len(destination), len(destination_alpha))
        imgs, alphas = [], []
        for i in range(n):
            d = destination[i]
            H, W = d.shape[:2]
            assert source[i].shape[2] == d.shape[2], "inputs need the same number of channels"
            da = _fit(destination_alpha[i][..., None], H, W)
            s = _fit(source[i], H, W)
            sa = _fit(source_alpha[i][..., None], H, W)
            oi, oa = porter_duff_composite(s, sa, d, da, PorterDuffMode[mode])
            imgs.append(oi)
            alphas.append(oa[..., 0])
        return (torch.stack(imgs), torch.stack(alphas))


class SplitImageWithAlpha:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"image": ("IMAGE",)}}
    CATEGORY = "mask/compositing"
    RETURN_TYPES = ("IMAGE", "MASK")
    FUNCTION = "split_image_with_alpha"

    def split_image_with_alpha(self, image):
        rgb = image[..., :3]
        a = image[..., 3] if image.shape[-1] > 3 else torch.ones_like(image[..., 0])
        return (rgb, 1.0 - a)


class JoinImageWithAlpha:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"image": ("IMAGE",), "alpha": ("MASK",)}}
    CATEGORY = "mask/compositing"
    RETURN_TYPES = ("IMAGE",)
    FUNCTION = "join_image_with_alpha"

    def join_image_with_alpha(self, image, alpha):
        n = min(len(image), len(alpha))
        a = F.interpolate(alpha.reshape(-1, 1, alpha.shape[-2], alpha.shape[-1]).float(),
                          size=image.shape[1:3], mode="bilinear")[:, 0]
        return (torch.cat([image[:n, ..., :3], (1.0 - a[:n])[..., None]], dim=-1),)


# ---------------------------------------------------------------- morphology / edges
def _dilate(x, k):
    p = k // 2
    return F.max_pool2d(F.pad(x, (p, k - 1 - p, p, k - 1 - p), mode="replicate"), k, stride=1)


def _erode(x, k):
    return -_dilate(-x, k)


class Morphology:
    OPS = ["erode", "dilate", "open", "close", "gradient", "bottom_hat", "top_hat"]

    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"image": ("IMAGE",), "operation": (s.OPS,),
                             "kernel_size": ("INT", {"default": 3, "min": 3, "max": 999, "step": 1})}}
    RETURN_TYPES = ("IMAGE",)
    FUNCTION = "process"
    CATEGORY = "image/postprocessing"

    def process(self, image, operation, kernel_size):
        x = image.to(_dev()).movedim(-1, 1).float()
        k = kernel_size
        if operation == "erode":
            y = _erode(x, k)
        elif operation == "dilate":
            y = _dilate(x, k)
        elif operation == "open":
            y = _dilate(_erode(x, k), k)
        elif operation == "close":
            y = _erode(_dilate(x, k), k)
        elif operation == "gradient":
            y = _dilate(x, k) - _erode(x, k)
        elif operation == "top_hat":
            y = x - _dilate(_erode(x, k), k)
        elif operation == "bottom_hat":
            y = _erode(_dilate(x, k), k) - x
        else:
            raise ValueError(f"Invalid operation {operation} for morphology")
        return (y.movedim(1, -1).to(dm.intermediate_device()),)


def canny_edges(img_bchw, low, high):
    """Canny on [B,C,H,W] in 0..1 -> (magnitude, edges) each [B,1,H,W]."""
    if img_bchw.shape[1] == 3:
        gray = (0.299 * img_bchw[:, 0] + 0.587 * img_bchw[:, 1] + 0.114 * img_bchw[:, 2])[:, None]
    else:
        gray = img_bchw[:, :1]
    ax = torch.arange(5, dtype=gray.dtype, device=gray.device) - 2
    g1 = torch.exp(-ax ** 2 / 2.0)
    g1 = g1 / g1.sum()
    blur = F.conv2d(F.pad(gray, (2, 2, 2, 2), mode="reflect"), (g1[:, None] * g1[None, :])[None, None])
    sx = torch.tensor([[-1., 0., 1.], [-2., 0., 2.], [-1., 0., 1.]], dtype=gray.dtype, device=gray.device)
    p = F.pad(blur, (1, 1, 1, 1), mode="replicate")
    gx = F.conv2d(p, sx[None, None])
    gy = F.conv2d(p, sx.t()[None, None])
    mag = torch.sqrt(gx * gx + gy * gy + 1e-6)
    ang = torch.rad2deg(torch.atan2(gy, gx)) % 180.0
    # quantised direction -> neighbour offsets (0, 45, 90, 135 degrees)
    q = (((ang + 22.5) // 45) % 4).long()
    mp = F.pad(mag, (1, 1, 1, 1))
    H, W = mag.shape[-2:]

    def shift(dy, dx):
        return mp[..., 1 + dy:1 + dy + H, 1 + dx:1 + dx + W]
    offs = [((0, 1), (0, -1)), ((1, 1), (-1, -1)), ((1, 0), (-1, 0)), ((1, -1), (-1, 1))]
    n1 = torch.zeros_like(mag)
    n2 = torch.zeros_like(mag)
    for i, (a, b) in enumerate(offs):
        sel = q == i
        n1 = torch.where(sel, shift(*a), n1)
        n2 = torch.where(sel, shift(*b), n2)
    nms = torch.where((mag >= n1) & (mag >= n2), mag, torch.zeros_like(mag))
    strong = nms > high
    weak = (nms > low) & ~strong
    edges = strong.float()
    for _ in range(max(H, W)):            # hysteresis: grow strong edges through weak pixels
        grown = (F.max_pool2d(edges, 3, stride=1, padding=1) > 0) & weak
        new = torch.maximum(edges, grown.float())
        if torch.equal(new, edges):
            break
        edges = new
    return mag, edges


class Canny:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"image": ("IMAGE",),
                             "low_threshold": ("FLOAT", {"default": 0.4, "min": 0.01, "max": 0.99, "step": 0.01}),
                             "high_threshold": ("FLOAT", {"default": 0.8, "min": 0.01, "max": 0.99, "step": 0.01})}}
    RETURN_TYPES = ("IMAGE",)
    FUNCTION = "detect_edge"
    CATEGORY = "image/preprocessors"

    def detect_edge(self, image, low_threshold, high_threshold):
        _, edges = canny_edges(image.to(_dev()).movedim(-1, 1).float(), low_threshold, high_threshold)
        return (edges.to(dm.intermediate_device()).repeat(1, 3, 1, 1).movedim(1, -1),)


NODE_CLASS_MAPPINGS = {
    "ImageCrop": ImageCrop, "RepeatImageBatch": RepeatImageBatch, "ImageFromBatch": ImageFromBatch,
    "SaveAnimatedWEBP": SaveAnimatedWEBP, "SaveAnimatedPNG": SaveAnimatedPNG, "ImageBlend": ImageBlend,
    "ImageBlur": ImageBlur, "ImageQuantize": ImageQuantize, "ImageSharpen": ImageSharpen,
    "ImageScaleToTotalPixels": ImageScaleToTotalPixels, "PorterDuffImageComposite": PorterDuffImageComposite,
    "SplitImageWithAlpha": SplitImageWithAlpha, "JoinImageWithAlpha": JoinImageWithAlpha,
    "Morphology": Morphology, "Canny": Canny,
}
NODE_DISPLAY_NAME_MAPPINGS = {"PorterDuffImageComposite": "Porter-Duff Image Composite",
                              "SplitImageWithAlpha": "Split Image with Alpha",
                              "JoinImageWithAlpha": "Join Image with Alpha", "Morphology": "ImageMorphology"}
