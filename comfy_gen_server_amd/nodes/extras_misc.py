"""API / delivery nodes: websocket image output, Stability SD3 API client, save+preview with an
optional S3 upload (parity: ``custom_nodes/websocket_image_save.py``, ``nodes.py:1468-1747``;
SURVEY C19, C63).

External services are reached only when a workflow actually runs these nodes: SD3 needs
``STABILITY_API_KEY`` and network access, S3 upload needs ``boto3`` plus the ``DO_*`` credentials
(both absent on the benchmark boxes -- the nodes fail with a clear error instead of hanging).
"""
from __future__ import annotations

import json
import os
import random
import time
from typing import BinaryIO
from urllib.parse import urlparse

import torch

from ..utils import folder_paths
from ..utils.image_format import bytes_to_tensor, convert_image_format, tensor_to_bytes
from ..utils.progress import ProgressBar
from . import helpers as NH


class SaveImageWebsocket:
    """Sends each image as a binary PNG preview frame on the prompt's websocket (no file)."""
    RETURN_TYPES = ()
    FUNCTION = "save_images"
    OUTPUT_NODE = True
    CATEGORY = "api/image"

    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"images": ("IMAGE",)}}

    def save_images(self, images):
        from PIL import Image
        import numpy as np
        pbar = ProgressBar(images.shape[0])
        for step, image in enumerate(images):
            arr = np.clip(255.0 * image.float().cpu().numpy(), 0, 255).astype(np.uint8)
            pbar.update_absolute(step, images.shape[0], ("PNG", Image.fromarray(arr), None))
        return {}

    @classmethod
    def IS_CHANGED(s, images):
        return time.time()


_ASPECTS = ["21:9", "16:9", "5:4", "3:2", "1:1", "2:3", "4:5", "9:16", "9:21"]


class SDAPI:
    RETURN_TYPES = ("IMAGE",)
    FUNCTION = "generate"
    CATEGORY = "sd3"

    @classmethod
    def INPUT_TYPES(s):
        return {"required": {
            "positive": ("STRING", {"default": "Worlds colliding", "multiline": True}),
            "negative": ("STRING", {"default": "best quality, high quality", "multiline": True}),
            "aspect_ratio": (_ASPECTS, {"default": "1:1"}),
            "seed": ("INT", {"default": 0, "min": 0, "max": 4294967294}),
            "output_format": (["png", "jpeg", "webp"], {"default": "png"}),
            "model": (["sd3", "sd3-turbo"],)},
            "optional": {"image": ("IMAGE",),
                         "strength": ("FLOAT", {"default": 0.7, "min": 0, "max": 1.0, "step": 0.01})}}

    @staticmethod
    def request_fields(positive, negative, aspect_ratio, seed, output_format, model, image, strength):
        """(files, data) of the multipart request (stable-image/generate/sd3)."""
        data = {"prompt": positive, "model": model, "seed": seed, "output_format": output_format}
        if model == "sd3":
            data["negative_prompt"] = negative
        if image is None:
            data.update(mode="text-to-image", aspect_ratio=aspect_ratio)
            files = {"none": ""}
        else:
            data.update(mode="image-to-image", strength=strength)
            files = {"image": ("image.png", image, "image/png")}
        return files, data

    @convert_image_format
    def generate(self, positive: str, negative: str, aspect_ratio, seed, output_format, model,
                 image: BinaryIO = None, strength=None):
        key = os.getenv("STABILITY_API_KEY")
        if not key:
            raise RuntimeError("SDAPI: STABILITY_API_KEY is not set")
        import requests
        files, data = self.request_fields(positive, negative, aspect_ratio, seed, output_format, model, image,
                                          strength)
        r = requests.post("https://api.stability.ai/v2beta/stable-image/generate/sd3",
                          headers={"authorization": key, "accept": "image/*"}, files=files, data=data, timeout=120)
        if r.status_code != 200:
            raise RuntimeError(f"SDAPI: HTTP {r.status_code}: {r.text[:200]}")
        return (bytes_to_tensor(r.content),)


def _write_png_bytes(content, prefix, out_dir, kind):
    full, filename, counter, subfolder, _ = folder_paths.get_save_image_path(prefix, out_dir)
    name = f"{filename}_{counter:05}_.png"
    if isinstance(content, torch.Tensor):
        content = tensor_to_bytes(content)
    with open(os.path.join(full, name), "wb") as f:
        f.write(content)
    return {"filename": name, "subfolder": subfolder, "type": kind}


class SDAPISaveImage:
    RETURN_TYPES = ()
    FUNCTION = "save"
    OUTPUT_NODE = True
    CATEGORY = "sd3"

    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"image_content": ("IMAGE",), "filename_prefix": ("STRING", {"default": "SDAPI"})}}

    def save(self, image_content, filename_prefix="SDAPI"):
        return {"ui": {"images": [_write_png_bytes(image_content, filename_prefix,
                                                   folder_paths.get_output_directory(), "output")]}}


class SDAPIPreviewImage:
    RETURN_TYPES = ()
    FUNCTION = "preview"
    OUTPUT_NODE = True
    CATEGORY = "sd3"

    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"image_content": ("IMAGE",)}}

    @convert_image_format
    def preview(self, image_content: bytes):
        prefix = "_temp_" + "".join(random.choice("abcdefghijklmnopqrstupvxyz") for _ in range(5))
        return {"ui": {"images": [_write_png_bytes(image_content, prefix, folder_paths.get_temp_directory(),
                                                   "temp")]}}


class SaveAndPreviewImage:
    """Always writes a temp preview; additionally saves to the output folder ("local") or uploads the
    first image to an S3-compatible bucket ("s3") and reports its URL in the UI payload."""
    RETURN_TYPES = ()
    FUNCTION = "save_and_preview_images"
    OUTPUT_NODE = True
    CATEGORY = "image"

    def __init__(self):
        self.temp_prefix_append = "_temp_" + "".join(random.choice("abcdefghijklmnopqrstupvxyz") for _ in range(5))

    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"images": ("IMAGE",), "filename_prefix": ("STRING", {"default": "ComfyUI"}),
                             "save_type": (["local", "s3"], {"default": "local"}),
                             "bucket_name": ("STRING", {"default": "my-bucket"})},
                "hidden": {"prompt": "PROMPT", "extra_pnginfo": "EXTRA_PNGINFO"}}

    @staticmethod
    def _save(images, prefix, out_dir, kind, compress, prompt, extra_pnginfo):
        from ..utils.imageio import save_png_batch
        full, filename, counter, subfolder, _ = folder_paths.get_save_image_path(
            prefix, out_dir, images[0].shape[1], images[0].shape[0])
        meta = None
        if not NH.args_disable_metadata():
            meta = {}
            if prompt is not None:
                meta["prompt"] = json.dumps(prompt)
            for k, v in (extra_pnginfo or {}).items():
                meta[k] = json.dumps(v)
        names = save_png_batch(images, full, filename, counter, meta, compress)
        return [{"filename": n, "subfolder": subfolder, "type": kind} for n in names]

    def save_and_preview_images(self, images, filename_prefix="ComfyUI", save_type="local", bucket_name="my-bucket",
                                prompt=None, extra_pnginfo=None):
        results = self._save(images, filename_prefix + self.temp_prefix_append, folder_paths.get_temp_directory(),
                             "temp", 1, prompt, extra_pnginfo)
        if save_type == "local":
            self._save(images, filename_prefix, folder_paths.get_output_directory(), "output", 4, prompt,
                       extra_pnginfo)
        elif save_type == "s3":
            url = self.upload_to_s3(images[:1], results[0]["filename"], bucket_name)
            results[-1]["output"] = {"image_url": url}
        return {"ui": {"images": results}}

    @convert_image_format
    def upload_to_s3(self, image_data: bytes, filename, bucket_name):
        try:
            import boto3
        except ImportError as e:
            raise RuntimeError("SaveAndPreviewImage: save_type 's3' needs boto3") from e
        session = boto3.Session(aws_access_key_id=os.getenv("DO_ACCESS_KEY_ID"),
                                aws_secret_access_key=os.getenv("DO_SECRET_ACCESS_KEY"),
                                region_name=os.getenv("REGION_NAME"))
        client = session.client("s3", endpoint_url=os.getenv("DO_ENDPOINT_URL"))
        bucket = os.getenv("BUCKET_NAME") or bucket_name
        key = f"comfy-test/{filename}"
        client.put_object(Bucket=bucket, Key=key, Body=image_data, ACL="public-read")
        host = urlparse(client.meta.endpoint_url).hostname
        return f"https://{bucket}.{host}/{key}"


NODE_CLASS_MAPPINGS = {
    "SaveImageWebsocket": SaveImageWebsocket, "SDAPI": SDAPI, "SDAPISaveImage": SDAPISaveImage,
    "SDAPIPreviewImage": SDAPIPreviewImage, "SaveAndPreviewImage": SaveAndPreviewImage,
}
