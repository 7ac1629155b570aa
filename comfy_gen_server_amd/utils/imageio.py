"""Image I/O at the node boundary (PIL codecs; SURVEY §2.3 'keep PIL for codecs').

* ``save_png_batch`` — PNG with ``prompt`` / workflow tEXt chunks (``nodes.py:1810-1837``); the
  batch is converted to uint8 on the device in one op and encoded by a thread pool (PNG encode of
  large batches is CPU-heavy: SURVEY §7.5 item 6). In a thread that opted in (``defer_saves``: the
  worker loop; ``CGS_ASYNC_SAVE=0`` turns it off) the encodes run behind the caller: the worker loop
  starts the next prompt while they finish and reports the
  prompt complete once its files are on disk (``take_pending``); ``/view`` waits for a file still
  being written (``pending``); each file is written to ``<name>.part`` and renamed into place.
* ``load_image_frames`` — multi-frame images, EXIF transpose, alpha -> inverted MASK
  (``nodes.py:1866-1893``).
"""
from __future__ import annotations

import concurrent.futures as cf
import logging
import os
import threading

import numpy as np
import torch
from PIL import Image, ImageOps, ImageSequence
from PIL.PngImagePlugin import PngInfo

_POOL = None


def _pool():
    global _POOL
    if _POOL is None:
        _POOL = cf.ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 4))
    return _POOL


def to_uint8_cpu(images: torch.Tensor) -> np.ndarray:
    u8 = (images.detach().clamp(0, 1) * 255.0 + 0.5).to(torch.uint8)
    return u8.cpu().numpy()


def encode_png(arr: np.ndarray, metadata: dict | None = None, compress_level=4) -> bytes:
    import io
    img = Image.fromarray(arr)
    info = None
    if metadata:
        info = PngInfo()
        for k, v in metadata.items():
            info.add_text(k, v)
    bio = io.BytesIO()
    img.save(bio, format="PNG", pnginfo=info, compress_level=compress_level)
    return bio.getvalue()


def _claim(folder, filename, counter):
    """Create ``{filename}_{counter:05}_.png`` exclusively, bumping the counter past names another
    writer (another rank / thread saving with the same prefix) took meanwhile."""
    while True:
        name = f"{filename}_{counter:05}_.png"
        try:
            os.close(os.open(os.path.join(folder, name), os.O_CREAT | os.O_EXCL | os.O_WRONLY, 0o644))
            return name, counter
        except FileExistsError:
            counter += 1


def reserve_png_names(folder, filename, counter, count):
    """Claim ``count`` consecutive free ``{filename}_{counter:05}_.png`` names (empty files)."""
    os.makedirs(folder, exist_ok=True)
    names = []
    for _ in range(count):
        name, counter = _claim(folder, filename, counter)
        counter += 1
        names.append(name)
    return names


_PENDING: dict = {}          # absolute path -> future of an encode still in flight
_plock = threading.Lock()
_tl = threading.local()      # futures the calling thread started since its last take_pending()


def defer_saves(on: bool = True):
    """Opt the calling thread into deferred saves (the server's worker loop, bench --via-executor): its
    PNG encodes return at once and are collected with ``take_pending``. Other callers keep the
    synchronous behaviour (files on disk when the node returns)."""
    _tl.defer = bool(on)


def async_saves() -> bool:
    return getattr(_tl, "defer", False) and os.environ.get("CGS_ASYNC_SAVE", "1") != "0"


def write_png_files(images, paths, metadata=None, compress_level=4, wait=None):
    """Encode ``images`` (B, H, W, C float in [0, 1]) to ``paths`` on the thread pool. The device ->
    host copy happens here; the encodes are waited for unless ``CGS_ASYNC_SAVE`` is on (``wait=None``),
    in which case the caller collects them with ``take_pending``."""
    arrs = to_uint8_cpu(images)

    def work(a, p):
        img = Image.fromarray(a)
        info = None
        if metadata:
            info = PngInfo()
            for k, v in metadata.items():
                info.add_text(k, v)
        tmp = p + ".part"
        img.save(tmp, format="PNG", pnginfo=info, compress_level=compress_level)
        os.replace(tmp, p)
    jobs = [_pool().submit(work, a, p) for a, p in zip(arrs, paths)]
    if wait is None:
        wait = not async_saves()
    if wait:
        for j in jobs:
            j.result()
        return []
    aps = [os.path.abspath(p) for p in paths]
    with _plock:
        for ap, j in zip(aps, jobs):
            _PENDING[ap] = j
    # outside the lock: a future that already finished runs its callback right here, in this thread
    for ap, j in zip(aps, jobs):
        j.add_done_callback(lambda f, ap=ap: _drop_pending(ap, f))
    _tl.futs = getattr(_tl, "futs", []) + jobs
    return jobs


def _drop_pending(ap, f):
    with _plock:
        if _PENDING.get(ap) is f:
            del _PENDING[ap]


def take_pending() -> list:
    """The encode futures this thread started since the last call (a prompt's saves)."""
    futs = getattr(_tl, "futs", [])
    _tl.futs = []
    return futs


def wait_futures(futs) -> list:
    """Wait for ``futs``; returns the error strings of the ones that failed."""
    errs = []
    for f in futs:
        try:
            f.result()
        except Exception as e:   # a write error fails the prompt that saved the file
            logging.error("image save failed: %s", e)
            errs.append(f"{type(e).__name__}: {e}")
    return errs


def pending(path):
    """The in-flight encode of ``path`` (or None)."""
    with _plock:
        return _PENDING.get(os.path.abspath(path))


def flush():
    with _plock:
        futs = list(_PENDING.values())
    wait_futures(futs)


def save_png_batch(images, folder, filename, counter, metadata=None, compress_level=4):
    names = reserve_png_names(folder, filename, counter, images.shape[0])
    write_png_files(images, [os.path.join(folder, n) for n in names], metadata, compress_level)
    return names


def load_image_frames(image_path):
    img = Image.open(image_path)
    output_images, output_masks = [], []
    w = h = None
    excluded = ["MPO"]
    for i in ImageSequence.Iterator(img):
        i = ImageOps.exif_transpose(i)
        if i.mode == "I":
            i = i.point(lambda v: v * (1 / 255))
        image = i.convert("RGB")
        if len(output_images) == 0:
            w, h = image.size
        if image.size[0] != w or image.size[1] != h:
            continue
        image = torch.from_numpy(np.array(image).astype(np.float32) / 255.0)[None,]
        if "A" in i.getbands():
            mask = np.array(i.getchannel("A")).astype(np.float32) / 255.0
            mask = 1.0 - torch.from_numpy(mask)
        else:
            mask = torch.zeros((64, 64), dtype=torch.float32, device="cpu")
        output_images.append(image)
        output_masks.append(mask.unsqueeze(0))
    if len(output_images) > 1 and img.format not in excluded:
        return torch.cat(output_images, dim=0), torch.cat(output_masks, dim=0)
    return output_images[0], output_masks[0]


def load_mask_channel(image_path, channel):
    i = Image.open(image_path)
    i = ImageOps.exif_transpose(i)
    if i.getbands() != ("R", "G", "B", "A"):
        if i.mode == "I":
            i = i.point(lambda v: v * (1 / 255))
        i = i.convert("RGBA")
    c = channel[0].upper()
    if c in i.getbands():
        mask = torch.from_numpy(np.array(i.getchannel(c)).astype(np.float32) / 255.0)
        if c == "A":
            mask = 1.0 - mask
    else:
        mask = torch.zeros((64, 64), dtype=torch.float32, device="cpu")
    return mask.unsqueeze(0)
