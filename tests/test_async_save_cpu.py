"""Deferred PNG saves (utils/imageio.py): a thread that opted in gets its encodes back as futures, the
files appear whole (``.part`` + rename) once they finish, ``pending`` names the in-flight ones for
``/view``; threads that did not opt in keep synchronous saves."""
import os
import threading

import numpy as np
import torch
from PIL import Image

from comfy_gen_server_amd.utils import imageio


def test_deferred_saves_complete_and_are_collected(tmp_path):
    imgs = torch.rand(3, 64, 48, 3)
    out = {}

    def worker():
        imageio.defer_saves(True)
        names = imageio.save_png_batch(imgs, str(tmp_path), "deferred", 1, {"prompt": "{}"})
        futs = imageio.take_pending()
        out["names"], out["futs"] = names, futs
        out["errs"] = imageio.wait_futures(futs)
        out["again"] = imageio.take_pending()
    t = threading.Thread(target=worker)
    t.start()
    t.join()
    assert len(out["futs"]) == 3 and out["errs"] == [] and out["again"] == []
    for i, n in enumerate(out["names"]):
        p = tmp_path / n
        assert imageio.pending(str(p)) is None
        arr = np.asarray(Image.open(p))
        ref = (imgs[i].clamp(0, 1) * 255 + 0.5).to(torch.uint8).numpy()
        assert arr.shape == (64, 48, 3) and np.array_equal(arr, ref)
    assert not [f for f in os.listdir(tmp_path) if f.endswith(".part")]


def test_saves_stay_synchronous_without_opt_in(tmp_path):
    names = imageio.save_png_batch(torch.rand(2, 16, 16, 3), str(tmp_path), "sync", 1)
    assert imageio.take_pending() == []
    assert all(os.path.getsize(tmp_path / n) > 0 for n in names)
