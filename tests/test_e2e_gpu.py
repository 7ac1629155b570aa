"""End-to-end prompt on the device: synthetic ldm checkpoint on disk -> CheckpointLoaderSimple (bytes
uploaded straight into HBM through the pinned double-buffered H2D path) -> CLIPTextEncode x2 ->
KSampler -> VAEDecode -> SaveImage, through validate_prompt + PromptExecutor; the image must match
the same prompt executed on the CPU to bf16 tolerance."""
import os

import numpy as np
import pytest
import torch

from comfy_gen_server_amd.runtime import device as dm

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu_env(tmp_path_factory):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    prev = dm.cpu_state
    dm.set_cpu_mode(False)
    base = tmp_path_factory.mktemp("cgs_gpu")
    from comfy_gen_server_amd.utils import folder_paths
    folder_paths.set_base_path(str(base))
    for d in ("models/checkpoints", "output", "input", "temp"):
        os.makedirs(base / d, exist_ok=True)
    from comfy_gen_server_amd.tools.synth import write_checkpoint
    write_checkpoint("tiny", str(base / "models/checkpoints/tiny.safetensors"), dtype=torch.float32)
    from comfy_gen_server_amd.graph import registry
    registry.init_nodes(custom_nodes=False)
    yield base
    dm.set_cpu_mode(prev == dm.CPUState.CPU)


def _graph(seed):
    return {
        "4": {"class_type": "CheckpointLoaderSimple", "inputs": {"ckpt_name": "tiny.safetensors"}},
        "5": {"class_type": "EmptyLatentImage", "inputs": {"width": 64, "height": 64, "batch_size": 2}},
        "6": {"class_type": "CLIPTextEncode", "inputs": {"text": "a photo of a cat", "clip": ["4", 1]}},
        "7": {"class_type": "CLIPTextEncode", "inputs": {"text": "blurry", "clip": ["4", 1]}},
        "3": {"class_type": "KSampler", "inputs": {"seed": seed, "steps": 3, "cfg": 5.0, "sampler_name": "euler",
                                                  "scheduler": "normal", "denoise": 1.0, "model": ["4", 0],
                                                  "positive": ["6", 0], "negative": ["7", 0], "latent_image": ["5", 0]}},
        "8": {"class_type": "VAEDecode", "inputs": {"samples": ["3", 0], "vae": ["4", 2]}},
        "9": {"class_type": "SaveImage", "inputs": {"filename_prefix": "gpu", "images": ["8", 0]}},
    }


def _run(p, pid):
    from comfy_gen_server_amd.graph.executor import PromptExecutor
    from comfy_gen_server_amd.graph.validation import validate_prompt
    ok, err, outputs, node_errors = validate_prompt(p)
    assert ok, (err, node_errors)
    ex = PromptExecutor()
    ex.execute(p, pid, {}, outputs)
    assert ex.success, ex.status_messages
    return ex.outputs_ui["9"]["images"]


def test_prompt_end_to_end_on_device(gpu_env):
    from PIL import Image
    from comfy_gen_server_amd.runtime.checkpoint import load_state_dict
    sd = load_state_dict(str(gpu_env / "models/checkpoints/tiny.safetensors"), device=dm.get_torch_device())
    assert next(iter(sd.values())).device.type == "cuda"            # direct HBM load path
    imgs = _run(_graph(7), "gpu-1")
    assert len(imgs) == 2
    a = np.asarray(Image.open(os.path.join(gpu_env, "output", imgs[0]["filename"]))).astype(np.float32)
    assert a.shape == (64, 64, 3) and a.std() > 0
    dm.set_cpu_mode(True)                                            # same prompt on the CPU
    try:
        imgs_c = _run(_graph(7), "cpu-1")
    finally:
        dm.set_cpu_mode(False)
    b = np.asarray(Image.open(os.path.join(gpu_env, "output", imgs_c[0]["filename"]))).astype(np.float32)
    assert np.abs(a - b).mean() < 6.0, np.abs(a - b).mean()          # bf16 device vs fp32 host, 8-bit images
