"""End-to-end plumbing slice on the CPU (SURVEY §7.2 step 1 / BASELINE config 1 in miniature):
synthetic ldm checkpoint on disk -> CheckpointLoaderSimple (detection) -> CLIPTextEncode x2 ->
EmptyLatentImage -> KSampler -> VAEDecode -> SaveImage, through validate_prompt + PromptExecutor."""
import json
import os

import pytest
import torch

from comfy_gen_server_amd.runtime import device as dm


@pytest.fixture(scope="module")
def env(tmp_path_factory):
    dm.set_cpu_mode(True)
    base = tmp_path_factory.mktemp("cgs")
    from comfy_gen_server_amd.utils import folder_paths
    folder_paths.set_base_path(str(base))
    for d in ("models/checkpoints", "output", "input", "temp", "models/loras"):
        os.makedirs(base / d, exist_ok=True)
    from comfy_gen_server_amd.tools.synth import write_checkpoint
    write_checkpoint("tiny", str(base / "models/checkpoints/tiny.safetensors"), dtype=torch.float32)
    from comfy_gen_server_amd.graph import registry
    registry.init_nodes(custom_nodes=False)
    return base


def graph(sampler="euler_ancestral", scheduler="normal", steps=2, seed=3):
    return {
        "4": {"class_type": "CheckpointLoaderSimple", "inputs": {"ckpt_name": "tiny.safetensors"}},
        "5": {"class_type": "EmptyLatentImage", "inputs": {"width": 64, "height": 64, "batch_size": 2}},
        "6": {"class_type": "CLIPTextEncode", "inputs": {"text": "a (photo:1.2) of a cat", "clip": ["4", 1]}},
        "7": {"class_type": "CLIPTextEncode", "inputs": {"text": "blurry", "clip": ["4", 1]}},
        "3": {"class_type": "KSampler", "inputs": {"seed": seed, "steps": steps, "cfg": 7.0, "sampler_name": sampler,
                                                  "scheduler": scheduler, "denoise": 1.0, "model": ["4", 0],
                                                  "positive": ["6", 0], "negative": ["7", 0], "latent_image": ["5", 0]}},
        "8": {"class_type": "VAEDecode", "inputs": {"samples": ["3", 0], "vae": ["4", 2]}},
        "9": {"class_type": "SaveImage", "inputs": {"filename_prefix": "e2e", "images": ["8", 0]}},
    }


def test_detect_tiny_checkpoint(env):
    from comfy_gen_server_amd.runtime.checkpoint import load_state_dict
    from comfy_gen_server_amd.runtime.detection import model_config_from_unet
    sd = load_state_dict(str(env / "models/checkpoints/tiny.safetensors"))
    mc = model_config_from_unet(sd, "model.diffusion_model.")
    assert type(mc).__name__ == "TinySD"


def test_prompt_end_to_end(env):
    from comfy_gen_server_amd.graph.validation import validate_prompt
    from comfy_gen_server_amd.graph.executor import PromptExecutor
    p = graph()
    ok, err, outputs, node_errors = validate_prompt(p)
    assert ok, (err, node_errors)
    ex = PromptExecutor()
    ex.execute(p, "pid-1", {}, outputs)
    assert ex.success, ex.status_messages
    imgs = ex.outputs_ui["9"]["images"]
    assert len(imgs) == 2
    path = os.path.join(env, "output", imgs[0]["filename"])
    assert os.path.exists(path)
    from PIL import Image
    im = Image.open(path)
    assert im.size == (64, 64)
    assert "prompt" in im.info and json.loads(im.info["prompt"])["3"]["class_type"] == "KSampler"
    # second run: everything cached except nothing changed -> SaveImage re-runs? (output node cached too)
    ex.execute(p, "pid-2", {}, outputs)
    cached = [m for m in ex.status_messages if m[0] == "execution_cached"][0][1]["nodes"]
    assert "4" in cached and "3" in cached
    # change the seed: sampler + downstream re-run, loader stays cached
    p2 = graph(seed=4)
    ok, err, outputs, _ = validate_prompt(p2)
    ex.execute(p2, "pid-3", {}, outputs)
    cached = [m for m in ex.status_messages if m[0] == "execution_cached"][0][1]["nodes"]
    assert "4" in cached and "3" not in cached


@pytest.mark.parametrize("sampler", ["euler", "heun", "dpm_2", "dpm_2_ancestral", "lms", "dpmpp_2s_ancestral",
                                     "dpmpp_sde", "dpmpp_2m", "dpmpp_2m_sde", "dpmpp_3m_sde", "ddpm", "lcm", "ddim",
                                     "uni_pc", "uni_pc_bh2", "heunpp2", "dpm_fast", "dpm_adaptive"])
def test_every_sampler_runs(env, sampler):
    from comfy_gen_server_amd.graph.validation import validate_prompt
    from comfy_gen_server_amd.graph.executor import PromptExecutor
    p = graph(sampler=sampler, steps=3)
    ok, err, outputs, _ = validate_prompt(p)
    assert ok
    ex = PromptExecutor()
    ex.execute(p, "s", {}, outputs)
    assert ex.success, [m for m in ex.status_messages if m[0] == "execution_error"]


@pytest.mark.parametrize("scheduler", ["normal", "karras", "exponential", "sgm_uniform", "simple", "ddim_uniform"])
def test_every_scheduler_runs(env, scheduler):
    from comfy_gen_server_amd.graph.validation import validate_prompt
    from comfy_gen_server_amd.graph.executor import PromptExecutor
    p = graph(scheduler=scheduler, steps=2)
    ok, err, outputs, _ = validate_prompt(p)
    ex = PromptExecutor()
    ex.execute(p, "s", {}, outputs)
    assert ex.success


def test_validation_errors(env):
    from comfy_gen_server_amd.graph.validation import validate_prompt
    p = graph()
    p["3"]["inputs"]["sampler_name"] = "nope"
    p["3"]["inputs"]["steps"] = 0
    ok, err, outputs, node_errors = validate_prompt(p)
    assert not ok
    types = {e["type"] for e in node_errors["3"]["errors"]}
    assert "value_not_in_list" in types and "value_smaller_than_min" in types
    p = graph()
    p["8"]["inputs"]["samples"] = ["4", 0]   # MODEL into LATENT
    ok, err, outputs, node_errors = validate_prompt(p)
    assert not ok and node_errors["8"]["errors"][0]["type"] == "return_type_mismatch"
    ok, err, _, _ = validate_prompt({"1": {"class_type": "EmptyLatentImage", "inputs": {}}})
    assert not ok and err["type"] == "prompt_no_outputs"
