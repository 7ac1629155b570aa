"""Custom-node import surface: reference-style custom nodes import ``comfy.*``,
``folder_paths``, ``nodes``, ``node_helpers``, ``latent_preview``, ``server`` — these resolve to this
engine's modules through ``compat.install()``. The reference's own bundled node
(``/root/reference/custom_nodes/websocket_image_save.py``) is loaded UNMODIFIED from a temp
``custom_nodes/`` dir and run in a prompt."""
import os
import shutil

import pytest
import torch

from comfy_gen_server_amd.runtime import device as dm

REF_NODE = "/root/reference/custom_nodes/websocket_image_save.py"


def test_alias_modules_resolve():
    from comfy_gen_server_amd import compat
    compat.install()
    import comfy.utils
    import comfy.model_management
    import comfy.samplers
    import comfy.sample
    import comfy.sd
    import comfy.model_patcher
    import comfy.ops
    import comfy.k_diffusion.sampling
    import folder_paths
    import nodes
    import node_helpers
    import latent_preview
    import server
    from comfy_extras.nodes_upscale_model import ImageUpscaleWithModel  # noqa: F401
    from comfy_gen_server_amd.runtime import device, patcher
    from comfy_gen_server_amd.api import server as api_server
    assert comfy.model_management is device
    assert comfy.model_management.get_torch_device is device.get_torch_device
    assert comfy.model_patcher.ModelPatcher is patcher.ModelPatcher
    assert "euler_ancestral" in comfy.samplers.KSampler.SAMPLERS
    assert callable(comfy.sample.prepare_noise) and callable(comfy.sd.load_checkpoint_guess_config)
    assert callable(comfy.utils.load_torch_file) and callable(comfy.utils.common_upscale)
    assert comfy.utils.ProgressBar(3).total == 3
    assert comfy.ops.disable_weight_init.Linear is not None
    assert callable(comfy.k_diffusion.sampling.sample_euler)
    assert callable(folder_paths.get_filename_list) and callable(node_helpers.conditioning_set_values)
    assert callable(latent_preview.get_previewer)
    assert server.PromptServer is api_server.PromptServer
    assert "KSampler" in nodes.NODE_CLASS_MAPPINGS or hasattr(nodes, "common_ksampler")
    assert nodes.MAX_RESOLUTION >= 8192


@pytest.mark.skipif(not os.path.exists(REF_NODE), reason="reference checkout not present")
def test_reference_websocket_node_loads_and_runs(tmp_path):
    dm.set_cpu_mode(True)
    cn = tmp_path / "custom_nodes"
    cn.mkdir()
    shutil.copy(REF_NODE, cn / "websocket_image_save.py")
    from comfy_gen_server_amd.graph import registry
    from comfy_gen_server_amd.graph.validation import validate_prompt
    from comfy_gen_server_amd.graph.executor import PromptExecutor
    from comfy_gen_server_amd.utils import progress
    registry.init_nodes(custom_nodes=False)
    times = registry.load_custom_nodes([str(cn)])
    assert times and all(ok for _, _, ok in times), times
    assert "SaveImageWebsocket" in registry.NODE_CLASS_MAPPINGS
    frames = []
    old = progress.PROGRESS_BAR_HOOK
    progress.set_progress_bar_global_hook(lambda v, t, preview: frames.append((v, t, preview)))
    try:
        p = {"1": {"class_type": "EmptyImage", "inputs": {"width": 32, "height": 24, "batch_size": 2, "color": 255}},
             "2": {"class_type": "SaveImageWebsocket", "inputs": {"images": ["1", 0]}}}
        ok, err, outputs, node_errors = validate_prompt(p)
        assert ok, (err, node_errors)
        ex = PromptExecutor()
        ex.execute(p, "ws-1", {}, outputs)
        assert ex.success, ex.status_messages
    finally:
        progress.set_progress_bar_global_hook(old)
    assert [f[0] for f in frames] == [0, 1] and all(f[1] == 2 for f in frames)
    fmt, img, _ = frames[0][2]
    assert fmt == "PNG" and img.size == (32, 24)
