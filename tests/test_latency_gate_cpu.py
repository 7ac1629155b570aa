"""Latency mode only row-shards networks whose every layer is band-aware (Stable Cascade's
depthwise convs / GRN / attention would treat band edges as image edges and return wrong images):
``LatencyParallel._spatial_ok`` accepts the openaimodel UNet, refuses Cascade and video UNets."""
import torch

from comfy_gen_server_amd.parallel.latency import LatencyParallel


class _Owner:
    def __init__(self, net):
        self.diffusion_model = net

    def apply_model(self, x, t, **c):
        return x


def _lp(Q=2):
    lp = object.__new__(LatencyParallel)
    lp.spatial, lp.Q = object(), Q
    return lp


def test_spatial_gate_unet_only():
    from comfy_gen_server_amd.models import cascade as SC
    from comfy_gen_server_amd.tools.synth import build_pipeline
    from test_cascade import _tiny_c
    patcher, _, _ = build_pipeline("tiny", device=torch.device("cpu"), dtype=torch.float32, seed=0,
                                   with_clip=False, with_vae=False)
    x = torch.zeros(2, 4, 32, 32)
    lp = _lp()
    assert lp._spatial_ok(x, {}, patcher.model.apply_model)
    assert not lp._spatial_ok(x, {}, _Owner(SC.StageC(**_tiny_c())).apply_model)
    assert not lp._spatial_ok(x, {}, None)                    # unknown callable: replicated, never sharded
    net = patcher.model.diffusion_model
    net.row_shardable = False                                 # video UNets (temporal layers) set this
    assert not lp._spatial_ok(x, {}, patcher.model.apply_model)
    net.row_shardable = True
    assert not lp._spatial_ok(x, {"transformer_options": {"patches": {"attn1_patch": [1]}}},
                              patcher.model.apply_model)
