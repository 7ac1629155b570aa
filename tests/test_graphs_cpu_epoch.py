"""Per-model weight epochs: patching one model retires only the graph plans captured over it."""
import torch.nn as nn

from comfy_gen_server_amd.models import layers


def test_stamp_epoch_is_per_model_tree():
    a = nn.Sequential(nn.Linear(2, 2), nn.Sequential(nn.Linear(2, 2)))
    b = nn.Sequential(nn.Linear(2, 2))
    assert layers.module_epoch(a) == 0 and layers.module_epoch(b) == 0
    ea = layers.stamp_epoch(a)
    assert layers.module_epoch(a) == ea and layers.module_epoch(a[1][0]) == ea
    assert layers.module_epoch(b) == 0                  # b's plans survive a's patch
    eb = layers.stamp_epoch(b)
    assert eb > ea and layers.module_epoch(a) == ea and layers.module_epoch(b) == eb
    layers.invalidate_all(a)
    assert layers.module_epoch(a) > eb and layers.module_epoch(b) == eb
