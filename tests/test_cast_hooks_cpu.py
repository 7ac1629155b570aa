"""``comfy.ops.CastWeightBiasOp`` semantics on our layers (custom nodes set per-layer
``weight_function`` / ``bias_function`` hooks, ``comfy/ops.py:22-37``) and the reference's named
argparse groups (``comfy/cli_args.py``) through the compat layer."""
import torch
import torch.nn.functional as F

from comfy_gen_server_amd import compat_names
from comfy_gen_server_amd.models import layers


def test_linear_and_conv_apply_weight_hooks():
    torch.manual_seed(0)
    lin = layers.Linear(8, 5)
    conv = layers.Conv2d(3, 4, 3, padding=1)
    for m in (lin, conv):
        torch.nn.init.normal_(m.weight)
        torch.nn.init.normal_(m.bias)
        assert isinstance(m, layers.CastWeightBiasOp) and m.weight_function is None
    x, xi = torch.randn(2, 8), torch.randn(1, 3, 6, 6)
    wf, bf = (lambda w: w * 0.5 + 0.1), (lambda b: b - 1.0)
    lin.weight_function, lin.bias_function = wf, bf
    conv.weight_function, conv.bias_function = wf, bf
    torch.testing.assert_close(lin(x), F.linear(x, wf(lin.weight), bf(lin.bias)), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(conv(xi), F.conv2d(xi, wf(conv.weight), bf(conv.bias), padding=1),
                               rtol=1e-5, atol=1e-5)
    ops_names = compat_names.extra_names("comfy.ops")
    w, b = ops_names["cast_bias_weight"](lin, x.double())
    assert w.dtype == torch.float64 and torch.allclose(w, wf(lin.weight.double()))


def test_cli_group_names_are_the_real_groups():
    names = compat_names.extra_names("comfy.cli_args")
    flags = {a.option_strings[0] for a in names["fp_group"]._group_actions}
    assert flags == {"--force-fp32", "--force-fp16"}
    assert "--lowvram" in {a.option_strings[0] for a in names["vram_group"]._group_actions}
