"""PhotoMaker ID-fusion parity against the reference module itself
(comfy_extras/nodes_photomaker.py FuseModule / MLP, imported read-only in a subprocess, CPU fp32):
same random weights, same prompt embeddings / ID embeddings / class-token mask. The CLIP-ViT-L
vision tower in front of it is the shared CLIP vision model (C44)."""
import os
import subprocess
import sys

import pytest

REF = "/root/reference"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "comfy_extras")),
                                reason="reference tree not mounted")

_SCRIPT = r'''
import sys, types
sys.path.insert(0, REF); sys.argv = ["x", "--cpu"]
import comfy.options; comfy.options.enable_args_parsing()
sys.modules.setdefault("torchsde", types.ModuleType("torchsde"))
import torch, comfy.ops
from comfy_extras.nodes_photomaker import FuseModule as RefFuse
sys.path.insert(0, ROOT)
from comfy_gen_server_amd.models.layers import init_random_
from comfy_gen_server_amd.nodes.extras_conditioning import FuseModule
torch.manual_seed(0)
ours = FuseModule(64)
init_random_(ours, seed=1)
ref = RefFuse(64, comfy.ops.manual_cast)
m, u = ref.load_state_dict(ours.state_dict(), strict=False)
assert not m and not u, (m, u)
prompt = torch.randn(1, 9, 64)
ids = torch.randn(1, 2, 1, 64)
mask = torch.zeros(1, 9, dtype=torch.bool)
mask[0, 3] = mask[0, 4] = True
with torch.no_grad():
    a = ours(prompt.clone(), ids, mask)
    b = ref(prompt.clone(), ids, mask)
err = (a - b).abs().max().item()
assert err < 1e-4 * max(1.0, b.abs().max().item()), err
assert torch.equal(a[0, :3], prompt[0, :3]) and (a[0, 3:5] - prompt[0, 3:5]).abs().max() > 1e-3
print("photomaker fuse", err)
'''


def test_photomaker_fuse_matches_reference():
    code = f"REF = {REF!r}\nROOT = {ROOT!r}\n" + _SCRIPT
    env = dict(os.environ, CGS_FORCE_CPU="1", PYTHONDONTWRITEBYTECODE="1")
    r = subprocess.run([sys.executable, "-c", code], cwd="/tmp", env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "photomaker fuse" in r.stdout
