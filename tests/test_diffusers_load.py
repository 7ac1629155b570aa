"""diffusers-folder loading: a tiny random pipeline written in diffusers layout loads back to the
same UNet / VAE outputs (parity target: comfy/diffusers_load.py, comfy/diffusers_convert.py)."""
import os
import re

import torch

from comfy_gen_server_amd.runtime.convert import unet_to_diffusers


def _vae_to_diffusers(sd, n_up):
    out = {}
    for k, v in sd.items():
        nk = re.sub(r"^encoder\.down\.(\d+)\.block\.(\d+)\.", r"encoder.down_blocks.\1.resnets.\2.", k)
        nk = re.sub(r"^encoder\.down\.(\d+)\.downsample\.conv\.", r"encoder.down_blocks.\1.downsamplers.0.conv.", nk)
        nk = re.sub(r"^decoder\.up\.(\d+)\.block\.(\d+)\.",
                    lambda m: f"decoder.up_blocks.{n_up - 1 - int(m.group(1))}.resnets.{m.group(2)}.", nk)
        nk = re.sub(r"^decoder\.up\.(\d+)\.upsample\.conv\.",
                    lambda m: f"decoder.up_blocks.{n_up - 1 - int(m.group(1))}.upsamplers.0.conv.", nk)
        nk = re.sub(r"\.mid\.block_(\d+)\.", lambda m: f".mid_block.resnets.{int(m.group(1)) - 1}.", nk)
        nk = nk.replace(".nin_shortcut.", ".conv_shortcut.").replace("norm_out", "conv_norm_out")
        if ".mid.attn_1." in nk:
            head, tail = nk.split(".mid.attn_1.")
            name, rest = tail.split(".", 1)
            name = {"norm": "group_norm", "q": "to_q", "k": "to_k", "v": "to_v", "proj_out": "to_out.0"}[name]
            if rest == "weight" and v.ndim == 4:
                v = v[:, :, 0, 0]
            nk = f"{head}.mid_block.attentions.0.{name}.{rest}"
        out[nk] = v.contiguous()
    return out


def test_load_diffusers_folder(tmp_path):
    from safetensors.torch import save_file
    from comfy_gen_server_amd.runtime.diffusers import load_diffusers
    from comfy_gen_server_amd.tools.synth import build_pipeline
    p, clip, vae = build_pipeline("tiny", device=torch.device("cpu"), dtype=torch.float32, seed=0)
    cfg = p.model.model_config.unet_config
    inv = {v: k for k, v in unet_to_diffusers(cfg).items()}
    ldm = p.model.diffusion_model.state_dict()
    assert all(k in inv for k in ldm)
    os.makedirs(tmp_path / "unet")
    os.makedirs(tmp_path / "vae")
    save_file({inv[k]: v.contiguous() for k, v in ldm.items()},
              str(tmp_path / "unet" / "diffusion_pytorch_model.safetensors"))
    vsd = vae.first_stage_model.state_dict()
    n_up = len(vae.first_stage_model.decoder.up)
    dvsd = _vae_to_diffusers(vsd, n_up)
    assert not any(".up." in k or ".down." in k or "attn_1" in k for k in dvsd)
    save_file(dvsd, str(tmp_path / "vae" / "diffusion_pytorch_model.safetensors"))

    unet, clip2, vae2 = load_diffusers(str(tmp_path), output_clip=False)
    assert clip2 is None
    x = torch.randn(1, 4, 16, 16)
    t = torch.tensor([500.0])
    c = torch.randn(1, 77, cfg["context_dim"])
    kw = {"y": torch.randn(1, cfg["adm_in_channels"])} if cfg.get("adm_in_channels") else {}
    a = p.model.diffusion_model(x, t, context=c, **kw)
    b = unet.model.diffusion_model.float()(x, t, context=c, **kw)
    assert torch.allclose(a, b, atol=1e-5)

    img = torch.rand(1, 64, 64, 3)
    z1, z2 = vae.encode(img), vae2.encode(img)
    assert torch.allclose(z1.float(), z2.float(), atol=1e-3, rtol=1e-3)
    assert torch.allclose(vae.decode(z1).float(), vae2.decode(z1).float(), atol=1e-3)
