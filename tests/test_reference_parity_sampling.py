"""Sampler / scheduler / cond-batching parity against the reference's own sources (imported
read-only in a subprocess with a CPU argv, same recipe as test_reference_parity.py).

* all 6 schedulers: ``comfy/samplers.py:660-677`` ``calculate_sigmas`` on the default SD1.x
  discrete schedule, compared exactly;
* every k-diffusion sampler (``comfy/k_diffusion/sampling.py``) + UniPC bh1/bh2
  (``comfy/extra_samplers/uni_pc.py``) on a deterministic nonlinear toy denoiser: ODE samplers
  exactly; stochastic samplers with a zero noise source (their deterministic part exactly — the
  noise stream itself is different by design: counter-based per image, sampling/rng.py);
* ``calc_cond_batch`` with areas, masks, strengths and timestep ranges (``comfy/samplers.py:131-228``).
Skipped where the reference tree is not mounted."""
import os
import subprocess
import sys

import pytest

REF = "/root/reference"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "comfy")), reason="reference tree not mounted")

_HEAD = r'''
import sys, types
sys.path.insert(0, "{REF}"); sys.argv = ["x", "--cpu"]
import comfy.options; comfy.options.enable_args_parsing()
for _m in ("torchsde", "blake3"):
    sys.modules.setdefault(_m, types.ModuleType(_m))
import torch
sys.path.insert(0, "{ROOT}")
from comfy_gen_server_amd.runtime import device as dm
dm.set_cpu_mode(True)
torch.manual_seed(0)

def close(a, b, tol=1e-5, what=""):
    err = (a - b).abs().max().item()
    scale = b.abs().max().item() + 1e-6
    assert err <= tol * max(1.0, scale), (what, err, scale)
    return err
'''

_SCHED = r'''
import comfy.samplers as RS, comfy.model_sampling as RMS
from comfy_gen_server_amd.sampling import schedulers as OS, model_sampling as OMS
class RM(RMS.ModelSamplingDiscrete, RMS.EPS): pass
class OM(OMS.ModelSamplingDiscrete, OMS.EPS): pass
rms, oms = RM(None), OM(None)
close(oms.sigmas, rms.sigmas, 1e-6, "sigma table")
for name in RS.SCHEDULER_NAMES:
    for steps in (1, 2, 7, 20, 33):
        close(OS.calculate_sigmas(oms, name, steps), RS.calculate_sigmas(rms, name, steps), 1e-5, (name, steps))
for s in (14.6, 3.0, 0.5, 0.03):
    t = torch.tensor([s])
    close(oms.timestep(t).float(), rms.timestep(t).float(), 1e-6, ("timestep", s))
    close(oms.sigma(oms.timestep(t)), rms.sigma(rms.timestep(t)), 1e-6, ("sigma", s))
for p in (0.0, 0.3, 0.999, 1.0):
    assert abs(oms.percent_to_sigma(p) - rms.percent_to_sigma(p)) < 1e-6 * max(1, rms.percent_to_sigma(p)), p
print("schedulers ok")
'''

_SAMPLERS = r'''
import comfy.k_diffusion.sampling as R
import comfy.extra_samplers.uni_pc as RU
import comfy.samplers as RS, comfy.model_sampling as RMS
from comfy_gen_server_amd.sampling import k_samplers as O, uni_pc as OU

class RM(RMS.ModelSamplingDiscrete, RMS.EPS): pass

class _NS:
    pass

class Toy:   # deterministic, nonlinear, sigma-dependent "denoiser" (+ the model_sampling path ddpm reads)
    def __init__(self):
        self.inner_model = _NS()
        self.inner_model.inner_model = _NS()
        self.inner_model.inner_model.model_sampling = RM(None)
    def __call__(self, x, sigma, **kw):
        s = sigma.reshape(-1, 1, 1, 1).to(x.dtype)
        return torch.tanh(0.7 * x) / (1 + s * s) + 0.05 * torch.sin(3 * x) * s / (1 + s)

model = Toy()
x0 = torch.randn(2, 4, 8, 8) * 14.6
sig = RS.calculate_sigmas(RM(None), "karras", 10)
zero = lambda a, b: torch.zeros_like(x0)
def run(mod, name, **kw):
    fn = getattr(mod, "sample_" + name)
    return fn(model, x0.clone(), sig.clone(), extra_args={}, disable=True, **kw)
ode = ["euler", "heun", "dpm_2", "lms", "dpmpp_2m", "heunpp2"]
for name in ode:
    print(name, close(run(O, name), run(R, name), 1e-4, name))
noisy = ["euler_ancestral", "dpm_2_ancestral", "dpmpp_2s_ancestral", "dpmpp_sde", "dpmpp_2m_sde", "dpmpp_3m_sde",
         "ddpm", "lcm"]
for name in noisy:
    print(name, close(run(O, name, noise_sampler=zero), run(R, name, noise_sampler=zero), 1e-4, name))
print("dpmpp_2m_sde heun", close(run(O, "dpmpp_2m_sde", noise_sampler=zero, solver_type="heun"),
                                 run(R, "dpmpp_2m_sde", noise_sampler=zero, solver_type="heun"), 1e-4))
print("euler_a eta .5", close(run(O, "euler_ancestral", noise_sampler=zero, eta=0.5),
                              run(R, "euler_ancestral", noise_sampler=zero, eta=0.5), 1e-4))
smin, smax = float(sig[-2]), float(sig[0])
a = O.sample_dpm_fast(model, x0.clone(), smin, smax, 8, extra_args={}, disable=True)
b = R.sample_dpm_fast(model, x0.clone(), smin, smax, 8, extra_args={}, disable=True)
print("dpm_fast", close(a, b, 1e-4))
a = O.sample_dpm_adaptive(model, x0.clone(), smin, smax, extra_args={}, disable=True)
b = R.sample_dpm_adaptive(model, x0.clone(), smin, smax, extra_args={}, disable=True)
print("dpm_adaptive", close(a, b, 1e-4))
# UniPC: the reference converts D(x) -> eps -> x0 in the tensor dtype (predict_eps_sigma +
# data_prediction), this engine uses D(x) directly; compared in fp64 so the algorithm (orders,
# B(h), rho solves, corrector) is pinned tightly, and in fp32 at rounding level
for v in ("bh1", "bh2"):
    a = OU.sample_unipc(model, x0.double(), sig.double(), extra_args={}, disable=True, variant=v)
    b = RU.sample_unipc(model, x0.double(), sig.double(), extra_args={}, disable=True, variant=v)
    print("uni_pc fp64", v, close(a, b, 1e-9))
    a = OU.sample_unipc(model, x0.clone(), sig.clone(), extra_args={}, disable=True, variant=v)
    b = RU.sample_unipc(model, x0.clone(), sig.clone(), extra_args={}, disable=True, variant=v)
    print("uni_pc fp32", v, close(a, b, 2e-3))
print("samplers ok")
'''

_COND = r'''
import comfy.samplers as RS, comfy.conds as RC
from comfy_gen_server_amd.sampling import samplers as OS, conds as OC

class Toy:
    """apply_model(x, t, c_crossattn) = x * mean(context) + t (per batch row)."""
    def apply_model(self, input_x, timestep_, **c):
        ctx = c["c_crossattn"]
        return input_x * ctx.mean(dim=(1, 2)).reshape(-1, 1, 1, 1) + timestep_.reshape(-1, 1, 1, 1) * 0.01
    def memory_required(self, shape):
        return 0

def conds_for(lib):
    C = lib.CONDCrossAttn
    g = torch.Generator().manual_seed(1)
    ctx = [torch.randn(1, 7, 8, generator=g) for _ in range(5)]
    mask = (torch.rand(1, 16, 16, generator=g) > 0.5).float()
    pos = [
        {"model_conds": {"c_crossattn": C(ctx[0])}},
        {"model_conds": {"c_crossattn": C(ctx[1])}, "area": (8, 8, 4, 4), "strength": 0.7},
        {"model_conds": {"c_crossattn": C(ctx[2])}, "mask": mask, "mask_strength": 0.5},
        {"model_conds": {"c_crossattn": C(ctx[3])}, "timestep_start": 999.0, "timestep_end": 5.0},
    ]
    neg = [{"model_conds": {"c_crossattn": C(ctx[4])}, "area": (16, 8, 0, 8)},
           {"model_conds": {"c_crossattn": C(ctx[0])}}]
    return pos, neg

x = torch.randn(2, 4, 16, 16)
for sigma in (10.0, 2.0, 1.0):
    t = torch.full((2,), sigma)
    rp, rn = conds_for(RC)
    op, on = conds_for(OC)
    ref = RS.calc_cond_batch(Toy(), [rp, rn], x, t, {})
    tok = OS.current_sigma.set(sigma)
    try:
        ours = OS.calc_cond_batch(Toy(), [op, on], x, t, {})
    finally:
        OS.current_sigma.reset(tok)
    for a, b in zip(ours, ref):
        print("cond", sigma, close(a, b, 1e-5))
    # plain cond+uncond fast path (one entry each)
    ref = RS.calc_cond_batch(Toy(), [rp[:1], rn[1:]], x, t, {})
    ours = OS.calc_cond_batch(Toy(), [op[:1], on[1:]], x, t, {})
    for a, b in zip(ours, ref):
        close(a, b, 1e-5, "fast path")
print("cond ok")
'''


def _run(body, tmp_path):
    script = tmp_path / "parity.py"
    script.write_text(_HEAD.replace("{REF}", REF).replace("{ROOT}", ROOT) + body)
    r = subprocess.run([sys.executable, str(script)], capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, CGS_FORCE_CPU="1", OMP_NUM_THREADS="4"))
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-4000:])
    return r.stdout


def test_schedulers_match_reference(tmp_path):
    assert "schedulers ok" in _run(_SCHED, tmp_path)


def test_samplers_match_reference(tmp_path):
    assert "samplers ok" in _run(_SAMPLERS, tmp_path)


def test_cond_batching_matches_reference(tmp_path):
    assert "cond ok" in _run(_COND, tmp_path)


_TOK = r'''
import os, tempfile
import comfy.sd1_clip as R
from comfy_gen_server_amd.models import text_encoders as O
from safetensors.torch import save_file
d = tempfile.mkdtemp()
g = torch.Generator().manual_seed(3)
save_file({"emb_params": torch.randn(3, 768, generator=g)}, os.path.join(d, "myemb.safetensors"))
prompts = [
    "a photo of a cat",
    "a (photo:1.3) of a ((cat)), [dog] (nested (emphasis:0.5) here:1.2)",
    "escaped \\(not weighted\\) text and (weighted \\) inside:1.1)",
    "newline\nseparated   spaces,and,commas!! unicode: café üñîçødé",
    " ".join(["word%d" % i for i in range(120)]),
    "supercalifragilisticexpialidocious antidisestablishmentarianism " * 12,
    "embedding:myemb, a painting (embedding:myemb:1.4) and embedding:missing_one",
    "",
    "(unclosed paren and: colon",
]
for kw in (dict(), dict(pad_with_end=False), dict(pad_to_max_length=False), dict(has_start_token=True, min_length=80)):
    rt = R.SDTokenizer(embedding_directory=d, **kw)
    ot = O.SDTokenizer(embedding_directory=d, **kw)
    for p in prompts:
        for wid in (False, True):
            a = ot.tokenize_with_weights(p, return_word_ids=wid)
            b = rt.tokenize_with_weights(p, return_word_ids=wid)
            assert len(a) == len(b), (p, kw, len(a), len(b))
            for ca, cb in zip(a, b):
                assert len(ca) == len(cb), (p, kw, len(ca), len(cb))
                for ta, tb in zip(ca, cb):
                    assert len(ta) == len(tb)
                    if isinstance(tb[0], torch.Tensor):
                        assert isinstance(ta[0], torch.Tensor) and torch.allclose(ta[0].float(), tb[0].float()), p
                    else:
                        assert ta[0] == tb[0], (p, kw, ta, tb)
                    assert abs(ta[1] - tb[1]) < 1e-6, (p, kw, ta, tb)
                    if wid:
                        assert ta[2] == tb[2], (p, kw, ta, tb)
print("tokenizer ok")
'''


def test_tokenizer_emphasis_ti_chunking_match_reference(tmp_path):
    """Prompt emphasis / escapes / 77-token chunking / long-word splitting / textual inversion /
    word ids (comfy/sd1_clip.py:201-480) against the reference SDTokenizer (transformers CLIPTokenizer
    on comfy/sd1_tokenizer) -- this engine uses its own byte-level BPE."""
    assert "tokenizer ok" in _run(_TOK, tmp_path)


_LORA = r'''
import types, copy
import comfy.lora as RL, comfy.model_patcher as RP, comfy.utils as RUt
from comfy_gen_server_amd.runtime import lora as OL, patcher as OP
from comfy_gen_server_amd.tools import synth
g = torch.Generator().manual_seed(7)
rn = lambda *s: torch.randn(*s, generator=g) * 0.1
W = {"lin": rn(64, 48), "conv": rn(32, 16, 3, 3)}
lora = {}
to_load = {}
def add(prefix, target, entries):
    to_load[prefix] = target
    for k, v in entries.items():
        lora[prefix + "." + k] = v
# Linear targets (out 64, in 48), rank 4
add("l_lora", "lin.lora", {"lora_up.weight": rn(64, 4), "lora_down.weight": rn(4, 48), "alpha": torch.tensor(2.0)})
add("l_dora", "lin.dora", {"lora_up.weight": rn(64, 4), "lora_down.weight": rn(4, 48), "alpha": torch.tensor(4.0),
                           "dora_scale": rn(64, 1).abs() + 0.5})
add("l_diffusers", "lin.diffusers", {"lora_linear_layer.up.weight": rn(64, 4), "lora_linear_layer.down.weight": rn(4, 48)})
add("l_loha", "lin.loha", {"hada_w1_a": rn(64, 4), "hada_w1_b": rn(4, 48), "hada_w2_a": rn(64, 4), "hada_w2_b": rn(4, 48),
                           "alpha": torch.tensor(3.0)})
add("l_lokr", "lin.lokr", {"lokr_w1": rn(8, 6), "lokr_w2_a": rn(8, 2), "lokr_w2_b": rn(2, 8), "alpha": torch.tensor(1.0)})
add("l_glora", "lin.glora", {"a1.weight": rn(4, 48), "a2.weight": rn(48, 4), "b1.weight": rn(4, 48), "b2.weight": rn(64, 4),
                             "alpha": torch.tensor(2.0)})
add("l_diff", "lin.diff", {"diff": rn(64, 48)})
# Conv targets (32, 16, 3, 3): LoCon with mid, LoHa with Tucker cores, LoKr full
add("c_locon", "conv.locon", {"lora_up.weight": rn(32, 4, 1, 1), "lora_down.weight": rn(4, 16, 1, 1),
                              "lora_mid.weight": rn(4, 4, 3, 3), "alpha": torch.tensor(2.0)})
add("c_lora", "conv.lora", {"lora_up.weight": rn(32, 4, 1, 1), "lora_down.weight": rn(4, 16, 3, 3)})
add("c_loha", "conv.loha", {"hada_w1_a": rn(4, 32), "hada_w1_b": rn(4, 16), "hada_w2_a": rn(4, 32), "hada_w2_b": rn(4, 16),
                            "hada_t1": rn(4, 4, 3, 3), "hada_t2": rn(4, 4, 3, 3), "alpha": torch.tensor(2.0)})
add("c_lokr", "conv.lokr", {"lokr_w1": rn(4, 2), "lokr_w2": rn(8, 8, 3, 3)})
pr = RL.load_lora(lora, to_load)
po = OL.load_lora(lora, to_load)
assert set(pr) == set(po), (set(pr) ^ set(po))
fake = types.SimpleNamespace()
fake.calculate_weight = lambda p, w, k: RP.ModelPatcher.calculate_weight(fake, p, w, k)
for key in sorted(pr):
    base = W[key.split(".")[0]]
    assert pr[key][0] == po[key][0], key
    for strength, smodel in ((1.0, 1.0), (0.6, 0.9)):
        a = OP.calculate_weight([(strength, po[key], smodel)], base.clone(), key)
        b = fake.calculate_weight([(strength, pr[key], smodel)], base.clone(), key)
        close(a, b, 1e-5, key)
# key maps: SDXL UNet (ldm + diffusers names) and SDXL CLIP-L/G
unet_cfg = dict(synth.SDXL_UNET, num_head_channels=64)
from comfy_gen_server_amd.models.unet import UNetModel
with torch.device("meta"):
    net = UNetModel(**unet_cfg, dtype=torch.float16, device=torch.device("meta"))
keys = ["diffusion_model." + k for k in net.state_dict().keys()]
fm = types.SimpleNamespace(state_dict=lambda: {k: None for k in keys},
                           model_config=types.SimpleNamespace(unet_config=unet_cfg))
ko = OL.model_lora_keys_unet(fm, {})
kr = RL.model_lora_keys_unet(fm, {})
assert ko == kr, (len(ko), len(kr), sorted(set(ko.items()) ^ set(kr.items()))[:5])
from comfy_gen_server_amd.runtime import families
ct = families.SDXL(dict(synth.SDXL_UNET)).clip_target()
with torch.device("meta"):
    cm = ct.stack(dtype=torch.float16, device=torch.device("meta"))
ck = {k: None for k in cm.state_dict().keys()}
cf = types.SimpleNamespace(state_dict=lambda: ck)
co, cr = OL.model_lora_keys_clip(cf, {}), RL.model_lora_keys_clip(cf, {})
assert co == cr and len(co) > 100, (len(co), len(cr))
print("lora ok", len(ko), len(co))
'''


def test_lora_lycoris_patches_and_key_maps_match_reference(tmp_path):
    """LoRA / LoCon (mid) / DoRA / diffusers / LoHa (+Tucker) / LoKr / GLoRA / diff patches parsed and
    merged exactly like comfy/lora.py:14-166 + comfy/model_patcher.py:316-452; UNet (ldm + diffusers
    names) and CLIP-L/G key maps equal to comfy/lora.py:169-241 on the SDXL architecture."""
    assert "lora ok" in _run(_LORA, tmp_path)


_DETECT = r'''
import copy
import comfy.model_detection as RD, comfy.supported_models as RSM
from comfy_gen_server_amd.runtime import detection as OD
from comfy_gen_server_amd.models.unet import UNetModel
from comfy_gen_server_amd.tools import synth
TEMPORAL = dict(use_temporal_resblock=True, use_temporal_attention=True, extra_ff_mix_layer=True,
                use_spatial_context=True, merge_strategy="learned_with_images", merge_factor=0.0,
                video_kernel_size=[3, 1, 1], channel_mult=[1, 2, 4, 4], num_res_blocks=[2, 2, 2, 2],
                num_head_channels=64, num_heads=-1, num_classes="sequential",
                transformer_depth_output=[1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0])
BASES = {"SD15": synth.SD15_UNET, "SD20": synth.SD21_UNET, "SDXL": synth.SDXL_UNET,
         "SDXLRefiner": synth.SDXL_REFINER_UNET}
def full_config(F):
    names = [c.__name__ for c in F.__mro__]
    base = next((BASES[n] for n in names if n in BASES), synth.SD15_UNET)
    cfg = copy.deepcopy(base)
    cfg.update(num_heads=-1, num_head_channels=64)
    part = {k: v for k, v in F.unet_config.items()}
    cfg.update(part)
    cfg.update(F.unet_extra_config)
    if cfg.get("adm_in_channels") and cfg.get("num_classes") is None:
        cfg["num_classes"] = "sequential"
    if cfg.get("use_temporal_resblock"):
        for k, v in TEMPORAL.items():
            cfg.setdefault(k, v) if k in part else cfg.__setitem__(k, v)
    td = cfg["transformer_depth"]
    nrb = cfg.get("num_res_blocks", [2] * len(cfg["channel_mult"]))
    if isinstance(nrb, int):
        nrb = [nrb] * len(cfg["channel_mult"])
    levels = len(td) // nrb[0] if len(td) % nrb[0] == 0 else len(cfg["channel_mult"])
    if len(td) != sum(nrb):       # KOALA-style shorter lists -> one res block per level
        cfg["num_res_blocks"] = [1] * len(td)
        cfg["channel_mult"] = cfg["channel_mult"][:len(td)]
        nrb = cfg["num_res_blocks"]
    if "transformer_depth_output" not in part:
        out = []
        for lvl in range(len(cfg["channel_mult"])):
            d = td[sum(nrb[:lvl])] if sum(nrb[:lvl]) < len(td) else 0
            out += [d] * (nrb[lvl] + 1)
        cfg["transformer_depth_output"] = out
    cfg["transformer_depth_middle"] = cfg.get("transformer_depth_middle", max(td))
    if cfg.get("num_classes") == 1000:
        cfg["num_classes"] = 1000
    cfg.pop("image_size", None)
    cfg.pop("use_checkpoint", None)
    return cfg
ok, skipped = [], []
for F in RSM.models:
    if F.__name__.startswith("Stable_Cascade"):
        continue
    cfg = full_config(F)
    try:
        with torch.device("meta"):
            net = UNetModel(**cfg, dtype=torch.float16, device=torch.device("meta"))
    except Exception as e:
        skipped.append((F.__name__, repr(e)[:120]))
        continue
    sd = {"model.diffusion_model." + k: v for k, v in net.state_dict().items()}
    if F.__name__ == "Stable_Zero123":
        sd["cc_projection.weight"] = torch.empty(768, 772, device="meta")
        sd["cc_projection.bias"] = torch.empty(768, device="meta")
    r = RD.model_config_from_unet(sd, "model.diffusion_model.")
    o = OD.model_config_from_unet(sd, "model.diffusion_model.")
    rn = type(r).__name__ if r is not None else None
    on = type(o).__name__ if o is not None else None
    assert rn == on, (F.__name__, rn, on)
    if r is not None:
        for k, v in r.unet_config.items():
            if k in o.unet_config:
                ov = o.unet_config[k]
                assert ov == v or (isinstance(v, (list, tuple)) and list(ov) == list(v)), (F.__name__, k, v, ov)
    ok.append((F.__name__, rn))
print("detect ok", ok, "skipped", skipped)
assert len(ok) >= 14, (ok, skipped)
'''


def test_architecture_detection_matches_reference(tmp_path):
    """``model_config_from_unet`` on meta-tensor state dicts of every UNet family of the reference's
    registry (comfy/model_detection.py:32-183, supported_models.py:479-481): the same family class is
    picked in the same registry order and the detected unet_config agrees key by key. (Stable Cascade
    B/C use their own stage models: tests/test_cascade.py.)"""
    out = _run(_DETECT, tmp_path)
    assert "detect ok" in out, out


_CASCADE_CN = r'''
import copy
import comfy.ops
from comfy.ldm.cascade.stage_c import StageC as RC
from comfy.ldm.cascade.stage_b import StageB as RB
from comfy.ldm.cascade.stage_a import StageA as RA
from comfy.cldm.cldm import ControlNet as RCN
from comfy_gen_server_amd.models import cascade as SC
from comfy_gen_server_amd.models.cldm import ControlNet as OCN
from comfy_gen_server_amd.models.layers import init_random_
from comfy_gen_server_amd.tools.synth import TINY_UNET
ops_ = comfy.ops.disable_weight_init

def load_same(ours, ref):
    sd = ours.state_dict()
    m, u = ref.load_state_dict(sd, strict=False)
    bufs = {n for n, _ in ref.named_buffers()}
    assert not [k for k in m if k not in bufs] and not u, (m[:5], u[:5])

# Stage C (prior) with ControlNet-style residuals
cc = dict(c_in=16, c_out=16, c_r=16, c_cond=32, c_hidden=[32, 32], nhead=[2, 2], blocks=[[1, 1], [1, 1]],
          block_repeat=[[1, 1], [2, 1]], level_config=["CTA", "CTA"], c_clip_text=24, c_clip_text_pooled=24,
          c_clip_img=768, c_clip_seq=2, switch_level=[False])
oc = SC.StageC(**cc); init_random_(oc, seed=7)
rc = RC(**cc, operations=ops_); load_same(oc, rc)
g = torch.Generator().manual_seed(0)
x = torch.randn(2, 16, 6, 6, generator=g); r = torch.tensor([0.3, 0.7])
ct, ctp, ci = torch.randn(2, 7, 24, generator=g), torch.randn(2, 1, 24, generator=g), torch.randn(2, 1, 768, generator=g)
with torch.no_grad():
    print("stage_c", close(oc(x, r, ct, ctp, ci), rc(x, r, ct, ctp, ci), 2e-4))
# Stage B (decoder)
bc = dict(c_in=4, c_out=4, c_r=16, patch_size=2, c_cond=32, c_hidden=[16, 24, 32], nhead=[-1, 2, 2],
          blocks=[[1, 1, 1], [1, 1, 1]], block_repeat=[[1, 1, 1], [2, 1, 1]], level_config=["CT", "CTA", "CTA"],
          c_clip=24, c_clip_seq=2, c_effnet=16)
ob = SC.StageB(**bc); init_random_(ob, seed=8)
rb = RB(**bc, operations=ops_); load_same(ob, rb)
xb = torch.randn(2, 4, 16, 16, generator=g); eff = torch.randn(2, 16, 3, 3, generator=g)
clip = torch.randn(2, 1, 24, generator=g)
with torch.no_grad():
    print("stage_b", close(ob(xb, torch.tensor([0.5, 0.25]), eff, clip), rb(xb, torch.tensor([0.5, 0.25]), eff, clip), 2e-4))
# Stage A (VQGAN): encode (no quantize) and decode
oa = SC.StageA(levels=2, bottleneck_blocks=2, c_hidden=32, c_latent=4, codebook_size=64); init_random_(oa, seed=9)
oa.eval()
ra = RA(levels=2, bottleneck_blocks=2, c_hidden=32, c_latent=4, codebook_size=64); load_same(oa, ra); ra.eval()
img = torch.rand(1, 3, 32, 32, generator=g)
with torch.no_grad():
    ea, eb = oa.encode(img), ra.encode(img)
    ea, eb = (ea[0] if isinstance(ea, tuple) else ea), (eb[0] if isinstance(eb, tuple) else eb)
    print("stage_a enc", close(ea, eb, 2e-4))
    print("stage_a dec", close(oa.decode(eb), ra.decode(eb), 2e-4))
# cldm ControlNet (SD-style, tiny): per-block residual outputs
cfg = copy.deepcopy(TINY_UNET)
cfg.update(num_heads=2, num_head_channels=-1)
ocn = OCN(hint_channels=3, **cfg); init_random_(ocn, seed=3)
rcfg = dict(cfg); rcfg.pop("out_channels", None)
rcn = RCN(hint_channels=3, operations=ops_, **rcfg); load_same(ocn, rcn)
xh = torch.randn(2, 4, 8, 8, generator=g); hint = torch.rand(2, 3, 64, 64, generator=g)
ts = torch.tensor([500.0, 20.0]); ctx = torch.randn(2, 9, 64, generator=g)
with torch.no_grad():
    a = ocn(x=xh, hint=hint, timesteps=ts, context=ctx)
    b = rcn(x=xh, hint=hint, timesteps=ts, context=ctx)
assert len(a) == len(b), (len(a), len(b))
for i, (u, v) in enumerate(zip(a, b)):
    close(u, v, 2e-4, ("controlnet out", i))
print("cascade/controlnet ok")
'''


def test_stage_c_b_and_controlnet_match_reference_modules(tmp_path):
    """Stable Cascade Stage C / Stage B / Stage A and the cldm ControlNet, loaded with the same random weights
    into this engine's modules and the reference's (comfy/ldm/cascade/stage_{c,b,a}.py,
    comfy/cldm/cldm.py:285-311), give the same outputs (fp32, CPU)."""
    assert "cascade/controlnet ok" in _run(_CASCADE_CN, tmp_path)
