"""fp32-I/O kernels (csrc/kernels/f32.hip, ops/f32.py) against float64 PyTorch references, and the
``--fp32-vae`` / ``--force-fp32`` paths end to end with no vendor-library call (``ops.stats``)."""
import math

import pytest
import torch
import torch.nn.functional as F

from comfy_gen_server_amd import _native, ops

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _native_loaded(cuda):
    assert _native.load_kernels() is not None, _native.kernels_error()
    assert _native.has_kernel("cgs_gemm_f32")
    ops.reset_stats()
    yield


def _err(a, b):
    """max |a - b| relative to max |b| (fp32 kernel vs float64 oracle)."""
    return ((a.double().cpu() - b.double().cpu()).abs().max() / (b.double().abs().max() + 1e-30)).item()


def _lib_calls():
    return {k: v for k, v in ops.stats().items() if k[1] == "lib"}


@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (300, 200, 132), (1, 77, 768), (4096, 1280, 320), (333, 5, 4)])
@pytest.mark.parametrize("epi", ["none", "bias", "bias_res", "gelu"])
def test_linear_f32(cuda, M, N, K, epi):
    torch.manual_seed(0)
    x = torch.randn(M, K, device=cuda)
    w = torch.randn(N, K, device=cuda) / math.sqrt(K)
    b = torch.randn(N, device=cuda) if epi != "none" else None
    r = torch.randn(M, N, device=cuda) if epi == "bias_res" else None
    y = ops.linear(x, w, b, residual=r, act="gelu" if epi == "gelu" else None)
    ref = x.double().cpu() @ w.double().cpu().t()
    if b is not None:
        ref = ref + b.double().cpu()
    if epi == "gelu":
        ref = F.gelu(ref)
    if r is not None:
        ref = ref + r.double().cpu()
    assert y.dtype == torch.float32 and ops.stats().get(("gemm", "hip"), 0) == 1 and not _lib_calls()
    assert _err(y, ref) < 2e-6


@pytest.mark.parametrize("N,Cin,H,W,Cout,k,s,p,up,c2,res", [
    (2, 8, 17, 13, 12, 3, 1, 1, False, 0, False), (1, 64, 32, 32, 64, 3, 1, 1, False, 0, True),
    (2, 16, 9, 9, 32, 3, 2, 0, False, 0, False), (1, 32, 8, 12, 16, 3, 1, 1, True, 0, False),
    (2, 32, 10, 10, 24, 3, 1, 1, False, 16, True), (1, 3, 20, 20, 16, 3, 1, 1, False, 0, False),
    (2, 4, 16, 16, 128, 3, 1, 1, False, 0, False), (1, 128, 16, 16, 3, 3, 1, 1, False, 0, False),
    (1, 64, 12, 12, 64, 1, 1, 0, False, 0, True)])
def test_conv_f32(cuda, N, Cin, H, W, Cout, k, s, p, up, c2, res):
    torch.manual_seed(1)
    x = torch.randn(N, Cin, H, W, device=cuda).contiguous(memory_format=torch.channels_last)
    x2 = torch.randn(N, c2, H, W, device=cuda) if c2 else None
    w = torch.randn(Cout, Cin + c2, k, k, device=cuda) / math.sqrt((Cin + c2) * k * k)
    b = torch.randn(Cout, device=cuda)
    xin = x if x2 is None else torch.cat([x, x2], 1)
    xr = xin.double().cpu()
    if up:
        xr = F.interpolate(xr, scale_factor=2.0, mode="nearest")
    ref = F.conv2d(xr, w.double().cpu(), b.double().cpu(), s, p)
    r = torch.randn(ref.shape, device=cuda) if res else None
    if r is not None:
        ref = ref + r.double().cpu()
    y = ops.conv2d(x, w, b, s, p, residual=r, upsample2x=up, x2=x2)
    assert ops.stats().get(("conv", "hip"), 0) == 1 and not _lib_calls()
    assert y.shape == ref.shape and _err(y, ref) < 2e-6


@pytest.mark.parametrize("N,C,H,W,G,c2,silu,pre,shift", [
    (2, 320, 32, 32, 32, 0, True, True, 0.0), (1, 128, 64, 64, 32, 0, False, False, 30.0),
    (3, 64, 5, 7, 32, 0, True, False, 0.0), (2, 640, 16, 16, 32, 640, True, True, 1.0),
    (1, 1280, 8, 8, 32, 0, False, True, 0.0), (2, 512, 33, 17, 32, 0, True, False, 5.0)])
def test_groupnorm_f32(cuda, N, C, H, W, G, c2, silu, pre, shift):
    torch.manual_seed(2)
    x = (torch.randn(N, C, H, W, device=cuda) * 2 + shift).contiguous(memory_format=torch.channels_last)
    x2 = torch.randn(N, c2, H, W, device=cuda) if c2 else None
    Ct = C + c2
    w, b = torch.randn(Ct, device=cuda), torch.randn(Ct, device=cuda)
    pa = torch.randn(N, Ct, device=cuda) if pre else None
    y = ops.group_norm(x, G, w, b, 1e-6, silu=silu, pre_add=pa, x2=x2)
    xr = (x if x2 is None else torch.cat([x, x2], 1)).double().cpu()
    if pa is not None:
        xr = xr + pa.double().cpu()[:, :, None, None]
    ref = F.group_norm(xr, G, w.double().cpu(), b.double().cpu(), 1e-6)
    if silu:
        ref = F.silu(ref)
    assert ops.stats().get(("groupnorm", "hip"), 0) == 1 and not _lib_calls()
    assert _err(y, ref) < 1e-5


@pytest.mark.parametrize("rows,C", [(1000, 320), (77, 768), (5, 1280), (4096, 64)])
def test_layernorm_f32(cuda, rows, C):
    torch.manual_seed(3)
    x = torch.randn(rows, C, device=cuda) * 3 + 7
    w, b = torch.randn(C, device=cuda), torch.randn(C, device=cuda)
    y = ops.layer_norm(x, w, b, 1e-5)
    ref = F.layer_norm(x.double().cpu(), (C,), w.double().cpu(), b.double().cpu(), 1e-5)
    assert ops.stats().get(("layernorm", "hip"), 0) == 1 and not _lib_calls()
    assert _err(y, ref) < 1e-5


def _attn_ref(q, k, v, heads, mask=None, causal=False, kp=None):
    B, Sq, HD = q.shape
    D = HD // heads
    qh = q.double().cpu().reshape(B, Sq, heads, D).transpose(1, 2)
    kh = k.double().cpu().reshape(B, -1, heads, D).transpose(1, 2)
    vh = v.double().cpu().reshape(B, -1, heads, D).transpose(1, 2)
    s = qh @ kh.transpose(-1, -2) / math.sqrt(D)
    if mask is not None:
        s = s + mask.double().cpu()
    if causal:
        s = s.masked_fill(torch.ones(Sq, s.shape[-1], dtype=torch.bool).triu(1), float("-inf"))
    if kp is not None:
        s = s.masked_fill(~kp.cpu()[:, None, None, :], float("-inf"))
    return (s.softmax(-1) @ vh).transpose(1, 2).reshape(B, Sq, HD)


@pytest.mark.parametrize("B,heads,Sq,Sk,D,kind", [(2, 10, 256, 256, 64, "plain"), (1, 1, 1024, 1024, 512, "plain"),
                                                  (2, 8, 77, 77, 64, "causal"), (2, 4, 100, 77, 40, "padding"),
                                                  (1, 2, 64, 96, 32, "mask")])
def test_attention_f32(cuda, B, heads, Sq, Sk, D, kind):
    torch.manual_seed(4)
    q = torch.randn(B, Sq, heads * D, device=cuda)
    k = torch.randn(B, Sk, heads * D, device=cuda)
    v = torch.randn(B, Sk, heads * D, device=cuda)
    mask = torch.randn(B, heads, Sq, Sk, device=cuda) if kind == "mask" else None
    kp = None
    if kind == "padding":
        kp = torch.ones(B, Sk, dtype=torch.bool, device=cuda)
        kp[0, 50:] = False
    o = ops.attention(q, k, v, heads, mask=mask, causal=kind == "causal", key_padding=kp)
    ref = _attn_ref(q, k, v, heads, mask, kind == "causal", kp)
    assert ops.stats().get(("attention", "hip"), 0) == 1 and not _lib_calls()
    assert _err(o, ref) < 1e-5


@pytest.mark.parametrize("kind", ["float3d", "bool3d", "bool2d"])
def test_attention_f32_mask_forms(cuda, kind):
    """Masks in the forms custom nodes pass through optimized_attention: a per-image [B, Sq, Sk] float bias
    (broadcast over heads, not over images), a bool keep-mask (False -> -inf, not an additive 0 / 1) and a
    2-D [Sq, Sk] keep-mask."""
    torch.manual_seed(6)
    B, heads, Sq, Sk, D = 3, 2, 48, 40, 32
    q, k, v = (torch.randn(B, S, heads * D, device=cuda) for S in (Sq, Sk, Sk))
    if kind == "float3d":
        mask = torch.randn(B, Sq, Sk, device=cuda)
        add = mask[:, None]
    else:
        keep = torch.rand((B, Sq, Sk) if kind == "bool3d" else (Sq, Sk), device=cuda) > 0.3
        keep[..., 0] = True                      # every row keeps a key
        mask = keep
        add = torch.zeros(keep.shape, device=cuda).masked_fill(~keep, float("-inf"))
        add = add[:, None] if kind == "bool3d" else add[None, None]
    o = ops.attention(q, k, v, heads, mask=mask)
    ref = _attn_ref(q, k, v, heads, add.expand(B, heads, Sq, Sk))
    assert ops.stats().get(("attention", "hip"), 0) == 1 and not _lib_calls()
    assert _err(o, ref) < 1e-5


def test_attention_f32_chunked(cuda, monkeypatch):
    """Score chunks smaller than the query length (the 1 GiB bound at VAE sizes)."""
    from comfy_gen_server_amd.ops import f32
    monkeypatch.setattr(f32, "SCORE_BUDGET", 3 * 100 * 2)
    torch.manual_seed(5)
    q, k, v = (torch.randn(2, 250, 2 * 64, device=cuda) for _ in range(3))
    o = ops.attention(q, k, v, 2)
    assert _err(o, _attn_ref(q, k, v, 2)) < 1e-5


def test_fp32_vae_decode_stays_on_hip(cuda):
    """--fp32-vae: the SDXL VAE decoder in fp32 runs every conv / GroupNorm / attention / GEMM on the
    fp32 kernels (no ``lib`` stats entry) and matches the fp32 torch reference of the same weights."""
    from comfy_gen_server_amd.ops.dispatch import torch_reference
    from comfy_gen_server_amd.runtime.sd import VAE
    from comfy_gen_server_amd.models.layers import init_random_fast_
    vae = VAE(sd=None, device=cuda, dtype=torch.float32)
    vae.first_stage_model.to(cuda)
    init_random_fast_(vae.first_stage_model, seed=9)
    torch.manual_seed(6)
    z = torch.randn(1, 4, 32, 32, device=cuda)
    m = vae.first_stage_model
    with torch.inference_mode():
        ops.reset_stats()
        y = m.decode(z)
        st = ops.stats()
        with torch_reference():
            ref = m.decode(z)
    assert y.dtype == torch.float32 and torch.isfinite(y).all()
    assert not {k: v for k, v in st.items() if k[1] == "lib"}, st
    assert st.get(("conv", "hip"), 0) > 10 and st.get(("groupnorm", "hip"), 0) > 10, st
    assert st.get(("attention", "hip"), 0) >= 1, st
    assert _err(y, ref) < 1e-4


def test_force_fp32_pipeline_stays_on_hip(cuda):
    """--force-fp32: the SD1.5 architecture (random init) entirely in fp32 -- CLIP, the UNet steps and
    the VAE -- runs with no vendor-library call and a finite image."""
    from comfy_gen_server_amd.parallel.dp import Job, generate_local
    from comfy_gen_server_amd.tools.synth import build_pipeline
    with torch.inference_mode():
        patcher, clip, vae = build_pipeline("sd15", device=cuda, dtype=torch.float32, seed=3)
        ops.reset_stats()
        img = generate_local(patcher, clip, vae, Job(batch=1, steps=2, seed=7, width=256, height=256), 0, 1)
        torch.cuda.synchronize()
    st = ops.stats()
    assert not _lib_calls(), st
    assert st.get(("gemm", "hip"), 0) > 0 and st.get(("conv", "hip"), 0) > 0 and st.get(("attention", "hip"), 0) > 0
    assert img.shape[0] == 1 and torch.isfinite(img.float()).all()
