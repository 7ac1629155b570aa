"""HBM weight arena (C27): C++ best-fit offset allocator + slab placement of module weights."""
import random

import pytest
import torch

from comfy_gen_server_amd import _native
from comfy_gen_server_amd.runtime import arena as A


def _allocators():
    out = [A._PyArena]
    rt = _native.load_runtime()
    if rt is not None and hasattr(rt, "Arena"):
        out.append(rt.Arena)
    return out


@pytest.mark.parametrize("cls", _allocators(), ids=lambda c: c.__module__ + "." + c.__name__)
def test_allocator_best_fit_and_coalescing(cls):
    a = cls(1 << 20, 256)
    x, y, z = a.alloc(1000), a.alloc(5000), a.alloc(300)
    assert (x, y, z) == (0, 1024, 6144)
    assert a.free(y) and not a.free(y)                       # double free refused
    w = a.alloc(4000)                                        # best fit: y's hole, not the tail
    assert w == 1024
    assert a.free(w) and a.free(x) and a.free(z)
    st = a.stats()
    assert st["used"] == 0 and st["free_blocks"] == 1 and st["largest_free"] == 1 << 20
    assert a.alloc(2 << 20) == -1                            # does not fit


@pytest.mark.parametrize("cls", _allocators(), ids=lambda c: c.__module__ + "." + c.__name__)
def test_allocator_random_stress(cls):
    rng = random.Random(0)
    cap = 64 << 20
    a = cls(cap, 256)
    live = {}
    for _ in range(3000):
        if live and rng.random() < 0.45:
            off = rng.choice(list(live))
            assert a.free(off)
            del live[off]
        else:
            n = rng.randint(1, 1 << 20)
            off = a.alloc(n)
            if off < 0:
                continue
            assert off % 256 == 0
            need = (n + 255) // 256 * 256
            for o, s in live.items():                        # no overlap with any live block
                assert off + need <= o or o + s <= off
            live[off] = need
    assert a.stats()["used"] == sum(live.values())
    for off in list(live):
        assert a.free(off)
    assert a.stats()["free_blocks"] == 1 and a.stats()["used"] == 0


def _tiny():
    from comfy_gen_server_amd.models.layers import init_random_
    from comfy_gen_server_amd.models.unet import UNetModel
    from comfy_gen_server_amd.tools.synth import TINY_UNET
    m = UNetModel(**dict(TINY_UNET, num_heads=2, num_head_channels=-1))
    init_random_(m, seed=1)
    return m


def test_weight_arena_place_forward_evict():
    m = _tiny()
    x = torch.randn(1, 4, 16, 16)
    t = torch.tensor([10.0])
    ctx = torch.randn(1, 5, 64)
    with torch.no_grad():
        ref = m(x, t, context=ctx)
    nbytes = sum(p.numel() * p.element_size() for p in m.parameters())
    wa = A.WeightArena(nbytes * 2, "cpu")
    placed = wa.place_module(m)
    assert placed > 0 and all(wa.owns(p) for p in m.parameters())
    with torch.no_grad():
        out = m(x, t, context=ctx)
    assert torch.equal(out, ref)
    st = wa.stats()
    assert st["live_blocks"] == len(wa.blocks[id(m)]) and st["used"] >= nbytes
    assert wa.evict_module(m, "cpu") > 0
    assert wa.stats()["used"] == 0 and not any(wa.owns(p) for p in m.parameters())
    with torch.no_grad():
        assert torch.equal(m(x, t, context=ctx), ref)


def test_weight_arena_inference_mode_module():
    """A model built under inference_mode (bench / synth pipelines) placed from normal mode: its
    buffers stay usable by view ops in both modes (a plain ``.data`` swap onto a normal slab view
    broke every later ``sigmas[-1]``: "Inference tensors do not track version counter")."""
    from comfy_gen_server_amd.sampling.model_sampling import ModelSamplingDiscrete
    with torch.inference_mode():
        m = _tiny()
        ms = ModelSamplingDiscrete()
    holder = torch.nn.Module()
    holder.unet, holder.ms = m, ms
    nbytes = sum(t.numel() * t.element_size() for t in list(holder.parameters()) + list(holder.buffers()))
    wa = A.WeightArena(nbytes * 2, "cpu")
    assert wa.place_module(holder) > 0
    assert wa.owns(ms.sigmas) and ms.sigmas.is_inference()
    want = float(ms.sigmas[-1])          # view op outside inference mode
    with torch.inference_mode():
        assert float(ms.sigma_max) == want
        out = m(torch.randn(1, 4, 16, 16), torch.tensor([10.0]), context=torch.randn(1, 5, 64))
    assert torch.isfinite(out).all()


def test_weight_arena_full_rolls_back():
    m = _tiny()
    wa = A.WeightArena(64 * 1024, "cpu")
    with pytest.raises(A.ArenaFull):
        wa.place_module(m)
    assert wa.stats()["used"] == 0
    assert not any(wa.owns(p) for p in m.parameters())


@pytest.mark.gpu
def test_patcher_places_weights_in_arena(cuda, monkeypatch):
    """With CGS_WEIGHT_ARENA_GB, loading a model places its weights in the slab; a LoRA-style weight
    patch is written into the same blocks; unloading evicts them."""
    from comfy_gen_server_amd.runtime import device as dm, patcher as P
    monkeypatch.setenv("CGS_WEIGHT_ARENA_GB", "1")
    A._ARENAS.clear()
    m = _tiny().to(torch.bfloat16)
    p = P.ModelPatcher(m, load_device=cuda, offload_device=torch.device("cpu"))
    dm.load_models_gpu([p])
    wa = A.get(cuda)
    assert wa is not None and all(wa.owns(t) for t in m.parameters())
    key = next(k for k, _ in m.named_parameters() if k.endswith("weight") and _.dim() == 2)
    w = dict(m.named_parameters())[key]
    before = w.detach().clone()
    p.add_patches({key: (torch.ones_like(before, device="cpu"),)}, 0.5)
    dm.load_models_gpu([p])
    w = dict(m.named_parameters())[key]
    assert wa.owns(w) and torch.allclose(w.float(), before.float() + 0.5, atol=1e-2)
    dm.unload_all_models()
    assert wa.stats()["used"] == 0
    A._ARENAS.clear()
