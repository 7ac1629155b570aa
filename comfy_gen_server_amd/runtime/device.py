"""Device, dtype and HBM-residency manager.

Replaces ``comfy/model_management.py`` (C27). MI355X design: 288 GB of HBM3E per GPU means the
whole working set of a node (SDXL UNet + refiner + ControlNets + VAE + CLIP-L/G + Cascade C/B/A)
fits at once, so the manager is a *residency set*, not an LRU swapper:

  * ``load_models_gpu`` moves a ModelPatcher's module to the device once (patched weights merged
    on the device) and keeps it resident across prompts; eviction only happens when a new load
    would exceed the HBM budget (``CGS_HBM_BUDGET_GB``, default: 90 % of device memory), and then
    least-recently-used unpinned models go first (no lowvram partial streaming path is needed on
    the hot path; the CPU fallback keeps everything on the host).
  * dtype policy: bf16 for UNet / VAE / text encoders on gfx950 (the MFMA-native dtype);
    fp32 on the CPU.
  * the interrupt flag (C10) lives here as in the reference.
"""
from __future__ import annotations

import gc
import logging
import os
import threading
import time

import torch

_state_lock = threading.RLock()


class VRAMState:
    DISABLED = 0
    NO_VRAM = 1
    LOW_VRAM = 2
    NORMAL_VRAM = 3
    HIGH_VRAM = 4
    SHARED = 5


class CPUState:
    GPU = 0
    CPU = 1


_force_cpu = os.environ.get("CGS_FORCE_CPU", "0") == "1"
cpu_state = CPUState.CPU if (_force_cpu or not torch.cuda.is_available()) else CPUState.GPU
vram_state = VRAMState.HIGH_VRAM if cpu_state == CPUState.GPU else VRAMState.DISABLED
_device_index = int(os.environ.get("LOCAL_RANK", os.environ.get("CGS_DEVICE", "0")))


def set_cpu_mode(flag: bool = True):
    global cpu_state, vram_state
    cpu_state = CPUState.CPU if flag else CPUState.GPU
    vram_state = VRAMState.DISABLED if flag else VRAMState.HIGH_VRAM


def set_device_index(i: int):
    global _device_index
    _device_index = i


def is_device_cuda():
    return cpu_state == CPUState.GPU


def get_torch_device() -> torch.device:
    if cpu_state == CPUState.CPU:
        return torch.device("cpu")
    return torch.device("cuda", _device_index % max(1, torch.cuda.device_count()))


def get_torch_device_name(device=None):
    device = device or get_torch_device()
    if device.type == "cuda":
        try:
            return f"{device} {torch.cuda.get_device_name(device)} : native"
        except Exception:
            return str(device)
    return str(device)


def get_total_memory(dev=None, torch_total_too=False):
    dev = dev or get_torch_device()
    if dev.type == "cpu":
        import psutil
        t = psutil.virtual_memory().total
        return (t, t) if torch_total_too else t
    free, total = torch.cuda.mem_get_info(dev)
    if torch_total_too:
        return total, torch.cuda.memory_reserved(dev)
    return total


def get_free_memory(dev=None, torch_free_too=False):
    dev = dev or get_torch_device()
    if dev.type == "cpu":
        import psutil
        f = psutil.virtual_memory().available
        return (f, f) if torch_free_too else f
    free, _ = torch.cuda.mem_get_info(dev)
    st = torch.cuda.memory_stats(dev)
    reserved = st.get("reserved_bytes.all.current", 0)
    active = st.get("active_bytes.all.current", 0)
    f_torch = reserved - active
    # the weight arena's slab is one "active" allocation to torch; its unused part is free for weights
    total_free = free + f_torch + _arena_free(dev)
    return (total_free, f_torch) if torch_free_too else total_free


def _arena_free(dev) -> int:
    from . import arena
    a = arena._ARENAS.get(dev.index if dev.index is not None else torch.cuda.current_device())
    if a is None:
        return 0
    s = a.stats()
    return int(s["capacity"] - s["used"])


def _hbm_bytes(m) -> int:
    """HBM a resident model holds outside the weight arena (arena blocks are inside the slab, which
    _evict_for charges once, whole)."""
    from . import arena
    if not arena._ARENAS:
        return m.size()
    owners = list(arena._ARENAS.values())
    n = 0
    for t in list(m.model.model.parameters()) + list(m.model.model.buffers()):
        if not any(a.owns(t) for a in owners):
            n += t.numel() * t.element_size()
    return n


def hbm_budget(dev=None) -> int:
    dev = dev or get_torch_device()
    env = os.environ.get("CGS_HBM_BUDGET_GB")
    if env:
        return int(float(env) * (1 << 30))
    return int(get_total_memory(dev) * 0.9)


# ---------------------------------------------------------------- dtypes
_args = {"force_fp32": False, "force_fp16": False, "bf16_unet": False, "fp16_unet": False,
         "fp8_e4m3fn_unet": False, "fp8_e5m2_unet": False, "fp32_vae": False, "fp16_vae": False,
         "bf16_vae": False, "cpu_vae": False, "fp32_text_enc": False, "fp16_text_enc": False,
         "disable_smart_memory": False}


def configure(**kw):
    _args.update({k: v for k, v in kw.items() if k in _args})


def _fp16_on_device(what: str):
    """fp16 requested for a device model. The hand-written MI355X kernels are bf16 (same MFMA rate,
    wider exponent); fp16 would route every op through the vendor libraries. So fp16 requests run the
    bf16 HIP path unless ``CGS_ALLOW_LIB=1`` asks for real fp16 through the libraries."""
    import os
    if os.environ.get("CGS_ALLOW_LIB", "0") == "1":
        return torch.float16
    key = "_fp16_warned_" + what
    if not _args.get(key):
        _args[key] = True
        logging.warning("%s: fp16 requested; MI355X kernels run bf16 (set CGS_ALLOW_LIB=1 for fp16 through "
                        "the vendor libraries)", what)
    return torch.bfloat16


def unet_dtype(device=None, model_params=0, supported_dtypes=(torch.bfloat16, torch.float16, torch.float32)):
    device = device or get_torch_device()
    if _args["force_fp32"] or device.type == "cpu":
        return torch.float32
    if _args["fp8_e4m3fn_unet"]:
        return torch.float8_e4m3fn
    if _args["fp8_e5m2_unet"]:
        return torch.float8_e5m2
    if _args["fp16_unet"] and torch.float16 in supported_dtypes:
        return _fp16_on_device("unet") if device.type == "cuda" and torch.bfloat16 in supported_dtypes \
            else torch.float16
    if torch.bfloat16 in supported_dtypes:
        return torch.bfloat16
    return torch.float16 if torch.float16 in supported_dtypes else torch.float32


def unet_manual_cast(weight_dtype, inference_device, supported_dtypes=()):
    if weight_dtype in (torch.float32, torch.bfloat16, torch.float16):
        return None
    return torch.bfloat16 if inference_device.type != "cpu" else torch.float32


def text_encoder_dtype(device=None):
    device = device or get_torch_device()
    if _args["fp32_text_enc"] or device.type == "cpu":
        return torch.float32
    if _args["fp16_text_enc"]:
        return _fp16_on_device("text encoder") if device.type == "cuda" else torch.float16
    return torch.bfloat16


def vae_dtype(device=None):
    device = device or get_torch_device()
    if _args["fp32_vae"] or device.type == "cpu":
        return torch.float32
    if _args["fp16_vae"]:
        return _fp16_on_device("vae") if device.type == "cuda" else torch.float16
    return torch.bfloat16


def unet_offload_device():
    return get_torch_device() if vram_state == VRAMState.HIGH_VRAM else torch.device("cpu")


def unet_inital_load_device(parameters, dtype):
    return get_torch_device()


def text_encoder_device():
    return get_torch_device()


def text_encoder_offload_device():
    return unet_offload_device()


def vae_device():
    return torch.device("cpu") if _args["cpu_vae"] else get_torch_device()


def vae_offload_device():
    return unet_offload_device()


def intermediate_device():
    """Where node outputs (conds, latents, images) live between nodes. With 288 GB of HBM we keep
    them on the device (``--gpu-only`` semantics of the reference) to avoid per-node D2H copies."""
    return get_torch_device()


def dtype_size(dtype):
    return torch.tensor([], dtype=dtype).element_size()


def module_size(module):
    return sum(p.numel() * p.element_size() for p in module.parameters()) + \
        sum(b.numel() * b.element_size() for b in module.buffers())


def cast_to_device(tensor, device, dtype, copy=False):
    return tensor.to(device=device, dtype=dtype, copy=copy, non_blocking=False)


def soft_empty_cache(force=False):
    if cpu_state == CPUState.GPU and force:
        torch.cuda.empty_cache()


def synchronize():
    if cpu_state == CPUState.GPU:
        torch.cuda.synchronize()


# ---------------------------------------------------------------- residency set
class LoadedModel:
    def __init__(self, patcher):
        self.model = patcher
        self.device = patcher.load_device
        self.last_used = time.monotonic()
        self.pinned = False

    def size(self):
        return self.model.model_size()

    def __eq__(self, other):
        return isinstance(other, LoadedModel) and self.model is other.model


current_loaded_models: list[LoadedModel] = []


def _evict_for(need: int, device, keep):
    if device.type != "cuda":
        return
    from . import arena
    budget = hbm_budget(device)
    key = device.index if device.index is not None else torch.cuda.current_device()
    slab = arena._ARENAS[key].slab.numel() if key in arena._ARENAS else 0
    # the slab counts once, whole; arena-resident weights live inside it (not charged twice)
    used = slab + sum(_hbm_bytes(m) for m in current_loaded_models if m.device == device)
    if used + need <= budget:
        return
    cands = sorted([m for m in current_loaded_models if m.device == device and m not in keep and not m.pinned],
                   key=lambda m: m.last_used)
    for m in cands:
        logging.info("evicting %s to make room", m.model.model.__class__.__name__)
        freed = _hbm_bytes(m)
        m.model.unpatch_model(m.model.offload_device)
        current_loaded_models.remove(m)
        used -= freed
        if used + need <= budget:
            break
    soft_empty_cache(True)


def load_models_gpu(models, memory_required=0, force_patch_weights=False):
    """Make every ModelPatcher in ``models`` resident on its load device with patches applied."""
    with _state_lock:
        keep = []
        for p in models:
            lm = LoadedModel(p)
            if lm in current_loaded_models:
                idx = current_loaded_models.index(lm)
                cur = current_loaded_models[idx]
                cur.last_used = time.monotonic()
                if cur.model.patches_uuid_applied != p.patches_uuid:
                    cur.model.patch_model(cur.device, force=True)
                keep.append(cur)
                continue
            # another clone of the same base module may be resident with different patches
            for other in list(current_loaded_models):
                if other.model.model is p.model and other.model is not p:
                    other.model.unpatch_model(other.device)
                    current_loaded_models.remove(other)
            need = 0 if p.is_resident_on(lm.device) else p.model_size()
            if need and lm.device.type == "cuda":    # what the arena's free space will take is already paid
                need = max(0, need - _arena_free(lm.device))
            _evict_for(need + memory_required, lm.device, keep)
            p.patch_model(lm.device)
            current_loaded_models.insert(0, lm)
            keep.append(lm)


def load_model_gpu(model):
    return load_models_gpu([model])


def loaded_models(only_currently_used=False):
    return [m.model for m in current_loaded_models]


def cleanup_models(keep_clone_weights_loaded=False):
    with _state_lock:
        for m in list(current_loaded_models):
            import sys
            if sys.getrefcount(m.model) <= 2 and not (keep_clone_weights_loaded and m.model.model is not None):
                current_loaded_models.remove(m)


def unload_all_models():
    with _state_lock:
        for m in list(current_loaded_models):
            m.model.unpatch_model(m.model.offload_device)
        current_loaded_models.clear()
    gc.collect()
    soft_empty_cache(True)


def free_memory(memory_required, device, keep_loaded=()):
    with _state_lock:
        _evict_for(memory_required, device, [LoadedModel(k) for k in keep_loaded])


# ---------------------------------------------------------------- interrupt (C10)
class InterruptProcessingException(Exception):
    pass


interrupt_processing_mutex = threading.RLock()
interrupt_processing = False


def interrupt_current_processing(value=True):
    global interrupt_processing
    with interrupt_processing_mutex:
        interrupt_processing = value


def processing_interrupted():
    with interrupt_processing_mutex:
        return interrupt_processing


def throw_exception_if_processing_interrupted():
    global interrupt_processing
    from ..sched import spmd
    if spmd.active() is not None:      # SPMD prompts stop only where every rank agrees (spmd.SPMD.execute)
        return
    with interrupt_processing_mutex:
        if interrupt_processing:
            interrupt_processing = False
            raise InterruptProcessingException()
