"""Import surface for ComfyUI custom nodes (the reference's own
``custom_nodes/websocket_image_save.py:5`` does ``import comfy.utils``).

Custom nodes written against the reference import its top-level modules — ``comfy.*``,
``folder_paths``, ``nodes``, ``node_helpers``, ``latent_preview``, ``server``, ``execution``,
``comfy_extras.*``. ``install()`` puts a meta-path finder in front of the normal import system that
resolves exactly those names to this package's modules (no reference code, no copies): a name maps
either to one module of ours (``comfy.samplers`` -> ``sampling.samplers``) or to a *facade* module
that forwards attribute lookups, in order, to several of ours plus a few reference-named wrappers
(``comfy.utils.load_torch_file`` -> ``runtime.checkpoint.load_state_dict``). Attributes are looked
up on every access, so state such as ``PromptServer.instance`` or the progress-bar hook is always
the live one. The finder sits first on ``sys.meta_path`` and answers only for the names above.
"""
from __future__ import annotations

import importlib
import importlib.abc
import importlib.machinery
import sys
import types

_PKG = "comfy_gen_server_amd"

# alias -> one module of this package
DIRECT = {
    "comfy.model_management": "runtime.device",
    "comfy.samplers": "sampling.samplers",
    "comfy.sample": "sampling.sample",
    "comfy.sampler_helpers": "sampling.sampler_helpers",
    "comfy.model_sampling": "sampling.model_sampling",
    "comfy.conds": "sampling.conds",
    "comfy.k_diffusion.sampling": "sampling.k_samplers",
    "comfy.extra_samplers.uni_pc": "sampling.uni_pc",
    "comfy.sd": "runtime.sd",
    "comfy.model_patcher": "runtime.patcher",
    "comfy.model_base": "runtime.model_base",
    "comfy.model_detection": "runtime.detection",
    "comfy.supported_models": "runtime.families",
    "comfy.supported_models_base": "runtime.families",
    "comfy.latent_formats": "runtime.latent_formats",
    "comfy.controlnet": "runtime.controlnet",
    "comfy.clip_vision": "runtime.clip_vision",
    "comfy.lora": "runtime.lora",
    "comfy.diffusers_load": "runtime.diffusers",
    "comfy.diffusers_convert": "runtime.convert",
    "comfy.cli_args": "cli_args",
    "comfy.sd1_clip": "models.text_encoders",
    "comfy.sdxl_clip": "models.text_encoders",
    "comfy.clip_model": "models.clip",
    "comfy.gligen": "models.gligen",
    "comfy.taesd.taesd": "models.taesd",
    "comfy.cldm.cldm": "models.cldm",
    "comfy.t2i_adapter.adapter": "models.t2i_adapter",
    "comfy.ldm.modules.attention": "models.attention",
    "comfy.ldm.modules.diffusionmodules.openaimodel": "models.unet",
    "comfy.ldm.modules.diffusionmodules.model": "models.vae",
    "comfy.ldm.cascade.stage_c": "models.cascade",
    "comfy.ldm.cascade.stage_b": "models.cascade",
    "comfy.ldm.cascade.stage_a": "models.cascade",
    "folder_paths": "utils.folder_paths",
    "node_helpers": "nodes.helpers",
    "latent_preview": "utils.preview",
    "execution": "graph.executor",
    "comfy_extras.chainner_models.model_loading": "models.upscalers",
}

# alias -> facade over several modules (searched in order) + reference-named wrappers
FACADES = {
    "comfy.utils": ["utils.image", "utils.progress", "runtime.checkpoint", "runtime.convert"],
    "comfy.ops": ["models.layers"],
    "nodes": ["graph.registry", "nodes.core"],
    "server": ["api.server"],
}
# packages that only hold submodules
PACKAGES = {"comfy", "comfy.k_diffusion", "comfy.extra_samplers", "comfy.taesd", "comfy.cldm", "comfy.t2i_adapter",
            "comfy.ldm", "comfy.ldm.modules", "comfy.ldm.modules.diffusionmodules", "comfy.ldm.cascade",
            "comfy_extras", "comfy_extras.chainner_models"}


def _extras(module):
    """Reference-named helpers a facade adds on top of its source modules."""
    name = module.__name__
    if name == "comfy.utils":
        from .runtime import checkpoint
        from .utils import progress

        def load_torch_file(ckpt, safe_load=False, device=None):
            return checkpoint.load_state_dict(ckpt, safe_load=safe_load, device=device)

        def save_torch_file(sd, ckpt, metadata=None):
            return checkpoint.save_state_dict(sd, ckpt, metadata=metadata)

        def set_progress_bar_enabled(enabled):
            progress.set_progress_bar_enabled(enabled)
        return {"load_torch_file": load_torch_file, "save_torch_file": save_torch_file,
                "set_progress_bar_enabled": set_progress_bar_enabled}
    if name == "nodes":
        from .graph import registry
        return {"MAX_RESOLUTION": 16384, "init_extra_nodes": registry.init_nodes}
    if name == "comfy.ops":
        from .models import layers

        class disable_weight_init:          # comfy/ops.py:39-163 (no-init, cast-on-call layers)
            Linear = layers.Linear
            Conv2d = layers.Conv2d
            Conv3d = layers.Conv3d
            GroupNorm = layers.GroupNorm
            LayerNorm = layers.LayerNorm
            Embedding = layers.Embedding

        class manual_cast(disable_weight_init):
            pass
        return {"disable_weight_init": disable_weight_init, "manual_cast": manual_cast}
    return {}


class _Facade(types.ModuleType):
    def __init__(self, name, sources):
        super().__init__(name)
        self.__dict__["_sources"] = sources
        self.__dict__["_extra"] = None

    def __getattr__(self, attr):
        if attr.startswith("__"):
            raise AttributeError(attr)
        extra = self.__dict__["_extra"]
        if extra is None:
            from . import compat_names
            extra = dict(compat_names.extra_names(self.__name__))
            extra.update(_extras(self))
            self.__dict__["_extra"] = extra
        if attr in extra:
            return extra[attr]
        for src in self.__dict__["_sources"]:
            mod = importlib.import_module(f"{_PKG}.{src}")
            if hasattr(mod, attr):
                return getattr(mod, attr)
        raise AttributeError(f"module {self.__name__!r} has no attribute {attr!r}")

    def __dir__(self):
        names = set(self.__dict__)
        for src in self.__dict__["_sources"]:
            names |= set(dir(importlib.import_module(f"{_PKG}.{src}")))
        return sorted(names)


class _ExtrasNodes(_Facade):
    """``comfy_extras.nodes_<x>``: any extra node class by name, from whichever module holds it."""

    def __init__(self, name):
        super().__init__(name, [])

    def __getattr__(self, attr):
        if attr.startswith("__"):
            raise AttributeError(attr)
        from .graph import registry
        registry.init_nodes(custom_nodes=False)
        cls = registry.NODE_CLASS_MAPPINGS.get(attr)
        if cls is not None:
            return cls
        if attr == "NODE_CLASS_MAPPINGS":
            return dict(registry.NODE_CLASS_MAPPINGS)
        for m in registry._CORE_MODULES:
            try:
                mod = importlib.import_module(f"{_PKG}.nodes.{m}")
            except ModuleNotFoundError:
                continue
            if hasattr(mod, attr):
                return getattr(mod, attr)
        raise AttributeError(f"module {self.__name__!r} has no attribute {attr!r}")


class _Loader(importlib.abc.Loader):
    def create_module(self, spec):
        name = spec.name
        if name in DIRECT:
            mod = importlib.import_module(f"{_PKG}.{DIRECT[name]}")
            from . import compat_names
            compat_names.inject(name, mod)     # reference-named extras on our module itself
            return mod
        if name in FACADES:
            return _Facade(name, FACADES[name])
        if name.startswith("comfy_extras.nodes_"):
            return _ExtrasNodes(name)
        mod = types.ModuleType(name)
        mod.__path__ = []
        return mod

    def exec_module(self, module):
        pass


class _Finder(importlib.abc.MetaPathFinder):
    def find_spec(self, fullname, path=None, target=None):
        if fullname in DIRECT or fullname in FACADES or fullname in PACKAGES or \
                fullname.startswith("comfy_extras.nodes_"):
            is_pkg = fullname in PACKAGES
            return importlib.machinery.ModuleSpec(fullname, _LOADER, is_package=is_pkg)
        return None


_LOADER = _Loader()
_FINDER = _Finder()


def install():
    """Idempotent: put the alias finder first on ``sys.meta_path``."""
    if _FINDER not in sys.meta_path:
        sys.meta_path.insert(0, _FINDER)
    return _FINDER


def uninstall():
    if _FINDER in sys.meta_path:
        sys.meta_path.remove(_FINDER)
    for name in list(sys.modules):
        if name in DIRECT or name in FACADES or name in PACKAGES or name.startswith("comfy_extras.nodes_"):
            del sys.modules[name]
