"""Node registry + custom-node loader (parity: ``nodes.py:2146-2400``, ``main.py:9-46``; C12).

``NODE_CLASS_MAPPINGS`` / ``NODE_DISPLAY_NAME_MAPPINGS`` / ``EXTENSION_WEB_DIRS`` are module-level
dicts so custom nodes and the server share one registry. ``init_nodes()`` imports the core and
extra node modules of this package, then every ``custom_nodes/*`` file or package (merging their
mappings without overriding existing names, registering ``WEB_DIRECTORY``), logging import times;
``execute_prestartup_scripts()`` runs each custom node's ``prestartup_script.py`` first.
"""
from __future__ import annotations

import importlib
import importlib.util
import logging
import os
import sys
import time
import traceback

NODE_CLASS_MAPPINGS: dict = {}
NODE_DISPLAY_NAME_MAPPINGS: dict = {}
EXTENSION_WEB_DIRS: dict = {}
LOADED_MODULE_DIRS: dict = {}

_CORE_MODULES = ["core", "extras_sampling", "extras_latent", "extras_image", "extras_mask", "extras_model", "extras_merge",
                 "extras_conditioning", "extras_cascade", "extras_video", "extras_upscale", "extras_misc"]
_initialized = False


def register(mappings: dict, display: dict | None = None, override=False):
    for k, v in mappings.items():
        if override or k not in NODE_CLASS_MAPPINGS:
            NODE_CLASS_MAPPINGS[k] = v
    if display:
        for k, v in display.items():
            NODE_DISPLAY_NAME_MAPPINGS.setdefault(k, v)


def load_custom_node(module_path, ignore=set(), module_parent="custom_nodes"):
    module_name = os.path.basename(module_path)
    if os.path.isfile(module_path):
        sp = os.path.splitext(module_path)
        module_name = sp[0]
    try:
        logging.debug("Trying to load custom node %s", module_path)
        if os.path.isfile(module_path):
            spec = importlib.util.spec_from_file_location(module_name, module_path)
            module_dir = os.path.split(module_path)[0]
        else:
            spec = importlib.util.spec_from_file_location(module_name, os.path.join(module_path, "__init__.py"))
            module_dir = module_path
        module = importlib.util.module_from_spec(spec)
        sys.modules[module_name] = module
        spec.loader.exec_module(module)
        LOADED_MODULE_DIRS[module_name] = os.path.abspath(module_dir)
        if hasattr(module, "WEB_DIRECTORY") and getattr(module, "WEB_DIRECTORY") is not None:
            web_dir = os.path.abspath(os.path.join(module_dir, getattr(module, "WEB_DIRECTORY")))
            if os.path.isdir(web_dir):
                EXTENSION_WEB_DIRS[module_name] = web_dir
        if hasattr(module, "NODE_CLASS_MAPPINGS") and getattr(module, "NODE_CLASS_MAPPINGS") is not None:
            for name, cls in module.NODE_CLASS_MAPPINGS.items():
                if name not in ignore:
                    NODE_CLASS_MAPPINGS[name] = cls
                    cls.RELATIVE_PYTHON_MODULE = f"{module_parent}.{module_name}"
            if hasattr(module, "NODE_DISPLAY_NAME_MAPPINGS") and getattr(module, "NODE_DISPLAY_NAME_MAPPINGS") is not None:
                NODE_DISPLAY_NAME_MAPPINGS.update(module.NODE_DISPLAY_NAME_MAPPINGS)
            return True
        logging.warning("Skip %s module for custom nodes due to the lack of NODE_CLASS_MAPPINGS.", module_path)
        return False
    except Exception:
        logging.warning(traceback.format_exc())
        logging.warning("Cannot import %s module for custom nodes", module_path)
        return False


def execute_prestartup_scripts(custom_node_dirs=None):
    if custom_node_dirs is None:
        from ..utils import folder_paths
        custom_node_dirs = folder_paths.get_folder_paths("custom_nodes")
    for d in custom_node_dirs:
        if not os.path.isdir(d):
            continue
        for p in sorted(os.listdir(d)):
            mp = os.path.join(d, p)
            if os.path.isfile(mp) or mp.endswith(".disabled") or mp == "__pycache__":
                continue
            script = os.path.join(mp, "prestartup_script.py")
            if os.path.exists(script):
                try:
                    spec = importlib.util.spec_from_file_location(p + "_prestartup", script)
                    m = importlib.util.module_from_spec(spec)
                    spec.loader.exec_module(m)
                except Exception as e:
                    logging.warning("Failed to execute startup-script %s / %s", script, e)


def load_custom_nodes(dirs=None):
    from ..utils import folder_paths
    from .. import compat
    compat.install()          # `import comfy.utils`, `folder_paths`, `nodes`, `server`, ... resolve to this engine
    base_names = set(NODE_CLASS_MAPPINGS.keys())
    dirs = dirs if dirs is not None else folder_paths.get_folder_paths("custom_nodes")
    times = []
    for d in dirs:
        if not os.path.isdir(d):
            continue
        for p in sorted(os.listdir(d)):
            mp = os.path.join(d, p)
            if os.path.isfile(mp) and os.path.splitext(mp)[1] != ".py":
                continue
            if mp.endswith(".disabled") or p == "__pycache__":
                continue
            t0 = time.perf_counter()
            ok = load_custom_node(mp, base_names)
            times.append((time.perf_counter() - t0, mp, ok))
    if times:
        logging.info("Import times for custom nodes:")
        for t, mp, ok in sorted(times):
            logging.info("%6.1f seconds%s: %s", t, "" if ok else " (IMPORT FAILED)", mp)
    return times


def init_nodes(custom_nodes=True, custom_dirs=None):
    global _initialized
    if not _initialized:
        for m in _CORE_MODULES:
            try:
                mod = importlib.import_module(f"comfy_gen_server_amd.nodes.{m}")
            except ModuleNotFoundError as e:
                if e.name == f"comfy_gen_server_amd.nodes.{m}":
                    continue
                raise
            register(getattr(mod, "NODE_CLASS_MAPPINGS", {}), getattr(mod, "NODE_DISPLAY_NAME_MAPPINGS", {}))
        _initialized = True
    if custom_nodes:
        load_custom_nodes(custom_dirs)
    return NODE_CLASS_MAPPINGS


def node_info(node_class: str) -> dict:
    """/object_info schema for one class (server.py:574-592)."""
    obj = NODE_CLASS_MAPPINGS[node_class]
    info = {"input": obj.INPUT_TYPES(), "output": obj.RETURN_TYPES,
            "output_is_list": getattr(obj, "OUTPUT_IS_LIST", [False] * len(obj.RETURN_TYPES)),
            "output_name": getattr(obj, "RETURN_NAMES", obj.RETURN_TYPES), "name": node_class,
            "display_name": NODE_DISPLAY_NAME_MAPPINGS.get(node_class, node_class),
            "description": getattr(obj, "DESCRIPTION", ""),
            "category": getattr(obj, "CATEGORY", "sd"),
            "output_node": bool(getattr(obj, "OUTPUT_NODE", False))}
    if hasattr(obj, "RELATIVE_PYTHON_MODULE"):
        info["python_module"] = obj.RELATIVE_PYTHON_MODULE
    else:
        info["python_module"] = "nodes"
    return info


def interrupt_processing(value=True):
    from ..runtime import device as dm
    dm.interrupt_current_processing(value)


def before_node_execution():
    from ..runtime import device as dm
    dm.throw_exception_if_processing_interrupted()
