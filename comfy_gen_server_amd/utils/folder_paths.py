"""Model / file registry (parity: ``folder_paths.py:1-267``; C15).

Maps model kinds to search directories + extensions, mtime-validated filename cache, annotated
filepaths (``name [input|output|temp]``), auto-incrementing save paths with %width%/%height%
substitution and path-escape guards, and extra roots from ``extra_model_paths.yaml``.
"""
from __future__ import annotations

import logging
import os
import time

supported_pt_extensions = {".ckpt", ".pt", ".bin", ".pth", ".safetensors", ".pkl", ".sft"}

base_path = os.environ.get("CGS_BASE_DIR", os.getcwd())
models_dir = os.path.join(base_path, "models")
folder_names_and_paths: dict[str, tuple[list[str], set[str]]] = {}


def _reset_defaults():
    global folder_names_and_paths
    folder_names_and_paths = {
        "checkpoints": ([os.path.join(models_dir, "checkpoints")], supported_pt_extensions),
        "configs": ([os.path.join(models_dir, "configs")], {".yaml"}),
        "loras": ([os.path.join(models_dir, "loras")], supported_pt_extensions),
        "vae": ([os.path.join(models_dir, "vae")], supported_pt_extensions),
        "clip": ([os.path.join(models_dir, "clip")], supported_pt_extensions),
        "unet": ([os.path.join(models_dir, "unet")], supported_pt_extensions),
        "clip_vision": ([os.path.join(models_dir, "clip_vision")], supported_pt_extensions),
        "style_models": ([os.path.join(models_dir, "style_models")], supported_pt_extensions),
        "embeddings": ([os.path.join(models_dir, "embeddings")], supported_pt_extensions),
        "diffusers": ([os.path.join(models_dir, "diffusers")], {"folder"}),
        "vae_approx": ([os.path.join(models_dir, "vae_approx")], supported_pt_extensions),
        "controlnet": ([os.path.join(models_dir, "controlnet"), os.path.join(models_dir, "t2i_adapter")],
                       supported_pt_extensions),
        "gligen": ([os.path.join(models_dir, "gligen")], supported_pt_extensions),
        "upscale_models": ([os.path.join(models_dir, "upscale_models")], supported_pt_extensions),
        "custom_nodes": ([os.path.join(base_path, "custom_nodes")], set()),
        "hypernetworks": ([os.path.join(models_dir, "hypernetworks")], supported_pt_extensions),
        "photomaker": ([os.path.join(models_dir, "photomaker")], supported_pt_extensions),
        "classifiers": ([os.path.join(models_dir, "classifiers")], {""}),
    }


_reset_defaults()
output_directory = os.path.join(base_path, "output")
temp_directory = os.path.join(base_path, "temp")
input_directory = os.path.join(base_path, "input")
user_directory = os.path.join(base_path, "user")
filename_list_cache: dict = {}


def set_base_path(path: str):
    """Re-root every default directory (used by tests and the server's --base-directory)."""
    global base_path, models_dir, output_directory, temp_directory, input_directory, user_directory
    base_path = path
    models_dir = os.path.join(path, "models")
    output_directory = os.path.join(path, "output")
    temp_directory = os.path.join(path, "temp")
    input_directory = os.path.join(path, "input")
    user_directory = os.path.join(path, "user")
    _reset_defaults()
    filename_list_cache.clear()


def set_output_directory(d):
    global output_directory
    output_directory = d


def set_temp_directory(d):
    global temp_directory
    temp_directory = d


def set_input_directory(d):
    global input_directory
    input_directory = d


def get_output_directory():
    return output_directory


def get_temp_directory():
    return temp_directory


def get_input_directory():
    return input_directory


def get_user_directory():
    return user_directory


def get_directory_by_type(type_name):
    return {"output": get_output_directory(), "temp": get_temp_directory(), "input": get_input_directory()}.get(type_name)


def annotated_filepath(name):
    for tag, fn in (("[output]", get_output_directory), ("[input]", get_input_directory), ("[temp]", get_temp_directory)):
        if name.endswith(tag):
            return name[:-len(tag)].rstrip(), fn()
    return name, None


def get_annotated_filepath(name, default_dir=None):
    name, base_dir = annotated_filepath(name)
    if base_dir is None:
        base_dir = default_dir if default_dir is not None else get_input_directory()
    return os.path.join(base_dir, name)


def exists_annotated_filepath(name):
    name, base_dir = annotated_filepath(name)
    if base_dir is None:
        base_dir = get_input_directory()
    return os.path.exists(os.path.join(base_dir, name))


def add_model_folder_path(folder_name, full_folder_path):
    if folder_name in folder_names_and_paths:
        if full_folder_path not in folder_names_and_paths[folder_name][0]:
            folder_names_and_paths[folder_name][0].append(full_folder_path)
    else:
        folder_names_and_paths[folder_name] = ([full_folder_path], set())
    filename_list_cache.pop(folder_name, None)


def get_folder_paths(folder_name):
    return folder_names_and_paths[folder_name][0][:]


def recursive_search(directory, excluded_dir_names=None):
    if not os.path.isdir(directory):
        return [], {}
    excluded = set(excluded_dir_names or [])
    result = []
    dirs = {}
    try:
        dirs[directory] = os.path.getmtime(directory)
    except FileNotFoundError:
        logging.warning("Directory %s not found", directory)
    for root, subdirs, files in os.walk(directory, followlinks=True, topdown=True):
        subdirs[:] = [d for d in subdirs if d not in excluded]
        for f in files:
            result.append(os.path.relpath(os.path.join(root, f), directory))
        for d in subdirs:
            p = os.path.join(root, d)
            try:
                dirs[p] = os.path.getmtime(p)
            except FileNotFoundError:
                continue
    return result, dirs


def filter_files_extensions(files, extensions):
    return sorted(f for f in files if os.path.splitext(f)[-1].lower() in extensions or len(extensions) == 0)


def get_full_path(folder_name, filename):
    if folder_name not in folder_names_and_paths:
        return None
    filename = os.path.relpath(os.path.join("/", filename), "/")
    for x in folder_names_and_paths[folder_name][0]:
        full = os.path.join(x, filename)
        if os.path.isfile(full):
            return full
    return None


def get_filename_list_(folder_name):
    output_list = set()
    folders = folder_names_and_paths[folder_name]
    output_folders = {}
    for x in folders[0]:
        files, dirs = recursive_search(x, excluded_dir_names=[".git"])
        output_list.update(filter_files_extensions(files, folders[1]))
        output_folders.update(dirs)
    return sorted(output_list), output_folders, time.perf_counter()


def cached_filename_list_(folder_name):
    if folder_name not in filename_list_cache:
        return None
    out = filename_list_cache[folder_name]
    for x, mt in out[1].items():
        if not os.path.exists(x) or os.path.getmtime(x) != mt:
            return None
    for x in folder_names_and_paths[folder_name][0]:
        if os.path.isdir(x) and x not in out[1]:
            return None
    return out


def get_filename_list(folder_name):
    out = cached_filename_list_(folder_name)
    if out is None:
        out = get_filename_list_(folder_name)
        filename_list_cache[folder_name] = out
    return list(out[0])


def get_save_image_path(filename_prefix, output_dir, image_width=0, image_height=0):
    def map_filename(filename):
        plen = len(os.path.basename(filename_prefix))
        prefix = filename[:plen + 1]
        try:
            digits = int(filename[plen + 1:].split("_")[0])
        except ValueError:
            digits = 0
        return digits, prefix

    def compute_vars(inp, w, h):
        return inp.replace("%width%", str(w)).replace("%height%", str(h))

    filename_prefix = compute_vars(filename_prefix, image_width, image_height)
    subfolder = os.path.dirname(os.path.normpath(filename_prefix))
    filename = os.path.basename(os.path.normpath(filename_prefix))
    full_output_folder = os.path.join(output_dir, subfolder)
    if os.path.commonpath((output_dir, os.path.abspath(full_output_folder))) != output_dir:
        raise Exception("Saving image outside the output folder is not allowed."
                        f"\n full_output_folder: {os.path.abspath(full_output_folder)}"
                        f"\n         output_dir: {output_dir}"
                        f"\n         commonpath: {os.path.commonpath((output_dir, os.path.abspath(full_output_folder)))}")
    try:
        counter = max(filter(lambda a: os.path.normcase(a[1][:-1]) == os.path.normcase(filename) and a[1][-1] == "_",
                             map(map_filename, os.listdir(full_output_folder))))[0] + 1
    except (ValueError, FileNotFoundError):
        os.makedirs(full_output_folder, exist_ok=True)
        counter = 1
    return full_output_folder, filename, counter, subfolder, filename_prefix


def load_extra_path_config(yaml_path):
    import yaml
    with open(yaml_path, "r") as stream:
        config = yaml.safe_load(stream)
    for c in config or {}:
        conf = config[c]
        if conf is None:
            continue
        base = None
        if "base_path" in conf:
            base = conf.pop("base_path")
        for x, y in conf.items():
            for p in y.split("\n"):
                if not p:
                    continue
                full = p
                if base is not None:
                    full = os.path.join(base, full)
                logging.info("Adding extra search path %s %s", x, full)
                add_model_folder_path(x, full)
