"""Installer for a ROCm / MI355X box (C61; the role of the reference's ``install.py``, which creates a
venv, pip-installs requirements and picks a CUDA/ROCm PyTorch wheel).

    python -m comfy_gen_server_amd.install [--venv DIR] [--pip] [--no-build] [--base-directory DIR]

Steps, each reported and skippable:

1. ``--venv DIR``: create a virtual environment WITH the system site-packages, so the ROCm PyTorch of
   the image (and RCCL) stays the one in use -- never a wheel from a package index; then re-run this
   installer inside it.
2. Python dependencies: every module the engine imports is checked; ``--pip`` installs the missing
   pure-Python ones with pip (off by default: MI355X hosts are often offline). PyTorch itself must
   be a ROCm build (``torch.version.hip``); a CUDA or CPU-only build is reported, not replaced.
3. Native build: ``build_native.py`` compiles the HIP kernels for gfx950 and the C++ runtime
   in-tree (``hipcc`` from ``/opt/rocm``).
4. Layout: ``models/<kind>/``, ``input/``, ``output/``, ``temp/`` under the base directory and an
   ``extra_model_paths.yaml`` template.
5. The doctor report (ROCm version, GPUs + ISA, exported kernels, RCCL / gloo, IPC env).
"""
from __future__ import annotations

import argparse
import importlib
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# import name -> pip name (pure-Python dependencies of the engine and its API surface)
REQUIRED = {"numpy": "numpy", "safetensors": "safetensors", "aiohttp": "aiohttp", "yaml": "pyyaml",
            "PIL": "pillow", "scipy": "scipy", "einops": "einops", "psutil": "psutil", "tqdm": "tqdm"}
OPTIONAL = {"grpc": "grpcio", "google.protobuf": "protobuf", "transformers": "transformers",
            "tokenizers": "tokenizers", "prometheus_client": "prometheus_client"}
MODEL_DIRS = ["checkpoints", "configs", "loras", "vae", "clip", "unet", "clip_vision", "style_models",
              "embeddings", "diffusers", "vae_approx", "controlnet", "gligen", "upscale_models",
              "hypernetworks", "photomaker", "classifiers"]


def missing(mods: dict) -> list:
    out = []
    for mod, pip_name in mods.items():
        try:
            importlib.import_module(mod)
        except Exception:
            out.append(pip_name)
    return out


def torch_status() -> dict:
    try:
        import torch
    except Exception as e:       # pragma: no cover - the image always has torch
        return {"ok": False, "detail": f"torch not importable: {e}"}
    hip = getattr(torch.version, "hip", None)
    if not hip:
        return {"ok": False, "detail": f"torch {torch.__version__} is not a ROCm build; install the ROCm wheel "
                                      f"that matches /opt/rocm (this engine targets gfx950 only)"}
    return {"ok": True, "detail": f"torch {torch.__version__} (HIP {hip})"}


def make_layout(base: str) -> list:
    made = []
    for d in [os.path.join("models", m) for m in MODEL_DIRS] + ["input", "output", "temp"]:
        p = os.path.join(base, d)
        if not os.path.isdir(p):
            os.makedirs(p, exist_ok=True)
            made.append(p)
    tmpl = os.path.join(ROOT, "deploy", "extra_model_paths.yaml.example")
    dst = os.path.join(base, "extra_model_paths.yaml.example")
    if os.path.exists(tmpl) and not os.path.exists(dst):
        shutil.copyfile(tmpl, dst)
        made.append(dst)
    return made


def create_venv(path: str) -> str:
    subprocess.run([sys.executable, "-m", "venv", "--system-site-packages", path], check=True)
    py = os.path.join(path, "bin", "python")
    print(f"install: venv at {path} (system site-packages kept: the image's ROCm PyTorch/RCCL)")
    return py


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="set up comfy_gen_server_amd on a ROCm box")
    ap.add_argument("--venv", default=None, help="create a venv here (system site-packages) and install into it")
    ap.add_argument("--pip", action="store_true", help="pip-install missing pure-Python dependencies")
    ap.add_argument("--no-build", action="store_true", help="skip the native (HIP / C++) build")
    ap.add_argument("--base-directory", default=ROOT, help="where models/, input/, output/ live")
    a = ap.parse_args(argv)
    if a.venv and os.path.realpath(sys.prefix) != os.path.realpath(a.venv):
        py = create_venv(a.venv)
        rest = [x for x in (argv if argv is not None else sys.argv[1:])]
        return subprocess.call([py, "-m", "comfy_gen_server_amd.install"] + rest, cwd=ROOT)
    rc = 0
    ts = torch_status()
    print(f"install: {ts['detail']}")
    rc |= 0 if ts["ok"] else 1
    req, opt = missing(REQUIRED), missing(OPTIONAL)
    if req or opt:
        print(f"install: missing required {req or '-'}; optional {opt or '-'}")
        if a.pip and (req or opt):
            r = subprocess.call([sys.executable, "-m", "pip", "install"] + req + opt)
            if r != 0:
                print("install: pip failed (offline host?); install the packages from a local wheelhouse")
            req = missing(REQUIRED)
        rc |= 1 if req else 0
    if not a.no_build:
        print("install: building the native libraries (hipcc --offload-arch=gfx950)")
        r = subprocess.call([sys.executable, os.path.join(ROOT, "build_native.py")], cwd=ROOT)
        rc |= 1 if r else 0
    made = make_layout(a.base_directory)
    print(f"install: layout under {a.base_directory} ({len(made)} entries created)")
    from .tools import doctor
    rep = doctor.report()
    for w in rep["warnings"]:
        print(f"install: warning: {w}")
    print("install: done" if rc == 0 else "install: finished with problems (see above)")
    return rc


if __name__ == "__main__":
    sys.exit(main())
