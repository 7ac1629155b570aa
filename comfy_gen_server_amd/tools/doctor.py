"""Installation check / setup (the role of the reference's ``install.py`` / updater scripts, C61,
for a ROCm box): reports the ROCm + PyTorch stack, the GPUs and their ISA, whether the in-tree native
libraries are built and export every kernel the op layer binds, the distributed backends, and the
environment settings the multi-process path needs. ``--build`` (re)builds the native libraries.

    python -m comfy_gen_server_amd.tools.doctor [--build] [--json]
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import subprocess
import sys


def report() -> dict:
    import torch
    from .. import _native
    r = {"python": sys.version.split()[0], "torch": torch.__version__, "hip": getattr(torch.version, "hip", None),
         "rocm_path": os.environ.get("ROCM_PATH", "/opt/rocm"), "hipcc": shutil.which("hipcc") or
         (os.path.exists("/opt/rocm/bin/hipcc") and "/opt/rocm/bin/hipcc") or None}
    try:
        with open(os.path.join(r["rocm_path"], ".info", "version")) as f:
            r["rocm_version"] = f.read().strip()
    except OSError:
        r["rocm_version"] = None
    gpus = []
    if torch.cuda.is_available():
        for i in range(torch.cuda.device_count()):
            p = torch.cuda.get_device_properties(i)
            gpus.append({"index": i, "name": p.name, "arch": getattr(p, "gcnArchName", "?"),
                         "hbm_gib": round(p.total_memory / 2 ** 30, 1), "cus": p.multi_processor_count})
    r["gpus"] = gpus
    lib = _native.load_kernels()
    r["kernels_lib"] = bool(lib)
    r["kernels_missing"] = [] if not lib else [n for n in _native.KERNEL_SIGNATURES if getattr(lib, n, None) is None]
    r["kernels_error"] = None if lib else _native.kernels_error()
    rt = _native.load_runtime()
    r["runtime_lib"] = bool(rt)
    import torch.distributed as dist
    r["distributed"] = {"available": dist.is_available(), "nccl(rccl)": dist.is_nccl_available(),
                        "gloo": dist.is_gloo_available()}
    r["env"] = {"HSA_ENABLE_IPC_MODE_LEGACY": os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY"),
                "GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES")}
    warn = []
    if gpus and any(g["arch"].split(":")[0] != "gfx950" for g in gpus):
        warn.append("kernels are built for gfx950 (MI355X) only")
    if not r["kernels_lib"] or r["kernels_missing"]:
        warn.append("native kernels missing: run `python build_native.py` (or doctor --build)")
    if not r["runtime_lib"]:
        warn.append("C++ runtime (_cgs_runtime) missing: safetensors/BPE/BLAKE3 fall back to Python")
    if len(gpus) > 1 and r["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] != "0":
        warn.append("set HSA_ENABLE_IPC_MODE_LEGACY=0 for multi-process RCCL (dmabuf IPC)")
    r["warnings"] = warn
    return r


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args(argv)
    if a.build:
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        subprocess.run([sys.executable, os.path.join(root, "build_native.py")], check=True)
    r = report()
    if a.json:
        print(json.dumps(r, indent=1))
    else:
        for k, v in r.items():
            print(f"{k:>16}: {v}")
    return 0 if not r["warnings"] else 1


if __name__ == "__main__":
    sys.exit(main())
