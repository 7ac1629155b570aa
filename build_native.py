#!/usr/bin/env python3
"""Build the in-tree native libraries (no JIT cache, no pip install — the .so files live in
``comfy_gen_server_amd/lib`` and travel with the repo snapshot to the GPU box).

  libcgs_kernels.so   hipcc --offload-arch=gfx950, every csrc/kernels/*.hip (plain HIP C++, no hipify)
  _cgs_runtime*.so    g++ (pybind11) — csrc/runtime/*.cpp (safetensors, BPE, BLAKE3, job queue)

Incremental: each source compiles to an object in build/ only when it is newer than its object.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "comfy_gen_server_amd")
KDIR = os.path.join(PKG, "csrc", "kernels")
RDIR = os.path.join(PKG, "csrc", "runtime")
LIB = os.path.join(PKG, "lib")
BUILD = os.path.join(ROOT, "build", "native")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")
ARCH = os.environ.get("CGS_OFFLOAD_ARCH", "gfx950")


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("command failed:\n" + " ".join(cmd) + "\n" + r.stdout)
    return r.stdout


def _stale(src, obj, deps=()):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(p) > t for p in (src,) + tuple(deps))


def build_kernels(verbose=False):
    os.makedirs(BUILD, exist_ok=True)
    os.makedirs(LIB, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(KDIR, "*.hip")))
    headers = glob.glob(os.path.join(KDIR, "*.h"))
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-mcode-object-version=5",
             "-Wno-unused-result", "-munsafe-fp-atomics"]
    jobs = []
    objs = []
    for s in srcs:
        o = os.path.join(BUILD, os.path.basename(s) + ".o")
        objs.append(o)
        if _stale(s, o, headers):
            jobs.append([HIPCC] + flags + ["-c", s, "-o", o])
    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 4)) as ex:
        for out in ex.map(_run, jobs):
            if verbose and out.strip():
                print(out)
    so = os.path.join(LIB, "libcgs_kernels.so")
    if jobs or not os.path.exists(so):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", so] + objs)
    return so


def build_runtime(verbose=False):
    srcs = sorted(glob.glob(os.path.join(RDIR, "*.cpp")))
    if not srcs:
        return None
    import pybind11
    os.makedirs(BUILD, exist_ok=True)
    ext = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    so = os.path.join(LIB, "_cgs_runtime" + ext)
    inc = [pybind11.get_include(), sysconfig.get_paths()["include"]]
    flags = ["-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-Wall", "-Wno-unused-function"]
    headers = glob.glob(os.path.join(RDIR, "*.h"))
    objs, jobs = [], []
    for s in srcs:
        o = os.path.join(BUILD, "rt_" + os.path.basename(s) + ".o")
        objs.append(o)
        if _stale(s, o, headers):
            jobs.append(["g++"] + flags + [f"-I{i}" for i in inc] + ["-c", s, "-o", o])
    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 4)) as ex:
        for out in ex.map(_run, jobs):
            if verbose and out.strip():
                print(out)
    if jobs or not os.path.exists(so):
        _run(["g++", "-shared", "-fPIC", "-o", so] + objs + ["-lpthread"])
    return so


def build_sanitized(kinds: str, verbose=False):
    """CPU sanitizer build of the host runtime as a standalone threaded stress binary
    (csrc/runtime/tests/stress_main.cpp + every runtime source except the pybind module), e.g.
    ``--sanitize=address,undefined`` or ``--sanitize=thread``. Returns the binary path."""
    kinds = ",".join(k.strip() for k in kinds.split(",") if k.strip())
    tag = kinds.replace(",", "_")
    out_dir = os.path.join(ROOT, "build", "sanitize")
    os.makedirs(out_dir, exist_ok=True)
    srcs = [s for s in sorted(glob.glob(os.path.join(RDIR, "*.cpp"))) if not s.endswith("module.cpp")]
    srcs.append(os.path.join(RDIR, "tests", "stress_main.cpp"))
    exe = os.path.join(out_dir, f"runtime_stress_{tag}")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", f"-fsanitize={kinds}",
           "-fno-sanitize-recover=all", "-o", exe] + srcs + ["-lpthread"]
    out = _run(cmd)
    if verbose and out.strip():
        print(out)
    return exe


def build_all(verbose=False):
    k = build_kernels(verbose)
    r = build_runtime(verbose)
    return k, r


if __name__ == "__main__":
    san = [a.split("=", 1)[1] for a in sys.argv[1:] if a.startswith("--sanitize=")]
    if san:
        for kinds in san:
            exe = build_sanitized(kinds, verbose="-v" in sys.argv)
            print("built", exe)
            r = subprocess.run([exe, os.path.join(ROOT, "build", "sanitize")])
            if r.returncode != 0:
                sys.exit(r.returncode)
    else:
        k, r = build_all(verbose="-v" in sys.argv)
        print("built", k, r)
