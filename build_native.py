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
import json
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


# Private-memory (scratch) budget of the MFMA main-loop kernels, bytes per lane. A kernel whose
# accumulator / fragment arrays fall out of registers (SROA failing on a grown epilogue) runs ~10x
# slower with identical results -- round 3 shipped one such v7 build -- so the build fails instead.
SCRATCH_BUDGET = {"gemm_bf16_nt_v7_kernel": 128, "conv_nhwc_v7_kernel": 128, "attn_fwd_d64": 64}


def _resources(out):
    """kernel -> {vgpr, agpr, scratch, spill} from -Rpass-analysis=kernel-resource-usage remarks."""
    res, cur = {}, None
    for line in out.splitlines():
        if "remark:" not in line:
            continue
        txt = line.split("remark:", 1)[1].split("[-Rpass", 1)[0].strip()
        key, _, val = txt.partition(":")
        val = val.strip()
        if key == "Function Name":
            cur = val
            res[cur] = {}
        elif cur is not None and key in ("VGPRs", "AGPRs", "ScratchSize [bytes/lane]", "VGPRs Spill"):
            res[cur][{"VGPRs": "vgpr", "AGPRs": "agpr", "ScratchSize [bytes/lane]": "scratch",
                      "VGPRs Spill": "spill"}[key]] = int(val.split()[0])
    return res


def _check_resources(report):
    if not report:
        return
    path = os.path.join(BUILD, "kernel_resources.json")
    old = {}
    if os.path.exists(path):
        with open(path) as f:
            old = json.load(f)
    old.update(report)
    with open(path, "w") as f:
        json.dump(old, f, indent=1, sort_keys=True)
    bad = [(k, v.get("scratch", 0), lim) for k, v in report.items() for pat, lim in SCRATCH_BUDGET.items()
           if pat in k and v.get("scratch", 0) > lim]
    if bad:
        raise RuntimeError("MFMA kernels over their scratch budget (arrays out of registers):\n" +
                           "\n".join(f"  {k}: {s} B/lane > {lim}" for k, s, lim in bad))


def build_kernels(verbose=False):
    os.makedirs(BUILD, exist_ok=True)
    os.makedirs(LIB, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(KDIR, "*.hip")))
    headers = glob.glob(os.path.join(KDIR, "*.h"))
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-mcode-object-version=5",
             "-Wno-unused-result", "-munsafe-fp-atomics", "-Rpass-analysis=kernel-resource-usage"]
    jobs = []
    objs = []
    for s in srcs:
        o = os.path.join(BUILD, os.path.basename(s) + ".o")
        objs.append(o)
        if _stale(s, o, headers):
            jobs.append([HIPCC] + flags + ["-c", s, "-o", o])
    report = {}
    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 4)) as ex:
        for out in ex.map(_run, jobs):
            report.update(_resources(out))
            if verbose:
                print("\n".join(l for l in out.splitlines() if "remark" not in l))
    _check_resources(report)
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
