"""Ablation of the one-wave-per-SIMD "w5" GEMM loop (csrc/kernels/gemm_w5.hip, DBG template bits) against
v7 and hipBLASLt on one box, interleaved rounds in one process.

  dbg 0 full loop; 1 no main-loop DMAs; 2 no fragment reads; 3 neither; 4 no per-stage wait + barrier;
  7 MFMAs only (the issue ceiling of the wave tile)

python tools/probes/w5_ablate.py [M N K ...] [--rounds R] [--iters I] [--only name,...]
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch
import torch.nn.functional as F

from comfy_gen_server_amd import _native
from comfy_gen_server_amd.ops import core


def bench(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main(argv):
    rounds, iters, only = 5, 10, None
    shapes = []
    nums = []
    i = 0
    while i < len(argv):
        if argv[i] == "--rounds":
            rounds = int(argv[i + 1]); i += 2
        elif argv[i] == "--iters":
            iters = int(argv[i + 1]); i += 2
        elif argv[i] == "--only":
            only = set(argv[i + 1].split(",")); i += 2
        else:
            nums.append(int(argv[i])); i += 1
    for j in range(0, len(nums), 3):
        shapes.append(tuple(nums[j:j + 3]))
    if not shapes:
        shapes = [(8192, 8192, 8192), (16384, 3840, 1280), (65536, 1920, 640)]
    lib = _native.load_kernels()
    assert lib is not None, _native.kernels_error()
    dev = torch.device("cuda", 0)
    stream = core._stream()
    for M, N, K in shapes:
        a = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).to(torch.bfloat16)
        b = torch.zeros(N, device=dev, dtype=torch.bfloat16)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        cands = {}
        for d in (0, 1, 2, 3, 4, 7):
            cands[f"w5d{d}"] = (lambda d=d: lib.cgs_gemm_bf16_w5_dbg(a.data_ptr(), w.data_ptr(), out.data_ptr(),
                                                                    b.data_ptr(), None, M, N, K, K, K, N, 0, 1, 1.0,
                                                                    d, stream))
        for d in (0, 1, 2, 3):
            for gc, tag in ((0, "p"), (1 << 30, "np")):
                cands[f"w6d{d}{tag}"] = (lambda d=d, gc=gc: lib.cgs_gemm_bf16_w6(
                    a.data_ptr(), w.data_ptr(), out.data_ptr(), b.data_ptr(), None, None, None, M, N, K, K, K, N, 0, 1,
                    1.0, d, 4, gc, 256, stream))
        cands["v7"] = lambda: lib.cgs_gemm_bf16_v(a.data_ptr(), w.data_ptr(), out.data_ptr(), b.data_ptr(), None, M, N,
                                                  K, K, K, N, 0, 1, 1.0, 7, stream)
        cands["v6"] = lambda: lib.cgs_gemm_bf16_v(a.data_ptr(), w.data_ptr(), out.data_ptr(), b.data_ptr(), None, M, N,
                                                  K, K, K, N, 0, 1, 1.0, 6, stream)
        cands["lib"] = lambda: F.linear(a, w, b)
        if only:
            cands = {k: v for k, v in cands.items() if k in only}
        ref = (a.float() @ w.float().t())
        for k in ("w5d0", "v7", "w6d0p", "w6d0np"):
            if k in cands:
                out.zero_()
                assert cands[k]() == 0, k
                torch.cuda.synchronize()
                err = (out.float() - ref).abs().max().item() / ref.abs().max().item()
                print(f"{M}x{N}x{K} {k} max rel err {err:.2e}", flush=True)
        del ref
        times = {k: [] for k in cands}
        for _ in range(rounds):
            for k, f in cands.items():
                times[k].append(bench(f, iters))
        fl = 2.0 * M * N * K
        print(f"== {M}x{N}x{K}: " + "  ".join(f"{k} {fl / statistics.median(t) / 1e9:.0f}" for k, t in times.items()),
              flush=True)
        del a, w, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main(sys.argv[1:])
