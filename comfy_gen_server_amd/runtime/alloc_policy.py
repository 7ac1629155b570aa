"""HBM allocator policy (C57; the reference's ``cuda_malloc.py`` picks ``backend:cudaMallocAsync`` for
the CUDA caching allocator before torch is imported).

On ROCm the caching allocator reads ``PYTORCH_HIP_ALLOC_CONF`` (``PYTORCH_CUDA_ALLOC_CONF`` is
honoured too) when it first allocates. The server composes one conf string from its flags and
the MI355X defaults, keeping every key the user already set:

* ``garbage_collection_threshold:0.9`` -- with 288 GB of HBM per GPU the cache grows large across
  prompts of different resolutions; past 90 % of the pool, unused cached blocks are returned
  before an allocation can fail (the reference instead empties the cache between prompts, which
  ROCm skips: ``model_management.py:839-841``);
* ``max_split_size_mb:1024`` -- blocks above 1 GiB (VAE decodes at 1024² x 8, checkpoint staging)
  are never split, so the large-tensor pool cannot fragment;
* ``--cuda-malloc`` -> ``backend:cudaMallocAsync`` (the stream-ordered hipMallocAsync allocator),
  ``--disable-cuda-malloc`` -> the native caching allocator (the default here: hipGraph plans use
  its private pools);
* ``--alloc-expandable`` -> ``expandable_segments:True`` (virtual-memory growth of one segment).

``configure(args)`` must run before the first device allocation; ``main`` calls it right after
argument parsing, before any model is built.
"""
from __future__ import annotations

import os

ENV_KEYS = ("PYTORCH_HIP_ALLOC_CONF", "PYTORCH_CUDA_ALLOC_CONF")
DEFAULTS = {"garbage_collection_threshold": "0.9", "max_split_size_mb": "1024"}


def parse_conf(s: str | None) -> dict:
    out = {}
    for part in (s or "").split(","):
        part = part.strip()
        if not part:
            continue
        k, _, v = part.partition(":")
        out[k.strip()] = v.strip()
    return out


def compose(existing: str | None, cuda_malloc=False, disable_cuda_malloc=False, expandable=False) -> str:
    """Conf string: the user's keys win, then flag-derived keys, then the MI355X defaults."""
    conf = dict(DEFAULTS)
    if expandable:
        conf["expandable_segments"] = "True"
    if cuda_malloc and not disable_cuda_malloc:
        conf = {"backend": "cudaMallocAsync"}      # the async backend takes no caching-allocator knobs
    conf.update(parse_conf(existing))
    return ",".join(f"{k}:{v}" for k, v in conf.items())


def configure(args=None) -> str:
    existing = os.environ.get(ENV_KEYS[0]) or os.environ.get(ENV_KEYS[1])
    s = compose(existing, cuda_malloc=bool(getattr(args, "cuda_malloc", False)),
                disable_cuda_malloc=bool(getattr(args, "disable_cuda_malloc", False)),
                expandable=bool(getattr(args, "alloc_expandable", False)))
    for k in ENV_KEYS:
        os.environ[k] = s
    return s
