"""Allocator policy (C57, reference cuda_malloc.py)."""
from comfy_gen_server_amd.runtime import alloc_policy as ap


def test_compose_defaults_flags_and_user_keys():
    assert ap.parse_conf(ap.compose(None)) == {"garbage_collection_threshold": "0.9", "max_split_size_mb": "1024"}
    c = ap.parse_conf(ap.compose(None, expandable=True))
    assert c["expandable_segments"] == "True"
    assert ap.parse_conf(ap.compose(None, cuda_malloc=True)) == {"backend": "cudaMallocAsync"}
    assert "backend" not in ap.parse_conf(ap.compose(None, cuda_malloc=True, disable_cuda_malloc=True))
    user = ap.parse_conf(ap.compose("max_split_size_mb:256,roundup_power2_divisions:4"))
    assert user["max_split_size_mb"] == "256" and user["roundup_power2_divisions"] == "4"
    assert user["garbage_collection_threshold"] == "0.9"


def test_configure_sets_both_env_names(monkeypatch):
    for k in ap.ENV_KEYS:
        monkeypatch.delenv(k, raising=False)

    class A:
        cuda_malloc = False
        disable_cuda_malloc = False
        alloc_expandable = True
    s = ap.configure(A())
    import os
    assert os.environ["PYTORCH_HIP_ALLOC_CONF"] == s == os.environ["PYTORCH_CUDA_ALLOC_CONF"]
    assert "expandable_segments:True" in s
