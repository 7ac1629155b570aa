"""The packaged tuning table (data/tune_mi355x.json) names only kernels the dispatchers know: a choice the op's
name -> variant map does not contain would raise (conv) or silently run the default path (GEMM) on every call
of that shape. Keys parse as the ops build them."""
import json

from comfy_gen_server_amd.ops import autotune, core

CONV = {"v2", "v4", "v5", "v6", "v7", "v8", "v6n128", "v6w4", "auto"}
GEMM = ({"v7", "v6", "v5", "v4", "v8", "w6", "w6n160", "v6m128", "v6w4", "hip", "lib"} | set(core._SMALL_NAMES)
        | set(core._SPLITK))
LNFOLD = {"v7", "v8", "v6", "w6", "w6n160", "v6m128", "v6w4"} | set(core._SMALL_NAMES) | set(core._SPLITK)
ATTN = {"d64", "d64q128", "generic", "d64ks2", "d64ks4"}
ALLOWED = {"conv": CONV, "gemm": GEMM, "gemm_lnfold": LNFOLD, "gemm_geglu": {"v5", "v6", "v7", "w6", "w6n160"},
           "attention_grid2": ATTN, "attention": {"hip", "lib"}}


def test_packaged_table_choices_are_dispatchable():
    with open(autotune.DEFAULT_TABLE) as f:
        table = json.load(f)
    bad = []
    for key, choice in table.items():
        if key.startswith("_"):
            continue
        kind = key.split("|")[0]
        assert kind in ALLOWED, key
        if choice not in ALLOWED[kind]:
            bad.append((key, choice))
    assert not bad, bad


def test_packaged_table_keys_parse():
    with open(autotune.DEFAULT_TABLE) as f:
        table = json.load(f)
    for key in table:
        if key.startswith("_"):
            continue
        parts = key.split("|")
        nums = parts[1:11] if parts[0] == "conv" else parts[1:]
        assert all(p.lstrip("-").isdigit() for p in nums), key
        if parts[0] in ("gemm", "gemm_lnfold", "gemm_geglu"):
            assert len(parts) == 5, key
