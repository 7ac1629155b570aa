"""Candidate gates of the device op layer that decide what the autotuner may time (no GPU needed):
split-K GEMM candidates (ops/core.py ``_splitk_cands``) and the Cascade fusion switches (models/cascade.py
``_fuse``)."""
from comfy_gen_server_amd.ops import core


def _gate(monkeypatch):
    monkeypatch.setattr(core._native, "has_kernel", lambda name: True)
    monkeypatch.setattr(core, "_underfilled", lambda M, N: True)
    return lambda name: name


def test_splitk_candidates_default_from_long_k(monkeypatch):
    run = _gate(monkeypatch)
    monkeypatch.delenv("CGS_SPLITK", raising=False)
    long_k = [n for n, _ in core._splitk_cands(1152, 2048, 8192, core.EPI_BIAS | core.EPI_RESIDUAL, run)]
    assert "sk4v8" in long_k and "sk2v8" in long_k            # Cascade Stage C K = 8192 at batch 1
    assert core._splitk_cands(2048, 1280, 1280, core.EPI_BIAS, run) == []     # SDXL batch-1 K: single pass
    monkeypatch.setenv("CGS_SPLITK", "1")
    assert core._splitk_cands(2048, 1280, 1280, core.EPI_BIAS, run)
    monkeypatch.setenv("CGS_SPLITK", "0")
    assert core._splitk_cands(1152, 2048, 8192, core.EPI_BIAS, run) == []


def test_splitk_slices_keep_whole_k_steps(monkeypatch):
    run = _gate(monkeypatch)
    monkeypatch.setenv("CGS_SPLITK", "1")
    for name, _ in core._splitk_cands(512, 1280, 1280, core.EPI_BIAS, run):
        s = core._SPLITK[name][1]
        assert 1280 % (32 * s) == 0 and 1280 // s >= 256
    # epilogues the reduce pass cannot apply (GEGLU) never get split-K candidates
    assert core._splitk_cands(512, 1280, 8192, core.EPI_BIAS | core.EPI_GEGLU, run) == []


def test_cascade_fusion_switches(monkeypatch):
    from comfy_gen_server_amd.models import cascade as SC
    for k in ("AFFLN", "TSBATCH", "ATTNLN", "DWLN", "GRNFOLD", "GELU_EPI", "LNFOLD"):
        monkeypatch.delenv(f"CGS_CASCADE_{k}", raising=False)
    assert SC._fuse("AFFLN") and SC._fuse("TSBATCH")           # measured wins: on
    assert not SC._fuse("ATTNLN") and not SC._fuse("DWLN") and not SC._fuse("GRNFOLD")
    assert not SC._fuse("GELU_EPI", 1152) and SC._fuse("GELU_EPI", 4608)     # rows threshold
    monkeypatch.setenv("CGS_CASCADE_TSBATCH", "0")
    assert not SC._fuse("TSBATCH")
