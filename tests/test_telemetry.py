"""Observability and failure-injection hooks: per-node and per-step
counters, Prometheus lines, per-prompt profiler traces, injected node / OOM / step faults becoming
structured execution errors while the executor keeps serving, JSON logs."""
import json
import logging
import os

import pytest

from test_e2e_cpu import env, graph  # noqa: F401


def _run(p, pid):
    from comfy_gen_server_amd.graph.executor import PromptExecutor
    from comfy_gen_server_amd.graph.validation import validate_prompt
    ok, err, outputs, node_errors = validate_prompt(p)
    assert ok, (err, node_errors)
    ex = PromptExecutor()
    ex.execute(p, pid, {}, outputs)
    return ex


def test_counters_and_prometheus(env):  # noqa: F811
    from comfy_gen_server_amd.utils import telemetry
    before = telemetry.snapshot()
    ex = _run(graph(seed=11, steps=3), "tele-1")
    assert ex.success
    snap = telemetry.snapshot()
    assert snap["sampler_steps_total"] - before.get("sampler_steps_total", 0) == 3
    assert snap["nodes"]["KSampler"]["calls"] >= 1 and snap["nodes"]["VAEDecode"]["seconds"] > 0
    assert snap["images_saved_total"] >= 2 and snap["sampler_step_ms_avg"] > 0
    text = "\n".join(telemetry.prometheus_lines())
    assert "cgs_sampler_steps_total" in text and 'cgs_node_seconds_total{class_type="KSampler"}' in text


@pytest.mark.parametrize("spec,kind", [("node:VAEDecode", "InjectedFault"), ("oom:KSampler", "OutOfMemoryError"),
                                       ("step:1", "InjectedFault")])
def test_injected_faults_become_execution_errors(env, monkeypatch, spec, kind):  # noqa: F811
    monkeypatch.setenv("CGS_FAULT", spec + "!")
    ex = _run(graph(seed=12, steps=2), "fault-1")
    assert not ex.success
    err = [m for m in ex.status_messages if m[0] == "execution_error"]
    assert err and kind in err[0][1]["exception_type"]
    monkeypatch.delenv("CGS_FAULT")
    assert _run(graph(seed=12, steps=2), "fault-2").success      # executor keeps serving


def test_profile_trace_per_prompt(env, tmp_path, monkeypatch):  # noqa: F811
    from comfy_gen_server_amd.utils import telemetry
    monkeypatch.setenv("CGS_PROFILE_DIR", str(tmp_path))
    with telemetry.maybe_profile("prof-1"):
        assert _run(graph(seed=13, steps=1), "prof-1").success
    trace = json.load(open(tmp_path / "prof-1.json"))
    names = {e.get("name", "") for e in trace.get("traceEvents", [])}
    assert any(n.startswith("node:KSampler") for n in names) and "prompt:prof-1" in names


def test_json_logs(capsys):
    from comfy_gen_server_amd.utils.telemetry import JsonFormatter
    rec = logging.LogRecord("cgs", logging.INFO, __file__, 1, "hello %s", ("world",), None)
    d = json.loads(JsonFormatter().format(rec))
    assert d["msg"] == "hello world" and d["level"] == "INFO"


@pytest.mark.parametrize("site", ["vae_decode", "vae_encode"])
def test_vae_oom_falls_back_to_tiled(monkeypatch, caplog, site):
    """An HBM OOM in the batched VAE pass retries as the 3-pass tiled pass (reference
    comfy/sd.py:300-302 / 326-328), driven by the ``oom:vae_*`` fault site."""
    import logging
    import torch
    from comfy_gen_server_amd.runtime import device as dm
    from comfy_gen_server_amd.tools.synth import build_pipeline
    from comfy_gen_server_amd.utils import telemetry
    dm.set_cpu_mode(True)
    _, _, vae = build_pipeline("tiny", device=torch.device("cpu"), dtype=torch.float32, seed=1, with_clip=False)
    g = torch.Generator().manual_seed(0)
    lat = torch.randn(1, 4, 8, 8, generator=g)
    px = torch.rand(1, 64, 64, 3, generator=g)
    ref = vae.decode(lat) if site == "vae_decode" else vae.encode(px)
    monkeypatch.setenv("CGS_FAULT", f"oom:{site}")
    telemetry._fired.clear()
    with caplog.at_level(logging.WARNING):
        out = vae.decode(lat) if site == "vae_decode" else vae.encode(px)
    assert any("retrying with tiled" in r.message for r in caplog.records)
    assert out.shape == ref.shape
    assert (out - ref).abs().max().item() < 1e-3   # tiles cover the whole (small) input: same result
