"""Failure handling of the node-wide serving cluster (sched/cluster.py, sched/spmd.py) on the CPU,
through the prompt API with injected faults (``CGS_FAULT``, utils/telemetry.py):

* a node that raises on ONE rank of an SPMD prompt stops every rank at the same agreement point:
  the prompt reports the error, no rank hangs, and the next SPMD prompt runs normally;
* a rank that DIES inside the sampler: the prompt is re-run whole on a surviving rank and resolves
  within 60 s; later prompts keep running on the survivors.
"""
import time

import pytest

from test_sched_cpu import _get, _graph, _images, _post, _start, _stop, _wait


@pytest.fixture
def fault_env(monkeypatch):
    def set_(spec):
        monkeypatch.setenv("CGS_FAULT", spec)
    return set_


def test_node_error_on_one_rank_fails_the_prompt_on_every_rank(tmp_path_factory, fault_env):
    fault_env("node:VAEDecode@1")                      # rank 1's first VAEDecode raises
    proc, url, base = _start(tmp_path_factory, 3)
    try:
        a = _post(url + "/prompt", {"prompt": _graph(5, 6, "fail")})["prompt_id"]
        ha = _wait(url, [a], timeout=120)[a]
        b = _post(url + "/prompt", {"prompt": _graph(6, 6, "ok")})["prompt_id"]
        hb = _wait(url, [b], timeout=120)[b]
    finally:
        _stop(proc)
    assert ha["status"]["status_str"] == "error", ha["status"]
    msgs = [m for m in ha["status"]["messages"] if m[0] == "execution_error"]
    assert any("injected fault" in str(m[1].get("exception_message", "")) for m in msgs), msgs
    assert hb["status"]["status_str"] == "success", hb["status"]
    assert hb["metrics"]["ranks"] == "all" and len(_images(base, hb)) == 6


def test_rank_death_mid_prompt_reruns_on_survivors(tmp_path_factory, fault_env):
    fault_env("node_exit:KSampler@2")                  # rank 2 exits inside its first KSampler
    proc, url, base = _start(tmp_path_factory, 3)
    try:
        t0 = time.time()
        a = _post(url + "/prompt", {"prompt": _graph(7, 6, "died")})["prompt_id"]
        ha = _wait(url, [a], timeout=120)[a]
        dt = time.time() - t0
        more = [_post(url + "/prompt", {"prompt": _graph(30 + i, 1, f"after{i}")})["prompt_id"] for i in range(3)]
        hm = _wait(url, more, timeout=120)
        stats = _get(url + "/queue")
    finally:
        _stop(proc)
    assert ha["status"]["status_str"] == "success", ha["status"]
    assert isinstance(ha["metrics"]["ranks"], int) and ha["metrics"]["ranks"] != 2   # re-run on a survivor
    assert len(_images(base, ha)) == 6
    assert dt < 60, dt
    assert all(e["status"]["status_str"] == "success" for e in hm.values())
    assert {e["metrics"]["ranks"] for e in hm.values()} <= {0, 1}
    assert stats["queue_running"] == [] and stats["queue_pending"] == []
