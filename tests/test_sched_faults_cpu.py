"""Failure handling of the node-wide serving cluster (sched/cluster.py, sched/spmd.py) on the CPU,
through the prompt API with injected faults (``CGS_FAULT``, utils/telemetry.py):

* a node that raises on ONE rank of an SPMD prompt stops every rank at the same agreement point:
  the prompt reports the error, no rank hangs, and the next SPMD prompt runs normally;
* a rank that DIES inside the sampler of an SPMD prompt: the prompt is re-run on the surviving rank
  prefix (its shards re-queued to the survivors) and resolves within 60 s; a replacement rank is
  spawned, the node re-rendezvouses (generation 1), and the next batch-6 prompt runs on all 3 ranks.
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


def test_rank_death_mid_prompt_reruns_on_survivors_and_node_recovers(tmp_path_factory, fault_env):
    fault_env("node_exit:KSampler@2")                  # rank 2 exits inside its first KSampler
    proc, url, base = _start(tmp_path_factory, 3)
    try:
        t0 = time.time()
        a = _post(url + "/prompt", {"prompt": _graph(7, 6, "died")})["prompt_id"]
        ha = _wait(url, [a], timeout=120)[a]
        dt = time.time() - t0
        more = [_post(url + "/prompt", {"prompt": _graph(30 + i, 1, f"after{i}")})["prompt_id"] for i in range(3)]
        hm = _wait(url, more, timeout=120)
        deadline = time.time() + 180                   # the replacement rank comes up; the node regroups
        while time.time() < deadline:
            cl = _get(url + "/system_stats")["cluster"]
            if cl["generation"] >= 1 and not cl["dead"]:
                break
            time.sleep(0.5)
        b = _post(url + "/prompt", {"prompt": _graph(8, 6, "whole")})["prompt_id"]
        hb = _wait(url, [b], timeout=120)[b]
        stats = _get(url + "/queue")
    finally:
        _stop(proc)
    assert ha["status"]["status_str"] == "success", ha["status"]
    assert ha["metrics"]["ranks"] == [0, 1], ha["metrics"]      # re-run SPMD on the surviving prefix
    assert ha["metrics"]["images_per_rank"] == {"0": 3, "1": 3}, ha["metrics"]
    assert len(_images(base, ha)) == 6
    assert dt < 60, dt
    assert all(e["status"]["status_str"] == "success" for e in hm.values())
    assert cl["generation"] >= 1 and cl["dead"] == [], cl
    assert hb["status"]["status_str"] == "success", hb["status"]
    assert hb["metrics"]["ranks"] == "all" and hb["metrics"]["images_per_rank"] == {"0": 2, "1": 2, "2": 2}
    assert len(_images(base, hb)) == 6
    assert stats["queue_running"] == [] and stats["queue_pending"] == []


def test_failed_sharded_save_leaves_no_placeholders(tmp_path_factory, fault_env):
    """Rank 1 fails inside SaveImage after rank 0 reserved the batch's names: the prompt fails and the
    names rank 1 never wrote are removed (no zero-byte PNGs); the other ranks' images stay whole."""
    import os
    fault_env("node:SaveImageWrite@1")
    proc, url, base = _start(tmp_path_factory, 3)
    try:
        a = _post(url + "/prompt", {"prompt": _graph(9, 6, "half")})["prompt_id"]
        ha = _wait(url, [a], timeout=120)[a]
    finally:
        _stop(proc)
    assert ha["status"]["status_str"] == "error", ha["status"]
    files = [f for f in os.listdir(os.path.join(base, "output")) if f.startswith("half")]
    sizes = {f: os.path.getsize(os.path.join(base, "output", f)) for f in files}
    assert len(files) == 4 and all(v > 0 for v in sizes.values()), sizes
