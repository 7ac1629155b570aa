"""Deferred PNG saves (utils/imageio.py): a thread that opted in gets its encodes back as futures, the
files appear whole (``.part`` + rename) once they finish, ``pending`` names the in-flight ones for
``/view``; threads that did not opt in keep synchronous saves."""
import os
import threading

import numpy as np
import torch
from PIL import Image

from comfy_gen_server_amd.utils import imageio


def test_deferred_saves_complete_and_are_collected(tmp_path):
    imgs = torch.rand(3, 64, 48, 3)
    out = {}

    def worker():
        imageio.defer_saves(True)
        names = imageio.save_png_batch(imgs, str(tmp_path), "deferred", 1, {"prompt": "{}"})
        futs = imageio.take_pending()
        out["names"], out["futs"] = names, futs
        out["errs"] = imageio.wait_futures(futs)
        out["again"] = imageio.take_pending()
    t = threading.Thread(target=worker)
    t.start()
    t.join()
    assert len(out["futs"]) == 3 and out["errs"] == [] and out["again"] == []
    for i, n in enumerate(out["names"]):
        p = tmp_path / n
        assert imageio.pending(str(p)) is None
        arr = np.asarray(Image.open(p))
        ref = (imgs[i].clamp(0, 1) * 255 + 0.5).to(torch.uint8).numpy()
        assert arr.shape == (64, 48, 3) and np.array_equal(arr, ref)
    assert not [f for f in os.listdir(tmp_path) if f.endswith(".part")]


def test_saves_stay_synchronous_without_opt_in(tmp_path):
    names = imageio.save_png_batch(torch.rand(2, 16, 16, 3), str(tmp_path), "sync", 1)
    assert imageio.take_pending() == []
    assert all(os.path.getsize(tmp_path / n) > 0 for n in names)


def test_prompt_completions_ordered_with_snapshot_outputs(monkeypatch):
    """Prompt N's slow PNG encode finishes behind prompt N+1's execute(), which rewrites the
    executor's outputs_ui in place: /history must still get N's own outputs, in submission order,
    and a failing encode wait must still complete the prompt (main._OrderedFinisher)."""
    import concurrent.futures as cf
    import time

    from comfy_gen_server_amd import main as M
    from comfy_gen_server_amd.graph import executor as X

    pool = cf.ThreadPoolExecutor(2)

    class FakeExec:
        def __init__(self, server):
            self.outputs_ui, self.success, self.status_messages = {}, True, []

        def execute(self, prompt, prompt_id, extra, outs):
            self.outputs_ui.pop("9", None)                      # the executor's in-place rewrite
            self.outputs_ui["9"] = {"images": [f"{prompt_id}.png"]}
            delay = prompt["delay"]
            imageio._tl.futs = [pool.submit(time.sleep, delay)]
            if prompt.get("fail"):
                def boom():
                    time.sleep(0.05)
                    raise OSError("disk full")
                imageio._tl.futs.append(pool.submit(boom))

        def reset(self):
            pass

    monkeypatch.setattr(X, "PromptExecutor", FakeExec)

    class Q:
        class ExecutionStatus(dict):
            def __init__(self, **kw):
                super().__init__(**kw)

        def __init__(self, items):
            self.items, self.done = list(items), []

        def get(self, timeout=None):
            if self.items:
                return self.items.pop(0)
            time.sleep(0.01)
            return None

        def task_done(self, item_id, outputs, status):
            self.done.append((item_id, outputs, status["status_str"]))

        def get_flags(self):
            return {}

    class S:
        client_id, last_prompt_id, last_node_id = None, None, None

        def __init__(self):
            self.metrics = {"prompts_total": 0, "execution_seconds_total": 0.0, "prompts_failed": 0}

        def send_sync(self, *a, **k):
            pass

    items = [((0, "p1", {"delay": 0.4}, {}, []), 1), ((1, "p2", {"delay": 0.0}, {}, []), 2),
             ((2, "p3", {"delay": 0.0, "fail": True}, {}, []), 3)]
    q, srv, stop = Q(items), S(), threading.Event()
    fin = M._OrderedFinisher()
    t = threading.Thread(target=M.prompt_worker, args=(q, srv, stop), kwargs={"finisher": fin}, daemon=True)
    t.start()
    t0 = time.time()
    while len(q.done) < 3 and time.time() - t0 < 10:
        time.sleep(0.01)
    stop.set()
    t.join(5)
    assert [d[0] for d in q.done] == [1, 2, 3]
    assert q.done[0][1] == {"9": {"images": ["p1.png"]}} and q.done[1][1] == {"9": {"images": ["p2.png"]}}
    assert [d[2] for d in q.done] == ["success", "success", "error"]
    assert srv.metrics["prompts_total"] == 3 and srv.metrics["prompts_failed"] == 1
    pool.shutdown()
