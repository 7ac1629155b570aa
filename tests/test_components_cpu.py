"""CPU tests for smaller components that had no direct test: the prompt-queue journal,
the image-format decorator (C17), the latent2rgb previewer (C16), latent formats (C35) and
hypernetwork patches (C53)."""
import numpy as np
import torch

from comfy_gen_server_amd.graph.queue import PromptQueue
from comfy_gen_server_amd.runtime import latent_formats as LF
from comfy_gen_server_amd.utils import image_format as IF
from comfy_gen_server_amd.utils.preview import Latent2RGBPreviewer


class _Srv:
    def __init__(self):
        self.updates = 0

    def queue_updated(self):
        self.updates += 1


def test_queue_journal_replays_pending_and_history(tmp_path):
    j = str(tmp_path / "queue.jsonl")
    q = PromptQueue(_Srv(), journal_path=j)
    q.put((0, "p-a", {"1": {}}, {}, ["1"]))
    q.put((1, "p-b", {"2": {}}, {}, ["2"]))
    item, i = q.get(timeout=1)
    assert item[1] == "p-a"
    q.task_done(i, {"1": {"images": []}})
    # a restarted server replays the journal: p-b is still queued, p-a is in history
    q2 = PromptQueue(_Srv(), journal_path=j)
    running, pending = q2.get_current_queue()
    assert running == [] and [p[1] for p in pending] == ["p-b"]
    assert "p-a" in q2.history and q2.history["p-a"]["outputs"] == {"1": {"images": []}}


def test_queue_journal_one_record_per_mutation_and_replay(tmp_path):
    """Every mutation is one journal record (deleting the last pending item is one ``delete``, not a
    delete plus a wipe); history deletes / wipes and queue deletes survive a restart; a torn last line
    (crash mid-write) is ignored."""
    import json
    j = tmp_path / "queue.jsonl"
    q = PromptQueue(_Srv(), journal_path=str(j))
    for n, pid in enumerate(["a", "b", "c", "d"]):
        q.put((n, pid, {}, {}, []))
    assert q.delete_queue_item(lambda it: it[1] == "b")
    for _ in range(2):
        item, i = q.get(timeout=1)
        q.task_done(i, {}, q.ExecutionStatus("success", True, []))
    q.delete_history_item("a")
    assert q.delete_queue_item(lambda it: it[1] == "d")            # the last pending item
    assert not q.delete_queue_item(lambda it: it[1] == "zz")
    ops = [json.loads(ln)["op"] for ln in j.read_text().splitlines()]
    assert ops == ["put"] * 4 + ["delete", "done", "done", "history_delete", "delete"], ops
    with open(j, "a") as f:
        f.write('{"op": "put", "item": [9, "torn"')               # crash mid-write
    q2 = PromptQueue(_Srv(), journal_path=str(j))
    assert q2.get_current_queue() == ([], []) and list(q2.history) == ["c"]
    assert q2.history["c"]["status"]["status_str"] == "success"
    q2.put((10, "e", {}, {}, []))
    q2.wipe_history()
    q3 = PromptQueue(_Srv(), journal_path=str(j))
    assert q3.history == {} and [it[1] for it in q3.get_current_queue()[1]] == ["e"]
    assert q3.get_history(max_items=5) == {}


def test_image_format_decorator_converts_by_annotation():
    img = torch.rand(1, 12, 10, 3)
    seen = {}

    @IF.convert_image_format
    def takes_tensor(image: torch.Tensor):
        seen["t"] = image
        return image

    @IF.convert_image_format
    def takes_bytes(data: bytes):
        seen["b"] = data
        return data

    png = takes_bytes(img)
    assert isinstance(png, bytes) and png[:8] == b"\x89PNG\r\n\x1a\n"
    t = takes_tensor(png)
    assert t.shape[-3:] == (12, 10, 3)
    assert (t.reshape(12, 10, 3) - img[0]).abs().max() <= 1.0 / 255 + 1e-6   # 8-bit round trip


def test_latent2rgb_preview_cpu_matches_linear_map():
    fmt = LF.SDXL()
    prev = Latent2RGBPreviewer(fmt.latent_rgb_factors)
    x0 = torch.randn(2, 4, 6, 5)
    pil = prev.decode_latent_to_preview(x0)
    assert pil.size == (5, 6)
    f = torch.tensor(fmt.latent_rgb_factors)
    ref = ((torch.einsum("chw,cr->hwr", x0[0], f) + 1.0) / 2.0).clamp(0, 1)
    got = torch.from_numpy(np.asarray(pil).astype(np.float32)) / 255.0
    assert (got - ref).abs().max() <= 1.0 / 255 + 1e-6


def test_latent_formats_scale_round_trip():
    for cls, scale in ((LF.SD15, 0.18215), (LF.SDXL, 0.13025)):
        fmt = cls()
        assert abs(fmt.scale_factor - scale) < 1e-9
        z = torch.randn(1, 4, 8, 8)
        assert torch.allclose(fmt.process_out(fmt.process_in(z)), z, atol=1e-6)


def test_hypernetwork_patch_from_file(tmp_path):
    from comfy_gen_server_amd.nodes.extras_merge import load_hypernetwork_patch
    torch.manual_seed(0)

    def mlp_sd(dim, hidden):
        return {"linear.0.weight": torch.randn(hidden, dim) * 0.1, "linear.0.bias": torch.zeros(hidden),
                "linear.1.weight": torch.randn(dim, hidden) * 0.1, "linear.1.bias": torch.zeros(dim)}
    sd = {768: [mlp_sd(768, 32), mlp_sd(768, 32)], "activation_func": "relu", "is_layer_norm": False}
    path = str(tmp_path / "hn.pt")
    torch.save(sd, path)
    patch = load_hypernetwork_patch(path, 0.5)
    assert patch is not None and 768 in patch.hypernet
    q, k, v = torch.randn(1, 5, 320), torch.randn(1, 7, 768), torch.randn(1, 7, 768)
    q2, k2, v2 = patch(q, k, v, {})
    w = sd[768][0]
    ref_k = k + (torch.relu(k @ w["linear.0.weight"].T) @ w["linear.1.weight"].T) * 0.5
    assert torch.equal(q2, q) and torch.allclose(k2, ref_k, atol=1e-5)
    # other context widths pass through untouched
    k3 = torch.randn(1, 7, 1024)
    assert torch.equal(patch(q, k3, k3, {})[1], k3)


def test_taesd_preview_cpu_matches_direct_decode():
    """TAESD previews share the async previewer (side stream on the GPU); on the CPU the image is the
    direct decode of the first latent."""
    from comfy_gen_server_amd.models.layers import init_random_
    from comfy_gen_server_amd.models.taesd import TAESD
    from comfy_gen_server_amd.utils.preview import TAESDPreviewerImpl
    t = TAESD(None, None, latent_channels=4)
    init_random_(t, seed=3)
    prev = TAESDPreviewerImpl(t)
    x0 = torch.randn(2, 4, 8, 8)
    fmt, pil, res = prev.decode_latent_to_preview_image("JPEG", x0)
    with torch.no_grad():
        ref = t.decode(x0[:1])[0].movedim(0, 2).clamp(0, 1)
    got = torch.from_numpy(np.asarray(pil).astype(np.float32)) / 255.0
    assert pil.size == (64, 64) and fmt == "JPEG" and res == 512
    assert (got - ref).abs().max() <= 1.0 / 255 + 1e-5
