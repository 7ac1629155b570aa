"""SPMD sharding of per-image conditioning and masks (sched/spmd.py), checked directly:

* ControlNet hint batches (and the hints of a chained ControlNet), ``concat_latent_image`` /
  ``concat_mask`` and batch-sized cond tensors are cut to the rank's ``[off, off + n)`` window; batch-1
  conditioning is left alone and the caller's objects are never mutated;
* a LATENT that is already sharded (second sampler) gets its full-batch ``noise_mask`` sliced;
* a batch smaller than the node runs replicated (no empty shards).
"""
import torch

from comfy_gen_server_amd.runtime.controlnet import ControlBase
from comfy_gen_server_amd.sched import spmd


class _CN(ControlBase):
    def copy(self):
        c = _CN()
        self.copy_to(c)
        return c


class _Comm:
    def __init__(self, rank, world):
        self.rank, self.world, self.enabled = rank, world, True


def _ctx(rank, world):
    c = spmd.SPMD.__new__(spmd.SPMD)
    c.comm = _Comm(rank, world)
    c.rank, c.world = rank, world
    c.images_sampled = 0
    c.mode = "spmd"
    c.latency = None
    c._seq, c._stage = 0, 2
    return c


def test_shard_conds_slices_batch_sized_conditioning():
    total, off, n = 6, 2, 2
    hint = torch.arange(total, dtype=torch.float32).reshape(total, 1, 1, 1).expand(total, 3, 8, 8).contiguous()
    prev = _CN().set_cond_hint(hint * 10)
    cn = _CN().set_cond_hint(hint)
    cn.set_previous_controlnet(prev)
    one = _CN().set_cond_hint(hint[:1])                     # batch-1 hint: broadcast, not sliced
    cli = torch.arange(total, dtype=torch.float32).reshape(total, 1, 1, 1).expand(total, 4, 4, 4)
    cond = torch.randn(total, 77, 32)                        # one prompt per image
    conds = [[cond, {"control": cn, "concat_latent_image": cli, "concat_mask": cli[:, :1], "pooled_output":
                     torch.randn(1, 32)}],
             [torch.randn(1, 77, 32), {"control": one}]]
    out = spmd.shard_conds(conds, (off, n, total))
    c0 = out[0][1]
    assert torch.equal(out[0][0], cond[off:off + n])
    assert torch.equal(c0["control"].cond_hint_original[:, 0, 0, 0], torch.tensor([2.0, 3.0]))
    assert torch.equal(c0["control"].previous_controlnet.cond_hint_original[:, 0, 0, 0], torch.tensor([20.0, 30.0]))
    assert torch.equal(c0["concat_latent_image"][:, 0, 0, 0], torch.tensor([2.0, 3.0]))
    assert c0["concat_mask"].shape[0] == n and c0["pooled_output"].shape[0] == 1
    assert out[1][1]["control"] is one                       # nothing to cut: same object
    # the caller's conditioning is untouched
    assert cn.cond_hint_original.shape[0] == total and prev.cond_hint_original.shape[0] == total
    assert conds[0][1]["concat_latent_image"].shape[0] == total
    assert spmd.shard_conds(conds, None) is conds


def test_shard_latent_second_sampler_and_replicated_small_batch():
    ctx = _ctx(1, 3)
    mask = torch.arange(6, dtype=torch.float32).reshape(6, 1, 1, 1)
    with spmd.activate(ctx):
        # first sampler: shard of rank 1 of 6 images = [2, 4)
        local, inds, shard = spmd.shard_latent({"samples": torch.zeros(6, 4, 8, 8), "noise_mask": mask})
        assert shard == (2, 2, 6) and inds == [2, 3] and local["samples"].shape[0] == 2
        assert torch.equal(local["noise_mask"].flatten(), torch.tensor([2.0, 3.0]))
        # second sampler on the already-sharded latent, full-batch mask set in between
        local2, inds2, shard2 = spmd.shard_latent({"samples": local["samples"], "dp_shard": shard,
                                                  "noise_mask": mask})
        assert shard2 == shard and inds2 == [2, 3]
        assert torch.equal(local2["noise_mask"].flatten(), torch.tensor([2.0, 3.0]))
        # 2 images on 3 ranks: replicated, never an empty shard
        local3, inds3, shard3 = spmd.shard_latent({"samples": torch.zeros(2, 4, 8, 8)})
        assert shard3 is None and local3["samples"].shape[0] == 2
    assert ctx.images_sampled == 2 + 2 + 2


def test_prompt_batch_traces_the_sampler_input():
    from comfy_gen_server_amd.sched.cluster import choose_mode, prompt_batch
    g = {"1": {"class_type": "LoadImage", "inputs": {"image": "x.png"}},
         "2": {"class_type": "RepeatImageBatch", "inputs": {"image": ["1", 0], "amount": 8}},
         "4": {"class_type": "CheckpointLoaderSimple", "inputs": {"ckpt_name": "m"}},
         "5": {"class_type": "VAEEncodeForInpaint", "inputs": {"pixels": ["2", 0], "vae": ["4", 2],
                                                               "mask": ["6", 0], "grow_mask_by": 6}},
         "6": {"class_type": "SolidMask", "inputs": {"value": 1.0, "width": 64, "height": 64}},
         "3": {"class_type": "KSampler", "inputs": {"latent_image": ["5", 0], "model": ["4", 0]}}}
    assert prompt_batch(g) == 8 and choose_mode(g, {}, 8) == "spmd"
    g["2"]["inputs"]["amount"] = 1
    assert prompt_batch(g) == 1 and choose_mode(g, {}, 8) == "single"
