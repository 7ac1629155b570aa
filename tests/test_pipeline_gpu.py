"""Prompt-level multi-stream pipelining (``DataParallelGenerator.run_many``) on the GPU: job n's VAE
decode runs on a side stream while job n+1 samples; results equal the one-job-at-a-time path."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_run_many_pipelined_matches_sequential(cuda):
    from comfy_gen_server_amd.parallel.dp import DataParallelGenerator, Job
    from comfy_gen_server_amd.tools.synth import build_pipeline
    with torch.inference_mode():
        patcher, clip, vae = build_pipeline("tiny", device=cuda, dtype=torch.bfloat16, seed=5)
        gen = DataParallelGenerator(patcher, clip, vae)
        jobs = [Job(batch=2, steps=4, seed=s, width=128, height=128) for s in (11, 12, 13)]
        seq = [gen.run(j).clone() for j in jobs]
        torch.cuda.synchronize()
        piped = [x.clone() for x in gen.run_many(iter(jobs), pipeline=True)]
        torch.cuda.synchronize()
    assert len(piped) == 3
    for a, b in zip(piped, seq):
        assert a.shape == b.shape and a.dtype == torch.uint8
        assert (a.int() - b.int()).abs().max().item() <= 1


@pytest.mark.parametrize("family", ["sd15", "sd21", "sdxl_refiner"])
def test_family_pipeline_captures_and_stays_native(cuda, family):
    """Full-size SD1.5 / SD2.x / SDXL-refiner architectures (random init) through CLIP -> captured Euler-a
    steps -> VAE: every step graph captures (no silent eager fallback, as Stable Cascade had) and no op
    leaves the HIP kernels for a vendor library."""
    from comfy_gen_server_amd import ops
    from comfy_gen_server_amd.parallel.dp import Job, generate_local
    from comfy_gen_server_amd.sampling import step_graph
    from comfy_gen_server_amd.tools.synth import build_pipeline
    with torch.inference_mode():
        patcher, clip, vae = build_pipeline(family, device=cuda, dtype=torch.bfloat16, seed=3)
        before = dict(step_graph.stats)
        ops.reset_stats()
        img = generate_local(patcher, clip, vae, Job(batch=2, steps=4, seed=7, width=256, height=256), 0, 2)
        torch.cuda.synchronize()
    st = ops.stats()
    lib = {k: v for k, v in st.items() if k[1] == "lib"}
    assert not lib, lib
    assert step_graph.stats.get("capture_failed", 0) == before.get("capture_failed", 0)
    assert step_graph.stats["replay"] > before["replay"]
    assert img.shape[0] == 2 and torch.isfinite(img.float()).all()


def test_taesd_preview_is_async_on_gpu(cuda):
    """TAESD previews decode on a side stream: a step's call returns at once (an earlier preview or
    None), never more than `depth` decodes are queued, and the blocking last call returns the newest
    step's image, equal to a direct decode."""
    import numpy as np
    from comfy_gen_server_amd.models.layers import init_random_
    from comfy_gen_server_amd.models.taesd import TAESD
    from comfy_gen_server_amd.utils.preview import TAESDPreviewerImpl
    t = TAESD(None, None, latent_channels=4)
    init_random_(t, seed=3)
    t = t.to(cuda)
    prev = TAESDPreviewerImpl(t)
    xs = [torch.randn(1, 4, 64, 64, device=cuda) for _ in range(6)]
    with torch.inference_mode():
        outs = [prev.decode_latent_to_preview_image("JPEG", x, block=(i == 5)) for i, x in enumerate(xs)]
        ref = t.decode(xs[-1])[0].movedim(0, 2).clamp(0, 1).float().cpu()
    assert prev.submitted + prev.skipped == 6 and len(prev._pending) == 0
    last = outs[-1][1]
    got = torch.from_numpy(np.asarray(last).astype(np.float32)) / 255.0
    assert last.size == (512, 512)
    assert (got - ref).abs().max() <= 2.0 / 255, (got - ref).abs().max()
