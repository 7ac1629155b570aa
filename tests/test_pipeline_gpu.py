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
