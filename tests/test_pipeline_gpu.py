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
