"""Device RNG kernels (csrc/kernels/rng.hip, K18) vs their bit-exact torch mirror (sampling/rng.py).

The uniforms are 24-bit exact on both sides; only libm-level differences of log/sin/cos remain,
so the tolerance is a few fp32 ulps."""
import pytest
import torch

from comfy_gen_server_amd import ops, _native

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _native_loaded(cuda):
    assert _native.load_kernels() is not None, _native.kernels_error()
    ops.reset_stats()
    yield


@pytest.mark.parametrize("shape,inds,stream", [((3, 4, 8, 8), [0, 1, 2], 0), ((2, 4, 128, 128), [5, 6], 19),
                                               ((1, 3, 5, 7), [9], 2), ((4, 16, 24, 24), [100, 101, 102, 103], 7)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_philox_randn_matches_mirror(cuda, shape, inds, stream, dtype):
    z = ops.philox_randn(shape, 1234567, inds, stream, device=cuda, dtype=dtype)
    assert ops.stats().get(("rng", "hip"), 0) >= 1
    ref = ops.philox_randn(shape, 1234567, inds, stream).to(dtype)
    tol = 2e-5 if dtype == torch.float32 else 1e-2
    assert torch.allclose(z.cpu().float(), ref.float(), atol=tol, rtol=tol), (z.cpu().float() - ref.float()).abs().max()


def test_philox_randn_device_step(cuda):
    step = torch.tensor([3], dtype=torch.int64, device=cuda)
    z = ops.philox_randn((2, 4, 16, 16), 5, [0, 1], 10, device=cuda, dev_step=step)
    ref = ops.philox_randn((2, 4, 16, 16), 5, [0, 1], 13)
    assert torch.allclose(z.cpu(), ref, atol=2e-5)


def test_philox_randn_statistics(cuda):
    z = ops.philox_randn((8, 4, 128, 128), 42, range(8), 0, device=cuda).double()
    assert abs(z.mean().item()) < 5e-3 and abs(z.std().item() - 1) < 5e-3
    assert abs((z ** 4).mean().item() - 3) < 0.05          # Gaussian kurtosis
    c = torch.corrcoef(z.view(8, -1))
    assert (c - torch.eye(8, dtype=c.dtype, device=c.device)).abs().max() < 0.02


def test_euler_ancestral_philox_equals_unfused(cuda):
    torch.manual_seed(0)
    x = torch.randn(3, 4, 32, 32, device=cuda)
    den = torch.randn(3, 4, 32, 32, device=cuda)
    fused = ops.euler_ancestral_philox(x, den, 2.5, 1.7, 0.9, 99, [4, 5, 6], 11)
    noise = ops.philox_randn(x.shape, 99, [4, 5, 6], 11, device=cuda)
    ref = x + (x - den) / 2.5 * (1.7 - 2.5) + noise * 0.9
    assert torch.allclose(fused, ref, atol=1e-5, rtol=1e-5)
    assert ops.stats().get(("euler", "hip"), 0) >= 1


@pytest.mark.parametrize("ta,tb", [(1.0, 1.5), (0.1, 3.9), (2.0, 2.0001), (0.0, 4.0)])
def test_brownian_increment_matches_mirror(cuda, ta, tb):
    shape = (2, 4, 16, 16)
    w = ops.brownian_increment(shape, 7, [3, 4], 0.0, 4.0, ta, tb, 1e-4, 24, 1.0, device=cuda)
    ref = ops.brownian_increment(shape, 7, [3, 4], 0.0, 4.0, ta, tb, 1e-4, 24, 1.0)
    assert torch.allclose(w.cpu(), ref, atol=5e-5, rtol=1e-4), (w.cpu() - ref).abs().max()


def test_brownian_increment_variance_and_additivity(cuda):
    shape = (4, 4, 64, 64)
    inc = lambda a, b: ops.brownian_increment(shape, 1, range(4), 0.0, 8.0, a, b, 1e-4, 24, 1.0, device=cuda)  # noqa
    w = inc(1.0, 3.0).double()
    assert abs(w.var().item() - 2.0) < 0.05
    # W(3)-W(1) = (W(2)-W(1)) + (W(3)-W(2)) from the same tree
    assert torch.allclose(inc(1.0, 2.0) + inc(2.0, 3.0), inc(1.0, 3.0), atol=1e-4)
