"""The workload models' pooling on the HIP kernels: fp8a_avg_pool2d_plane (MobileNetV2's head
nn.AvgPool2d(input_size // 32), models/mobilenet_v2.py) against ATen's avg_pool2d on the same
device -- the window summed in row-major order in fp32 and divided once, so the same bits."""
import pytest
import torch
from torch import nn

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.mark.parametrize("shape,k,s", [((512, 1280, 7, 7), 7, 7), ((3, 5, 7, 7), 7, 7), ((2, 3, 9, 8), (7, 6), (3, 4)),
                                       ((4, 6, 14, 14), 14, 14), ((1, 2, 1, 1), 1, 1), ((2, 129, 8, 8), 8, 8)])
def test_avg_pool_plane_matches_aten(shape, k, s):
    from fp8_quantization_amd import _lib
    from fp8_quantization_amd.approx_ops import AvgPool2d
    g = torch.Generator().manual_seed(shape[1])
    x = (torch.randn(*shape, generator=g) * 3).to(DEV)
    x.view(-1)[min(5, x.numel() - 2)] = float("inf")
    x.view(-1)[-1] = float("nan")
    m = AvgPool2d(k, s)
    assert isinstance(m, nn.AvgPool2d)
    orig = nn.functional.avg_pool2d
    try:
        nn.functional.avg_pool2d = lambda *a, **kw: (_ for _ in ()).throw(AssertionError("torch pooling"))
        y = m(x)
    finally:
        nn.functional.avg_pool2d = orig
    ref = orig(x, k, s)
    assert y.shape == ref.shape
    assert torch.equal(torch.isnan(y), torch.isnan(ref))
    fin = ~torch.isnan(ref)
    assert torch.equal(y[fin], ref[fin])
    with pytest.raises(AssertionError):  # a window with more than one output per plane
        L = _lib.load()
        _lib.check(L.fp8a_avg_pool2d_plane(_lib.dev_ptr(x), _lib.dev_ptr(y), shape[0], shape[1], shape[2] * 2,
                                           shape[3], shape[2], shape[3], 1, 1, _lib.stream_ptr(x.device)), "pool")


def test_avg_pool_other_geometry_runs_torch():
    from fp8_quantization_amd.approx_ops import AvgPool2d
    x = torch.randn(2, 3, 14, 14, device=DEV)
    assert torch.equal(AvgPool2d(7)(x), nn.functional.avg_pool2d(x, 7))
