"""The depthwise forms conv_dwx_kernel (band-staged) and conv_dwg_kernel (fp32 gather)
(csrc/conv_tbx.h) against the word-image form conv_tbx_kernel on E4M3 depthwise layers.

All compute the same tensor-bias table terms in the same (ky, kx) order, so the outputs must be
BIT-identical; conv_tbx_kernel itself is pinned to the oracle per term and per layer in
tests/test_gpu_tbx.py (which runs on the default form).  Covered here: every MobileNetV2 depthwise shape
(batch 2), ragged widths (Wo % 4 != 0, 1-pixel planes), a 5x3 kernel with dilation, the fused
input quantizer (qin), the BN + ReLU6 epilogue, and an off-grid input (gate raised: both return
the gated exact kernel's result).  The per-launch path option is fp8a_set_option("dwx", 0 / 1 / 2 / 3).
"""
import numpy as np
import pytest
import torch
from torch import nn

from tests import golden_io as gio

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
E, M = 4, 3


@pytest.fixture(scope="module", autouse=True)
def _native():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device")
    from fp8_quantization_amd import _lib
    _lib.load()


def _grid(rng, shape, bias, zero_frac=0.0, lo=3):
    expo = rng.integers(lo, 16, size=shape)
    mant = rng.integers(0, 8, size=shape)
    v = np.ldexp(1.0 + mant / 8.0, expo - bias) * rng.choice([-1.0, 1.0], size=shape)
    v[rng.random(shape) < zero_frac] = 0.0
    return v.astype(np.float32)


class _Both:
    """fn() under each depthwise form (option "dwx": 1 band-staged, 2 fp32 gather, 3 column gather
    over the word image), each paired
    with the word-image form (0) for _same."""

    def __init__(self, fn):
        from fp8_quantization_amd import _lib
        old = _lib.set_option("dwx", 0)
        try:
            self.ref = fn()
            self.runs = []
            for mode in (1, 2, 3):
                _lib.set_option("dwx", mode)
                self.runs.append((mode, fn()))
        finally:
            _lib.set_option("dwx", old)


def _both(fn):
    return _Both(fn)


def _same(both, what):
    def bits(t):
        return t.cpu().numpy() if torch.is_tensor(t) else t
    b = bits(both.ref)
    for mode, a in both.runs:
        a = bits(a)
        same = (a.view(np.uint32) == b.view(np.uint32)) | ((a == 0) & (b == 0))
        assert same.all(), f"{what} (dwx={mode}): {np.count_nonzero(~same)} outputs differ, first at {np.argwhere(~same)[0]}"


# (C, H, stride): the 17 depthwise layers of MobileNetV2 at 224 (distinct shapes)
MBV2_DW = [(32, 112, 1), (96, 112, 2), (144, 56, 1), (144, 56, 2), (192, 28, 1), (192, 28, 2), (384, 14, 1),
           (576, 14, 1), (576, 14, 2), (960, 7, 1)]
TAB = None


def _tab():
    global TAB
    if TAB is None:
        TAB = torch.as_tensor(gio.load("g2_matmul.npz")["E4M3_table_nocomp"])
    return TAB


@pytest.mark.parametrize("C,H,s", MBV2_DW)
def test_mbv2_depthwise_identical(C, H, s):
    from fp8_quantization_amd import approx_conv2d
    rng = np.random.default_rng(C * 7 + H + s)
    bA, bR = 10, 9
    x = torch.from_numpy(_grid(rng, (2, C, H, H), bA, zero_frac=0.4)).to(DEV)
    bW = rng.integers(12, 16, size=C).astype(np.int32)
    w = torch.from_numpy(_grid(rng, (C, 1, 3, 3), bW[:, None, None, None])).to(DEV)
    r = _both(lambda: approx_conv2d(x, w, E, M, bA, torch.from_numpy(bW), bR, _tab(), with_approx=True,
                                    with_s2nn2s_opt=True, quant_btw_mult_accu=True, stride=(s, s),
                                    padding=(1, 1), groups=C))
    _same(r, f"C={C} H={H} s={s}")


@pytest.mark.parametrize("shape", [(3, 5, 9, 9, 1, (3, 3), (1, 1), (1, 1)),
                                   (2, 7, 13, 11, 2, (3, 3), (1, 1), (1, 1)),
                                   (1, 4, 1, 1, 1, (3, 3), (1, 1), (1, 1)),
                                   (2, 6, 10, 7, 1, (5, 3), (2, 1), (2, 1)),
                                   (2, 9, 17, 30, 2, (3, 3), (0, 0), (1, 1)),
                                   (64, 3, 6, 6, 1, (3, 3), (1, 1), (1, 1))])
def test_ragged_shapes_identical(shape):
    from fp8_quantization_amd import approx_conv2d
    Bn, C, H, W, s, k, pad, dil = shape
    rng = np.random.default_rng(Bn * 1000 + C * 10 + H)
    bA, bR = 11, 8
    x = torch.from_numpy(_grid(rng, (Bn, C, H, W), bA, zero_frac=0.3)).to(DEV)
    bW = rng.integers(11, 16, size=C).astype(np.int32)
    w = torch.from_numpy(_grid(rng, (C, 1) + k, bW[:, None, None, None])).to(DEV)
    r = _both(lambda: approx_conv2d(x, w, E, M, bA, torch.from_numpy(bW), bR, _tab(), with_approx=True,
                                    with_s2nn2s_opt=True, quant_btw_mult_accu=True, stride=(s, s), padding=pad,
                                    dilation=dil, groups=C))
    _same(r, f"shape {shape}")


@pytest.mark.parametrize("C,H,s", [(96, 28, 2), (144, 14, 1), (24, 9, 1)])
def test_fused_input_quantizer_and_bn_identical(C, H, s):
    """qin (the layer's E4M3 input quantizer applied inside the kernel) + BN + ReLU6 epilogue;
    the input quantizer's bias is returned identically too."""
    from fp8_quantization_amd import approx_conv2d
    from fp8_quantization_amd.approx_ops import bn_act_epilogue
    rng = np.random.default_rng(C + H)
    x = torch.from_numpy(rng.standard_normal((2, C, H, H)).astype(np.float32)).relu().to(DEV)
    bW = rng.integers(12, 16, size=C).astype(np.int32)
    w = torch.from_numpy(_grid(rng, (C, 1, 3, 3), bW[:, None, None, None])).to(DEV)
    mx = x.abs().max().reshape(1)
    ep = bn_act_epilogue(torch.randn(C, device=DEV) * 0.1, torch.rand(C, device=DEV) + 0.5,
                         torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV) * 0.1, 1e-5, nn.ReLU6())

    def run():
        y, ib, _ = approx_conv2d(x, w, E, M, None, torch.from_numpy(bW), 9, _tab(), with_approx=True,
                                 with_s2nn2s_opt=True, quant_btw_mult_accu=True, stride=(s, s), padding=(1, 1),
                                 groups=C, epilogue=ep, qin=(mx, 8, 3, 1))
        return y.cpu().numpy(), float(ib)
    r = _both(run)
    ys = _Both.__new__(_Both)
    ys.ref, ys.runs = r.ref[0], [(m, v[0]) for m, v in r.runs]
    _same(ys, f"qin C={C} H={H} s={s}")
    assert all(v[1] == r.ref[1] for _, v in r.runs)


def test_off_grid_input_gated_identical():
    from fp8_quantization_amd import approx_conv2d
    rng = np.random.default_rng(5)
    bA, bR = 10, 9
    xn = _grid(rng, (2, 8, 12, 12), bA, zero_frac=0.3)
    xn[1, 3, 5, 6] = 0.3  # off the E4M3 grid: the gate is raised and the exact kernel answers
    x = torch.from_numpy(xn).to(DEV)
    bW = np.full(8, 13, np.int32)
    w = torch.from_numpy(_grid(rng, (8, 1, 3, 3), 13)).to(DEV)
    r = _both(lambda: approx_conv2d(x, w, E, M, bA, torch.from_numpy(bW), bR, _tab(), with_approx=True,
                                    with_s2nn2s_opt=True, quant_btw_mult_accu=True, padding=(1, 1), groups=8))
    _same(r, "off-grid")
