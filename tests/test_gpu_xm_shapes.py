"""gemm_f8mx_kernel's tile shapes and its fp32-A staging (csrc/gemm_f8mx.h, XmCfg / AF32).

The narrow tiles (128 x 32, 256 x 16 outputs) and the in-kernel A decode (1x1 convs and matrix
A read as fp32, decoded while staged, instead of by the xm_decode_a pre-pass) change only the
schedule: every output is summed in the same order, so results must be BIT-identical to the
128 x 64 / pre-pass form (options "xm_ncg" = 4, "af32_maxct" = 0), and the oracle bar holds.
Covered: MobileNetV2's pointwise shapes (N = 16, 24, 32, 96, 160, 320), ragged M / N / K,
strided matrix rows (lda > K), split-K, the fused input quantizer (qin) with BN + ReLU6, a 1x1
stride-2 downsample, and off-grid A values caught by the in-kernel decode (fallback marks).
"""
import numpy as np
import pytest
import torch
from torch import nn

from oracle import oracle as orc
from tests import golden_io as gio
from tests.test_gpu_f8mx import FL, _close, _conv_raw, _conv_ref, _grid, _matmul_raw, _nhwc, _tab

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
E, M = 4, 3


@pytest.fixture(scope="module", autouse=True)
def _native():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device")
    from fp8_quantization_amd import _lib
    _lib.load()


def _with(opts, fn):
    from fp8_quantization_amd import _lib
    old = {k: _lib.set_option(k, v) for k, v in opts.items()}
    try:
        return fn()
    finally:
        for k, v in old.items():
            _lib.set_option(k, v)


WIDE = {"xm_ncg": 4, "af32_maxct": 0}               # the round-2 schedule
VARIANTS = [{"xm_ncg": 0, "af32_maxct": 1},          # the default choice
            {"xm_ncg": 0, "af32_maxct": 3},
            {"xm_ncg": 1, "af32_maxct": 64}, {"xm_ncg": 2, "af32_maxct": 64}, {"xm_ncg": 4, "af32_maxct": 64},
            {"xm_ncg": 1, "af32_maxct": 0}, {"xm_ncg": 2, "af32_maxct": 0}]


def _bits_equal(a, b, what):
    same = a.view(np.uint32) == b.view(np.uint32)
    assert same.all(), f"{what}: {np.count_nonzero(~same)} outputs differ, first at {np.argwhere(~same)[0]}"


@pytest.mark.parametrize("cfg", [
    dict(B=2, cin=32, cout=16, k=1, s=1, hw=20),     # MobileNetV2 projection, N = 16
    dict(B=2, cin=96, cout=24, k=1, s=1, hw=14),     # N = 24
    dict(B=3, cin=144, cout=32, k=1, s=1, hw=9),     # N = 32, ragged M
    dict(B=2, cin=384, cout=96, k=1, s=1, hw=7),     # N = 96
    dict(B=2, cin=576, cout=160, k=1, s=1, hw=7),    # N = 160
    dict(B=1, cin=960, cout=320, k=1, s=1, hw=7),    # N = 320
    dict(B=2, cin=13, cout=40, k=1, s=1, hw=11),     # K % 8 != 0, N = 40
    dict(B=2, cin=24, cout=48, k=1, s=2, hw=16),     # 1x1 stride-2 downsample
    dict(B=1, cin=2304, cout=24, k=1, s=1, hw=6),    # split-K on the in-kernel decode
    dict(B=2, cin=16, cout=24, k=3, s=1, hw=12),     # 3x3 (pre-pass word image) on a narrow tile
])
def test_conv_schedules_identical(cfg):
    rng = np.random.default_rng(cfg["cin"] * 7 + cfg["cout"])
    bA, bR = 10, 7
    x = _grid(rng, (cfg["B"], cfg["cin"], cfg["hw"], cfg["hw"]), bA, zero_frac=0.4, lo_code=1)
    bW = rng.integers(14, 17, size=cfg["cout"]).astype(np.int32)
    w = _grid(rng, (cfg["cout"], cfg["cin"], cfg["k"], cfg["k"]), bW[:, None, None, None], lo_code=2)
    pad = cfg["k"] // 2
    args = (cfg["s"], pad, 1, 1)
    base, flag = _with(WIDE, lambda: _conv_raw(x, w, bA, bW, bR, _tab(), FL, *args))
    assert flag == 0
    for v in VARIANTS:
        y, f = _with(v, lambda: _conv_raw(x, w, bA, bW, bR, _tab(), FL, *args))
        assert f == 0, f"{v}: fallback flag raised"
        _bits_equal(y, base, f"{cfg} {v}")
    if cfg["cin"] * cfg["cout"] <= 40000:
        ref, S = _conv_ref(x, w, bA, bW, bR, _tab(), FL, *args)
        _close(_nhwc(base), ref, S, str(cfg))


@pytest.mark.parametrize("shape", [(130, 300, 129), (257, 17, 5), (300, 64, 16), (1, 64, 1), (600, 96, 24)])
def test_matmul_schedules_identical(shape):
    Mr, K, N = shape
    rng = np.random.default_rng(Mr * 3 + K + N)
    bA, bR = 10, 7
    lda = K + 7
    Afull = _grid(rng, (Mr, lda), bA, zero_frac=0.4)
    bB = rng.integers(14, 17, size=N).astype(np.int32)
    W = _grid(rng, (N, K), bB[:, None])
    base, flag = _with(WIDE, lambda: _matmul_raw(Afull, lda, W, 1, K, Mr, N, K, bA, bB, bR, _tab(), FL))
    assert flag == 0
    for v in VARIANTS:
        C, f = _with(v, lambda: _matmul_raw(Afull, lda, W, 1, K, Mr, N, K, bA, bB, bR, _tab(), FL))
        assert f == 0
        _bits_equal(C, base, f"{shape} {v}")
    ref, S = orc.matmul(Afull[:, :K], W.T, E, M, bA, bB, bR, _tab(), FL, with_abs=True)
    _close(base, ref, S, str(shape))


@pytest.mark.parametrize("cin,cout,hw", [(96, 24, 14), (192, 64, 7), (32, 16, 10)])
def test_fused_input_quantizer_identical(cin, cout, hw):
    """qin (the E4M3 input quantizer applied to unquantized x inside the op) + BN + ReLU6: the
    in-kernel decode quantizes while staging; outputs and the quantizer's bias are identical."""
    from fp8_quantization_amd import approx_conv2d
    from fp8_quantization_amd.approx_ops import bn_act_epilogue
    rng = np.random.default_rng(cin + cout)
    x = torch.from_numpy(rng.standard_normal((2, cin, hw, hw)).astype(np.float32)).to(DEV)
    bW = rng.integers(14, 17, size=cout).astype(np.int32)
    w = torch.from_numpy(_grid(rng, (cout, cin, 1, 1), bW[:, None, None, None])).to(DEV)
    mx = x.abs().max().reshape(1)
    ep = bn_act_epilogue(torch.randn(cout, device=DEV) * 0.1, torch.rand(cout, device=DEV) + 0.5,
                         torch.rand(cout, device=DEV) + 0.5, torch.randn(cout, device=DEV) * 0.1, 1e-5, nn.ReLU6())

    def run():
        y, ib, _ = approx_conv2d(x, w, E, M, None, torch.from_numpy(bW), 9, torch.as_tensor(_tab()), with_approx=True,
                                 with_s2nn2s_opt=True, quant_btw_mult_accu=True, epilogue=ep, qin=(mx, 8, 3, 1))
        torch.cuda.synchronize()
        return y.cpu().numpy(), float(ib)
    base, bb = _with(WIDE, run)
    for v in VARIANTS:
        y, b = _with(v, run)
        _bits_equal(y, base, f"qin {cin}x{cout} {v}")
        assert b == bb


def test_in_kernel_decode_falls_back():
    """An off-grid activation of a 1x1 conv, seen by the in-kernel decode: the tile is marked,
    the flag raised, and the gated exact kernel's result is returned (oracle bar)."""
    rng = np.random.default_rng(3)
    bA, bR = 10, 7
    x = _grid(rng, (2, 32, 10, 10), bA, zero_frac=0.3)
    x[1, 5, 3, 7] = 0.3
    bW = np.full(24, 15, np.int32)
    w = _grid(rng, (24, 32, 1, 1), 15)
    for v in ({"xm_ncg": 0, "af32_maxct": 1}, {"xm_ncg": 1, "af32_maxct": 64}):
        y, flag = _with(v, lambda: _conv_raw(x, w, bA, bW, bR, _tab(), FL, 1, 0, 1, 1))
        assert flag != 0, f"{v}: the in-kernel decode did not flag the launch"
        ref, S = _conv_ref(x, w, bA, bW, bR, _tab(), FL, 1, 0, 1, 1)
        _close(_nhwc(y), ref, S, str(v))
