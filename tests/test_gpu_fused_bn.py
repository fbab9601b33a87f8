"""Fused eval-mode BatchNorm + activation epilogue (fp8a_conv2d_bn_act).

The fused store computes act(fma(acc, scale, shift)) on the same accumulator the unfused
launch writes, so the fused output equals the unfused output pushed through
y * scale + shift (rounded once) and the clamp: checked to within one fp32 rounding against a
float64 restatement, over every launch path of the conv entry (unsplit / split-K GEMM,
partial tiles, grouped, depthwise fast / direct / gated fallback, off-grid exact fallback,
v5).  At module level the fused BNFusedHijacker forward is compared with the unfused one
(F.batch_norm + activation module), and the G5 operator fixtures (tests/test_gpu_operator.py)
run through the fused form by default.
"""
import numpy as np
import pytest
import torch
from torch import nn

from oracle import oracle as orc
from tests import golden_io as gio

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _native():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device")
    from fp8_quantization_amd import _lib
    _lib.load()


def _grid(rng, E, M, shape, bias, zero_frac=0.3, bins=8):
    emax = 2 ** E - 1
    expo = rng.integers(max(0, emax - bins), emax + 1, size=shape)
    mant = rng.integers(0, 2 ** M, size=shape)
    v = np.where(expo == 0, np.ldexp(mant / 2 ** M, 1 - bias), np.ldexp(1.0 + mant / 2 ** M, expo - bias))
    v = v * rng.choice([-1.0, 1.0], size=shape)
    v[rng.random(shape) < zero_frac] = 0.0
    return v.astype(np.float32)


def _bn(rng, C):
    mean = rng.normal(0, 0.5, C).astype(np.float32)
    var = rng.uniform(0.2, 3.0, C).astype(np.float32)
    gamma = rng.normal(1, 0.3, C).astype(np.float32)
    beta = rng.normal(0, 0.2, C).astype(np.float32)
    return [torch.from_numpy(a).to(DEV) for a in (mean, var, gamma, beta)]


ACTS = {"none": None, "relu": nn.ReLU(), "relu6": nn.ReLU6(), "hardtanh": nn.Hardtanh(-0.5, 0.75)}


def _expect(y0, ep):
    ss, act, lo, hi = ep
    ss = ss.cpu().numpy().astype(np.float64)
    C = ss.shape[0]
    v = y0.astype(np.float64) * ss[:, 0].reshape(1, C, 1, 1) + ss[:, 1].reshape(1, C, 1, 1)
    if act:
        v = np.minimum(np.maximum(v, lo), hi)
    return v, np.abs(y0.astype(np.float64) * ss[:, 0].reshape(1, C, 1, 1)) + np.abs(ss[:, 1].reshape(1, C, 1, 1))


def _check(x, w, E, M, bA, bW, bR, tab, fl, act, seed, **conv):
    import fp8_quantization_amd as fa
    rng = np.random.default_rng(seed)
    Cout = w.shape[0]
    ep = fa.approx_ops.bn_act_epilogue(*_bn(rng, Cout), 1e-5, ACTS[act])
    args = (torch.from_numpy(x).to(DEV), torch.from_numpy(w).to(DEV), E, M, torch.tensor([bA], device=DEV),
            torch.from_numpy(bW).to(DEV), torch.tensor([bR], device=DEV), torch.as_tensor(tab))
    y0 = fa.approx_conv2d(*args, flags=fl, **conv).cpu().numpy()
    y1 = fa.approx_conv2d(*args, flags=fl, epilogue=ep, **conv).cpu().numpy()
    exp, mag = _expect(y0, ep)
    err = np.abs(y1.astype(np.float64) - exp)
    tol = 2.0 ** -23 * np.abs(exp) + 2.0 ** -45 * mag + 1e-38
    assert np.all(err <= tol), (act, float(np.max(err / (tol + 1e-30))))
    if act != "none":
        assert np.all(y1 >= ep[2]) and np.all(y1 <= ep[3])
    return y0, y1


@pytest.mark.parametrize("act", ["none", "relu", "relu6", "hardtanh"])
@pytest.mark.parametrize("shape", [
    # (Bn, Cin, H, Cout, k, stride, pad, groups): unsplit, split-K (2 tiles, K = 576),
    # a partial N tile (Cout 96), 1x1 stride 2, grouped
    (4, 16, 16, 64, 3, 1, 1, 1), (2, 64, 8, 64, 3, 1, 1, 1), (2, 32, 9, 96, 1, 2, 0, 1), (2, 24, 7, 48, 3, 1, 1, 2)])
def test_fused_epilogue_gemm_paths(shape, act):
    Bn, Cin, H, Cout, k, s, p, g = shape
    E, M = 4, 3
    rng = np.random.default_rng(sum(shape))
    x = _grid(rng, E, M, (Bn, Cin, H, H), 9)
    w = _grid(rng, E, M, (Cout, Cin // g, k, k), 12, zero_frac=0.1)
    bW = rng.integers(11, 14, Cout).astype(np.int32)
    tab = gio.load("g2_matmul.npz")["E4M3_table_nocomp"]
    fl = orc.flags_of(approx=True, s2n=True, qbma=True)
    _check(x, w, E, M, 9, bW, 10, tab, fl, act, Cout, stride=(s, s), padding=(p, p), groups=g)


@pytest.mark.parametrize("act", ["none", "relu6"])
@pytest.mark.parametrize("variant", ["fast", "gclip_direct", "offgrid_fallback", "s2n_off"])
def test_fused_epilogue_depthwise_paths(variant, act):
    E, M = 4, 3
    rng = np.random.default_rng(len(variant))
    C = 32
    x = _grid(rng, E, M, (2, C, 9, 9), 9)
    if variant == "offgrid_fallback":
        x[1, 5, 4, 4] = 0.123456
    w = _grid(rng, E, M, (C, 1, 3, 3), 12, zero_frac=0.0)
    bW = np.full(C, 12, np.int32)
    tab = gio.load("g2_matmul.npz")["E4M3_table_nocomp"]
    fl = orc.flags_of(approx=True, s2n=variant != "s2n_off", qbma=True, gclip=variant == "gclip_direct")
    _check(x, w, E, M, 9, bW, 10, tab, fl, act, 7, padding=(1, 1), groups=C)


def test_fused_epilogue_exact_fallback_gemm():
    E, M = 4, 3
    rng = np.random.default_rng(3)
    x = _grid(rng, E, M, (2, 16, 8, 8), 9)
    x[0, 2, 3, 3] = 0.3141  # off the E4M3 grid: the gated exact kernel recomputes the tile
    w = _grid(rng, E, M, (64, 16, 3, 3), 12)
    bW = np.full(64, 12, np.int32)
    tab = gio.load("g2_matmul.npz")["E4M3_table_nocomp"]
    _check(x, w, E, M, 9, bW, 10, tab, orc.flags_of(approx=True, s2n=True, qbma=True), "relu", 5, padding=(1, 1))


def test_fused_epilogue_v5():
    E, M = 4, 3
    rng = np.random.default_rng(4)
    x = _grid(rng, E, M, (2, 8, 6, 6), 9)
    w = _grid(rng, E, M, (16, 8, 3, 3), 12)
    bW = np.full(16, 12, np.int32)
    tab = gio.load("g2_matmul.npz")["E4M3_table_nocomp"]
    _check(x, w, E, M, 9, bW, 10, tab, orc.flags_v5(), "relu", 6, padding=(1, 1))


def test_bad_epilogue_shape_asserts():
    import fp8_quantization_amd as fa
    x = torch.zeros(1, 4, 4, 4, device=DEV)
    w = torch.zeros(8, 4, 1, 1, device=DEV)
    ep = (torch.zeros(4, 2, device=DEV), 0, 0.0, 0.0)
    with pytest.raises(AssertionError):
        fa.approx_conv2d(x, w, 4, 3, 9, torch.full((8,), 12, dtype=torch.int32, device=DEV), 10, None,
                         with_approx=False, epilogue=ep)


def _module(act, quantize_input):
    from fp8_quantization_amd.approx_calculation import QCustomBNConv2dTorch
    from fp8_quantization_amd.resnet_workload import approx_qparams
    qp = approx_qparams()
    qp["quantize_input"] = quantize_input
    torch.manual_seed(0)
    m = QCustomBNConv2dTorch(in_channels=16, out_channels=48, kernel_size=3, padding=1, bias=False,
                             activation=ACTS[act], **qp)
    with torch.no_grad():
        m.running_mean.normal_(0, 0.3)
        m.running_var.uniform_(0.3, 2.0)
        m.gamma.normal_(1, 0.2)
        m.beta.normal_(0, 0.2)
    return m.to(DEV).eval()


@pytest.mark.parametrize("quantize_input", [True, False])
@pytest.mark.parametrize("act", ["relu", "relu6", "none"])
def test_module_fused_matches_unfused(act, quantize_input):
    m = _module(act, quantize_input)
    m.quantized()
    m.estimate_ranges()
    x = torch.randn(4, 16, 12, 12, device=DEV)
    with torch.no_grad():
        m(x)
    m.fix_ranges()
    assert m._fused_epilogue() is not None
    with torch.no_grad():
        y1 = m(x).cpu().numpy()
        m.fuse_bn_act = False
        assert m._fused_epilogue() is None
        y0 = m(x).cpu().numpy()
    if quantize_input:   # no output quantizer: one fp32 rounding apart
        np.testing.assert_allclose(y1, y0, rtol=4e-7, atol=1e-6 * float(np.abs(y0).max()))
    else:                # the output FP8 quantizer may round a value lying on a tie differently
        diff = y1 != y0
        assert diff.mean() < 1e-3, diff.mean()
        rel = np.abs(y1 - y0)[diff] / np.maximum(np.abs(y0[diff]), 1e-30)
        assert rel.size == 0 or rel.max() <= 0.26


def test_module_cache_follows_running_stats():
    m = _module("relu", True)
    m.quantized()
    m.estimate_ranges()
    with torch.no_grad():
        m(torch.randn(2, 16, 8, 8, device=DEV))
    m.fix_ranges()
    a = m._fused_epilogue()[0].clone()
    with torch.no_grad():
        m.running_var.mul_(4.0)
    b = m._fused_epilogue()[0]
    torch.testing.assert_close(b[:, 0], a[:, 0] / 2, rtol=1e-4, atol=0)
