"""Fused input quantization (fp8a_conv2d_qin; hijacker.py `_fused_input_quantizer`).

Also the residual-block tail fused into the last conv's store (fp8a_conv2d_block,
model_wrap.fused_block_tail): logits with it on and off.

In the fixed-range approx forward the layer's input fake-quant (quantize_to_fp8_ste_MM,
fp8_quantizer.py:97-173) runs inside the approx op: inside the operand pre-decode of the E4M3
matrix-core (E4M3 / E5M2, the E3M4 / E2M5 tile-table, the v5 word) and tensor-bias table kernels and
of the v5 depthwise word form, or as one fake-quant pass into the workspace for every other path.  Checked here, bit for bit, against the unfused sequence (fp8a_fp8_quantize, then the
plain convolution): outputs, the quantizer's float / int32 bias, every path (E4M3, E3M4, E2M5
and v5 E5M2 GEMM and depthwise, with and without the BN epilogue); and at model level,
logits with the fusion on and off.
"""
import numpy as np
import pytest
import torch

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


@pytest.mark.parametrize("fmt", [(4, 3, "E4M3", "nocomp"), (3, 4, "E3M4", "comp3"), (2, 5, "E2M5", "comp5"),
                                 (2, 5, "E2M5", "nocomp"), (5, 2, "E5M2", "v5"), (5, 2, "E5M2", "v5_of_uf")])
@pytest.mark.parametrize("layer", ["gemm", "depthwise", "depthwise_s2", "conv1x1"])
@pytest.mark.parametrize("bn", [False, True])
def test_fused_equals_quantize_then_conv(fmt, layer, bn):
    from fp8_quantization_amd.approx_ops import approx_conv2d, bn_act_epilogue, fp8_fake_quantize
    E, M, fname, tname = fmt
    rng = np.random.default_rng(E * 1000 + sum(map(ord, layer)) * 2 + int(bn))
    C = 24
    if layer == "gemm":
        x = rng.standard_normal((2, C, 13, 13)).astype(np.float32)
        w_shape, groups, stride, pad = (40, C, 3, 3), 1, 1, 1
    elif layer == "conv1x1":
        x = rng.standard_normal((2, C, 9, 9)).astype(np.float32)
        w_shape, groups, stride, pad = (32, C, 1, 1), 1, 2, 0
    else:
        x = rng.standard_normal((2, C, 15, 15)).astype(np.float32)
        w_shape, groups, stride, pad = (C, 1, 3, 3), C, (2 if layer.endswith("s2") else 1), 1
    x = np.maximum(x, 0) * 0.7
    xt = torch.from_numpy(x).to(DEV)
    maxval = torch.tensor([float(x.max()) * 0.9], device=DEV)  # some values clip
    # per-channel quantized weights, as the weight quantizer gives them
    wf = torch.from_numpy((rng.standard_normal(w_shape) * 0.1).astype(np.float32)).to(DEV)
    wmax = wf.abs().reshape(w_shape[0], -1).amax(1)
    wq, wb = fp8_fake_quantize(wf, wmax, 8, M, per_row=True)
    bR = torch.tensor([2 ** (E - 1) + 6], dtype=torch.int32, device=DEV)
    if tname.startswith("v5"):  # the v5 adder model with the wrap (its matrix-core form) and its options
        tab = np.zeros((4, 4), np.int32)
        tab[1:, 1:] = rng.integers(-3, 4, (3, 3))
        fl = orc.flags_v5(True, tname == "v5_of_uf", tname == "v5_of_uf")
    else:
        tab = gio.load("g2_matmul.npz")[f"{fname}_table_{tname}"]
        fl = orc.flags_of(approx=True, s2n=True, qbma=True)
    ep = None
    if bn:
        cout = w_shape[0]
        g = torch.Generator().manual_seed(1)
        ep = bn_act_epilogue(torch.randn(cout, generator=g).to(DEV) * 0.1, torch.rand(cout, generator=g).to(DEV) + 0.5,
                             torch.randn(cout, generator=g).to(DEV), torch.randn(cout, generator=g).to(DEV) * 0.1,
                             1e-5, torch.nn.ReLU())
    args = dict(flags=fl, stride=(stride, stride), padding=(pad, pad), groups=groups, epilogue=ep)
    xq, xb = fp8_fake_quantize(xt, maxval, 8, M)
    y_ref = approx_conv2d(xq, wq, E, M, xb, wb, bR, torch.as_tensor(tab), **args)
    y, b, _ = approx_conv2d(xt, wq, E, M, None, wb, bR, torch.as_tensor(tab), qin=(maxval, 8, M, 1), **args)
    torch.cuda.synchronize()
    assert torch.equal(b, xb), "quantizer bias differs"
    assert torch.equal(b._fp8a_i32, xb._fp8a_i32), "int32 quantizer bias differs"
    assert torch.equal(y.view(torch.int32), y_ref.view(torch.int32)), f"{layer} {fname}: fused result differs"


@pytest.mark.parametrize("arch", ["resnet18", "resnet50", "mobilenet_v2"])
def test_model_logits_identical_with_and_without_fusion(arch):
    from fp8_quantization_amd import model_wrap
    from fp8_quantization_amd.mobilenet_workload import mobilenet_v2_approx
    from fp8_quantization_amd.quantization.hijacker import QuantizationHijacker
    from fp8_quantization_amd.approx_calculation import ApproxLinearMixin
    from fp8_quantization_amd.resnet_workload import resnet18_approx, resnet50_approx
    torch.manual_seed(0)
    if arch.startswith("resnet"):
        model = (resnet18_approx if arch == "resnet18" else resnet50_approx)(bn_stats_batches=1, device=DEV)
        shape = (3, 64, 64)
    else:
        model = mobilenet_v2_approx(input_size=64, bn_stats_batches=1, device=DEV)
        shape = (3, 64, 64)
    model = model.to(DEV).eval()
    g = torch.Generator().manual_seed(3)
    cal = torch.randn((4,) + shape, generator=g).to(DEV)
    x = torch.randn((6,) + shape, generator=g).to(DEV)
    with torch.no_grad():
        model.quantized()
        model.estimate_ranges()
        model(cal)
        model.fix_ranges()
        try:
            QuantizationHijacker.fuse_input_quant = False
            model_wrap.FUSE_BLOCK = False
            ApproxLinearMixin.fuse_linear_block = False
            ref = model(x)
            QuantizationHijacker.fuse_input_quant = True
            ApproxLinearMixin.fuse_linear_block = True
            got_qin = model(x)
            model_wrap.FUSE_BLOCK = True
            got = model(x)
        finally:
            QuantizationHijacker.fuse_input_quant = True
            ApproxLinearMixin.fuse_linear_block = True
            model_wrap.FUSE_BLOCK = True
    torch.cuda.synchronize()
    assert torch.equal(got_qin.view(torch.int32), ref.view(torch.int32)), "logits differ with the input fusion on"
    assert torch.equal(got.view(torch.int32), ref.view(torch.int32)), "logits differ with the block fusion on"


@pytest.mark.parametrize("case", ["plain", "splitk", "exact_fallback", "e3m4"])
@pytest.mark.parametrize("tail", ["relu_quant", "quant", "relu"])
def test_block_tail_equals_unfused(case, tail):
    """fp8a_conv2d_block's tail (residual add, clamp, output quantizer) in the GEMM store, the
    split-K reduction and the gated exact kernel, bit for bit against the separate ops."""
    from fp8_quantization_amd.approx_ops import approx_conv2d, bn_act_epilogue, fp8_fake_quantize
    E, M, fname, tname = (3, 4, "E3M4", "comp3") if case == "e3m4" else (4, 3, "E4M3", "nocomp")
    rng = np.random.default_rng(sum(map(ord, case + tail)))
    if case == "splitk":
        x = np.maximum(rng.standard_normal((1, 256, 7, 7)), 0).astype(np.float32)
        w_shape = (128, 256, 3, 3)
    else:
        x = np.maximum(rng.standard_normal((2, 32, 12, 12)), 0).astype(np.float32)
        w_shape = (48, 32, 3, 3)
    xt = torch.from_numpy(x).to(DEV)
    wf = torch.from_numpy((rng.standard_normal(w_shape) * 0.1).astype(np.float32)).to(DEV)
    wq, wb = fp8_fake_quantize(wf, wf.abs().reshape(w_shape[0], -1).amax(1), 8, M, per_row=True)
    if case == "exact_fallback":
        wq[3, 2, 1, 1] = 0.0123  # off the weight grid: the gated exact kernel recomputes the launch
    xq, xb = fp8_fake_quantize(xt, torch.tensor([float(x.max())], device=DEV), 8, M)
    bR = torch.tensor([2 ** (E - 1) + 5], dtype=torch.int32, device=DEV)
    tab = torch.as_tensor(gio.load("g2_matmul.npz")[f"{fname}_table_{tname}"])
    fl = orc.flags_of(approx=True, s2n=True, qbma=True)
    cout = w_shape[0]
    g = torch.Generator().manual_seed(2)
    ep = bn_act_epilogue(torch.randn(cout, generator=g).to(DEV) * 0.1, torch.rand(cout, generator=g).to(DEV) + 0.5,
                         torch.randn(cout, generator=g).to(DEV), torch.randn(cout, generator=g).to(DEV) * 0.1, 1e-5)
    args = dict(flags=fl, padding=(1, 1), epilogue=ep)
    base = approx_conv2d(xq, wq, E, M, xb, wb, bR, tab, **args)
    res = torch.randn(base.shape, generator=g).to(DEV)
    omax = torch.tensor([2.5], device=DEV)
    ref = base + res
    if "relu" in tail:
        ref = torch.relu(ref)
    oq = None
    if "quant" in tail:
        ref, ob_ref = fp8_fake_quantize(ref, omax, 8, M)
        oq = (omax, 8, M, 1)
    clamp = ("relu" in tail)
    y, ib, ob = approx_conv2d(xq, wq, E, M, xb, wb, bR, tab, post=(res, int(clamp), 0.0, float("inf"), oq), **args)
    torch.cuda.synchronize()
    assert ib is None
    if oq is not None:
        assert torch.equal(ob, ob_ref) and torch.equal(ob._fp8a_i32, ob_ref._fp8a_i32)
    ok = (y.view(torch.int32) == ref.view(torch.int32)) | ((y == 0) & (ref == 0))
    assert bool(ok.all()), f"{case} {tail}: {int((~ok).sum())} outputs differ"


_POOL_SHAPES = [(4, 64, 112, 112), (2, 5, 9, 16), (2, 3, 7, 9), (1, 5, 1, 1)]
_POOL_CFGS = [(3, 2, 1), (2, 2, 0), (3, 1, 1)]


# (every combination whose window fits the padded input: torch rejects the others)
@pytest.mark.parametrize("shape,cfg", [(sh, c) for sh in _POOL_SHAPES for c in _POOL_CFGS
                                       if sh[2] + 2 * c[2] >= c[0] and sh[3] + 2 * c[2] >= c[0]])
def test_max_pool2d_matches_torch(shape, cfg):
    """fp8a_max_pool2d (the ResNet stem pooling) against torch's max_pool2d, bit for bit, NaN included."""
    from fp8_quantization_amd.approx_ops import MaxPool2d
    k, s, p = cfg
    g = torch.Generator().manual_seed(sum(shape) + k)
    x = torch.randn(shape, generator=g).to(DEV)
    x.view(-1)[min(7, x.numel() - 1)] = float("nan")
    if x.shape[3] >= 10 and x.shape[2] >= 3:
        x[-1, -1, 1, 0] = float("nan")  # a left-edge window
        x[0, 0, 2, 8] = -0.0  # signed-zero ties keep the first in scan order
        x[0, 0, 2, 9] = 0.0
    mp = MaxPool2d.from_module(torch.nn.MaxPool2d(k, s, p))
    assert isinstance(mp, MaxPool2d)
    y = mp(x)
    ref = torch.nn.functional.max_pool2d(x, k, s, p)
    assert y.shape == ref.shape
    assert torch.equal(torch.isnan(y), torch.isnan(ref))
    assert torch.equal(torch.nan_to_num(y, nan=0.0), torch.nan_to_num(ref, nan=0.0))
