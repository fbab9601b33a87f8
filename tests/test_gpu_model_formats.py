"""Network-level parity of every approx product, per format (BASELINE configs 2 and 5).

A ResNet-18 and a ResNet-50 (random init, BN statistics from synthetic batches, 64x64 inputs)
are quantized as E4M3 / E3M4 / E2M5 approx_v9 (dnsmp_factor 3, withComp False: the E4M3 8x8
{0,1}, E3M4 16x16 and E2M5 32x32 error tables, s2n, qbma) and as E5M2 (BASELINE config 5's
expo_width = 5 point: the reference has no E5M2 table and raises, approx_matmul_whole_v9.py:588-590,
so it runs with the opt-in all-zero table, zero_table_ext; its arithmetic is pinned by the E5M2
G1 / G2 fixtures through the oracle), calibrated on one batch and run in the fixed-range state.  Two checks:
  * every approx product of the forward (ResNet-18: 20 convs + fc; ResNet-50: 53 convs + fc),
    run unfused so its operands are
    visible, against the CPU oracle on the captured operands and biases (im2col for convs):
    sums within 1e-5 * sum|term|; this pins the whole network's data, biases included, through
    the GPU path layer by layer;
  * the fused forward (input quantization and residual tails in the kernels) gives logits
    bit-identical to the unfused one (the BN + ReLU epilogue on in both: it is within one fp32
    rounding of F.batch_norm, not bit-identical -- tests/test_gpu_fused_bn.py).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

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


def _model(E, M, arch="resnet18", batch=2):
    from fp8_quantization_amd import resnet_workload as rw
    torch.manual_seed(E * 10 + M)
    m = getattr(rw, arch + "_approx")(bn_stats_batches=2, device=DEV, expo_width=E, mant_width=M, withComp=False)
    m = m.to(DEV).eval()
    g = torch.Generator().manual_seed(5)
    m.quantized()
    m.estimate_ranges()
    with torch.no_grad():
        m(torch.randn((4, 3, 64, 64), generator=g).to(DEV))
    m.fix_ranges()
    return m, torch.randn((batch, 3, 64, 64), generator=g).to(DEV)


def _ib(t):
    return int(t.reshape(-1)[0].item()) if isinstance(t, torch.Tensor) else int(t)


@pytest.mark.parametrize("fmt", [(4, 3), (3, 4), (2, 5), (5, 2)], ids=["E4M3", "E3M4", "E2M5", "E5M2"])
@pytest.mark.parametrize("arch", ["resnet18", "resnet50"])
def test_resnet_layers_match_oracle(arch, fmt, monkeypatch):
    from fp8_quantization_amd import approx_calculation as ac
    from fp8_quantization_amd import model_wrap
    from fp8_quantization_amd.quantization.hijacker import QuantizationHijacker
    from fp8_quantization_amd.quantization.quantized_folded_bn import BNFusedHijacker
    E, M = fmt
    model, x = _model(E, M, arch, batch=2 if arch == "resnet18" else 1)

    with torch.no_grad():
        fused = model(x).cpu().numpy()

    # the input-quantizer, block-tail and linear fusions are bit-identical to the separate passes;
    # the BN epilogue (fma(acc, scale, shift)) is within one fp32 rounding of F.batch_norm, so the
    # bit comparison keeps it on, and the operand capture below runs with it off
    monkeypatch.setattr(QuantizationHijacker, "fuse_input_quant", False)
    monkeypatch.setattr(model_wrap, "FUSE_BLOCK", False)
    monkeypatch.setattr(ac.ApproxLinearMixin, "fuse_linear_block", False)
    with torch.no_grad():
        unfused = model(x).cpu().numpy()
    assert np.array_equal(fused.view(np.uint32), unfused.view(np.uint32)), "fused and unfused logits differ"
    monkeypatch.setattr(BNFusedHijacker, "fuse_bn_act", False)
    calls = []
    conv0, mm0 = ac.approx_conv2d, ac.approx_matmul

    def conv(xq, w, E_, M_, bA, bW, bR, table=None, **kw):
        y = conv0(xq, w, E_, M_, bA, bW, bR, table, **kw)
        calls.append(("conv", xq.cpu(), w.cpu(), bA, bW, bR, table, kw, y.cpu()))
        return y

    def mm(a, b, E_, M_, bA, bB, bR, table=None, **kw):
        c = mm0(a, b, E_, M_, bA, bB, bR, table, **kw)
        calls.append(("mm", a.cpu(), b.cpu(), bA, bB, bR, table, kw, c.cpu()))
        return c

    monkeypatch.setattr(ac, "approx_conv2d", conv)
    monkeypatch.setattr(ac, "approx_matmul", mm)
    with torch.no_grad():
        model(x)
    assert len(calls) == (21 if arch == "resnet18" else 54), len(calls)  # convs + fc

    for i, (kind, a, b, bA, bB, bR, table, kw, out) in enumerate(calls):
        tab = np.ascontiguousarray(table.numpy(), np.int32)
        fl = int(kw["flags"])
        bBv = (bB.reshape(-1).cpu().numpy() if isinstance(bB, torch.Tensor) else np.array([bB])).astype(np.int32)
        if kind == "conv":
            assert kw.get("groups", 1) == 1 and kw.get("epilogue") is None
            cols = F.unfold(a, b.shape[2:], dilation=kw["dilation"], padding=kw["padding"], stride=kw["stride"])
            A = cols.transpose(1, 2).reshape(-1, cols.shape[1]).numpy()
            B = b.reshape(b.shape[0], -1).t().contiguous().numpy()
            got = out.permute(0, 2, 3, 1).reshape(-1, b.shape[0]).numpy()
        else:
            A, B, got = a.numpy(), b.contiguous().numpy(), out.numpy()
        ref, S = orc.matmul(A, B, E, M, _ib(bA), bBv, _ib(bR), tab, fl, with_abs=True)
        bad = np.abs(got.astype(np.float64) - ref) > gio.sum_tolerance(S.astype(np.float64))
        assert not bad.any(), f"layer {i} ({kind} {tuple(b.shape)}): {np.count_nonzero(bad)} outputs outside the bar"
