"""Per-layer parity of MobileNetV2 (BASELINE config 3) in the formats and modes G8 cannot pin.

A MobileNetV2 (width 0.5, 64x64 inputs, random init, BN statistics from synthetic batches) is
quantized, calibrated on one batch and run in the fixed-range state, unfused so every approx
product's operands are visible; each product (pointwise / strided convs, the depthwise convs --
single-output-channel groups, i.e. the reference's tensor-bias semantics, approx_calculation.py:
800-809 -- and the classifier) is checked against the CPU oracle on the captured operands and
biases (per group, im2col): sums within 1e-5 * sum|term|.  Before that, the fused forward must
give logits bit-identical to the unfused one (input quantization, block tails and the linear
fusion off; the BN epilogue, within one fp32 rounding of F.batch_norm, on in both).

Modes: E5M2 approx_v9 with the opt-in zero table (BASELINE config 3's format, which the
reference rejects: SURVEY F3); E5M2 in the v5 integer-adder mode with sim_hw_add_OFUF +
with_OF_opt + with_UF_opt live (config 3's switches; v9 ignores them; v5 has no
tensor-bias semantics, so its depthwise groups run the int-bias form); E4M3 approx_v9 (the
depthwise E4M3 table kernel) for comparison.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import oracle as orc
from tests import golden_io as gio

pytestmark = pytest.mark.gpu
DEV = "cuda:0"

MODES = {
    "e5m2_v9": dict(expo_width=5, mant_width=2),
    "e5m2_v5_ofuf": dict(expo_width=5, mant_width=2, withComp=True, approx_version=5, sim_hw_add_OFUF=True,
                         with_OF_opt=True, with_UF_opt=True),
    "e4m3_v9": dict(expo_width=4, mant_width=3),
}


@pytest.fixture(scope="module", autouse=True)
def _native():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device")
    from fp8_quantization_amd import _lib
    _lib.load()


def _ib(t):
    return int(t.reshape(-1)[0].item()) if isinstance(t, torch.Tensor) else int(t)


def _model(cfg):
    from fp8_quantization_amd.mobilenet_workload import mobilenet_v2_approx
    torch.manual_seed(31)
    m = mobilenet_v2_approx(input_size=64, width_mult=0.5, n_class=100, bn_stats_batches=2, device=DEV,
                            **dict(dict(withComp=False), **cfg)).to(DEV).eval()
    g = torch.Generator().manual_seed(6)
    m.quantized()
    m.estimate_ranges()
    with torch.no_grad():
        m(torch.randn((4, 3, 64, 64), generator=g).to(DEV))
    m.fix_ranges()
    return m, torch.randn((2, 3, 64, 64), generator=g).to(DEV)


def check_layer(kind, a, b, bA, bB, bR, table, kw, out, E, M):
    """One captured approx product vs the oracle (per group for convs)."""
    tab = np.ascontiguousarray(table.numpy(), np.int32)
    fl = int(kw["flags"])
    bBv = (bB.reshape(-1).cpu().numpy() if isinstance(bB, torch.Tensor) else np.array([bB])).astype(np.int32)
    if kind == "mm":
        ref, S = orc.matmul(a.numpy(), b.contiguous().numpy(), E, M, _ib(bA), bBv, _ib(bR), tab, fl, with_abs=True)
        return out.numpy(), ref, S
    g = kw.get("groups", 1)
    cin_g, cout_g = a.shape[1] // g, b.shape[0] // g
    got = out.permute(0, 2, 3, 1).reshape(-1, b.shape[0]).numpy()
    refs, sums = [], []
    for j in range(g):
        xs = a[:, j * cin_g:(j + 1) * cin_g]
        cols = F.unfold(xs, b.shape[2:], dilation=kw["dilation"], padding=kw["padding"], stride=kw["stride"])
        A = cols.transpose(1, 2).reshape(-1, cols.shape[1]).numpy()
        B = b[j * cout_g:(j + 1) * cout_g].reshape(cout_g, -1).t().contiguous().numpy()
        bb = bBv[j * cout_g:(j + 1) * cout_g] if bBv.size > 1 else bBv
        tb = cout_g == 1 and not (fl & orc.V5)  # single-column groups: the tensor-bias semantics
        r, s = orc.matmul(A, B, E, M, _ib(bA), bb, _ib(bR), tab, fl | (orc.TB if tb else 0), with_abs=True)
        refs.append(r)
        sums.append(s)
    return got, np.concatenate(refs, axis=1), np.concatenate(sums, axis=1)


@pytest.mark.parametrize("mode", list(MODES))
def test_mobilenet_v2_layers_match_oracle(mode, monkeypatch):
    from fp8_quantization_amd import approx_calculation as ac
    from fp8_quantization_amd import model_wrap
    from fp8_quantization_amd.quantization.hijacker import QuantizationHijacker
    from fp8_quantization_amd.quantization.quantized_folded_bn import BNFusedHijacker
    cfg = MODES[mode]
    E, M = cfg["expo_width"], cfg["mant_width"]
    model, x = _model(cfg)
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
    assert len(calls) == 53, len(calls)  # 52 convs (17 depthwise) + classifier
    assert sum(1 for c in calls if c[0] == "conv" and c[7].get("groups", 1) > 1) == 17
    for i, (kind, a, b, bA, bB, bR, table, kw, out) in enumerate(calls):
        got, ref, S = check_layer(kind, a, b, bA, bB, bR, table, kw, out, E, M)
        bad = np.abs(got.astype(np.float64) - ref) > gio.sum_tolerance(S.astype(np.float64))
        assert not bad.any(), f"layer {i} ({kind} {tuple(b.shape)}): {np.count_nonzero(bad)} outputs outside the bar"
