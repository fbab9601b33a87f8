"""Model-level parity for the ViT caller (BASELINE config 4): the reference's
vit_quantized_approx module tree (fp8_quantization_amd/vit_workload.py) on a small ViT
(32x32 images, 8x8 patches -> 17 tokens, hidden 64, 4 heads, MLP 256, 2 layers, 10 classes),
random init, calibrated on one batch and run in the fixed-range approx state.

Checks:
  * every approx product of the forward (per layer Q, K, V, attention output, MLP up / down on
    [B * 17, *] token rows, plus the classifier on the class tokens) against the CPU oracle on the
    captured operands and biases: sums within 1e-5 * sum|term| (the bar of every parity test);
  * the forward is deterministic (bit-identical logits on a second run), and the fused forward
    (input quantizer, bias and residual tails inside fp8a_matmul_block) gives logits
    bit-identical to the unfused one;
  * with the F4 extension switched off the encoder linears raise AssertionError on their 3-D
    inputs, as the reference's do (approx_matmul_whole_v9.py:20).
Reference-side parity of the whole model is unpinned: the reference cannot run this model
under approx_flag; each product is pinned through the oracle instead.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as orc
from tests import golden_io as gio

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
SMALL = dict(image_size=32, patch_size=8, hidden=64, layers=2, heads=4, mlp=256, num_labels=10)


@pytest.fixture(scope="module", autouse=True)
def _native():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device")
    from fp8_quantization_amd import _lib
    _lib.load()


def _model(E, M, flatten=True, with_comp=False):
    from fp8_quantization_amd.vit_workload import vit_b16_approx
    m = vit_b16_approx(flatten_token_rows=flatten, seed=E * 10 + M, expo_width=E, mant_width=M,
                       withComp=with_comp, **SMALL)
    m = m.to(DEV).eval()
    g = torch.Generator().manual_seed(3)
    xcal = torch.randn((4, 3, 32, 32), generator=g).to(DEV)
    xev = torch.randn((3, 3, 32, 32), generator=g).to(DEV)
    return m, xcal, xev


def _calibrate(m, xcal):
    m.quantized()
    m.estimate_ranges()
    with torch.no_grad():
        m(xcal)
    m.fix_ranges()


def _ib(t):
    return int(t.reshape(-1)[0].item()) if isinstance(t, torch.Tensor) else int(t)


@pytest.mark.parametrize("fmt", [(4, 3, False), (3, 4, True)], ids=["E4M3", "E3M4-comp"])
def test_vit_layers_match_oracle(fmt, monkeypatch):
    from fp8_quantization_amd import approx_calculation as ac
    from fp8_quantization_amd import model_wrap
    from fp8_quantization_amd.quantization.hijacker import QuantizationHijacker
    E, M, comp = fmt
    model, xcal, xev = _model(E, M, with_comp=comp)
    _calibrate(model, xcal)
    with torch.no_grad():
        fused = model(xev).cpu().numpy()
        fused2 = model(xev).cpu().numpy()
    assert np.array_equal(fused.view(np.uint32), fused2.view(np.uint32)), "forward is not deterministic"

    # unfused: separate input quantizer, product, bias, residual and block-quantizer passes
    monkeypatch.setattr(QuantizationHijacker, "fuse_input_quant", False)
    monkeypatch.setattr(ac.ApproxLinearMixin, "fuse_linear_block", False)
    monkeypatch.setattr(model_wrap, "FUSE_BLOCK", False)
    calls = []
    mm0 = ac.approx_matmul

    def mm(a, b, E_, M_, bA, bB, bR, table=None, **kw):
        c = mm0(a, b, E_, M_, bA, bB, bR, table, **kw)
        calls.append((a.cpu(), b.cpu(), bA, bB, bR, table, kw, c.cpu()))
        return c

    monkeypatch.setattr(ac, "approx_matmul", mm)
    with torch.no_grad():
        logits = model(xev).cpu().numpy()
    assert np.array_equal(fused.view(np.uint32), logits.view(np.uint32)), "fused and unfused logits differ"
    assert np.isfinite(logits).all()
    assert len(calls) == SMALL["layers"] * 6 + 1, len(calls)

    tokens = (SMALL["image_size"] // SMALL["patch_size"]) ** 2 + 1
    for i, (a, b, bA, bB, bR, table, kw, out) in enumerate(calls):
        rows = xev.shape[0] * (tokens if i < len(calls) - 1 else 1)
        assert a.shape[0] == rows, (i, tuple(a.shape))
        tab = np.ascontiguousarray(table.numpy(), np.int32)
        bBv = (bB.reshape(-1).cpu().numpy() if isinstance(bB, torch.Tensor) else np.array([bB])).astype(np.int32)
        ref, S = orc.matmul(a.numpy(), b.contiguous().numpy(), E, M, _ib(bA), bBv, _ib(bR), tab, int(kw["flags"]),
                            with_abs=True)
        bad = np.abs(out.numpy().astype(np.float64) - ref) > gio.sum_tolerance(S.astype(np.float64))
        assert not bad.any(), f"product {i} {tuple(a.shape)}x{tuple(b.shape)}: {np.count_nonzero(bad)} outside the bar"


def test_vit_without_token_flattening_raises_like_reference():
    model, xcal, _ = _model(4, 3, flatten=False)
    model.quantized()
    model.estimate_ranges()
    with pytest.raises(AssertionError):
        with torch.no_grad():
            model(xcal)


def test_vit_b16_full_size_forward():
    """The real ViT-B/16 shape (224x224, 197 tokens, 12 layers) through calibration and the
    approx forward: finite logits, every approx product launched on [B * 197, *] rows."""
    from fp8_quantization_amd.resnet_workload import approx_layer_shapes
    from fp8_quantization_amd.vit_workload import vit_approx_macs_per_image, vit_b16_approx
    m = vit_b16_approx(seed=0).to(DEV).eval()
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        shapes, hooks = approx_layer_shapes(m)
        _calibrate(m, torch.randn((2, 3, 224, 224), generator=g).to(DEV))
        for h in hooks:
            h.remove()
        out = m(torch.randn((2, 3, 224, 224), generator=g).to(DEV))
    assert out.shape == (2, 1000) and torch.isfinite(out).all()
    assert len(shapes) == 73
    assert sum(Mi * K * N for (_, Mi, K, N, _) in shapes) == vit_approx_macs_per_image()
