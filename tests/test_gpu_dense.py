"""The exact (non-approx) product on the block-scaled fp8 matrix core (csrc/gemm_dense.h): the
reference's `x @ y` of FP8-quantized operands (approx_calculation.py:797, 811; config 1).

Bar: |C - C64| <= 1e-5 * sum_k |a_k b_k| (fp32 summation order) against the float64
product, for E4M3 (e4m3 operands) and E5M2 (e5m2) grids over ragged shapes and strides, convs
with stride / padding / dilation; values off the fp8 grid (unquantized, a block spanning more
binades than e4m3 holds) go to the fp32 units and still meet the bar, and exactly their units are
recomputed; NaN / inf propagate as in torch's fp32 product.
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


def _q(x, E, M, per_row=False):
    mx = np.abs(x).max(axis=1) if per_row else np.abs(x).max()
    q, _ = orc.fp8_fake_quant(x, np.maximum(mx, 1e-30), E, M, per_row=per_row)
    return q.astype(np.float32)


def _operands(Mr, K, N, E, M, seed):
    rng = np.random.default_rng(seed)
    A = _q(np.maximum(rng.standard_normal((Mr, K)), 0.0).astype(np.float32) * 3.0, E, M) if K else \
        np.zeros((Mr, 0), np.float32)
    W = (rng.standard_normal((N, K)) * 0.05 * np.exp(rng.standard_normal((N, 1)))).astype(np.float32)
    Wq = _q(W, E, M, per_row=True) if K else W
    return A, np.ascontiguousarray(Wq.T)


def _tame(X):
    """Zero what lies more than 12 binades below its row's largest magnitude (so no 32-k block
    spans more than e4m3 holds): inputs whose fp32-unit count is exactly the off-grid ones."""
    mx = np.abs(X).max(axis=1, keepdims=True)
    return np.where(np.abs(X) >= mx * 2.0 ** -12, X, 0.0).astype(np.float32)


def _check(C, A, B):
    ref = A.astype(np.float64) @ B.astype(np.float64)
    S = np.abs(A.astype(np.float64)) @ np.abs(B.astype(np.float64))
    bad = np.abs(C.astype(np.float64) - ref) > gio.sum_tolerance(S)
    assert not bad.any(), f"{bad.sum()} outputs outside the bar"


FMTS = {"e4m3": (4, 3), "e5m2": (5, 2), "bf16": (4, 3)}  # (the bf16 form on E4M3-grid operands)


def _fmt(name):
    from fp8_quantization_amd import _lib
    return {"e4m3": _lib.DENSE_E4M3, "e5m2": _lib.DENSE_E5M2, "bf16": _lib.DENSE_BF16}[name]


def _stats():
    from fp8_quantization_amd import _lib
    return _lib.dense_stats(reset=True)


@pytest.mark.parametrize("fmt", ["e4m3", "e5m2", "bf16"])
@pytest.mark.parametrize("shape", [(1, 1, 1), (7, 33, 5), (130, 300, 129), (256, 4608, 64), (1000, 147, 1),
                                   (513, 64, 1000), (3, 0, 4)])
@pytest.mark.parametrize("layout", ["rowmajor", "transposed"])
def test_matmul_on_grid(shape, fmt, layout):
    from fp8_quantization_amd import _lib
    from fp8_quantization_amd.approx_ops import dense_matmul
    Mr, K, N = shape
    E, M = FMTS[fmt]
    A, B = _operands(Mr, K, N, E, M, sum(shape) + M)
    if layout == "rowmajor":
        tA, tB = torch.from_numpy(A).to(DEV), torch.from_numpy(B).to(DEV)
    else:  # A as a column-major view, B as weight.t() (the linear layers' operand)
        tA = torch.from_numpy(np.ascontiguousarray(A.T)).to(DEV).t()
        tB = torch.from_numpy(np.ascontiguousarray(B.T)).to(DEV).t()
    _stats()
    _lib.path_stats(reset=True)
    C = dense_matmul(tA, tB, _fmt(fmt)).cpu().numpy()
    st = _stats()
    assert _lib.path_stats(reset=True)["dense"] == 1
    if K == 0:
        assert not C.any()
    _check(C, A, B)
    # on-grid blocks are exact in the fp8 format unless one 32-k block spans more binades than
    # e4m3 holds (a column's 1.875 x 2^e maximum next to its smallest subnormal: ~19 binades vs
    # e4m3's 17.8) -- those few units run in fp32
    units = ((Mr + 127) // 128 * 2) * ((N + 127) // 128 * 2)
    assert st["fp32_units"] <= (0 if fmt == "bf16" else units // 10), st


@pytest.mark.parametrize("fmt", ["e4m3", "e5m2", "bf16"])
def test_off_grid_rows_take_the_fp32_units(fmt):
    from fp8_quantization_amd.approx_ops import dense_matmul
    E, M = FMTS[fmt]
    f = _fmt(fmt)
    Mr, K, N = 300, 200, 129
    A, B = _operands(Mr, K, N, E, M, 11)
    A, B = _tame(A), np.ascontiguousarray(_tame(B.T).T)
    A[70, 5] = np.float32(1.0 + 2.0 ** -20)  # off the grid: row 70 -> row unit 1
    _stats()
    C = dense_matmul(torch.from_numpy(A).to(DEV), torch.from_numpy(B).to(DEV), f).cpu().numpy()
    st = _stats()
    _check(C, A, B)
    assert st == dict(fp32_launches=1, fp32_units=(N + 127) // 128 * 2), st
    # wholly unquantized operands: every unit in fp32, same bar
    rng = np.random.default_rng(3)
    A2 = rng.standard_normal((Mr, K)).astype(np.float32)
    C2 = dense_matmul(torch.from_numpy(A2).to(DEV), torch.from_numpy(B).to(DEV), f).cpu().numpy()
    st = _stats()
    _check(C2, A2, B)
    assert st["fp32_units"] == (Mr + 63) // 64 * ((N + 127) // 128 * 2), st


def test_block_span_beyond_e4m3():
    """An E4M3-grid row whose 32-k block holds its top value and a value 17 binades lower: not
    exact under one e4m3 block scale -> its unit in fp32 (E5M2's range would hold it)."""
    from fp8_quantization_amd import _lib
    from fp8_quantization_amd.approx_ops import dense_matmul
    Mr, K, N = 64, 64, 64
    A, B = _operands(Mr, K, N, 4, 3, 5)
    B = np.ascontiguousarray(_tame(B.T).T)
    A[0, :] = 0.0
    A[0, 0] = np.float32(1.875 * 2.0 ** 3)
    A[0, 1] = np.float32(2.0 ** -14)
    _stats()
    C = dense_matmul(torch.from_numpy(A).to(DEV), torch.from_numpy(B).to(DEV), _lib.DENSE_E4M3).cpu().numpy()
    st = _stats()
    _check(C, A, B)
    assert st["fp32_units"] == 2, st  # (npad = 128: two column units of row unit 0)
    C = dense_matmul(torch.from_numpy(A).to(DEV), torch.from_numpy(B).to(DEV), _lib.DENSE_E5M2).cpu().numpy()
    # (B's E4M3 weights are not all e5m2-exact: the units recompute; the values stay right)
    _check(C, A, B)
    _stats()


def test_non_finite_like_torch():
    from fp8_quantization_amd import _lib
    from fp8_quantization_amd.approx_ops import dense_matmul
    Mr, K, N = 200, 96, 70
    A, B = _operands(Mr, K, N, 4, 3, 9)
    B[:, 3] = 0.0
    A[3, 5] = np.nan
    A[150, 2] = np.inf
    C = dense_matmul(torch.from_numpy(A).to(DEV), torch.from_numpy(B).to(DEV), _lib.DENSE_E4M3).cpu().numpy()
    ref = (torch.from_numpy(A).double() @ torch.from_numpy(B).double()).numpy()
    assert np.array_equal(np.isnan(C), np.isnan(ref))
    assert np.array_equal(np.isinf(C), np.isinf(ref)) and np.array_equal(np.sign(C[np.isinf(C)]), np.sign(ref[np.isinf(ref)]))
    fin = np.isfinite(ref)
    S = np.abs(A.astype(np.float64)) @ np.abs(B.astype(np.float64))
    with np.errstate(invalid="ignore"):
        assert np.all(np.abs(C[fin] - ref[fin]) <= gio.sum_tolerance(S[fin]))
    _stats()


@pytest.mark.parametrize("fmt", ["e4m3", "e5m2", "bf16"])
@pytest.mark.parametrize("geo", [
    # (Bn, Cin, H, W, Cout, kh, kw, stride, padding, dilation)
    (2, 16, 15, 17, 24, 3, 3, (2, 1), (1, 2), (1, 2)),
    (3, 64, 14, 14, 96, 1, 1, (1, 1), (0, 0), (1, 1)),
    (1, 256, 9, 9, 130, 3, 3, (1, 1), (1, 1), (1, 1)),
    (4, 3, 32, 32, 32, 3, 3, (2, 2), (1, 1), (1, 1)),
])
def test_conv_on_grid(geo, fmt):
    from fp8_quantization_amd import _lib
    from fp8_quantization_amd.approx_ops import dense_conv2d
    Bn, Cin, H, W, Cout, kh, kw, st, pd, dl = geo
    E, M = FMTS[fmt]
    rng = np.random.default_rng(Cin + Cout)
    x = _q(np.maximum(rng.standard_normal((Bn, Cin, H, W)), 0).astype(np.float32), E, M)
    w = _q((rng.standard_normal((Cout, Cin * kh * kw)) * 0.1).astype(np.float32), E, M, per_row=True)
    w = _tame(w).reshape(Cout, Cin, kh, kw)
    _stats()
    y = dense_conv2d(torch.from_numpy(x).to(DEV), torch.from_numpy(w).to(DEV), _fmt(fmt), st, pd, dl).cpu().numpy()
    stt = _stats()
    tx, tw = torch.from_numpy(x).double(), torch.from_numpy(w).double()
    ref = F.conv2d(tx, tw, None, st, pd, dl).numpy()
    S = F.conv2d(tx.abs(), tw.abs(), None, st, pd, dl).numpy()
    assert y.shape == ref.shape
    bad = np.abs(y.astype(np.float64) - ref) > gio.sum_tolerance(S)
    assert not bad.any(), f"{bad.sum()} outputs outside the bar"
    assert stt["fp32_units"] == 0, stt  # (weights within 12 binades of their channel's largest)


def test_module_exact_branch_runs_dense():
    """QCustomBNConv2dTorch / QCustomLinearTorch with approx_flag off route their exact product
    through the dense path once their operands are FP8-quantized (state flags on), matching
    F.conv2d / x @ y; with quantization off the product stays torch's fp32 contraction."""
    from fp8_quantization_amd import _lib
    from fp8_quantization_amd.approx_calculation import QCustomBNConv2dTorch, QCustomLinearTorch
    from fp8_quantization_amd.resnet_workload import approx_qparams
    torch.manual_seed(2)
    kw = approx_qparams(expo_width=4, mant_width=3, dnsmp_factor=3, withComp=False, with_approx=False)
    conv = QCustomBNConv2dTorch(in_channels=32, out_channels=48, kernel_size=3, padding=1, bias=False, **kw).to(DEV)
    lin = QCustomLinearTorch(in_features=96, out_features=40, bias=True, **kw).to(DEV)
    for m in (conv, lin):
        m.eval()
        m.approx_flag = False
    x = torch.relu(torch.randn(2, 32, 10, 10, device=DEV))
    z = torch.relu(torch.randn(8, 96, device=DEV))
    _lib.path_stats(reset=True)
    with torch.no_grad():
        w = conv.weight.detach()
        conv.run_forward(x, w, None)
        lin.run_forward(z, lin.weight.detach(), lin.bias.detach())
    assert _lib.path_stats(reset=True)["dense"] == 0  # quantization off: torch's contraction
    for m in (conv, lin):
        m.quantized()
    with torch.no_grad():
        y = conv.run_forward(x, w, None)
        yl = lin.run_forward(z, lin.weight.detach(), lin.bias.detach())
    assert _lib.path_stats(reset=True)["dense"] == 2
    # unquantized operands here: every unit is in fp32 -- still the torch product up to order
    ref = F.conv2d(x.double(), w.double(), None, 1, 1)
    S = F.conv2d(x.double().abs(), w.double().abs(), None, 1, 1)
    assert torch.all((y.double() - ref).abs() <= 1e-5 * S + 1e-30)
    refl = z.double() @ lin.weight.double().t() + lin.bias.double()
    Sl = z.double().abs() @ lin.weight.double().abs().t() + lin.bias.double().abs()
    assert torch.all((yl.double() - refl).abs() <= 1e-5 * Sl + 1e-30)
    _stats()


@pytest.mark.parametrize("fmt", ["e4m3", "e5m2", "bf16"])
def test_wide_range_pairs_exact(fmt):
    """Every pair of positions (i, j) of a 32-k block: 2^8 at i and 2^-9 at j (17 binades apart,
    both exact in the block's fp8 format) must sum exactly -- the matrix core's narrow first
    summation stage never sees two of them (one value per 8-byte operand group)."""
    from fp8_quantization_amd import _lib
    from fp8_quantization_amd.approx_ops import dense_matmul
    pairs = [(i, j) for i in range(32) for j in range(32) if i != j]
    lo = 2.0 ** -9 if fmt == "e4m3" else 2.0 ** -14  # (bf16: 2^-14 too)
    A = np.zeros((len(pairs), 64), np.float32)
    for r, (i, j) in enumerate(pairs):
        A[r, i] = 256.0
        A[r, 32 + j] = 256.0  # (the second block: the same pattern)
        A[r, j] = lo
        A[r, 32 + i] = lo
    B = np.ones((64, 16), np.float32)
    _stats()
    C = dense_matmul(torch.from_numpy(A).to(DEV), torch.from_numpy(B).to(DEV), _fmt(fmt)).cpu().numpy()
    assert _stats()["fp32_units"] == 0
    want = np.float32(512.0 + 2 * lo)
    bad = [pairs[r] for r in range(len(pairs)) if C[r, 0] != want]
    assert not bad, f"{len(bad)} pairs lose the small product, e.g. {bad[:8]}"


def test_bf16_form_has_no_range_limit():
    """The bf16 form holds a whole E4M3 tensor's range (and E3M4 / E2M5 values) in one block:
    no fp32 units where the e4m3 form needs them."""
    from fp8_quantization_amd import _lib
    from fp8_quantization_amd.approx_ops import dense_matmul
    for (E, M) in ((4, 3), (3, 4), (2, 5)):
        A, B = _operands(300, 256, 96, E, M, E)
        A[:, 0] = np.float32(1.875 * 2.0 ** 3)
        A[:, 1] = np.float32(2.0 ** -14)
        _stats()
        C = dense_matmul(torch.from_numpy(A).to(DEV), torch.from_numpy(B).to(DEV), _lib.DENSE_BF16).cpu().numpy()
        assert _stats()["fp32_units"] == 0
        _check(C, A, B)
